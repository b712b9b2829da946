"""Multi-process (gloo, CPU) tests of the view-parallel path's collective logic.

The HIP kernels are exercised by the GPU tests; here the compute engine is the CPU
oracle, so what is tested is exactly ``mvdet_amd.parallel``: view ownership, the
rank-major slot order, the in-place all-gather of the slab, row bands and the
assembly of the map bands — for uneven view splits (empty slots) and B > 1.
"""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mvdet_amd import parallel
from oracle import cpu_path, fixtures, kornia_warp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleEngine:
    """CPU stand-in for ``pipeline.ProjectFuse`` built on the oracle (test only)."""

    def __init__(self, proj_mats, src_hw, grid_hw, C, params, slot_views, all_views=True, parts=None,
                 part_channels=None):
        self.pm, self.src_hw, self.grid_hw, self.C, self.params = proj_mats, src_hw, grid_hw, C, params
        self.slot_views = slot_views
        # channel parts (ViewPartialSum's split): camera s = channels [c0, c0 + part_channels) of view v
        self.parts, self.cp = parts, part_channels
        self.slot_of = {v: s for s, v in enumerate(slot_views) if v is not None}
        self._ws = {}

    def workspace(self, B, device, band=None, slab_rows=None, tag=0):
        from mvdet_amd.pipeline import band_rows
        H, W = self.grid_hw
        band = (0, H) if band is None else tuple(band)
        slab_rows = (0, H) if slab_rows is None else tuple(slab_rows)
        key = (B, band, slab_rows, tag)
        if key not in self._ws:
            y1r, y2r = band_rows(band[0], band[1], H)
            mid = self.params["map_classifier.0.weight"].shape[0]
            self._ws[key] = SimpleNamespace(
                slab=torch.zeros(len(self.slot_views), B, self.C, slab_rows[1] - slab_rows[0], W), band=band,
                slab_rows=slab_rows, y1=torch.zeros(B, mid, y1r[1] - y1r[0], W), y1_rows=y1r, y2_rows=y2r)
        return self._ws[key]

    # partial-sum mode: conv1 over this slab's views only, then the band fusion from summed y1
    def conv1_partial(self, ws, mc, out, mark=None, band_rows=0):
        w1 = self.params["map_classifier.0.weight"]
        H = self.grid_hw[0]
        full = torch.zeros(ws.slab.shape[1], w1.shape[0], H, self.grid_hw[1])
        for s, v in enumerate(self.slot_views):
            if v is None:
                continue
            if self.parts is None:
                full += torch.nn.functional.conv2d(ws.slab[s], w1[:, v * self.C:(v + 1) * self.C], padding=1)
            else:
                pv, c0 = self.parts[v]
                a = pv * self.C + c0
                full += torch.nn.functional.conv2d(ws.slab[s][:, :self.cp], w1[:, a:a + self.cp], padding=1)
        if not band_rows:
            return out.copy_(full)
        for p in range(-(-H // band_rows)):  # the band-major layout of ProjectFuse.conv1_partial
            a, b = p * band_rows, min(H, (p + 1) * band_rows)
            out[p, :, :, :b - a] = full[:, :, a:b]
        return out

    def finish_from_y1(self, ws, mc, mark=None):
        F = torch.nn.functional
        p = self.params
        H, W = self.grid_hw
        B = ws.y1.shape[0]
        nc = len(self.pm) * self.C
        cm = cpu_path.coord_map(H, W)
        coord = F.conv2d(cm, p["map_classifier.0.weight"][:, nc:nc + 2], p["map_classifier.0.bias"], padding=1)
        (a1, b1), (a2, b2), (r0, r1) = ws.y1_rows, ws.y2_rows, ws.band
        Y1 = torch.zeros(B, ws.y1.shape[1], H, W)
        Y1[:, :, a1:b1] = F.relu(ws.y1 + coord[:, :, a1:b1])
        y2 = F.relu(F.conv2d(Y1, p["map_classifier.2.weight"], p["map_classifier.2.bias"], padding=2, dilation=2))
        Y2 = torch.zeros_like(y2)
        Y2[:, :, a2:b2] = y2[:, :, a2:b2]
        return F.conv2d(Y2, p["map_classifier.4.weight"], None, padding=4, dilation=4)[:, :, r0:r1]

    # band exchange: the view windows written straight into the send chunks
    def window_buffer(self, n, B, rows, device):
        return torch.zeros(n, B, self.C, rows, self.grid_hw[1])

    def warp_windows(self, dsts, cams, feats, row0s, nonfinite=None):
        for d, v, f, r0 in zip(dsts, cams, feats, row0s):
            M = torch.as_tensor(np.asarray(self.pm[v])).reshape(1, 3, 3).repeat(f.shape[0], 1, 1).float()
            d.copy_(kornia_warp.warp_perspective(f, M, list(self.grid_hw))[:, :, r0:r0 + d.shape[2]])

    def warp_views_upsampled(self, ws, cams, feats):
        """a4 + a5: the 3x bilinear upsample of backbone-resolution maps (``:65``), then the warp."""
        for v, f in zip(cams, feats):
            self.warp_view(ws, v, torch.nn.functional.interpolate(f.float(), list(self.src_hw), mode="bilinear"))

    def warp_view(self, ws, v, feat):
        B = feat.shape[0]
        pv = v if self.parts is None else self.parts[v][0]
        M = torch.as_tensor(np.asarray(self.pm[pv])).reshape(1, 3, 3).repeat(B, 1, 1).float()
        ws.slab[self.slot_of[v], :, :feat.shape[1]] = kornia_warp.warp_perspective(feat, M, list(self.grid_hw))

    def fuse(self, ws, mc, mark=None):
        """The oracle convs on the slab's rows (a band-local window is exact 7 rows inside its
        cuts, which the band is), then the band's rows."""
        B = ws.slab.shape[1]
        lo, hi = ws.slab_rows
        views = [ws.slab[self.slot_of[v]] for v in range(len(self.pm))]
        coord = cpu_path.coord_map(*self.grid_hw)[:, :, lo:hi].repeat(B, 1, 1, 1)
        out = cpu_path.fuse(torch.cat(views + [coord], 1), self.params)
        return out[:, :, ws.band[0] - lo:ws.band[1] - lo]


def _case():
    from mvdet_amd.synthetic import wildtrack_like
    ds = wildtrack_like(3, 4, seed=21, img_shape=(72, 128), worldgrid_shape=(52, 100))
    from mvdet_amd.geometry import projection_matrices
    pm = [M.numpy() for M in projection_matrices(ds)]
    C, B = 8, 2
    up = ds.upsample_shape
    feats = [torch.from_numpy(fixtures.feature_input((B, C, *up), seed=300 + v)) for v in range(3)]
    params = {k: torch.from_numpy(v) for k, v in fixtures.head_params(3, seed=5, C=C).items()}
    return pm, tuple(up), tuple(ds.reducedgrid_shape), C, B, feats, params


MODES = {"gather": parallel.ViewParallel, "partial": parallel.ViewPartialSum, "bands": parallel.ViewBands}


def _backbone_maps(up, C, B):
    """Backbone-resolution maps (src / 3) whose 3x upsample is the warp's source (``:64-65``)."""
    g = torch.Generator().manual_seed(77)
    return [torch.randn(B, C, up[0] // 3, up[1] // 3, generator=g).clamp_min_(0) for _ in range(3)]


def _worker(rank, world, port, out_dir, mode="gather", frames=1, weights=None, split=False, k=0, backbone=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    pm, up, grid, C, B, feats, params = _case()
    kw = {} if weights is None else {"view_weights": weights}
    if split:  # channel parts of the views (C = 8 here: parts down to 2 channels)
        kw.update(channels=C, min_part=2, parts_k=k)
        if backbone:  # the owners' backbone-resolution maps cross (channels-last wire format)
            feats = _backbone_maps(up, C, B)
            kw.update(fetch_hw=feats[0].shape[2:], fetch_channels_last=True)
    vp = MODES[mode](lambda sv, **kw: OracleEngine(pm, up, grid, C, params, sv, **kw), pm, grid, rank, world, **kw)
    with torch.no_grad():
        if frames == 1:
            outs = [vp.step(vp.workspace(B, "cpu"), [feats[v] for v in vp.my_views], None)]
        else:  # FramePipeline: frame f uses the features scaled by (f + 1)
            pipe = parallel.FramePipeline(vp, B, "cpu")
            outs = [pipe.submit([(f + 1) * feats[v] for v in vp.my_views], None) for f in range(frames)]
            lag = 2 if pipe.fetching else 1
            assert all(o is None for o in outs[:lag]) and all(o is not None for o in outs[lag:])
            outs = outs[lag:] + pipe.drain_all(None)
            assert pipe.drain(None) is None
    torch.save({"outs": outs, "band": vp.band, "views": vp.my_views, "parts": getattr(vp, "my_parts", None),
                "recv": [list(map(list, ps)) for ps in getattr(vp, "recv_parts", [])]},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "gather"), (3, "gather"), (4, "gather"), (2, "partial"), (3, "partial"),
                                        (4, "partial"), (8, "gather"), (8, "partial"), (2, "bands"), (3, "bands"),
                                        (4, "bands"), (8, "bands")])
def test_view_parallel_matches_single_process_oracle(world, mode, tmp_path):
    """gather: slab all-gather + row bands.  partial: conv1 partial sums over each rank's
    views + reduce-scatter by band + edge-row halo (world 2: 7-row bands use the edge
    all-gather; world 3: 5-row bands fall back to whole bands; world 4: a rank with no view
    contributes zeros; world 8, the driver's node size: five ranks without views, 7-row bands).
    bands: all-to-all of each band's input row window (windows shifted inside the grid at the
    edges; ranks without views send nothing), fusion from the band-local slab."""
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), mode), nprocs=world, join=True)
    pm, up, grid, C, B, feats, params = _case()
    with torch.no_grad():
        ref = cpu_path.project_fuse(feats, pm, grid, params)
    bands = []
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["views"] == parallel.views_of(r, world, 3)
        tol = dict(rtol=1e-5, atol=1e-6) if mode == "partial" else dict(rtol=1e-6, atol=1e-7)  # summation order
        torch.testing.assert_close(res["outs"][0], ref, **tol)
        bands.append(tuple(res["band"]))
    assert bands[0][0] == 0 and bands[-1][1] == grid[0]
    assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))


def test_slot_order_and_bands():
    assert parallel.slot_views(2, 3) == [0, 2, 1, None]
    assert parallel.slot_views(7, 7) == list(range(7))
    assert parallel.slot_views(4, 7) == [0, 4, 1, 5, 2, 6, 3, None]
    assert parallel.slot_views(8, 7) == list(range(7)) + [None]
    assert [parallel.row_band(120, r, 8) for r in range(8)][-1] == (105, 120)
    assert [parallel.row_band(160, r, 6) for r in range(6)][-1] == (135, 160)
    assert parallel.row_band(5, 7, 8) == (5, 5)  # more ranks than rows: empty band
    from mvdet_amd.pipeline import band_rows
    assert band_rows(15, 30, 120) == ((9, 36), (11, 34))
    assert band_rows(0, 15, 120) == ((0, 21), (0, 19))


@pytest.mark.parametrize("world,mode", [(2, "bands"), (3, "partial"), (2, "gather")])
def test_frame_pipeline_returns_every_frame_in_order(world, mode, tmp_path):
    """FramePipeline (frame i's exchange overlapped with frame i-1's fusion, double buffers):
    4 frames with different inputs come back in order, each equal to its own single-process
    result (a buffer reused too early would mix frames)."""
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), mode, 4), nprocs=world, join=True)
    pm, up, grid, C, B, feats, params = _case()
    with torch.no_grad():
        refs = [cpu_path.project_fuse([(f + 1) * x for x in feats], pm, grid, params) for f in range(4)]
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert len(res["outs"]) == 4
        for f in range(4):
            torch.testing.assert_close(res["outs"][f], refs[f], rtol=1e-5, atol=1e-6)


def test_band_windows_cover_each_band():
    """ViewBands' input windows: E = ceil(H/P) + 14 rows, inside the grid, covering the band's
    rows +- 7 (clipped at the grid edges)."""
    for H, P in ((52, 2), (52, 3), (52, 8), (120, 7), (480, 7), (160, 6), (5, 8)):
        vb = SimpleNamespace(grid_hw=(H, 10), world=P, E=min(H, -(-H // P) + 14))
        for p in range(P):
            lo, hi = parallel.ViewBands.window(vb, p)
            r0, r1 = parallel.row_band(H, p, P)
            if r1 <= r0:
                r0, r1 = 0, 1
            assert 0 <= lo and hi <= H and hi - lo == vb.E
            assert lo <= max(0, r0 - 7) and min(H, r1 + 7) <= hi


def test_balanced_views_assignment():
    """Longest-processing-time dealing of views to ranks by their conv1 work (partial-sum mode)."""
    w = [0.37, 0.73, 0.82, 0.6, 0.58, 0.9, 0.82]
    for P in (2, 3, 4, 7, 8):
        a = parallel.balanced_views(w, P)
        assert sorted(v for vs in a for v in vs) == list(range(7)) and len(a) == P
        loads = [sum(w[v] for v in vs) for vs in a]
        mod = [sum(w[v] for v in parallel.views_of(r, P, 7)) for r in range(P)]
        assert max(loads) <= max(mod) + 1e-12
    assert parallel.balanced_views(w, 7) == [[5], [2], [6], [1], [3], [4], [0]]


@pytest.mark.parametrize("world", [2, 3])
def test_partial_mode_balanced_assignment_matches_oracle(world, tmp_path):
    """The partial-sum mode with views dealt by their conv1 work (``view_weights``): same map."""
    weights = [0.2, 0.9, 0.5]
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), "partial", 1, weights), nprocs=world, join=True)
    pm, up, grid, C, B, feats, params = _case()
    with torch.no_grad():
        ref = cpu_path.project_fuse(feats, pm, grid, params)
    assigned = []
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["views"] == parallel.balanced_views(weights, world)[r]
        assigned += res["views"]
        torch.testing.assert_close(res["outs"][0], ref, rtol=1e-5, atol=1e-6)
    assert sorted(assigned) == [0, 1, 2]


@pytest.mark.parametrize("world,k,backbone", [(2, 0, False), (4, 0, False), (5, 0, False), (2, 4, True),
                                              (4, 2, True), (8, 4, True)])
def test_partial_mode_channel_parts_match_oracle(world, k, backbone, tmp_path):
    """The partial-sum mode with views cut into channel parts (``mp_model.balanced_parts``; world 4, 5 and 8
    > 3 views: every view split, a rank holding parts of several views; ``k`` forces the split), pipelined
    over 4 frames (the slice exchange's 3-buffer rotation wraps): every rank's map equals the oracle's, the
    parts cover every (view, channel) exactly once, every rank was handed only the maps of the views it owns
    (``view_owners``) and received exactly the parts it holds of views owned elsewhere.  ``backbone``: the
    owners hold backbone-resolution maps, the slices cross in channels-last form and the warp upsamples."""
    weights = [0.9, 0.3, 0.6]
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), "partial", 4, weights, True, k, backbone), nprocs=world,
             join=True)
    pm, up, grid, C, B, feats, params = _case()
    if backbone:
        feats = [torch.nn.functional.interpolate(x, list(up), mode="bilinear") for x in _backbone_maps(up, C, B)]
    with torch.no_grad():
        refs = [cpu_path.project_fuse([(f + 1) * x for x in feats], pm, grid, params) for f in range(4)]
    covered = []
    assign, cp = parallel.balanced_parts(weights, world, C, min_part=2, k=k)
    owner = parallel.view_owners([w + 0.05 for w in weights], world)
    if world > 3:
        assert cp < C  # the split is exercised
    moved = 0
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert [tuple(p) for p in res["parts"]] == [tuple(p) for p in assign[r]]
        assert res["views"] == [v for v in range(3) if owner[v] == r]
        recv = sorted(tuple(p) for ps in res["recv"] for p in ps)
        assert recv == sorted(tuple(p) for p in assign[r] if owner[p[0]] != r)
        moved += len(recv)
        covered += [(v, c) for v, c0 in res["parts"] for c in range(c0, c0 + cp)]
        assert len(res["outs"]) == 4
        for f in range(4):
            torch.testing.assert_close(res["outs"][f], refs[f], rtol=1e-5, atol=1e-6)
    assert sorted(covered) == [(v, c) for v in range(3) for c in range(C)]
    if world > 3:
        assert moved > 0  # the slice exchange is exercised


def test_owner_affine_part_dealing():
    """Round 6: whole views (k = 1) stay on their owner (no slice crosses), every view has one owner and
    with P >= N no rank owns two views; parts go home when that costs little balance."""
    from mvdet_amd import mp_model
    w = [0.37, 0.73, 0.82, 0.6, 0.58, 0.9, 0.82]
    for P in (2, 3, 4, 7, 8):
        owner = mp_model.view_owners([x + 0.05 for x in w], P)
        assign, cp = mp_model.balanced_parts(w, P, 512, k=1)
        assert all(owner[v] == r for r, ps in enumerate(assign) for v, _ in ps)
        if P >= 7:
            assert len(set(owner)) == 7
        for k in (2, 4, 8):
            assign, cp = mp_model.balanced_parts(w, P, 512, k=k)
            assert cp == 512 // k and sorted(p for ps in assign for p in ps) == sorted(
                (v, j * cp) for v in range(7) for j in range(k))
            home = sum(owner[v] == r for r, ps in enumerate(assign) for v, _ in ps)
            plain = mp_model.balanced_parts(w, P, 512, k=k, affinity=0.0)[0]
            assert home >= sum(owner[v] == r for r, ps in enumerate(plain) for v, _ in ps)


def test_slice_exchange_cost_model():
    """mp_model's slice-exchange pricing (round 6): per (sender, receiver) link the bytes of the parts held away
    from their owner; whole views (k = 1) move nothing; the model's chosen split for the driver's node at cfg2
    (P = 8) cuts every view into 64-channel parts and each link carries at most one 3.7 MB backbone-map slice."""
    from mvdet_amd import mp_model
    w = [0.37, 0.73, 0.82, 0.6, 0.58, 0.9, 0.82]
    for P in (2, 4, 8):
        owner = mp_model.view_owners([x + 0.05 for x in w], P)
        a1, _ = mp_model.balanced_parts(w, P, 512, k=1)
        assert mp_model.fetch_link_bytes(a1, owner, P, 1.0).sum() == 0
        a8, cp = mp_model.balanced_parts(w, P, 512, k=8)
        links = mp_model.fetch_link_bytes(a8, owner, P, 1.0)
        moved = sum(owner[v] != q for q, ps in enumerate(a8) for v, _ in ps)
        assert links.sum() == moved and np.all(np.diag(links) == 0)
    pr = mp_model.predict_config(2, 8)["partial"]
    assert pr["parts_k"] == 8 and pr["fetch"] > 0
    part = 4.0 * 1 * 64 * mp_model.backbone_pixels(2)
    assert abs(part - 64 * 90 * 160 * 4) < 1
    assert pr["fetch_bytes_max_rank"] <= 8 * part
    assert mp_model.predict_config(2, 2)["partial"]["fetch"] == 0.0  # k = 1 at P = 2: no slice moves
