"""GPU tests of the multi-GPU building blocks on one device.

* Row bands: the fusion computed band by band (as each rank does after the
  all-gather) is bitwise identical to the whole-grid fusion.
* Rehearsals of both multi-GPU modes (slab all-gather; conv1 partial sums +
  reduce-scatter) with 2-4 ranks on the single GPU of the test box (gloo collectives
  staged through host memory): every rank's assembled map equals the single-process
  HIP result to fp32 summation-order rounding.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import assert_parity_t
from oracle import cpu_path, fixtures

pytestmark = pytest.mark.gpu


def _setup(seed=31, C=64, B=2):
    from mvdet_amd import synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.multiviewx_like(3, 4, seed=seed, img_shape=(216, 384), worldgrid_shape=(128, 200))
    up = tuple(ds.upsample_shape)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=50 + v) for v in range(3)]
    params = fixtures.head_params(3, seed=seed, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * 3 + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    return ds, projection_matrices(ds), up, tuple(ds.reducedgrid_shape), C, B, feats, mc


def _poison(feats):
    """+inf, NaN and -inf in three views' features near the image centre (sampled by the warps)."""
    feats = [f.clone() for f in feats]
    h, w = feats[0].shape[2:]
    feats[0][1, 5, h // 2, w // 2] = float("inf")
    feats[1][0, 17, h // 2 + 2, w // 2 - 3] = float("nan")
    feats[2][1, 40, h // 2 - 3, w // 2 + 4] = float("-inf")
    return feats


def _oracle_map(scale=1.0, poison=False):
    """The reference CPU path (kornia restatement + cat + F.conv2d, persp_trans_detector.py:69-82) on
    the same inputs as ``_setup``'s (features times ``scale``; ``poison``: with ``_poison``'s values)."""
    ds, pm, up, grid, C, B, feats, mc = _setup()
    if poison:
        feats = _poison(feats)
    params = {k: torch.from_numpy(v) for k, v in fixtures.head_params(3, seed=31, C=C).items()}
    with torch.no_grad():
        return cpu_path.project_fuse([scale * f for f in feats], [M.numpy() for M in pm], grid, params)


@pytest.mark.parametrize("wino", [False, True])
def test_band_fusion_matches_whole_grid(wino):
    """Row bands (the multi-GPU fusion) vs the whole grid: bitwise with the direct conv1 and conv2;
    with the row-Winograd convs a band's 3-row tiles start at its own first row, so its sums are
    grouped differently: fp32 rounding level."""
    from mvdet_amd import ProjectFuse
    from mvdet_amd.parallel import row_band
    ds, pm, up, grid, C, B, feats, mc = _setup()
    mc = mc.to("cuda:0")
    eng = ProjectFuse(pm, up, grid, C, split_k=False, wino_conv1=wino, wino_conv2=wino)  # split-K tails re-associate K sums
    with torch.no_grad():
        full = eng.project_fuse([f.cuda() for f in feats], mc).cpu()
        for P in (3, 5):
            parts = []
            for r in range(P):
                ws = eng.workspace(B, "cuda:0", row_band(grid[0], r, P))
                for v, f in enumerate(feats):
                    eng.warp_view(ws, v, f.cuda())
                parts.append(eng.fuse(ws, mc).cpu())
            if wino:
                torch.testing.assert_close(torch.cat(parts, 2), full, rtol=1e-4, atol=1e-5)
            else:
                assert torch.equal(torch.cat(parts, 2), full), P


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, mode="gather", backend="gloo", frames=1, poison=False, split=False,
            precision="bf16x3"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group(backend, rank=rank, world_size=world,
                            device_id=torch.device("cuda:0") if backend == "nccl" else None)
    from mvdet_amd import ProjectFuse
    from mvdet_amd.parallel import FramePipeline, ViewBands, ViewParallel, ViewPartialSum
    ds, pm, up, grid, C, B, feats, mc = _setup()
    if poison:  # frame 0 poisoned; with frames > 1 frame 1 is finite again (the guard must not fire)
        bad = _poison(feats)
        frame_feats = lambda f: bad if f == 0 else feats  # noqa: E731
    else:
        frame_feats = lambda f: [(f + 1) * x for x in feats]  # noqa: E731
    mc = mc.to("cuda:0")
    cls = {"gather": ViewParallel, "partial": ViewPartialSum, "bands": ViewBands}[mode]
    # split: the partial-sum mode's channel parts (16-channel parts allowed: C = 64 here)
    skw = dict(view_weights=[0.9, 0.3, 0.6], channels=C, min_part=16) if split else {}
    vp = cls(lambda sv, **kw: ProjectFuse(pm, up, grid, C, slot_views=sv, precision=precision, **kw), pm, grid, rank,
             world, **skw)
    with torch.no_grad():
        if frames == 1:
            outs = [vp.step(vp.workspace(B, "cuda:0"), [frame_feats(0)[v].cuda() for v in vp.my_views], mc)]
        else:  # frame f: the features scaled by (f + 1); exchange on a side stream under NCCL
            pipe = FramePipeline(vp, B, "cuda:0")
            outs = [pipe.submit([frame_feats(f)[v].cuda() for v in vp.my_views], mc) for f in range(frames)]
            lag = 2 if pipe.fetching else 1  # the channel-part mode's slice exchange adds a pipeline stage
            outs = outs[lag:] + pipe.drain_all(mc)
            assert len(outs) == frames
        torch.cuda.synchronize()
    if poison:  # did the guard fire for the poisoned frame (buffer 0) and only for it (buffer 1)?
        fired = ([int(fr.ws.nf2.item()) == fr.ws.nf2_tag for fr in pipe.frames[:frames]] if mode == "partial" else
                 [int(fr.gflag.item()) == fr.tag for fr in pipe.frames[:frames]])
        torch.save(fired, os.path.join(out_dir, f"fired{rank}.pt"))
    torch.save([o.cpu() for o in outs], os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,split,precision", [
    (2, "gather", False, "bf16x3"), (2, "partial", False, "bf16x3"), (4, "partial", False, "bf16x3"),
    (2, "bands", False, "bf16x3"), (3, "bands", False, "bf16x3"), (2, "partial", True, "bf16x3"),
    (4, "partial", True, "bf16x3"), (2, "bands", False, "fp32"), (3, "partial", True, "fp32")])
def test_rank_rehearsal_matches_single_process(world, mode, split, precision, tmp_path):
    """gather / partial-sum / band-exchange modes; world 4 (3 views) includes a rank without
    views and bands of 8 rows (edge-row halo exchange); bands at world 3: one view per rank,
    shifted windows at both grid edges; ``split``: the partial-sum mode on channel parts of the views
    (``mp_model.balanced_parts``; world 4 > 3 views splits every view; each rank handed only its owned
    views' features, the other parts through the slice exchange); ``precision="fp32"``: the fp32-MFMA
    engines (the band exchange's windows as fp32, warped in the reference's order)."""
    from mvdet_amd import ProjectFuse
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), mode, "gloo", 1, False, split, precision),
             nprocs=world, join=True)
    ds, pm, up, grid, C, B, feats, mc = _setup()
    mc = mc.to("cuda:0")
    with torch.no_grad():
        ref = ProjectFuse(pm, up, grid, C).project_fuse([f.cuda() for f in feats], mc).cpu()
    oracle = _oracle_map()
    for r in range(world):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)[0]
        # every rank's assembled map vs the reference's CPU path (the parity gate, and the 3xbf16 path's
        # 5e-5), and vs the single-process HIP map (different slot order / band-started Winograd tiles ->
        # different summation order in conv1: fp32-rounding level only)
        assert_parity_t(got, oracle, f"{mode} x{world} rank {r} map_result vs oracle", normwise_tol=5e-5)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mode,split", [("bands", False), ("gather", False), ("partial", False), ("partial", True)])
def test_frame_pipeline_on_rccl_streams(mode, split, tmp_path):
    """FramePipeline with the real RCCL backend (a one-rank world on the box's GPU): the exchange
    runs on the side stream behind events, the fusion of the previous frame on the compute
    stream; 4 frames with different inputs come back in order and equal the single-process
    maps (a missing wait or an early buffer reuse would mix frames).  ``split``: the channel-part
    mode's three-stage pipeline (fetch on the side stream, 3 rotating frame buffers)."""
    from mvdet_amd import ProjectFuse
    mp.spawn(_worker, args=(1, _free_port(), str(tmp_path), mode, "nccl", 4, False, split), nprocs=1, join=True)
    ds, pm, up, grid, C, B, feats, mc = _setup()
    mc = mc.to("cuda:0")
    eng = ProjectFuse(pm, up, grid, C)
    got = torch.load(tmp_path / "r0.pt", weights_only=True)
    assert len(got) == 4
    with torch.no_grad():
        for f in range(4):
            ref = eng.project_fuse([(f + 1) * x.cuda() for x in feats], mc).cpu()
            assert_parity_t(got[f], _oracle_map(f + 1.0), f"{mode} pipeline frame {f} vs oracle", normwise_tol=5e-5)
            torch.testing.assert_close(got[f], ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world,mode,split", [(2, "gather", False), (2, "partial", False), (3, "partial", False),
                                              (2, "bands", False), (3, "bands", False), (4, "partial", True)])
def test_rank_rehearsal_nonfinite_features(world, mode, split, tmp_path):
    """VERDICT r04 missing 2: the non-finite guard in the multi-rank modes.  +inf / NaN / -inf in three
    views' features (one rank's, or several ranks'), then a finite frame through the pipeline: every
    rank's map has the oracle's NaN / inf pattern (bands / gather: the window warps' reports, MAXed over
    the ranks, switch every rank to exchanged fp32 windows and the gated fp32-MFMA convs; partial: each
    rank's gated exact conv1 partial, the summed pre-activation's report, the gated exact conv2), and the
    finite frame after it is the fast path's."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), mode, "gloo", 2, True, split), nprocs=world,
             join=True)
    ref = _oracle_map(poison=True)
    nf = ~torch.isfinite(ref)
    assert 0 < int(nf.sum()) < ref.numel() and int(torch.isnan(ref).sum()) > 0  # the case discriminates
    ref_fin = _oracle_map()
    for r in range(world):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.load(tmp_path / f"fired{r}.pt", weights_only=True) == [True, False]
        assert_parity_t(got[0], ref, f"{mode} x{world} rank {r} poisoned frame (NaN / inf pattern included)")
        assert torch.isfinite(got[1]).all()
        assert_parity_t(got[1], ref_fin, f"{mode} x{world} rank {r} finite frame after it", normwise_tol=5e-5)


# -- BASELINE-size rehearsals of the modes mp_model picks for the driver's 8-GPU node

def _cfg_inputs(cfg):
    from mvdet_amd import synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    return spec, ds, projection_matrices(ds), up, grid


def _cfg_feats(cfg, spec, up, views):
    from mvdet_amd import synthetic
    half = cfg == 4
    return [synthetic.synthetic_features(spec["B"], spec["C"], [u // 3 for u in up], up, seed=1000 * cfg + v,
                                         device="cuda:0").to(torch.float16 if half else torch.float32) for v in views]


def _cfg_worker(rank, world, port, out_dir, cfg, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mvdet_amd import ProjectFuse, mp_model, synthetic
    from mvdet_amd.parallel import ViewBands, ViewParallel, ViewPartialSum
    spec, ds, pm, up, grid = _cfg_inputs(cfg)
    C, N = spec["C"], ds.num_cam
    params = fixtures.head_params(N, seed=cfg, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * N + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    mc = mc.to("cuda:0")
    kw = {}
    half = cfg == 4
    if mode == "partial":
        # as bench.py --gpus N runs it: views cut into channel parts dealt by their conv1 work (the split the
        # cost model predicts fastest), each rank holding only its OWNED views' backbone-resolution maps
        # (channels-last; fp16 NCHW at cfg4), the other holders' slices crossing in the slice exchange
        kw["view_weights"] = [float(a.mean()) for a in mp_model.config_inputs(cfg)[4]]
        kw["channels"] = C
        kw["parts_k"] = int(mp_model.predict_config(cfg, world)["partial"]["parts_k"])
        kw.update(fetch_hw=tuple(u // 3 for u in up), fetch_dtype=torch.float16 if half else torch.float32,
                  fetch_channels_last=not half)
    cls = {"gather": ViewParallel, "partial": ViewPartialSum, "bands": ViewBands}[mode]
    vp = cls(lambda sv, **k: ProjectFuse(pm, up, grid, C, slot_views=sv, **k), pm, grid, rank, world, **kw)
    if mode == "partial":
        feats = []
        for v in vp.my_views:
            x = synthetic.backbone_features(spec["B"], C, [u // 3 for u in up], seed=1000 * cfg + v, device="cuda:0")
            feats.append(x.half() if half else x.contiguous(memory_format=torch.channels_last))
    else:
        feats = _cfg_feats(cfg, spec, up, vp.my_views)
    with torch.no_grad():
        out = vp.step(vp.workspace(spec["B"], "cuda:0"), feats, mc)
        torch.cuda.synchronize()
    torch.save({"map": out.cpu(), "views": vp.my_views, "band": vp.band,
                "owner": getattr(vp, "owner", None)}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,world", [(3, 7), (5, 8), (4, 6), (2, 8)])
def test_chosen_mode_at_baseline_size_vs_oracle(cfg, world, tmp_path):
    """The mode ``mp_model.choose_mode`` picks for the config at ``world`` ranks (cfg3 at P = 7: partial;
    cfg5 at P = 8: bands; cfg4 at P = 6: partial; cfg2 at P = 8: partial — the partial-sum mode from each rank's
    owned backbone maps through the slice exchange, round 6), rehearsed with gloo ranks sharing the box's GPU at
    the BASELINE size: every rank's assembled map vs the oracle (warp of every view whole, convs on row
    bands +- 7) on the top and bottom edge bands and on bands across rank boundaries, at 5e-5 normwise."""
    from mvdet_amd import mp_model
    from mvdet_amd.parallel import row_band
    mode = mp_model.choose_mode(cfg, world)
    mp.spawn(_cfg_worker, args=(world, _free_port(), str(tmp_path), cfg, mode), nprocs=world, join=True)
    spec, ds, pm, up, grid = _cfg_inputs(cfg)
    H = grid[0]
    if mode == "partial" and cfg == 4:  # the ranks' inputs: fp16 backbone maps, upsampled inside the warp
        from mvdet_amd import synthetic
        feats = [torch.nn.functional.interpolate(
            synthetic.backbone_features(spec["B"], spec["C"], [u // 3 for u in up], seed=1000 * cfg + v,
                                        device="cuda:0").half().float(), list(up), mode="bilinear")
            for v in range(ds.num_cam)]
    else:
        feats = _cfg_feats(cfg, spec, up, range(ds.num_cam))
    warped = cpu_path.warp_views([f.float().cpu() for f in feats], [M.numpy() for M in pm], grid)
    del feats
    tp = {k: torch.from_numpy(v) for k, v in fixtures.head_params(ds.num_cam, seed=cfg, C=spec["C"]).items()}
    n = row_band(H, 0, world)[1]
    mid = (world // 2) * n
    bands = [(0, 16), (n - 8, n + 8), (mid - 8, mid + 8), (H - 16, H)]
    refs = [_oracle_band(warped, grid, tp, r0, r1) for r0, r1 in bands]
    for r in range(world):
        res = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert res["map"].shape == (spec["B"], 1) + grid
        if res["owner"] is not None:  # the rank was handed its owned views' maps only (the slice exchange)
            assert res["views"] == [v for v in range(ds.num_cam) if res["owner"][v] == r]
        for (r0, r1), ref in zip(bands, refs):
            assert_parity_t(res["map"][:, :, r0:r1], ref, f"cfg{cfg} {mode} x{world} rank {r} map rows {r0}:{r1}",
                            normwise_tol=5e-5)


def _oracle_band(warped, grid, params, r0, r1):
    """map rows [r0, r1) of the oracle from the warped views' rows [r0 - 7, r1 + 7) (clipped)."""
    H = grid[0]
    a, b = max(0, r0 - 7), min(H, r1 + 7)
    B = warped[0].shape[0]
    coord = cpu_path.coord_map(*grid)[:, :, a:b].repeat([B, 1, 1, 1])
    with torch.no_grad():
        out = cpu_path.fuse(torch.cat([w[:, :, a:b] for w in warped] + [coord], 1), params)
    return out[:, :, r0 - a:r1 - a]
