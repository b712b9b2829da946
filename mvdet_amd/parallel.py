"""View-parallel project+fuse across GPUs (one process per GPU, torch.distributed).

SURVEY §8(e).  The reference has no distributed code (everything on ``cuda:0``,
``persp_trans_detector.py:37-54``); this is the MI355X-native multi-GPU design the
north star asks for:

1. **Views shard across ranks.**  Rank ``r`` owns views ``{v : v % P == r}`` (its
   cameras' backbone + upsample run there) and warps them into its own slots of the
   view-major slab ``[S = P*Vmax, B, Cs, Ho, Wo]`` — slot ``r*Vmax + j`` holds view
   ``r + P*j`` (empty slots stay zero and get zero conv1 weights).
2. **One RCCL all-gather over xGMI** (``all_gather_into_tensor``, in place): the
   slab is rank-major, so every rank's chunk is already contiguous — no repack.
3. **Fusion by row band.**  Each rank runs conv1/conv2/conv3 only for output rows
   ``[r0, r1)`` (``ceil(Ho/P)`` rows), computing conv1 on the band + 6 halo rows and
   conv2 on the band + 4 (dilations 1, 2, 4 of ``:51-54``) from the gathered slab,
   so the 26-TFLOP fusion at config 3 is split P ways instead of replicated.
4. **A tiny all-gather of the map bands** assembles ``map_result`` on every rank.

``ViewPartialSum`` is the partial-sum alternative (SURVEY §8(e) "Alternative", §8(f)
row 3).  conv1 is linear in its input channels, so each rank computes conv1 over only
its own views' channels for the whole grid (no slab exchange at all), then
**reduce-scatters** those [B, 512, Ho, Wo] partial sums by row band (each rank receives
its band summed over all ranks), all-gathers the 6 edge rows of every band as halo, adds
the coord term + bias and ReLU, and runs conv2/conv3 on its band.  Per rank it moves
≈ (P-1)/P × 88.5 MB at config 2 instead of (P-1)/P × 620 MB, and conv1's FLOPs split
by views instead of by (band + halo) rows.

The compute engine is pluggable (``engine`` = ``pipeline.ProjectFuse`` on GPU; the
CPU gloo tests plug in an oracle engine), so the collective logic is tested without
a GPU.  With the ``gloo`` backend and CUDA tensors the collectives are staged
through host memory (used only for single-GPU rehearsals of the multi-rank path).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def views_of(rank: int, world: int, num_cam: int) -> List[int]:
    return [v for v in range(num_cam) if v % world == rank]


def slot_views(world: int, num_cam: int) -> List[Optional[int]]:
    """Rank-major slot order: slot r*Vmax + j holds view r + P*j (or None)."""
    vmax = math.ceil(num_cam / world)
    out: List[Optional[int]] = []
    for r in range(world):
        vs = views_of(r, world, num_cam)
        out += vs + [None] * (vmax - len(vs))
    return out


def row_band(H: int, rank: int, world: int) -> Tuple[int, int]:
    per = math.ceil(H / world)
    r0 = min(H, rank * per)
    return r0, min(H, r0 + per)


def _all_gather_inplace(full: torch.Tensor, rank: int, world: int, group=None) -> None:
    """``full`` is [world * n, ...]; this rank's chunk is ``full[rank*n:(rank+1)*n]``."""
    n = full.shape[0] // world
    mine = full[rank * n:(rank + 1) * n]
    if full.is_cuda and dist.get_backend(group) == "gloo":
        host = full.cpu()
        dist.all_gather_into_tensor(host, host[rank * n:(rank + 1) * n].clone(), group=group)
        full.copy_(host)
        return
    dist.all_gather_into_tensor(full, mine, group=group)


class ViewParallel:
    """Drives one rank's share of the view-parallel project+fuse."""

    def __init__(self, engine_factory, proj_mats: Sequence[torch.Tensor], grid_hw: Tuple[int, int],
                 rank: int, world: int, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.num_cam = len(proj_mats)
        self.grid_hw = (int(grid_hw[0]), int(grid_hw[1]))
        self.my_views = views_of(rank, world, self.num_cam)
        self.vmax = math.ceil(self.num_cam / world)
        self.engine = engine_factory(slot_views(world, self.num_cam))
        self.band = row_band(self.grid_hw[0], rank, world)
        self.band_rows = math.ceil(self.grid_hw[0] / world)
        self._out = {}

    def workspace(self, B: int, device):
        r0, r1 = self.band
        band = (r0, r1) if r1 > r0 else (0, 1)  # empty band (H < P): compute a dummy row
        return self.engine.workspace(B, device, band)

    def warp(self, ws, feats: Sequence[torch.Tensor]) -> None:
        """Warp this rank's views (``feats[j]`` is view ``my_views[j]``)."""
        if hasattr(self.engine, "warp_views"):
            self.engine.warp_views(ws, self.my_views, list(feats))
        else:
            for v, f in zip(self.my_views, feats):
                self.engine.warp_view(ws, v, f)

    def gather_views(self, ws) -> None:
        _all_gather_inplace(ws.slab, self.rank, self.world, self.group)

    def fuse_band(self, ws, map_classifier, mark=None) -> torch.Tensor:
        return self.engine.fuse(ws, map_classifier, mark=mark)

    def gather_map(self, band_out: torch.Tensor) -> torch.Tensor:
        """[B,1,rows,W] band of every rank -> [B,1,Ho,Wo] on every rank."""
        B, _, _, W = band_out.shape
        H = self.grid_hw[0]
        key = (band_out.device, B)
        buf = self._out.get(key)
        if buf is None:
            buf = torch.zeros((self.world, B, 1, self.band_rows, W), dtype=band_out.dtype, device=band_out.device)
            self._out[key] = buf
        r0, r1 = self.band
        if r1 > r0:
            buf[self.rank, :, :, :r1 - r0].copy_(band_out)
        _all_gather_inplace(buf, self.rank, self.world, self.group)
        full = buf.permute(1, 2, 0, 3, 4).reshape(B, 1, self.world * self.band_rows, W)
        return full[:, :, :H]

    def step(self, ws, feats, map_classifier, mark=None) -> torch.Tensor:
        if mark:
            mark("warp")
        self.warp(ws, feats)
        if mark:
            mark("allgather")
        self.gather_views(ws)
        band = self.fuse_band(ws, map_classifier, mark=mark)
        if mark:
            mark("gather_map")
        return self.gather_map(band)


def _reduce_scatter(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """``inp`` [world, *out.shape] summed over ranks; this rank's slice -> ``out``."""
    out = out.unsqueeze(0)
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        host = inp.cpu()
        res = torch.empty_like(out, device="cpu")
        dist.reduce_scatter_tensor(res, host, op=dist.ReduceOp.SUM, group=group)
        out.copy_(res)
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


class ViewPartialSum(ViewParallel):
    """Partial-sum view-parallel fusion: conv1 split by views, reduce-scatter by rows.

    The engine of rank r holds only r's views (``all_views=False`` slab); a rank with no
    view contributes zeros.  After the reduce-scatter, rank r owns the summed conv1
    pre-activation of rows ``[r*band, (r+1)*band)``; its halo rows (6 above and below:
    conv2's dilation 2 + conv3's 4) come from the neighbours' bands through one small
    all-gather of every band's top and bottom 6 rows (bands of fewer than 6 rows fall back
    to gathering whole bands)."""

    HALO = 6

    def __init__(self, engine_factory, proj_mats, grid_hw, rank, world, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.num_cam = len(proj_mats)
        self.grid_hw = (int(grid_hw[0]), int(grid_hw[1]))
        self.my_views = views_of(rank, world, self.num_cam)
        self.engine = engine_factory(self.my_views) if self.my_views else None
        self._factory = engine_factory
        self.band = row_band(self.grid_hw[0], rank, world)
        self.band_rows = math.ceil(self.grid_hw[0] / world)
        self._out = {}
        self._bufs = {}
        # a rank without views still runs the band fusion: give it an engine over view 0's
        # slot layout (its slab is never written or read) for the packed conv2 weights etc.
        self._fuse_engine = self.engine if self.engine is not None else engine_factory([0])
        for e in (self.engine, self._fuse_engine):  # the exchange sums fp32 partials into y1
            if e is not None and hasattr(e, "y1_split"):
                e.y1_split = False

    def workspace(self, B: int, device):
        r0, r1 = self.band
        band = (r0, r1) if r1 > r0 else (0, 1)
        return self._fuse_engine.workspace(B, device, band)

    def _buffers(self, ws):
        B, mid, _, W = ws.y1.shape
        H, P, n = self.grid_hw[0], self.world, self.band_rows
        key = (ws.y1.device, B)
        bufs = self._bufs.get(key)
        if bufs is None:
            dev = ws.y1.device
            e = min(self.HALO, n)
            bufs = dict(
                part=torch.zeros((B, mid, H, W), dtype=torch.float32, device=dev),
                stage=torch.zeros((P, B, mid, n, W), dtype=torch.float32, device=dev),
                mine=torch.zeros((B, mid, n, W), dtype=torch.float32, device=dev),
                edges=torch.zeros((P, 2, B, mid, e, W), dtype=torch.float32, device=dev),
                full=None if n >= self.HALO else torch.zeros((P, B, mid, n, W), dtype=torch.float32, device=dev))
            self._bufs[key] = bufs
        return bufs

    def conv1_partial(self, ws, map_classifier) -> None:
        bufs = self._buffers(ws)
        if self.engine is None:
            bufs["part"].zero_()
        else:
            self.engine.conv1_partial(ws, map_classifier, bufs["part"])
        H, n = self.grid_hw[0], self.band_rows
        for p in range(self.world):  # band-major staging for the reduce-scatter
            a, b = min(H, p * n), min(H, (p + 1) * n)
            if b > a:
                bufs["stage"][p, :, :, :b - a].copy_(bufs["part"][:, :, a:b])

    def exchange(self, ws) -> None:
        """Reduce-scatter of the partial sums by band, then the halo rows into ``ws.y1``."""
        bufs = self._buffers(ws)
        _reduce_scatter(bufs["mine"], bufs["stage"], self.group)
        H, P, n = self.grid_hw[0], self.world, self.band_rows
        a1, b1 = ws.y1_rows

        def rows_of(p):  # the summed rows of band p available locally after the exchange
            return min(H, p * n), min(H, (p + 1) * n)

        if bufs["full"] is not None:  # bands thinner than the halo: gather whole bands
            bufs["full"][self.rank].copy_(bufs["mine"])
            _all_gather_inplace(bufs["full"], self.rank, P, self.group)
            src = {p: bufs["full"][p] for p in range(P)}
            for p in range(P):
                a, b = rows_of(p)
                lo, hi = max(a, a1), min(b, b1)
                if hi > lo:
                    ws.y1[:, :, lo - a1:hi - a1].copy_(src[p][:, :, lo - a:hi - a])
            return
        e = self.HALO
        bufs["edges"][self.rank, 0].copy_(bufs["mine"][:, :, :e])
        r0, r1 = self.band
        if r1 > r0:
            last = r1 - r0
            bufs["edges"][self.rank, 1].copy_(bufs["mine"][:, :, max(0, last - e):max(0, last - e) + e])
        _all_gather_inplace(bufs["edges"], self.rank, P, self.group)
        # own band
        if r1 > r0:
            ws.y1[:, :, r0 - a1:r1 - a1].copy_(bufs["mine"][:, :, :r1 - r0])
        # halo above: the last rows of band rank-1; below: the first rows of band rank+1
        if self.rank > 0 and a1 < r0:
            pa, pb = rows_of(self.rank - 1)
            top0 = max(pa, pb - e)  # global row of edges[rank-1, 1][:, :, 0]
            ws.y1[:, :, :r0 - a1].copy_(bufs["edges"][self.rank - 1, 1][:, :, a1 - top0:r0 - top0])
        if self.rank + 1 < P and b1 > r1:
            na, _ = rows_of(self.rank + 1)
            ws.y1[:, :, r1 - a1:].copy_(bufs["edges"][self.rank + 1, 0][:, :, :b1 - na])

    def step(self, ws, feats, map_classifier, mark=None) -> torch.Tensor:
        if mark:
            mark("warp")
        if self.engine is not None:  # a rank with views fuses with the same engine
            self.warp(ws, feats)
        if mark:
            mark("conv1")
        self.conv1_partial(ws, map_classifier)
        if mark:
            mark("exchange")
        self.exchange(ws)
        band = self._fuse_engine.finish_from_y1(ws, map_classifier, mark=mark)
        if mark:
            mark("gather_map")
        return self.gather_map(band)


def bench_main(args) -> None:
    """``bench.py`` under torchrun with WORLD_SIZE > 1: frame-parallel (default, ``value``) and the
    view-parallel paths of the north star (RCCL), each timed with barrier + max over ranks."""
    import json
    import os
    import time

    import numpy as np

    from bench import BF16_MFMA_PEAK_TFS, DTYPE_LABEL, FP32_MFMA_PEAK_TFS, build_mc, head_params
    from . import synthetic
    from .geometry import projection_matrices
    from .pipeline import ProjectFuse

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MVBEV_DIST_BACKEND", "nccl")
    # one GPU per rank; on a 1-GPU rehearsal box (gloo) ranks share device 0
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, seed=args.config, C=C), dev)

    def run(mode):
        if mode == "frames":  # frame-parallel: each rank fuses its own frame batch, no collective
            eng = ProjectFuse(pm, up, (ho, wo), C, precision=args.precision,
                              wino_conv1=getattr(args, "conv1", "direct") == "wino")
            feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up,
                                                  seed=1000 * args.config + 100 * rank + v, device=dev)
                     for v in range(N)]
            ws = eng.workspace(B, dev)
            stages = ("warp", "conv1", "conv2", "conv3")
            K, W = args.steps, args.warmup
            ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(K)] for k in stages}
            end = [torch.cuda.Event(enable_timing=True) for _ in range(K)]

            def fstep(mark=None):
                if mark:
                    mark("warp")
                eng.warp_views(ws, list(range(N)), feats)
                return eng.fuse(ws, mc, mark=mark)

            with torch.no_grad():
                for _ in range(W):
                    fstep()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for i in range(K):
                    fstep(mark=lambda s: ev[s][i].record() if s in ev else None)  # (conv1's sub-stage marks)
                    end[i].record()
                torch.cuda.synchronize()
                dist.barrier()
                dt = time.perf_counter() - t0
            t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            nxt = {stages[i]: stages[i + 1] for i in range(len(stages) - 1)}
            stage_ms = {st: round(float(np.mean([ev[st][i].elapsed_time((ev[nxt[st]] if st in nxt else end)[i])
                                                 for i in range(K)])), 4) for st in stages}
            conv1_tfs = 2.0 * B * ho * wo * 9 * N * C * 512 / (stage_ms["conv1"] * 1e-3) / 1e12
            # the MFMA work conv1 executes (frustum-masked), as the single-GPU line reports it
            active = (eng.conv1_active_fraction(dev, ws.y1_rows[0], ws.y1_rows[1] - ws.y1_rows[0], grid=eng.wino_conv1)
                      if args.precision == "bf16x3" else 1.0)
            return dict(value=round(world * B * K / dt, 3), ms=round(dt * 1e3 / K, 4), stage_ms=stage_ms,
                        band=(0, ho), conv1_tfs=conv1_tfs * active, active=active)
        if mode == "partial":
            vp = ViewPartialSum(lambda sv: ProjectFuse(pm, up, (ho, wo), C, slot_views=sv, precision=args.precision,
                                                       all_views=False), pm, (ho, wo), rank, world)
            stages = ("warp", "conv1", "exchange", "conv2", "conv3", "gather_map")
        else:
            vp = ViewParallel(lambda sv: ProjectFuse(pm, up, (ho, wo), C, slot_views=sv, precision=args.precision),
                              pm, (ho, wo), rank, world)
            stages = ("warp", "allgather", "conv1", "conv2", "conv3", "gather_map")
        feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * args.config + v,
                                              device=dev) for v in vp.my_views]
        ws = vp.workspace(B, dev)
        K, W = args.steps, args.warmup
        ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(K)] for k in stages}
        end = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
        with torch.no_grad():
            for _ in range(W):
                vp.step(ws, feats, mc)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for i in range(K):
                vp.step(ws, feats, mc, mark=lambda s: ev[s][i].record())
                end[i].record()
            torch.cuda.synchronize()
            dist.barrier()
            dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        nxt = {stages[i]: stages[i + 1] for i in range(len(stages) - 1)}
        stage_ms = {}
        for st in stages:
            e2 = ev[nxt[st]] if st in nxt else end
            stage_ms[st] = round(float(np.mean([ev[st][i].elapsed_time(e2[i]) for i in range(K)])), 4)
        if mode == "partial":
            conv1_flop = 2.0 * B * ho * wo * 9 * len(vp.my_views) * C * 512
        else:
            y1r = ws.y1_rows
            conv1_flop = 2.0 * B * (y1r[1] - y1r[0]) * wo * 9 * N * C * 512
        conv1_tfs = conv1_flop / (stage_ms["conv1"] * 1e-3) / 1e12
        return dict(value=round(B * K / dt, 3), ms=round(dt * 1e3 / K, 4), stage_ms=stage_ms, band=vp.band,
                    conv1_tfs=conv1_tfs)

    mode = getattr(args, "mp_mode", "frames")
    res = run(mode)
    others = [m for m in ("frames", "partial", "gather") if m != mode]
    def run_alt(m):
        # a failure in a reported-alongside mode (raised on every rank alike, e.g. a collective
        # the fabric rejects) must not cost the `value` line of the mode measured above
        try:
            return run(m)
        except Exception as e:  # noqa: BLE001
            return {"error": f"{type(e).__name__}: {e}"[:300]}

    alts = {} if getattr(args, "no_alt", False) else {m: run_alt(m) for m in others}
    bf16 = args.precision == "bf16x3"
    achieved = res["conv1_tfs"] * (3 if bf16 else 1)
    peak = BF16_MFMA_PEAK_TFS if bf16 else FP32_MFMA_PEAK_TFS
    hows = {"frames": f"frame-parallel x{world}: each rank fuses its own frame batch (all views), no collective",
            "partial": f"view-parallel x{world} ({backend}): views' conv1 partial sums, reduce-scatter by row band "
                       "+ edge-row all-gather",
            "gather": f"view-parallel x{world} ({backend}): all-gather of the warped slab + row-band fusion"}
    if rank == 0:
        line = {
            "metric": "multi-view frames/sec (project+fuse)",
            "value": res["value"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["ms"],
            "higher_is_better": True,
            "scaling": "weak" if mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": DTYPE_LABEL[args.precision],
            "data": "synthetic (see single-GPU line)",
            "config": {"workload": f"cfg{args.config}: {spec['name']}", "views": N, "channels": C,
                       "batch": B * (world if mode == "frames" else 1), "batch_per_rank": B if mode == "frames" else None,
                       "src_hw": list(up), "grid_hw": [ho, wo], "precision": args.precision,
                       "parallelism": hows[mode]},
            "roofline": {"kernel": "conv1 on rank 0" + {"frames": " (all views, whole grid)",
                                                       "partial": " (partial over its views)",
                                                       "gather": " (row band + halo)"}[mode],
                         "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": None},
            "stages_ms_rank0": res["stage_ms"],
            "band_rank0": list(res["band"]),
        }
        if "active" in res:
            line["roofline"]["frustum_active_fraction"] = round(res["active"], 4)
        for m, r in alts.items():
            key = "frame_parallel" if m == "frames" else f"view_parallel_{m}"
            line[key] = r if "error" in r else {
                "value": r["value"], "ms_per_step": r["ms"], "scaling": "weak" if m == "frames" else "strong",
                "parallelism": hows[m], "stages_ms_rank0": r["stage_ms"]}
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()
