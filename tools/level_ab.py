"""A/B of the row-Winograd conv1 dispatched as the kernel deals it (heavy-first pixel tiles, XCD turns) vs
through the leveling schedule (ProjectFuse level_conv1: schedule.plan_level + the ring fixup), at a config:
the map difference, the planner's predicted makespans, and interleaved timings of conv1 alone and of the
whole frame.  python tools/level_ab.py [--config 2] [--batch 0] [--steps 200] [--rounds 3]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import ProjectFuse, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402
from bench import build_mc, head_params  # noqa: E402


def timed(fn, K):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(K):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--block-overhead", type=float, default=0.0, help="plan_level block overhead (0 = engine's)")
    ap.add_argument("--piece-overhead", type=float, default=0.0)
    ap.add_argument("--min-piece", type=int, default=0)
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = (args.batch or spec["B"]), spec["C"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    engs = {"plain": ProjectFuse(pm, up, grid, C), "level": ProjectFuse(pm, up, grid, C, level_conv1=True)}
    lv = engs["level"]
    if args.block_overhead:
        lv.LEVEL_BLOCK_OVERHEAD = args.block_overhead
    if args.piece_overhead:
        lv.LEVEL_PIECE_OVERHEAD = args.piece_overhead
    if args.min_piece:
        lv.LEVEL_MIN_PIECE = args.min_piece
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * args.config + v, device=dev)
             for v in range(N)]
    views = list(range(N))
    wss = {k: e.workspace(B, dev) for k, e in engs.items()}
    outs = {}
    with torch.no_grad():
        for k, e in engs.items():
            e.warp_views(wss[k], views, feats)
            outs[k] = e.fuse(wss[k], mc).clone()
        torch.cuda.synchronize()
        a, b = outs["plain"].double(), outs["level"].double()
        diff = float((a - b).norm() / max(a.norm(), 1e-30))
        sc = lv.conv1_level_schedule(dev, 0, grid[0], B)
        head = {"config": args.config, "B": B, "map_normwise_diff": diff, "items": sc.nitems, "fixups": sc.nfix,
                "predicted": round(sc.predicted, 1), "predicted_plain": round(sc.predicted_plain, 1),
                "overheads": [lv.LEVEL_BLOCK_OVERHEAD, lv.LEVEL_PIECE_OVERHEAD, lv.LEVEL_MIN_PIECE]}
        print(json.dumps(head), flush=True)
        assert diff < 2e-5, diff  # pieces change the fp32 summation order only (3xbf16 vs fp64: ~1e-5)
        init = {k: e.coord_term(mc[0]) for k, e in engs.items()}
        d1 = {k: e._conv1_desc(B) for k, e in engs.items()}

        def conv1(k):
            return lambda: engs[k].conv1_wino(wss[k], mc[0], d1[k], init[k])

        def frame(k):
            def f():
                engs[k].warp_views(wss[k], views, feats)
                engs[k].fuse(wss[k], mc)
            return f
        for r in range(args.rounds):
            res = {"round": r}
            for k in engs:
                res[f"conv1_{k}_ms"] = round(timed(conv1(k), args.steps), 4)
            for k in engs:
                res[f"frame_{k}_ms"] = round(timed(frame(k), args.steps), 4)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
