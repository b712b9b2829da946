"""Per-kernel micro-benchmark of the hot-path kernels at a BASELINE config (GPU box).

    python tools/kbench.py [--config 2] [--reps 20] [--only warp,warpup,conv1,conv2,conv3]

Times each stage alone with HIP events on torch's current stream (the stream the
kernels are launched on) and prints one JSON line per stage.  Used for A/B work on
the kernels and as the target of rocprofv3 --pmc passes.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import build_mc, head_params  # noqa: E402
from mvdet_amd import ProjectFuse, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    return float(np.median(t)), float(np.min(t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"],
                    help="conv1/conv2 arithmetic: fp32 MFMA or 3xbf16 split (fp32-class accuracy)")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="warp,conv1,conv2,conv3")
    ap.add_argument("--libs", default="", help="comma-separated libmvbev variants to A/B (interleaved rounds)")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--no-frustum", action="store_true", help="dense conv1 (no frustum mask)")
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    dev = torch.device("cuda:0")
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=args.precision, frustum=not args.no_frustum)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev) for v in range(N)]
    bfeats = [synthetic.backbone_features(B, C, [u // 3 for u in up], seed=v, device=dev) for v in range(N)]
    ws = eng.workspace(B, dev)
    with torch.no_grad():
        for v in range(N):
            eng.warp_view(ws, v, feats[v])
        eng.fuse(ws, mc)
        stages = {
            "warp": (lambda: eng.warp_views(ws, list(range(N)), feats), None),
            "warpup": (lambda: eng.warp_views_upsampled(ws, list(range(N)), bfeats), None),
            "warp1": (lambda: [eng.warp_view(ws, v, feats[v]) for v in range(N)], None),
            "conv1": (lambda: eng.conv1(ws, mc[0]), 2.0 * B * ho * wo * 9 * N * C * 512),
            "conv2": (lambda: eng.conv2(ws, mc[2]), 2.0 * B * ho * wo * 9 * 512 * 512),
            "conv3": (lambda: eng.conv3(ws, mc[4]), None),
        }
        from mvdet_amd import _native
        libs = [("default", _native.load())]
        for path in filter(None, args.libs.split(",")):
            libs.append((Path(path).stem, _native.load(path)))
        for rnd in range(args.rounds):
            for lname, lib in libs:
                _native._lib = lib
                for name in args.only.split(","):
                    fn, flop = stages[name]
                    med, mn = timeit(fn, args.reps)
                    rec = {"stage": name, "lib": lname, "round": rnd, "config": args.config,
                           "median_ms": round(med, 4), "min_ms": round(mn, 4)}
                    if flop:
                        rec["TFLOPs"] = round(flop / (med * 1e-3) / 1e12, 2)
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
