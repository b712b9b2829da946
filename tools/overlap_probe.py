"""Probe: frames/s of the cfg2 forward with 1 stream vs consecutive frames alternating over
S streams (one workspace each), so one frame's HBM-bound warp can overlap another frame's
MFMA-bound conv1.  Prints one JSON line per (streams, layout)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--streams", default="1,2,3")
    ap.add_argument("--layout", default="nchw")
    args = ap.parse_args()
    from bench import build_mc, head_params
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    dev = torch.device("cuda", 0)
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, seed=args.config, C=C), dev)
    eng = ProjectFuse(pm, up, tuple(ds.reducedgrid_shape), C, precision="bf16x3", wino_conv1=True, wino_conv2=True)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * args.config + v, device=dev)
             for v in range(N)]
    if args.layout == "channels_last":
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    views = list(range(N))
    smax = max(int(s) for s in args.streams.split(","))
    wss = [eng.workspace(B, dev) for _ in range(smax)]
    streams = [torch.cuda.Stream(dev) for _ in range(smax)]
    outs = [None] * smax
    with torch.no_grad():
        for ws in wss:  # warm every workspace on the default stream
            eng.warp_views(ws, views, feats)
            eng.fuse(ws, mc)
        torch.cuda.synchronize()
        for r in range(args.rounds):
            for S in [int(s) for s in args.streams.split(",")]:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    k = i % S
                    st = streams[k]
                    with torch.cuda.stream(st):
                        eng.warp_views(wss[k], views, feats)
                        outs[k] = eng.fuse(wss[k], mc)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(json.dumps({"round": r, "streams": S, "layout": args.layout,
                                  "fps": round(B * args.steps / dt, 2), "ms_per_frame": round(1e3 * dt / args.steps, 4)}),
                      flush=True)
        # the outputs agree with a single-stream frame
        with torch.cuda.stream(streams[0]):
            eng.warp_views(wss[0], views, feats)
            a = eng.fuse(wss[0], mc).clone()
        torch.cuda.synchronize()
        for k in range(1, smax):
            print(json.dumps({"check_stream": k, "equal": bool(torch.equal(a, outs[k]))}))


if __name__ == "__main__":
    main()
