"""Frame overlap A/B at a config: frames one after another on one stream (bench.py's step) against
frame i+1's warp on a side stream beside frame i's convs (two workspaces alternating), with the
convs' stream at default or high priority.  Prints one JSON line per round of the three variants
and checks the overlapped maps equal the sequential ones bitwise.
python tools/overlap_ab.py [--config 2] [--steps 200] [--rounds 3]"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import ProjectFuse, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402
from bench import build_mc, head_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(pm, up, grid, C)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * args.config + v, device=dev)
             for v in range(N)]
    views = list(range(N))
    ws = [eng.workspace(B, dev), eng.workspace(B, dev)]
    K = args.steps

    def sequential():
        out = None
        for _ in range(K):
            eng.warp_views(ws[0], views, feats)
            out = eng.fuse(ws[0], mc)
        return out

    def overlapped(prio):
        main_s = torch.cuda.Stream(dev, priority=prio)
        side = torch.cuda.Stream(dev)
        fused = [None, None]
        out = None
        main_s.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        for i in range(K):
            w = ws[i % 2]
            with torch.cuda.stream(side):
                if fused[i % 2] is not None:
                    side.wait_event(fused[i % 2])  # frame i-2's convs are done with this workspace
                eng.warp_views(w, views, feats)
                ready = torch.cuda.Event()
                ready.record(side)
            with torch.cuda.stream(main_s):
                main_s.wait_event(ready)
                out = eng.fuse(w, mc)
                done = torch.cuda.Event()
                done.record(main_s)
                fused[i % 2] = done
        torch.cuda.current_stream().wait_stream(main_s)
        torch.cuda.current_stream().wait_stream(side)
        return out

    variants = {"sequential": sequential, "overlap": lambda: overlapped(0), "overlap_hiprio": lambda: overlapped(-1)}
    with torch.no_grad():
        ref = None
        for name, fn in variants.items():  # warm-up + parity
            out = fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), name
        for r in range(args.rounds):
            res = {"round": r, "config": args.config, "steps": K}
            for name, fn in variants.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                res[name + "_fps"] = round(B * K / dt, 2)
                res[name + "_ms"] = round(1e3 * dt / K, 4)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
