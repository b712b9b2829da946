"""HIP-graph A/B of the inference frame at a config: the frame's launches issued eagerly (bench.py's
step) against the same launches captured once into a graph (torch.cuda.CUDAGraph over the engine's
ctypes launches on the capturing stream) and replayed.  Checks the replayed map equals the eager one
bitwise and prints one JSON line per round.  python tools/graph_ab.py [--config 2] [--steps 300]"""
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
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=4)
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
    ws = eng.workspace(B, dev)
    K = args.steps

    def frame():
        eng.warp_views(ws, views, feats)
        return eng.fuse(ws, mc)

    with torch.no_grad():
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                ref = frame()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        ref = ref.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = frame()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref), "graph replay differs from the eager frame"
        for r in range(args.rounds):
            res = {"round": r, "config": args.config, "steps": K}
            for name, fn in (("eager", frame), ("graph", g.replay)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(K):
                    fn()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                res[name + "_fps"] = round(B * K / dt, 2)
                res[name + "_ms"] = round(1e3 * dt / K, 4)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
