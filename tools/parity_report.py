"""Parity of the HIP path vs the CPU oracle at a BASELINE config, per stage (GPU box).

    python tools/parity_report.py [--config 2] [--precision fp32|bf16x3]
Prints one JSON line: normwise max|d|/max|ref| and the elementwise-gate violations for
every view's warp, conv1, conv2 and map_result.
"""
import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from helpers import parity_stats  # noqa: E402
from bench import build_mc  # noqa: E402
from mvdet_amd import ProjectFuse, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402
from oracle import cpu_path, fixtures  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--conv1", default="direct", choices=["direct", "wino"],
                    help="conv1 form (bf16x3): the direct ring conv or row-Winograd F(3,3) with the fused warp")
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C = spec["B"], spec["C"]
    if args.config == 4:
        B = 1  # keep the CPU oracle run short; the fp16-storage path is exercised per frame
    up = ds.upsample_shape
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * args.config + v)
             for v in range(ds.num_cam)]
    half = args.config == 4
    if half:
        feats = [f.half().float() for f in feats]  # the reference runs on the upcast fp16 values
    params = fixtures.head_params(ds.num_cam, seed=args.config, C=C)
    pm = projection_matrices(ds)
    eng = ProjectFuse(pm, tuple(up), tuple(ds.reducedgrid_shape), C, precision=args.precision,
                      slab_dtype=torch.float16 if half else torch.float32,
                      wino_conv1=args.conv1 == "wino" and args.precision == "bf16x3")
    mc = build_mc(C, ds.num_cam, params, "cuda:0")
    with torch.no_grad():
        got = eng.project_fuse([f.to("cuda:0", torch.float16 if half else torch.float32) for f in feats], mc)
        torch.cuda.synchronize()
        keep = {}
        ref = cpu_path.project_fuse(feats, [M.numpy() for M in pm], tuple(ds.reducedgrid_shape),
                                    {k: torch.from_numpy(v) for k, v in params.items()}, keep=keep)
    ws = eng.workspace(B, "cuda:0")
    with torch.no_grad():  # inference fuses conv2 into conv3 (no y2 in HBM): run conv2 alone for its parity
        eng.conv2(ws, mc[2])
    rep = {"config": args.config, "precision": args.precision, "slab": str(eng.slab_dtype),
           "conv1_form": "row-Winograd, warp writes T" if ws.t_from_warp else "direct"}
    if not ws.t_from_warp:  # the fused warp writes conv1's row transform, not the slab
        rep["warp_worst_normwise"] = max(parity_stats(eng.view_slice(ws, v).float().cpu(),
                                                      keep["warped"][v])["normwise"] for v in range(ds.num_cam))
    for name, g, r in (("conv1", eng.y1_fp32(ws), keep["conv1_relu"]), ("conv2", ws.y2, keep["conv2_relu"]),
                       ("map_result", got, ref)):
        s = parity_stats(g.cpu(), r)
        rep[name] = {"normwise": s["normwise"], "gate_violations": s["n_bad"]}
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
