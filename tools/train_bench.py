"""Training-step benchmark of the hot path on one GPU.

    python tools/train_bench.py [--config 2] [--steps 10] [--warmup 3] [--no-torch]

Step = forward + backward of warp + concat + fusion head over one frame batch (inputs
resident in HBM, grad w.r.t. the upsampled view features and all head parameters), as
``trainer.py:38-47`` runs it.  "native" = ``autograd.ProjectFuseFunction`` (HIP forward and
backward); "torch" = the reference's own op sequence on the GPU (grid_sample + cat +
nn.Conv2d under autograd, MIOpen convs), the path the detector would otherwise fall back
to.  Prints one JSON line with frames/s and per-stage ms (HIP events).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import build_mc, head_params  # noqa: E402
from mvdet_amd import ProjectFuse, autograd, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def torch_warp(feat, m, ho, wo):
    """kornia steps 3-6 in stock torch GPU ops (autograd through grid_sample)."""
    B = feat.shape[0]
    xs = (torch.linspace(0, wo - 1, wo, device=feat.device) / (wo - 1) - 0.5) * 2
    ys = (torch.linspace(0, ho - 1, ho, device=feat.device) / (ho - 1) - 0.5) * 2
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    pts = torch.stack([gx, gy, torch.ones_like(gx)], -1) @ m.T
    z = pts[..., 2:]
    scale = torch.where(z.abs() > 1e-8, 1.0 / (z + 1e-8), torch.ones_like(z))
    grid = (scale * pts[..., :2]).unsqueeze(0).expand(B, ho, wo, 2)
    return F.grid_sample(feat, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"])
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    dev = torch.device("cuda:0")
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=args.precision)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev).requires_grad_()
             for v in range(N)]
    gmap = torch.randn((B, 1, ho, wo), device=dev)
    res = {"config": f"cfg{args.config}: {spec['name']}", "precision": args.precision}

    def run(step, K, W, hook_stages=None):
        for _ in range(W):
            step(None)
        torch.cuda.synchronize()
        evs = []
        t0 = time.perf_counter()
        for i in range(K):
            marks = {}
            if hook_stages:
                autograd.set_stage_hook(lambda s: marks.setdefault(s, torch.cuda.Event(enable_timing=True)).record())
            step(i)
            autograd.set_stage_hook(None)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks["end"] = e
            evs.append(marks)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out = {"frames_per_s": round(B * K / dt, 3), "ms_per_step": round(dt * 1e3 / K, 3)}
        if hook_stages:
            names = [s for s in evs[0] if s != "end"]
            st = {}
            for a, b in zip(names, names[1:] + ["end"]):
                st[a] = round(float(np.mean([m[a].elapsed_time(m[b]) for m in evs])), 4)
            out["stages_ms"] = st
        return out

    def native_step(i):
        for f in feats:
            f.grad = None
        mc.zero_grad(set_to_none=True)
        out = autograd.project_fuse(eng, feats, mc)
        out.backward(gmap)

    res["native"] = run(native_step, args.steps, args.warmup, hook_stages=True)
    if not args.no_torch:
        ms = [eng.m_norm_cpu[v].to(dev) for v in range(N)]
        cmap = torch.from_numpy(np.stack(np.meshgrid(np.arange(wo) / (wo - 1) * 2 - 1,
                                                     np.arange(ho) / (ho - 1) * 2 - 1), 0)).float()[None].to(dev)

        def torch_step(i):
            for f in feats:
                f.grad = None
            mc.zero_grad(set_to_none=True)
            world = [torch_warp(f, m, ho, wo) for f, m in zip(feats, ms)]
            out = mc(torch.cat(world + [cmap.repeat(B, 1, 1, 1)], 1))
            out.backward(gmap)

        res["torch_gpu"] = run(torch_step, max(2, args.steps // 2), 1)
        res["speedup_vs_torch_gpu"] = round(res["native"]["frames_per_s"] / res["torch_gpu"]["frames_per_s"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
