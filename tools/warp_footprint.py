"""Source-read floor of the warp at a BASELINE config: distinct touched source pixels
(T_v) and the bytes of the 32/64/128-B granules that contain them, per
channel plane (NCHW fp32) — what an ideal gather must fetch from HBM.

    python tools/warp_footprint.py [--config 2]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def touched(M, H, W, ho, wo):
    v, u = np.meshgrid(np.arange(ho, dtype=np.float64), np.arange(wo, dtype=np.float64), indexing="ij")
    p = np.linalg.inv(M) @ np.stack([u.ravel(), v.ravel(), np.ones(u.size)])
    ok = np.abs(p[2]) > 1e-8
    zs = np.where(ok, p[2], 1.0)
    x = np.floor(np.where(ok, p[0] / zs, -10.0))
    y = np.floor(np.where(ok, p[1] / zs, -10.0))
    seen = np.zeros((H, W), bool)
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x + dx, y + dy
            inb = (xi >= 0) & (xi <= W - 1) & (yi >= 0) & (yi <= H - 1)
            seen[yi[inb].astype(np.int64), xi[inb].astype(np.int64)] = True
    inside = float(((x >= -1) & (x <= W - 1) & (y >= -1) & (y <= H - 1)).mean())
    return seen, inside


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    args = ap.parse_args()
    cfg = synthetic.CONFIGS[args.config]
    ds = cfg["make"]()
    C, B = cfg["C"], cfg["B"]
    H, W = ds.upsample_shape
    ho, wo = ds.reducedgrid_shape
    tot = {}
    for cam, M in enumerate(projection_matrices(ds)):
        seen, inside = touched(M.numpy(), H, W, ho, wo)
        r = {"pixels": int(seen.sum())}
        for g in (8, 16, 32):
            Wp = -(-W // g) * g
            s = np.zeros((H, Wp), bool)
            s[:, :W] = seen
            r[f"{4 * g}B"] = int(s.reshape(H, Wp // g, g).any(-1).sum()) * g
        print(f"view {cam}: inside {inside:.3f} " + " ".join(f"{k}={v / (H * W):.3f}" for k, v in r.items()))
        for k, v in r.items():
            tot[k] = tot.get(k, 0) + v
    for k, v in tot.items():
        print(f"read floor at {k:7s} granules: {4 * B * C * v / 1e9:.3f} GB")
    print(f"write: {4 * B * C * ds.num_cam * ho * wo / 1e9:.3f} GB; full source {4 * B * C * ds.num_cam * H * W / 1e9:.3f} GB")


if __name__ == "__main__":
    main()
