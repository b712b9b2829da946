"""Golden vectors for the post-processing row from the reference.

Runs ONLY in the build container (needs ``/root/reference``): imports the reference's own
``multiview_detector/utils/nms.py`` (it depends on torch only) by file path and records its
outputs on seeded inputs shaped like the evaluation loop's (``trainer.py:97-106,148-157``):
integer grid positions scaled by ``grid_reduce``, scores above ``cls_thres``, ties included.
The threshold / nonzero step of ``trainer.py:97-105`` is stock torch and is restated in
``run_trainer_case`` line by line; its NMS call is the reference function itself.

Usage:  python tools/gen_golden_nms.py        (writes tests/golden/nms_cases.npz)
"""
from __future__ import annotations

import importlib.util
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
REF_NMS = Path("/root/reference/multiview_detector/utils/nms.py")
OUT = ROOT / "tests" / "golden" / "nms_cases.npz"


def load_ref_nms():
    spec = importlib.util.spec_from_file_location("ref_nms", REF_NMS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.nms


def run_trainer_case(nms, map_res, frame, cls_thres, grid_reduce, indexing):
    """trainer.py:97-105 (threshold + nonzero + rows) and :148-156 (per-frame NMS)."""
    map_grid_res = map_res.detach().cpu().squeeze()
    v_s = map_grid_res[map_grid_res > cls_thres].unsqueeze(1)
    grid_ij = (map_grid_res > cls_thres).nonzero()
    grid_xy = grid_ij[:, [1, 0]] if indexing == "xy" else grid_ij
    rows = torch.cat([torch.ones_like(v_s) * frame, grid_xy.float() * grid_reduce, v_s], dim=1)
    res = rows[rows[:, 0] == frame, :]
    positions, scores = res[:, 1:3], res[:, 3]
    ids, count = nms(positions, scores, 20, np.inf)
    final = torch.cat([torch.ones([count, 1]) * frame, positions[ids[:count], :]], dim=1)
    return rows.numpy(), final.numpy()


def main():
    nms = load_ref_nms()
    rng = np.random.default_rng(2024)
    out = {}
    cases = [(50, 50 / 2.5, 50), (300, 20.0, np.inf), (1000, 20.0, np.inf), (64, 8.0, 10), (2000, 12.0, np.inf)]
    for i, (K, dist, top_k) in enumerate(cases):
        pts = (rng.integers(0, 120, size=(K, 2)) * 4).astype(np.float32)
        sc = rng.uniform(0.4, 1.0, size=K).astype(np.float32)
        sc[rng.integers(0, K, size=K // 5)] = np.float32(0.75)  # ties
        keep, count = nms(torch.from_numpy(pts), torch.from_numpy(sc), dist, top_k)
        out.update({f"c{i}_points": pts, f"c{i}_scores": sc, f"c{i}_dist": np.float64(dist),
                    f"c{i}_topk": np.float64(top_k), f"c{i}_keep": keep.numpy(), f"c{i}_count": np.int64(count)})
    # trainer-style maps: smooth blobs, threshold 0.4, Wildtrack 'ij' and MultiviewX 'xy'
    for j, (H, W, indexing) in enumerate([(120, 360, "ij"), (160, 250, "xy")]):
        yy, xx = np.mgrid[0:H, 0:W]
        m = np.zeros((H, W), np.float32)
        for _ in range(25):
            cy, cx = rng.uniform(0, H), rng.uniform(0, W)
            m += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * rng.uniform(1.5, 4) ** 2)).astype(np.float32)
        m += rng.uniform(0, 0.05, size=m.shape).astype(np.float32)
        rows, final = run_trainer_case(nms, torch.from_numpy(m)[None, None], 7, 0.4, 4, indexing)
        out.update({f"map{j}": m, f"map{j}_indexing": np.array(indexing), f"map{j}_rows": rows,
                    f"map{j}_final": final})
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items() if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
