"""Oracle: the reference's evaluation post-processing.  TEST INFRASTRUCTURE ONLY.

Restates:
* ``nms``            ``multiview_detector/utils/nms.py:7-43`` — greedy point NMS: scores sorted
  ascending (torch CPU sort), repeatedly take the last (largest) index, drop the candidates
  within ``dist_thres`` (kept only if distance > dist_thres), ``top_k`` largest considered.
* ``threshold_rows`` ``trainer.py:97-105`` — ``map > cls_thres``, ``nonzero`` (row-major),
  (frame, x, y, score) rows with grid coordinates scaled by ``grid_reduce``.
* ``frame_results``  ``trainer.py:148-156`` — per-frame NMS (dist 20, top_k inf), (frame, x, y).
Pinned by ``tests/golden/nms_cases.npz`` (the reference's own nms, ``tools/gen_golden_nms.py``).
"""
from __future__ import annotations

import numpy as np
import torch


def nms(points: torch.Tensor, scores: torch.Tensor, dist_thres=50 / 2.5, top_k=50):
    keep = torch.zeros_like(scores).long()
    if points.numel() == 0:
        return keep
    v, indices = scores.sort(0)
    top_k = min(top_k, len(indices))
    indices = indices[-top_k:]
    count = 0
    while indices.numel() > 0:
        idx = indices[-1]
        keep[count] = idx
        count += 1
        if indices.numel() == 1:
            break
        indices = indices[:-1]
        dists = torch.norm(points[idx, :] - points[indices, :], dim=1)
        indices = indices[dists > dist_thres]
    return keep, count


def threshold_rows(map_res: torch.Tensor, frame, cls_thres: float, grid_reduce: int, indexing: str):
    m = map_res.detach().cpu().squeeze()
    v_s = m[m > cls_thres].unsqueeze(1)
    grid_ij = (m > cls_thres).nonzero()
    grid_xy = grid_ij[:, [1, 0]] if indexing == "xy" else grid_ij
    return torch.cat([torch.ones_like(v_s) * frame, grid_xy.float() * grid_reduce, v_s], dim=1)


def frame_results(rows: torch.Tensor, dist_thres=20, top_k=np.inf):
    out = []
    for frame in np.unique(rows[:, 0].numpy()):
        res = rows[rows[:, 0] == frame, :]
        positions, scores = res[:, 1:3], res[:, 3]
        ids, count = nms(positions, scores, dist_thres, top_k)
        out.append(torch.cat([torch.ones([count, 1]) * frame, positions[ids[:count], :]], dim=1))
    return torch.cat(out, 0) if out else torch.empty((0, 3))
