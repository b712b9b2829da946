"""Evaluation post-processing on the GPU.

Drop-ins for the CPU loop of ``multiview_detector/trainer.py:97-106,148-157`` and for
``multiview_detector/utils/nms.py:7-43`` (same names, arguments and return values), on the
HIP kernels of ``libmvbev.so`` (``mvbev_threshold_points``, ``mvbev_point_nms_ws``):

* ``nms(points, scores, dist_thres=50/2.5, top_k=50) -> (keep, count)``: greedy point NMS.
  Returns ``keep`` alone for empty input, like the reference.  Equal scores are taken in the
  order torch's CPU ``scores.sort(0)`` leaves them (the kernel replays its introsort), so the
  kept set matches the reference's exactly, ties included.  That replay is of the sort the
  installed torch uses (validated on torch 2.10.0+rocm7.0's CPU ``sort``: libstdc++ ``std::sort``
  introsort of (score, index) pairs, NaN largest); a torch build with another sort (a stable or
  radix path, another libstdc++) could order equal scores differently, and
  ``tests/test_oracle.py::test_sort_order_restatement_matches_torch_cpu_sort`` — which compares the
  replay with the running torch's own ``sort`` on ties, NaN and introsort's heap-sort fallback —
  then fails rather than letting the kept set drift silently.
* ``threshold_rows(map_res, frame, cls_thres, grid_reduce, indexing)``: the (frame, x, y,
  score) rows of ``map_res > cls_thres`` in ``nonzero`` order.
* ``frame_results(rows, dist_thres=20, top_k=inf)``: per-frame NMS -> (frame, x, y) rows.
"""
from __future__ import annotations

import math

import torch

from . import _native
from .ops import _require_cuda, _stream

_CAP = 1 << 16  # threshold hits read back per map (the rest is counted, then re-run larger)


def _dev(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_cuda else t.to("cuda:0")


def nms(points: torch.Tensor, scores: torch.Tensor, dist_thres=50 / 2.5, top_k=50):
    keep = torch.zeros_like(scores).long()
    if points.numel() == 0:
        return keep  # (sic) nms.py:23-24 returns the tensor alone here
    pts = _dev(points).float().contiguous()
    sc = _dev(scores).float().contiguous()
    _require_cuda(pts, sc)
    K = sc.numel()
    k = K if (isinstance(top_k, float) and math.isinf(top_k)) else min(int(top_k), K)
    out = torch.empty(K, dtype=torch.int64, device=sc.device)
    cnt = torch.empty(1, dtype=torch.int32, device=sc.device)
    lib = _native.load()
    # any K (nms.py accepts any; trainer.py:154 hands it every map cell over cls_thres)
    nws = int(lib.mvbev_point_nms_workspace_bytes(K, max(k, 1)))
    ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=sc.device)
    st = lib.mvbev_point_nms_ws(pts.data_ptr(), sc.data_ptr(), K, float(dist_thres), max(k, 1),
                                out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), nws, _stream(sc))
    _native.check(st, "mvbev_point_nms_ws")
    return out.to(keep.device), int(cnt.item())


def threshold_rows(map_res: torch.Tensor, frame, cls_thres: float, grid_reduce: int, indexing: str = "ij"):
    """trainer.py:97-105 on the GPU: [n, 4] rows (frame, x, y, score) on the map's device."""
    m = _dev(map_res.detach()).squeeze().float().contiguous()
    _require_cuda(m)
    H, W = m.shape
    lib = _native.load()
    cap = _CAP
    while True:
        cnt = torch.zeros(1, dtype=torch.int32, device=m.device)
        ij = torch.empty((cap, 2), dtype=torch.int32, device=m.device)
        val = torch.empty(cap, dtype=torch.float32, device=m.device)
        st = lib.mvbev_threshold_points(m.data_ptr(), H, W, float(cls_thres), cnt.data_ptr(), ij.data_ptr(),
                                        val.data_ptr(), cap, _stream(m))
        _native.check(st, "mvbev_threshold_points")
        n = int(cnt.item())
        if n <= cap:
            break
        cap = n
    ij, val = ij[:n].float(), val[:n, None]
    xy = ij[:, [1, 0]] if indexing == "xy" else ij
    return torch.cat([torch.full_like(val, float(frame)), xy * grid_reduce, val], dim=1)


def frame_results(rows: torch.Tensor, dist_thres=20, top_k=math.inf) -> torch.Tensor:
    """trainer.py:148-156: per-frame NMS of the rows -> [m, 3] (frame, x, y)."""
    out = []
    for frame in torch.unique(rows[:, 0]).tolist():
        res = rows[rows[:, 0] == frame, :]
        positions, scores = res[:, 1:3], res[:, 3]
        ids, count = nms(positions, scores, dist_thres, top_k)
        ids = ids.to(positions.device)
        out.append(torch.cat([torch.full((count, 1), frame, device=positions.device),
                              positions[ids[:count], :]], dim=1))
    return torch.cat(out, 0) if out else torch.empty((0, 3), device=rows.device)
