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


# ---- torch's CPU sort order, restated (what nms.py:22's scores.sort(0) does on the CPU) ----------
# torch sorts (value, index) pairs with std::sort under KeyValueCompAsc (NaN largest): libstdc++'s
# introsort (median-of-three pivot to the front, unguarded Hoare partition, recursion while a
# range holds > 16 elements, depth limit 2 floor(log2 n) then heap sort, one final insertion
# sort).  Equal scores keep the order this process leaves them in.  The GPU kernel
# (mvdet_amd/csrc/postproc.hip, torch_cpu_sort) replays it level by level; ``std_sort_order``
# is the sequential form, ``level_sort_order`` the kernel's level-synchronous form, and the CPU
# tests pin both against torch.sort itself (random ties, NaN, sorted / reversed runs and
# ``killer_sequence`` inputs that reach the heap-sort fallback).

def _lt(a: float, b: float) -> bool:
    return (not np.isnan(a) and np.isnan(b)) or (a < b)


def _heap_sort(v, ix, f, l, lt=_lt):
    """libstdc++ __make_heap + __sort_heap over [f, l) (the depth-limit fallback)."""
    def adjust(hole, ln, vk, vi):
        top = second = hole
        while second < (ln - 1) // 2:
            second = 2 * (second + 1)
            if lt(v[f + second], v[f + second - 1]):
                second -= 1
            v[f + hole], ix[f + hole] = v[f + second], ix[f + second]
            hole = second
        if (ln & 1) == 0 and second == (ln - 2) // 2:
            second = 2 * (second + 1)
            v[f + hole], ix[f + hole] = v[f + second - 1], ix[f + second - 1]
            hole = second - 1
        parent = (hole - 1) // 2
        while hole > top and lt(v[f + parent], vk):
            v[f + hole], ix[f + hole] = v[f + parent], ix[f + parent]
            hole, parent = parent, (parent - 1) // 2
        v[f + hole], ix[f + hole] = vk, vi
    ln = l - f
    if ln >= 2:
        parent = (ln - 2) // 2
        while True:
            adjust(parent, ln, v[f + parent], ix[f + parent])
            if parent == 0:
                break
            parent -= 1
    last = l
    while last - f > 1:
        last -= 1
        vk, vi = v[last], ix[last]
        v[last], ix[last] = v[f], ix[f]
        adjust(0, last - f, vk, vi)


def _median_to_front(v, ix, f, l, lt=_lt):
    a, b, c = f + 1, f + (l - f) // 2, l - 1
    if lt(v[a], v[b]):
        pick = b if lt(v[b], v[c]) else (c if lt(v[a], v[c]) else a)
    else:
        pick = a if lt(v[a], v[c]) else (c if lt(v[b], v[c]) else b)
    v[f], v[pick] = v[pick], v[f]
    ix[f], ix[pick] = ix[pick], ix[f]


def _insertion_sort(v, ix, f, l, lt=_lt):
    for i in range(f + 1, l):
        vk, vi, j = v[i], ix[i], i
        while j > f and lt(vk, v[j - 1]):
            v[j], ix[j] = v[j - 1], ix[j - 1]
            j -= 1
        v[j], ix[j] = vk, vi


def std_sort_order(values, lt=_lt):
    """Indices of ``values`` in the order torch's CPU ``sort`` (ascending) returns them."""
    v = [float(x) for x in values]
    ix = list(range(len(v)))
    n = len(v)

    def partition(first, last, piv):
        while True:
            while lt(v[first], v[piv]):
                first += 1
            last -= 1
            while lt(v[piv], v[last]):
                last -= 1
            if not first < last:
                return first
            v[first], v[last] = v[last], v[first]
            ix[first], ix[last] = ix[last], ix[first]
            first += 1

    def loop(first, last, depth):
        while last - first > 16:
            if depth == 0:
                _heap_sort(v, ix, first, last, lt)
                return
            depth -= 1
            _median_to_front(v, ix, first, last, lt)
            cut = partition(first + 1, last, first)
            loop(cut, last, depth)
            last = cut

    if n > 1:
        loop(0, n, 2 * (n.bit_length() - 1))
        _insertion_sort(v, ix, 0, n, lt)
    return ix


def level_sort_order(values):
    """The same order, computed as the GPU kernel does: every range of one recursion depth
    partitioned at once, each Hoare partition from prefix counts (the k-th element >= p from the
    left swaps with the k-th element <= p from the right for k <= m = max_x min(#left stops before
    x, #right stops from x); cut = L_1 if m = 0 else min(L_{m+1}, R_m)), then a stable insertion
    sort per final range."""
    v = [float(x) for x in values]
    ix = list(range(len(v)))
    n = len(v)
    if n <= 1:
        return ix
    ranges, final = [(0, n, 2 * (n.bit_length() - 1))], []
    while ranges:
        nxt = []
        for f, l, d in ranges:
            if l - f <= 16:
                final.append((f, l))
                continue
            if d == 0:
                _heap_sort(v, ix, f, l)
                continue
            _median_to_front(v, ix, f, l)
            p = v[f]
            left = [i for i in range(f + 1, l) if not _lt(v[i], p)]
            right = [i for i in range(l - 1, f, -1) if not _lt(p, v[i])]
            inc_l = inc_r = m = 0
            for i in range(f + 1, l):
                inc_l += not _lt(v[i], p)
                inc_r += not _lt(p, v[i])
                m = max(m, min(inc_l, len(right) - inc_r))
            for k in range(m):
                a, b = left[k], right[k]
                v[a], v[b] = v[b], v[a]
                ix[a], ix[b] = ix[b], ix[a]
            cut = left[0] if m == 0 else min(left[m] if m < len(left) else l, right[m - 1])
            nxt += [(f, cut, d - 1), (cut, l, d - 1)]
        ranges = nxt
    for f, l in final:
        _insertion_sort(v, ix, f, l)
    return ix


def killer_sequence(n: int) -> np.ndarray:
    """McIlroy's adversary ("A killer adversary for quicksort", 1999) run against
    ``std_sort_order``: values are decided lazily so every median-of-three partition is lopsided,
    which drives the introsort to its heap-sort fallback.  float32 [n]."""
    gas = [True] * n
    val = [0.0] * n
    state = {"solid": 0, "cand": 0}

    def lt(a, b):  # a, b are the original indices (the sorted payload is the index itself)
        a, b = int(a), int(b)
        if gas[a] and gas[b]:
            x = a if a == state["cand"] else b
            gas[x], val[x] = False, float(state["solid"])
            state["solid"] += 1
        if gas[a]:
            state["cand"] = a
        elif gas[b]:
            state["cand"] = b
        va = np.inf if gas[a] else val[a]
        vb = np.inf if gas[b] else val[b]
        return va < vb

    std_sort_order(list(range(n)), lt=lt)
    out = [state["solid"] + i if g else x for i, (g, x) in enumerate(zip(gas, val))]
    return np.asarray(out, dtype=np.float32)
