"""Host-planned schedules for the LDS-DMA ring conv kernel (``mvbev_conv_schedule``).

A ring-kernel launch runs one block per (pixel tile, 128-channel Cout tile); a block's work is
its tile's active 16-channel K-chunks (all of K, or the camera slots a frustum mask enables).
The hardware hands block i to XCD i % 8 and, there, to the first free CU, so a launch whose
blocks do not fill the CUs evenly ends in a partial round: measured with block timestamps
(``tools/ring_stamps.py``), conv1's data gradient at cfg2 (2320 equal blocks on 256 CUs)
leaves 12.6 % of CU-time idle.  The planner here gives each XCD a contiguous share of the
blocks (the order the kernel uses without a schedule, kept for L2 locality), simulates the
first-free-CU dispatch inside each XCD, and cuts the blocks of each XCD's last, partial round
into K-pieces: the pieces write raw partial sums and ``conv_ring_fixup_kernel`` adds them in
K order (deterministic) and writes the tile as the kernel would.  The cut that minimises the
simulated makespan (with a per-block and a per-piece overhead) is kept; with none better the
schedule is plain (no pieces).

Schedules depend only on the geometry (mask, sizes), so callers build them once and reuse
them (``ProjectFuse`` caches per geometry).
"""
from __future__ import annotations

import ctypes
import heapq
from typing import List, Optional, Sequence, Tuple

import torch

from . import _native

XCDS = 8
BLOCK_OVERHEAD = 2.0   # chunk-times per block: pipeline fill from cold caches + epilogue
PIECE_OVERHEAD = 2.0   # extra per piece: partial store + its share of the fixup pass


def _xcd_makespan(works: Sequence[float], cus: int) -> float:
    h = [0.0] * cus
    for w in works:
        heapq.heappush(h, heapq.heappop(h) + w + BLOCK_OVERHEAD)
    return max(h) if works else 0.0


def _split_tail(queue: List[Tuple[int, int]], cus: int, kmax: int):
    """Best cut of one XCD's queue [(tile, chunks)]: the last m blocks in k pieces each.
    Returns (makespan, m, k)."""
    works = [float(c) for _, c in queue]
    best = (_xcd_makespan(works, cus), 0, 1)
    n = len(queue)
    for m in range(1, min(n, cus) + 1):
        head, tail = works[:n - m], works[n - m:]
        for k in (2, 3, 4, 6, 8, 12, 16):
            if k > kmax or any(c / k < 2 for c in tail):
                continue
            pieces = [c / k + PIECE_OVERHEAD for c in tail for _ in range(k)]
            t = _xcd_makespan(head + pieces, cus)
            if t < best[0] * 0.995:
                best = (t, m, k)
    return best


class ConvSchedule:
    """A ring-kernel schedule on ``device``: ``items`` [n, 4] int32 (tile, chunk begin, chunk
    end, partial slot or -1; tile -1 = idle block), ``fixups`` [f, 4] (tile, first slot,
    pieces, 0), the partial-sum workspace, and the ``mvbev_conv_schedule`` struct pointing at
    them.  ``predicted`` / ``predicted_plain``: simulated makespans (chunk-times) with and
    without the pieces."""

    def __init__(self, items, fixups, nslots: int, device, predicted: float, predicted_plain: float):
        dev = torch.device(device)
        self.items = torch.tensor(items if items else [[-1, 0, 0, -1]], dtype=torch.int32, device=dev).reshape(-1, 4)
        self.fixups = torch.tensor(fixups if fixups else [[0, 0, 0, 0]], dtype=torch.int32,
                                   device=dev).reshape(-1, 4)
        slot = int(_native.load().mvbev_conv_schedule_slot_bytes())
        self.partials = torch.empty(max(nslots, 1) * slot // 4, dtype=torch.float32, device=dev)
        self.nitems, self.nfix, self.nslots = len(items), len(fixups), nslots
        self.predicted, self.predicted_plain = predicted, predicted_plain
        self.c = _native.ConvSchedule(self.items.data_ptr(), self.nitems, self.fixups.data_ptr(), self.nfix,
                                      self.nslots, self.partials.data_ptr(),
                                      self.partials.numel() * self.partials.element_size())


def plan(blocks: Sequence[Tuple[int, int]], cus: int, device, split: bool = True,
         kmax: int = 16, force_pieces: int = 0, deal: int = 0) -> ConvSchedule:
    """``blocks``: the launch's (tile, active chunks) in run order (blocks with 0 chunks run
    their epilogue only).  Each XCD takes a contiguous share (equal chunk totals), in order — or, with
    ``deal`` = n_cot, the blocks' pixel tiles (tile // n_cot) are dealt to the XCDs in turn
    (the frustum-masked forward's heavy-first order: every XCD gets the same mix of heavy and
    light tiles, a pixel tile's Cout blocks stay together); with ``split`` each XCD's last
    round is cut into K-pieces where the simulation says so.  ``force_pieces`` > 1 (tests):
    every block in that many pieces.  (Measured on the masked conv1 forward: the tail cut
    ±1 %, cutting every block of > 96 / 128 / 160 chunks in place 6-10 % slower.)"""
    blocks = [(int(t), int(c)) for t, c in blocks]  # 0-chunk blocks still write their epilogue
    per = max(cus // XCDS, 1)
    total = sum(c for _, c in blocks)
    queues: List[List[Tuple[int, int]]] = [[] for _ in range(XCDS)]
    if deal:
        turn, last = -1, None
        for t, c in blocks:
            if t // deal != last:
                turn, last = turn + 1, t // deal
            queues[turn % XCDS].append((t, c))
    else:
        acc, x = 0, 0
        for t, c in blocks:  # contiguous shares by cumulative work
            while x < XCDS - 1 and acc >= total * (x + 1) / XCDS:
                x += 1
            queues[x].append((t, c))
            acc += c
    rows: List[List[Tuple[int, int, int, int]]] = []
    fixups: List[List[int]] = []
    nslots = 0
    pred = pred_plain = 0.0
    for q in queues:
        plain = _xcd_makespan([float(c) for _, c in q], per)
        pred_plain = max(pred_plain, plain)
        t, m, k = _split_tail(q, per, kmax) if split else (plain, 0, 1)
        if force_pieces > 1:
            t, m, k = plain, len(q), force_pieces
        pred = max(pred, t)
        head, tail = q[:len(q) - m], q[len(q) - m:]
        seq = [(tile, 0, c, -1) for tile, c in head]
        for tile, c in tail:
            fixups.append([tile, nslots, k, 0])
            for p in range(k):
                seq.append((tile, c * p // k, c * (p + 1) // k, nslots + p))
            nslots += k
        rows.append(seq)
    n = max(len(r) for r in rows) if rows else 0
    items = []
    for j in range(n):  # block 8 j + x runs queue x's j-th item
        for r in rows:
            items.append(list(r[j]) if j < len(r) else [-1, 0, 0, -1])
    while items and items[-1][0] < 0:
        items.pop()
    return ConvSchedule(items, fixups, nslots, device, pred, pred_plain)


def ring_blocks(B: int, tiles_y: int, tiles_x: int, n_cot: int, chunks: int,
                group_mask: Optional[Sequence[int]] = None, cpg: int = 0,
                out_mask: Optional[Sequence[int]] = None, cot_per_group: int = 1,
                order: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """A ring launch's (tile, active chunks) blocks in run order.  ``group_mask`` (per pixel
    tile ty * tiles_x + tx, input-side frustum mask): chunks = enabled groups x ``cpg``;
    ``out_mask``: Cout tile cot runs where bit cot // cot_per_group is set; ``order``: the
    (b, pixel tile) run order (``heavy_first_order``), else natural."""
    T = tiles_y * tiles_x
    pix = list(order) if order is not None else list(range(B * T))
    out = []
    for pt in pix:
        ptile = pt % T
        nch = chunks
        if group_mask is not None:
            nch = bin(int(group_mask[ptile]) & 0xFFFFFFFF).count("1") * cpg
        for cot in range(n_cot):
            if out_mask is not None and not (int(out_mask[ptile]) >> (cot // cot_per_group)) & 1:
                continue
            out.append((pt * n_cot + cot, nch))
    return out
