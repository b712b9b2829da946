"""Host-side model of conv_wino_kernel's beyond-L2 traffic at a BASELINE config.

Every workgroup (pixel tile, Cout tile) walks its units (active view chunk, xi) one per time
step; per unit it reads 24 KiB of G w (shared by every pixel tile with that view) and 8.5 KiB
of T (shared by the 4 Cout tiles of its pixel tile).  Workgroups are dispatched as the kernel
deals them (blockIdx & 7 = XCD, first free CU of 32 per XCD) and each XCD's 4 MiB L2 is an LRU
over those blocks.  Prints the bytes that miss L2 per launch for the current order and for
alternatives, to decide what to try on the GPU (the model ignores stalls and the Infinity
Cache; compare its current-order figure with the PMC's 4.7 GB before trusting a delta).

    python tools/l2sim.py [--config 2]
"""
from __future__ import annotations

import argparse
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import synthetic  # noqa: E402
from tools.mask_balance import tile_masks  # noqa: E402

WB, TB = 24 * 1024, 8704  # bytes per unit: G w (3 kernel columns x hi/lo x 128 Cout x 16 ch), T row
L2 = 4 << 20


def simulate(order, masks, cpg, n_cot=4, xcds=8, per=32, view_order=None, chunk_rot=None):
    """order: pixel-tile run order (slots); returns (miss bytes, makespan in units)."""
    npix = len(order)
    blocks = [[] for _ in range(xcds)]
    for x in range(xcds):
        q = 0
        while 8 * q + x < npix:
            for c in range(n_cot):
                blocks[x].append((order[8 * q + x], c))
            q += 1
    miss = 0
    makespan = 0
    for x in range(xcds):
        lru: OrderedDict = OrderedDict()
        used = 0
        queue = list(blocks[x])
        cus = [None] * per  # (iterator over units) per CU
        t = 0

        def units(tile, cot):
            views = [v for v in range(32) if (masks[tile] >> v) & 1]
            if view_order is not None:
                views = view_order(tile, views)
            for v in views:
                for ch in range(cpg):
                    ch2 = (ch + (chunk_rot(tile, v) if chunk_rot else 0)) % cpg
                    for xi in range(5):
                        yield ("w", v, ch2, xi, cot), WB
                        yield ("t", tile, v, ch2, xi), TB

        while queue or any(c is not None for c in cus):
            for i in range(per):
                if cus[i] is None and queue:
                    cus[i] = units(*queue.pop(0))
            for i in range(per):
                it = cus[i]
                if it is None:
                    continue
                for _ in range(2):
                    try:
                        key, nb = next(it)
                    except StopIteration:
                        cus[i] = None
                        break
                    if key in lru:
                        lru.move_to_end(key)
                    else:
                        miss += nb
                        lru[key] = nb
                        used += nb
                        while used > L2:
                            _, b = lru.popitem(last=False)
                            used -= b
            t += 1
        makespan = max(makespan, t)
    return miss, makespan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    args = ap.parse_args()
    cfg = synthetic.CONFIGS[args.config]
    ds = cfg["make"]()
    cpg = cfg["C"] // 16
    m = [int(v) for v in tile_masks(ds, 12)]
    bits = [bin(v).count("1") for v in m]
    T = len(m)
    heavy = sorted(range(T), key=lambda i: (-bits[i], m[i], i))
    print(f"{T} pixel tiles; active units/tile avg {np.mean(bits) * cpg * 5:.0f}")
    for name, order, vo in [
        ("current (heavy-first, masks grouped)", heavy, None),
        ("heavy-first, views walked most-common-first", heavy,
         lambda tile, views: sorted(views, key=lambda v: -sum((mm >> v) & 1 for mm in m))),
        ("heavy-first, views rotated by tile parity", heavy,
         lambda tile, views: views[tile % len(views):] + views[:tile % len(views)]),
    ]:
        ms, mk = simulate(order, m, cpg, view_order=vo)
        print(f"{name:50s} miss {ms / 1e9:.2f} GB  makespan {mk} unit-steps")


if __name__ == "__main__":
    main()
