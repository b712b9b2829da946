"""Load balance of the frustum-masked conv1 at a BASELINE config (host-side model).

Per output tile (tile_h x 32 pixels + 1-pixel halo) the views whose warp samples inside the
source (float64 restatement of ``mvbev_warp_tile_mask``), then a greedy list schedule of the
workgroups over the CUs in the kernel's dispatch order (heaviest pixel tiles first, dealt
round-robin over the 8 XCDs, 4 Cout tiles per pixel tile): makespan vs the perfect-balance
bound, in chunk units.

    python tools/mask_balance.py [--config 2] [--tile-h 12] [--split 1]
"""
from __future__ import annotations

import argparse
import heapq
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def tile_masks(ds, tile_h, tile_w=32, halo=1):
    H, W = ds.upsample_shape
    ho, wo = ds.reducedgrid_shape
    ty, tx = -(-ho // tile_h), -(-wo // tile_w)
    masks = np.zeros(ty * tx, dtype=np.int64)
    v, u = np.meshgrid(np.arange(ho, dtype=np.float64), np.arange(wo, dtype=np.float64), indexing="ij")
    for s, M in enumerate(projection_matrices(ds)):
        p = np.linalg.inv(M.numpy()) @ np.stack([u.ravel(), v.ravel(), np.ones(u.size)])
        z = np.where(np.abs(p[2]) > 1e-8, p[2], 1.0)
        x, y = p[0] / z, p[1] / z
        inside = ((x > -1) & (x < W) & (y > -1) & (y < H)).reshape(ho, wo)
        for t in range(ty * tx):
            r0, c0 = (t // tx) * tile_h, (t % tx) * tile_w
            if inside[max(0, r0 - halo):r0 + tile_h + halo, max(0, c0 - halo):c0 + tile_w + halo].any():
                masks[t] |= 1 << s
    return masks


def schedule(work, cus=256, xcds=8, n_cot=4):
    """Greedy list schedule: block i goes to XCD i % 8 and, there, to the first free CU."""
    order = sorted(range(len(work)), key=lambda i: -work[i])
    blocks = [work[t] for t in order for _ in range(n_cot)]
    per = cus // xcds
    heaps = [[0.0] * per for _ in range(xcds)]
    for i, w in enumerate(blocks):
        h = heaps[i % xcds]
        t = heapq.heappop(h)
        heapq.heappush(h, t + w)
    return max(max(h) for h in heaps), sum(blocks) / cus


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--tile-h", type=int, default=12)
    args = ap.parse_args()
    cfg = synthetic.CONFIGS[args.config]
    ds = cfg["make"]()
    cpg = cfg["C"] // 16
    m = tile_masks(ds, args.tile_h)
    bits = np.array([bin(int(x)).count("1") for x in m])
    work = (bits * cpg).tolist()
    dense = len(m) * ds.num_cam * cpg
    mk, lb = schedule(work)
    print(f"tile_h {args.tile_h}: {len(m)} pixel tiles, active fraction {sum(work) / dense:.3f}, "
          f"makespan {mk:.0f} chunks vs balanced {lb:.0f} ({mk / lb:.3f}x); dense makespan "
          f"{schedule([ds.num_cam * cpg] * len(m))[0]:.0f}")


def split_schedule(work, cap, cus=256, xcds=8, n_cot=4):
    """Items above `cap` chunks cut into equal K-pieces, then the same greedy schedule."""
    items = []
    for w in work:
        n = max(1, -(-w // cap))
        items += [w / n] * (n * n_cot)
    items.sort(reverse=True)
    per = cus // xcds
    heaps = [[0.0] * per for _ in range(xcds)]
    for i, w in enumerate(items):
        h = heaps[i % xcds]
        heapq.heappush(h, heapq.heappop(h) + w)
    return max(max(h) for h in heaps), sum(items) / cus, len(items)


def lpt_schedule(items, cus=256, xcds=8):
    """Items (descending) dealt to the least-loaded XCD, then the hardware's first-free-CU
    greedy inside each XCD; returns the makespan."""
    items = sorted(items, reverse=True)
    load = [0.0] * xcds
    lists = [[] for _ in range(xcds)]
    for w in items:
        x = min(range(xcds), key=lambda j: load[j])
        load[x] += w
        lists[x].append(w)
    per = cus // xcds
    mk = 0.0
    for lst in lists:
        h = [0.0] * per
        for w in lst:
            heapq.heappush(h, heapq.heappop(h) + w)
        mk = max(mk, max(h))
    return mk


if __name__ == "__main__":
    main()
