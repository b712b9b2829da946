"""List-scheduling model of conv1's workgroup makespan (CPU only; DESIGN.md §8 "Next").

Per (tile_h x 32) output tile the number of views whose frustum reaches the tile's 3x3 halo is taken from the
geometry (the normalised homographies of ``ProjectFuse``; a sample counts as inside within 5 % of the source
border, an approximation of ``mvbev_warp_tile_mask`` that needs no GPU).  A block costs active views x units
per view (F(3,3): 12 rows x 5/3 = 20, F(4,3): 16 rows x 6/4 = 24; halved with 64-Cout blocks), blocks are
dispatched heaviest first to the least-loaded of 256 CUs (one block per CU), and the makespan is compared
with the bound total / 256.

    PYTHONPATH=. python tools/makespan_model.py --config 2
"""
import argparse
import heapq
import warnings

import numpy as np

from mvdet_amd import synthetic
from mvdet_amd.geometry import projection_matrices
from mvdet_amd.pipeline import ProjectFuse


def lpt(costs, cus=256):
    h = [0.0] * cus
    for w in sorted(costs, reverse=True):
        heapq.heappush(h, heapq.heappop(h) + w)
    return max(h)


def main():
    warnings.filterwarnings("ignore")
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    eng = ProjectFuse(projection_matrices(ds), tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape), spec["C"])
    H, W = ds.reducedgrid_shape
    mats = [np.array(eng.m_norm_cpu[v].tolist(), dtype=np.float64) for v in range(ds.num_cam)]

    def active(y0, y1, x0, x1):
        ys, xs = np.mgrid[max(0, y0 - 1):min(H, y1 + 1), max(0, x0 - 1):min(W, x1 + 1)]
        p0 = np.stack([2 * xs / (W - 1) - 1, 2 * ys / (H - 1) - 1, np.ones(xs.shape)], -1)
        n = 0
        for m in mats:
            p = p0 @ m.T
            u, v = p[..., 0] / p[..., 2], p[..., 1] / p[..., 2]
            n += bool(((np.abs(u) <= 1.05) & (np.abs(v) <= 1.05) & (p[..., 2] > 0)).any())
        return n

    B = spec["B"]
    for name, th, per, n_cot in (("F(3,3) 128-Cout", 12, 20, 4), ("F(4,3) 128-Cout", 16, 24, 4),
                                 ("F(3,3) 64-Cout", 12, 10, 8), ("F(4,3) 64-Cout", 16, 12, 8)):
        costs = []
        for ty in range(-(-H // th)):
            for tx in range(-(-W // 32)):
                costs += [active(ty * th, ty * th + th, tx * 32, tx * 32 + 32) * per] * n_cot * B
        print(f"{name}: blocks {len(costs)}  bound {sum(costs) / 256:.1f}  makespan {lpt(costs):.1f} units")


if __name__ == "__main__":
    main()
