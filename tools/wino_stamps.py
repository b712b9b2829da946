"""Per-workgroup timeline of the row-Winograd conv1 at a config (diagnostic build with
-DMVBEV_WINO_STAMPS=1, loaded through MVBEV_LIB): CU busy fraction over the launch, and how the
last round tails off.  python tools/wino_stamps.py [--config 2] [--batch 1]"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd import ProjectFuse, _native, ops, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402
from bench import build_mc, head_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = (args.batch or spec["B"]), spec["C"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    dev = torch.device("cuda:0")
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(pm, up, grid, C, wino_conv1=True, wino_warp=False)
    ws = eng.workspace(B, dev)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev) for v in range(N)]
    eng.warp_views(ws, list(range(N)), feats)
    d1 = eng._conv1_desc(B)
    init = eng.coord_term(mc[0])
    eng.conv1_wino(ws, mc[0], d1, init)  # allocates wino_t and writes T (the product path)
    torch.cuda.synchronize()
    lib = _native.load()
    run = lambda: eng.conv1_wino(ws, mc[0], d1, init)
    res = []
    gmh = eng.conv1_mask(dev, 0, grid[0]).cpu().numpy().astype(np.uint32)
    dumps = []
    for rep in range(5):
        run()
        torch.cuda.synchronize()
        st = np.zeros(4 * 65536, dtype=np.int64)
        lib.mvbev_debug_wino_stamps.restype = ctypes.c_int
        assert lib.mvbev_debug_wino_stamps(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes)) == 0
        st = st.reshape(-1, 4)
        nwg = int((st[:, 1] > 0).sum())
        s = st[st[:, 1] > 0]
        t0, t1 = s[:, 0].min(), s[:, 1].max()
        span = (t1 - t0) / 100.0  # wall_clock64: 100 MHz -> us
        busy = ((s[:, 1] - s[:, 0]) / 100.0).sum()
        cus = len(np.unique(s[:, 2]))
        ends = np.sort(s[:, 1] - t0) / 100.0
        first_idle = None
        per_cu = {}
        for row in s:
            per_cu.setdefault(int(row[2]), []).append(row[1])
        last_end = sorted((max(v) - t0) / 100.0 for v in per_cu.values())
        dur = (s[:, 1] - s[:, 0]) / 100.0
        res.append({"wgs": nwg, "cus_seen": cus, "span_us": round(span, 1), "busy_frac": round(busy / (span * 256), 4),
                    "cu_last_end_us_p10_p50_max": [round(last_end[len(last_end) // 10], 1),
                                                   round(last_end[len(last_end) // 2], 1), round(last_end[-1], 1)],
                    "wg_us_min_med_max": [round(dur.min(), 1), round(float(np.median(dur)), 1), round(dur.max(), 1)]})
        pp = (s[:, 3] // 4) % gmh.size
        nch = np.array([bin(int(m)).count("1") for m in gmh[pp]])
        dumps.append(np.column_stack([s[:, 0] - t0, s[:, 1] - t0, s[:, 2], s[:, 3], nch]))
    if args.out:
        np.savez(args.out, *dumps)
    print(json.dumps({"config": args.config, "B": B, "runs": res}))


if __name__ == "__main__":
    main()
