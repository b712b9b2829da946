"""Per-block wall-clock spans of the ring conv kernel (diagnostics build, GPU box):

    make -C mvdet_amd/csrc exp NAME=stamp EXTRA=-DMVBEV_RING_STAMP=1
    python tools/ring_stamps.py mvdet_amd/lib/exp/libmvbev_stamp.so [--config 2] [--stage conv1]

Each block records s_memrealtime (100 MHz) at entry and after its epilogue plus its HW_ID /
XCC_ID; this reports the kernel span, every CU's busy time (sum of its blocks' spans) and the
idle fraction = 1 - busy / (CUs x span): the load-balance loss of the launch, measured.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import build_mc, head_params  # noqa: E402
from mvdet_amd import ProjectFuse, _native, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--stage", default="conv1", choices=["conv1", "conv2", "dgrad1", "dgrad1s"])
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    dev = torch.device("cuda:0")
    lib = _native.load(args.lib)
    _native._lib = lib
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(projection_matrices(ds), up, (ho, wo), C, wino_conv1=False)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev) for v in range(N)]
    ws = eng.workspace(B, dev)
    buf = np.zeros(16384 * 4, dtype=np.uint32)
    with torch.no_grad():
        for v in range(N):
            eng.warp_view(ws, v, feats[v])
        if args.stage.startswith("dgrad1"):  # conv1's data gradient as the training step runs it (kbench's setup)
            from tools.kbench import backward_stages
            run = backward_stages(eng, ws, mc, B, ho, wo, N, C, dev)[args.stage][0]
        else:
            run = (lambda: eng.conv1(ws, mc[0])) if args.stage.startswith("conv1") else (lambda: eng.conv2(ws, mc[2]))
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        lib.mvbev_debug_ring_stamps.restype = ctypes.c_int
        assert lib.mvbev_debug_ring_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size) == 0
    st = buf.reshape(-1, 4).astype(np.int64)
    bid = np.arange(len(st))
    bid = bid[st[:, 1] != 0]
    st = st[st[:, 1] != 0]
    # the last launch's blocks: entries whose start lies within the latest kernel span
    t1 = st[:, 1].max()
    bid = bid[st[:, 0] > t1 - 10_000_000]
    st = st[st[:, 0] > t1 - 10_000_000]  # 100 ms window
    t0 = st[:, 0].min()
    span = (t1 - t0) / 100.0  # us
    key = (st[:, 3] << 8) | ((st[:, 2] >> 8) & 0xFF)
    cus = {}
    for k, a, b in zip(key, st[:, 0], st[:, 1]):
        cus.setdefault(int(k), []).append((a - t0, b - t0))
    busy = np.array([sum(b - a for a, b in v) for v in cus.values()]) / 100.0
    last = np.array([max(b for _, b in v) for v in cus.values()]) / 100.0
    dur = (st[:, 1] - st[:, 0]) / 100.0
    out = {"stage": args.stage, "blocks": int(len(st)), "cus": len(cus), "span_us": round(span, 1),
           "busy_us_mean": round(float(busy.mean()), 1), "busy_us_min": round(float(busy.min()), 1),
           "idle_frac": round(1 - float(busy.sum()) / (len(cus) * span), 4),
           "cu_last_end_us_p10_p50_p90": [round(float(np.percentile(last, q)), 1) for q in (10, 50, 90)],
           "block_us_p10_p50_p90_max": [round(float(np.percentile(dur, q)), 1) for q in (10, 50, 90)] +
                                       [round(float(dur.max()), 1)]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
