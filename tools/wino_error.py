"""Rounding error of the row-Winograd conv forms under the kernels' 3xbf16 arithmetic (CPU, numpy).

Emulates one kernel column of conv1 along the rows (the row-Winograd direction): T = B^T d in fp32 then
split hi / lo bf16, G w in float64 then split, the three bf16 products hi*hi + hi*lo + lo*hi accumulated
in fp32 over K, then A^T in fp32 — for the F(3,3) form the kernels run (conv_bf16x3.hip "Row-Winograd")
and the F(4,3) candidate (points 0, +-1, +-2, inf), against the float64 direct correlation, and beside
the direct 3xbf16 conv of the same data.  Prints one JSON line per form: normwise error
max|y - ref| / max|ref| and the relative Frobenius error.

    python tools/wino_error.py [--K 3584] [--rows 48] [--cout 32] [--seed 0]
"""
import argparse
import json

import numpy as np

F33 = dict(
    m=3,
    BT=np.array([[2, -1, -2, 1, 0], [0, -2, -1, 1, 0], [0, 2, -3, 1, 0], [0, -1, 0, 1, 0], [0, 2, -1, -2, 1]], float),
    G=np.array([[1 / 2, 0, 0], [-1 / 2, -1 / 2, -1 / 2], [-1 / 6, 1 / 6, -1 / 6], [1 / 6, 1 / 3, 2 / 3], [0, 0, 1]]),
    AT=np.array([[1, 1, 1, 1, 0], [0, 1, -1, 2, 0], [0, 1, 1, 4, 1]], float),
)
F43 = dict(
    m=4,
    BT=np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                 [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], float),
    G=np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
                [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]]),
    AT=np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], float),
)


def bf16(x):
    """Round-to-nearest-even fp32 -> bf16 (as float32 values)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def split(x):
    x = np.asarray(x, dtype=np.float32)
    hi = bf16(x)
    return hi, bf16(x - hi)


def mm3(a_hi, a_lo, b_hi, b_lo):
    """[M, K] x [K, N] as the 3 bf16 products accumulated in fp32 (16-deep MFMA chunks, in K order)."""
    K = a_hi.shape[1]
    acc = np.zeros((a_hi.shape[0], b_hi.shape[1]), np.float32)
    for k0 in range(0, K, 16):
        s = slice(k0, k0 + 16)
        for a, b in ((a_hi, b_lo), (a_lo, b_hi), (a_hi, b_hi)):  # the kernels' pass order
            acc = (acc + (a[:, s].astype(np.float64) @ b[s].astype(np.float64)).astype(np.float32)).astype(np.float32)
    return acc


def wino(form, d, w):
    """d [K, H + 2] (zero-padded rows), w [Cout, K, 3] -> y [Cout, H] (correlation along the rows)."""
    m, BT, G, AT = form["m"], form["BT"], form["G"], form["AT"]
    n = BT.shape[0]
    K, Hp = d.shape
    H = Hp - 2
    tiles = -(-H // m)
    dp = np.zeros((K, tiles * m + 2), np.float32)
    dp[:, :Hp] = d
    gw = np.einsum("xt,oct->xoc", G, w.astype(np.float64))  # [n, Cout, K]
    y = np.zeros((w.shape[0], tiles * m), np.float32)
    for t in range(tiles):
        seg = dp[:, t * m:t * m + n].astype(np.float32)  # [K, n]
        T = (seg @ BT.T.astype(np.float32)).astype(np.float32)  # fp32 transform, [K, n]
        M = np.zeros((n, w.shape[0]), np.float32)
        for xi in range(n):
            th, tl = split(T[:, xi:xi + 1])
            wh, wl = split(gw[xi].astype(np.float32))
            M[xi] = mm3(wh, wl, th, tl)[:, 0]
        y[:, t * m:(t + 1) * m] = (AT.astype(np.float32) @ M).T
    return y[:, :H]


def direct3(d, w):
    K, Hp = d.shape
    H = Hp - 2
    wh, wl = split(w.reshape(w.shape[0], -1))
    y = np.zeros((w.shape[0], H), np.float32)
    for r in range(H):
        col = d[:, r:r + 3].reshape(-1, 1)  # [K*3, 1] in (k, tap) order = w's flattening
        ch, cl = split(col)
        y[:, r] = mm3(wh, wl, ch, cl)[:, 0]
    return y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=3584)
    ap.add_argument("--rows", type=int, default=48)
    ap.add_argument("--cout", type=int, default=32)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    K, H, Co = args.K, args.rows, args.cout
    # ReLU'd unit-normal features (the warped backbone maps), zero rows outside the grid; kaiming-uniform
    # weights of a 3x3 conv over K channels (nn.Conv2d's default init), one kernel column
    d = np.zeros((K, H + 2), np.float32)
    d[:, 1:-1] = np.maximum(rng.standard_normal((K, H)), 0).astype(np.float32)
    bound = 1.0 / np.sqrt(K * 9)
    w = rng.uniform(-bound, bound, (Co, K, 3)).astype(np.float32)
    ref = np.stack([sum(w[:, :, k].astype(np.float64) @ d[:, r + k].astype(np.float64) for k in range(3))
                    for r in range(H)], axis=1)
    scale = np.abs(ref).max()
    for name, y in (("direct_3xbf16", direct3(d, w)), ("F(3,3)_3xbf16", wino(F33, d, w)),
                    ("F(4,3)_3xbf16", wino(F43, d, w))):
        e = y.astype(np.float64) - ref
        print(json.dumps({"form": name, "K": K, "rows": H, "cout": Co, "seed": args.seed,
                          "normwise": float(np.abs(e).max() / scale),
                          "rel_fro": float(np.linalg.norm(e) / np.linalg.norm(ref))}), flush=True)


if __name__ == "__main__":
    main()
