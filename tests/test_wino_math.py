"""Host check of the row-Winograd identity the conv1 kernels implement (csrc/conv_bf16x3.hip,
"Row-Winograd conv1"): y = A^T [(G w) . (B^T d)] equals the 3-tap correlation
y_i = sum_kh w[kh] d[i + kh] for i < 3 over 5 input rows, with the constants as written in the
kernels (pack_wino_kernel's G rows, wino_rows_kernel's B^T rows, conv_wino_kernel's A^T rows).
Exact in rational arithmetic; plus a float32 3xbf16 emulation of the error budget."""
from fractions import Fraction as Fr

import numpy as np

AT = [[1, 1, 1, 1, 0], [0, 1, -1, 2, 0], [0, 1, 1, 4, 1]]
G = [[Fr(1, 2), 0, 0], [Fr(-1, 2), Fr(-1, 2), Fr(-1, 2)], [Fr(-1, 6), Fr(1, 6), Fr(-1, 6)],
     [Fr(1, 6), Fr(1, 3), Fr(2, 3)], [0, 0, 1]]
BT = [[2, -1, -2, 1, 0], [0, -2, -1, 1, 0], [0, 2, -3, 1, 0], [0, -1, 0, 1, 0], [0, 2, -1, -2, 1]]


def test_identity_exact():
    # the bilinear form's coefficient of w[k] d[l] in y_i must be [l == i + k]
    for i in range(3):
        for k in range(3):
            for l in range(5):
                c = sum(Fr(AT[i][j]) * Fr(G[j][k]) * Fr(BT[j][l]) for j in range(5))
                assert c == (1 if l == i + k else 0), (i, k, l, c)


def _bf16(x):
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


def _split(x):
    h = _bf16(x)
    return h, _bf16(np.asarray(x, np.float32) - h)


def test_error_budget_3xbf16():
    """Per kernel column: T and G w split hi/lo, products hi*hi + hi*lo + lo*hi in fp32-class
    accumulation; the Winograd result stays within a few times the direct 3xbf16 conv's error
    and far inside the north star's 1e-3 relative gate."""
    rng = np.random.default_rng(0)
    K, P = 1024, 64
    d = np.maximum(rng.standard_normal((5, K, P)), 0).astype(np.float32)   # ReLU features
    w = (rng.standard_normal((3, K)) * 0.03).astype(np.float32)
    ref = np.stack([sum(w[k].astype(np.float64)[:, None] * d[i + k] for k in range(3)).sum(0) for i in range(3)])
    Gf = np.array([[float(v) for v in r] for r in G], np.float32)
    V = np.einsum("jl,lkp->jkp", np.array(BT, np.float32), d).astype(np.float32)
    U = (Gf @ w).astype(np.float32)
    Vh, Vl = _split(V)
    Uh, Ul = _split(U)
    M = np.stack([(Uh[j].astype(np.float64)[:, None] * Vh[j] + Uh[j][:, None] * Vl[j] + Ul[j][:, None] * Vh[j]).sum(0)
                  for j in range(5)]).astype(np.float32)
    Y = np.array(AT, np.float32) @ M.reshape(5, -1)
    dh, dl = _split(d)
    wh, wl = _split(w)
    D = np.stack([sum((wh[k].astype(np.float64)[:, None] * dh[i + k] + wh[k][:, None] * dl[i + k]
                       + wl[k][:, None] * dh[i + k]).sum(0) for k in range(3)) for i in range(3)])
    e_w = np.linalg.norm(Y.reshape(3, P) - ref) / np.linalg.norm(ref)
    e_d = np.linalg.norm(D - ref) / np.linalg.norm(ref)
    assert e_w < 5e-5 and e_w < 6 * e_d + 1e-6, (e_w, e_d)
