"""Debug: the fused upsample-warp T of the NCHW and channels-last kernels vs the CPU oracle's
upsample + warp + B^T (float64 transform), per-element error statistics (cfg1, C=32, B=1)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from mvdet_amd import ops, synthetic  # noqa: E402
from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices  # noqa: E402
from oracle import cpu_path  # noqa: E402

BT = np.array([[2, -1, -2, 1, 0], [0, -2, -1, 1, 0], [0, 2, -3, 1, 0], [0, -1, 0, 1, 0], [0, 2, -1, -2, 1]], dtype=np.float64)
cfg, C, B = 1, 32, 1
DEV = "cuda:0"
ds = synthetic.CONFIGS[cfg]["make"]()
N = ds.num_cam
up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
pm = projection_matrices(ds)
ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in pm]
low = [u // 3 for u in up]
feats = [synthetic.backbone_features(B, C, low, seed=81 + v, device=DEV) for v in range(N)]
Ho, Wo = grid
r3 = 4 * (-(-Ho // 12))
numel = B * (N * C // 8) * 5 * r3 * Wo * 16


def run(src):
    t = torch.zeros(numel, dtype=torch.bfloat16, device=DEV)
    ops.warp_views_wino_rows_into(src, ms, t, list(range(N)), C, N * C, Ho, Wo, dst_zeroed=True, up_hw=up)
    h = t.view(B, N * C // 8, 5 * r3, 2, Wo, 8).float().cpu()
    return (h[:, :, :, 0] + h[:, :, :, 1]).permute(0, 1, 4, 2, 3).reshape(B, N * C, 5 * r3, Wo).double().numpy()


ta = run(feats)
tb = run([f.contiguous(memory_format=torch.channels_last) for f in feats])
warped = cpu_path.warp_views([cpu_path.upsample(f.cpu(), up) for f in feats], pm, grid)
x = torch.cat(warped, 1).double().numpy()  # [B, N*C, Ho, Wo]
ref = np.zeros_like(ta)
for q in range(r3):
    d = np.zeros((5, B, N * C, Wo))
    for m in range(5):
        row = 3 * q - 1 + m
        if 0 <= row < Ho:
            d[m] = x[:, :, row]
    ref[:, :, 5 * q:5 * q + 5] = np.einsum("xm,mbkw->bkxw", BT, d).transpose(0, 1, 2, 3)
for name, t in (("nchw", ta), ("cl", tb)):
    e = np.abs(t - ref)
    print(name, "max err", e.max(), "normwise", np.linalg.norm(t - ref) / np.linalg.norm(ref),
          "n>1e-4", int((e > 1e-4).sum()), "of", e.size)
    i = np.unravel_index(np.argmax(e), e.shape)
    print("   at", i, "got", t[i], "ref", ref[i], "other", (tb if name == "nchw" else ta)[i])
e = np.abs(ta - tb)
print("nchw vs cl: n>1e-4", int((e > 1e-4).sum()), "max", e.max())
bad = np.argwhere(e > 1e-4)
print("bad (b, k, T row, col) sample:", bad[:10].tolist())
print("bad views:", np.unique(bad[:, 1] // C).tolist(), "T rows % 5:", np.unique(bad[:, 2] % 5).tolist())
