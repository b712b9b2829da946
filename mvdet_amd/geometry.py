"""Host geometry of the hot path (rows a1-a3 of SURVEY §8(a)).

* ``imgcoord2worldgrid_matrices`` — the reference matrix chain
  (``persp_trans_detector.py:89-101``), float64 numpy.
* ``projection_matrices`` — the zoom chain of ``__init__`` (``:23-30``),
  including the reference's (H-ratio, W-ratio) image-zoom axis quirk.
* ``coord_map`` — ``create_coord_map`` (``:103-112``).
* ``kornia_src_norm_from_dst_norm`` — the fp32 3x3 kornia 0.6.11 hands to its
  ``transform_points`` (``normalize_homography`` then ``_torch_inverse_cast``),
  computed once on the host with the same torch fp32 ops, uploaded once.
* ``touched_footprint`` — T_v of SURVEY §8(d): distinct in-bounds bilinear
  source pixels, the basis of the warp's algorithmic byte count.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

PERMUTATION = np.array([[0, 1, 0], [1, 0, 0], [0, 0, 1]])


def imgcoord2worldgrid_matrices(intrinsic_matrices, extrinsic_matrices, worldgrid2worldcoord_mat,
                                num_cam: int) -> List[np.ndarray]:
    """Per camera ``P_swap @ inv(K @ [r1 r2 t] @ G)`` (``:89-101``)."""
    out = []
    for cam in range(num_cam):
        worldcoord2imgcoord = intrinsic_matrices[cam] @ np.delete(extrinsic_matrices[cam], 2, 1)
        worldgrid2imgcoord = worldcoord2imgcoord @ worldgrid2worldcoord_mat
        imgcoord2worldgrid = np.linalg.inv(worldgrid2imgcoord)
        out.append(PERMUTATION @ imgcoord2worldgrid)
    return out


def upsample_shape(img_shape: Sequence[int], img_reduce) -> List[int]:
    """``:23`` — warp-input (feature map) size."""
    return [int(x / img_reduce) for x in img_shape]


def projection_matrices(dataset) -> List[torch.Tensor]:
    """``:18-30``: ``Z_map @ imgcoord2worldgrid @ Z_img`` per camera (float64)."""
    i2w = imgcoord2worldgrid_matrices(dataset.base.intrinsic_matrices, dataset.base.extrinsic_matrices,
                                      dataset.base.worldgrid2worldcoord_mat, dataset.num_cam)
    ups = upsample_shape(dataset.img_shape, dataset.img_reduce)
    img_reduce = np.array(dataset.img_shape) / np.array(ups)
    img_zoom_mat = np.diag(np.append(img_reduce, [1]))
    map_zoom_mat = np.diag(np.append(np.ones([2]) / dataset.grid_reduce, [1]))
    return [torch.from_numpy(map_zoom_mat @ i2w[cam] @ img_zoom_mat) for cam in range(dataset.num_cam)]


def coord_map(ho: int, wo: int) -> torch.Tensor:
    """``create_coord_map([ho, wo, 1])`` → [1, 2, ho, wo] fp32 (x, y in [-1, 1])."""
    grid_x, grid_y = np.meshgrid(np.arange(wo), np.arange(ho))
    gx = torch.from_numpy(grid_x / (wo - 1) * 2 - 1).float()
    gy = torch.from_numpy(grid_y / (ho - 1) * 2 - 1).float()
    return torch.stack([gx, gy], dim=0).unsqueeze(0)


def _normal_transform_pixel(height: int, width: int, eps: float = 1e-14) -> torch.Tensor:
    tr = torch.tensor([[1.0, 0.0, -1.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]], dtype=torch.float32)
    wd = eps if width == 1 else width - 1.0
    hd = eps if height == 1 else height - 1.0
    tr[0, 0] = tr[0, 0] * 2.0 / wd
    tr[1, 1] = tr[1, 1] * 2.0 / hd
    return tr.unsqueeze(0)


def kornia_src_norm_from_dst_norm(M: torch.Tensor, src_hw, dst_hw) -> torch.Tensor:
    """kornia 0.6.11 ``warp_perspective`` steps 1-2 on the host, fp32:
    ``inv(N_dst @ (M @ inv(N_src)))`` → [B, 3, 3] (``M`` is src pix → dst pix)."""
    M = M.detach().to("cpu", torch.float32)
    n_src = _normal_transform_pixel(*src_hw)
    n_src_inv = torch.inverse(n_src)
    n_dst = _normal_transform_pixel(*dst_hw)
    dst_norm_trans_src_norm = n_dst @ (M @ n_src_inv)
    return torch.inverse(dst_norm_trans_src_norm)


def touched_footprint(M: np.ndarray, src_hw, dst_hw) -> int:
    """Distinct in-bounds source pixels that are a bilinear corner of at least one
    output sample, from float64 ``M^-1`` (SURVEY §8(d) T_v)."""
    H, W = src_hw
    ho, wo = dst_hw
    v, u = np.meshgrid(np.arange(ho, dtype=np.float64), np.arange(wo, dtype=np.float64), indexing="ij")
    p = np.linalg.inv(np.asarray(M, np.float64)) @ np.stack([u.ravel(), v.ravel(), np.ones(u.size)])
    ok = np.abs(p[2]) > 1e-8
    zs = np.where(ok, p[2], 1.0)
    x = np.floor(np.where(ok, p[0] / zs, -10.0))
    y = np.floor(np.where(ok, p[1] / zs, -10.0))
    seen = np.zeros((H, W), dtype=bool)
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x + dx, y + dy
            inb = (xi >= 0) & (xi <= W - 1) & (yi >= 0) & (yi <= H - 1)
            seen[yi[inb].astype(np.int64), xi[inb].astype(np.int64)] = True
    return int(seen.sum())
