"""Oracle: kornia 0.6.11 ``warp_perspective`` restated over torch-CPU ops.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

The reference calls ``kornia.geometry.transform.warp_perspective(img_feature,
proj_mat, self.reducedgrid_shape)`` at
``multiview_detector/models/persp_trans_detector.py:69`` (kornia pinned to
0.6.11 in ``requirements.txt:1``; not vendored, not installed here).  kornia's
function body is restated step by step below from the pinned release; the last
step is the real ``torch.nn.functional.grid_sample`` (ATen CPU kernel; formula
in ``torch/include/ATen/native/GridSampler.h:27-36`` unnormalize and the
bilinear corner/bounds logic of ``GridSamplerKernel.cpp``).

``closed_form_warp_f64`` is the independent float64 pin: bilinear sampling of
``src`` at ``M^-1 [u, v, 1]`` (perspective divide, zero padding, integer pixel
centres) — what the fp32 chain approximates.

PARITY STATUS — kornia parity unpinned: kornia itself is not importable here and
no reference fixture holds a kornia output, so the golden vectors
(``tools/gen_golden.py``) run the reference's own ``PerspTransDetector`` with kornia
stubbed by THIS restatement.  Every warp / fused-upsample / adjoint parity test
therefore checks against the restatement, not against kornia's own output.  An
error in the restatement is caught only by the float64 closed form above, which
the required tests ``tests/test_oracle.py::test_restatement_vs_closed_form`` (CPU)
and ``tests/test_gpu_parity.py::test_warp_vs_oracle_and_closed_form`` (HIP warp vs
both) check on every run.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


# --- kornia.geometry.conversions ------------------------------------------------

def normal_transform_pixel(height: int, width: int, eps: float = 1e-14,
                           dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """kornia 0.6.11 ``normal_transform_pixel``: pixel -> [-1, 1] (1x3x3)."""
    tr = torch.tensor([[1.0, 0.0, -1.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]], dtype=dtype)
    width_denom = eps if width == 1 else width - 1.0
    height_denom = eps if height == 1 else height - 1.0
    tr[0, 0] = tr[0, 0] * 2.0 / width_denom
    tr[1, 1] = tr[1, 1] * 2.0 / height_denom
    return tr.unsqueeze(0)


def _torch_inverse_cast(x: torch.Tensor) -> torch.Tensor:
    """kornia 0.6.11 ``_torch_inverse_cast``: inverse in f32/f64, cast back."""
    dtype = x.dtype if x.dtype in (torch.float32, torch.float64) else torch.float32
    return torch.inverse(x.to(dtype)).to(x.dtype)


def normalize_homography(dst_pix_trans_src_pix: torch.Tensor, dsize_src, dsize_dst) -> torch.Tensor:
    """kornia 0.6.11 ``normalize_homography``: N_dst @ (M @ N_src^-1)."""
    src_h, src_w = dsize_src
    dst_h, dst_w = dsize_dst
    src_norm_trans_src_pix = normal_transform_pixel(src_h, src_w).to(dst_pix_trans_src_pix)
    src_pix_trans_src_norm = _torch_inverse_cast(src_norm_trans_src_pix)
    dst_norm_trans_dst_pix = normal_transform_pixel(dst_h, dst_w).to(dst_pix_trans_src_pix)
    return dst_norm_trans_dst_pix @ (dst_pix_trans_src_pix @ src_pix_trans_src_norm)


def convert_points_to_homogeneous(points: torch.Tensor) -> torch.Tensor:
    return F.pad(points, [0, 1], "constant", 1.0)


def convert_points_from_homogeneous(points: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """kornia 0.6.11: scale = 1/(z+eps) where |z| > eps, else 1 (no z>0 mask)."""
    z_vec = points[..., -1:]
    mask = torch.abs(z_vec) > eps
    scale = torch.where(mask, 1.0 / (z_vec + eps), torch.ones_like(z_vec))
    return scale * points[..., :-1]


def transform_points(trans_01: torch.Tensor, points_1: torch.Tensor) -> torch.Tensor:
    """kornia 0.6.11 ``transform_points`` (homogeneous bmm + divide)."""
    shape_inp = list(points_1.shape)
    points_1 = points_1.reshape(-1, points_1.shape[-2], points_1.shape[-1])
    trans_01 = trans_01.reshape(-1, trans_01.shape[-2], trans_01.shape[-1])
    trans_01 = torch.repeat_interleave(trans_01, repeats=points_1.shape[0] // trans_01.shape[0], dim=0)
    points_1_h = convert_points_to_homogeneous(points_1)
    points_0_h = torch.bmm(points_1_h, trans_01.permute(0, 2, 1))
    points_0_h = torch.squeeze(points_0_h, dim=-1)
    points_0 = convert_points_from_homogeneous(points_0_h)
    shape_inp[-2] = points_0.shape[-2]
    shape_inp[-1] = points_0.shape[-1]
    return points_0.reshape(shape_inp)


def create_meshgrid(height: int, width: int, normalized_coordinates: bool = True,
                    dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """kornia 0.6.11 ``create_meshgrid``: [1, H, W, 2] ordered (x, y)."""
    xs = torch.linspace(0, width - 1, width, dtype=dtype)
    ys = torch.linspace(0, height - 1, height, dtype=dtype)
    if normalized_coordinates:
        xs = (xs / (width - 1) - 0.5) * 2
        ys = (ys / (height - 1) - 0.5) * 2
    base_grid = torch.stack(torch.meshgrid([xs, ys], indexing="ij"), dim=-1)
    return base_grid.permute(1, 0, 2).unsqueeze(0)


def src_norm_from_dst_norm(M: torch.Tensor, src_hw, dst_hw) -> torch.Tensor:
    """The fp32 3x3 kornia hands to ``transform_points`` (B x 3 x 3)."""
    return _torch_inverse_cast(normalize_homography(M, src_hw, dst_hw))


def warp_perspective(src: torch.Tensor, M: torch.Tensor, dsize, mode: str = "bilinear",
                     padding_mode: str = "zeros", align_corners: bool = True) -> torch.Tensor:
    """kornia 0.6.11 ``warp_perspective`` (default-argument path used at
    ``persp_trans_detector.py:69``)."""
    if not isinstance(src, torch.Tensor):
        raise TypeError(f"Input src type is not a torch.Tensor. Got {type(src)}")
    if not isinstance(M, torch.Tensor):
        raise TypeError(f"Input M type is not a torch.Tensor. Got {type(M)}")
    if not len(src.shape) == 4:
        raise ValueError(f"Input src must be a BxCxHxW tensor. Got {src.shape}")
    if not (len(M.shape) == 3 and M.shape[-2:] == (3, 3)):
        raise ValueError(f"Input M must be a Bx3x3 tensor. Got {M.shape}")
    B, _, H, W = src.size()
    h_out, w_out = dsize
    dst_norm_trans_src_norm = normalize_homography(M, (H, W), (h_out, w_out))
    src_norm_trans_dst_norm = _torch_inverse_cast(dst_norm_trans_src_norm)
    grid = create_meshgrid(h_out, w_out, True).to(src.dtype).repeat(B, 1, 1, 1)
    grid = transform_points(src_norm_trans_dst_norm[:, None, None], grid)
    return F.grid_sample(src, grid, align_corners=align_corners, mode=mode, padding_mode=padding_mode)


# --- float64 closed form (independent pin) ---------------------------------------

def closed_form_warp_f64(src: np.ndarray, M: np.ndarray, dsize) -> np.ndarray:
    """out[b, c, v, u] = bilinear(src[b, c], M_b^-1 [u, v, 1]) in float64.

    Zero padding, integer pixel centres (align_corners=True semantics), no
    cheirality mask; points with |z| <= 1e-8 keep their un-divided x, y in
    normalised coordinates exactly as kornia does (never hit in practice).
    """
    src = np.asarray(src, dtype=np.float64)
    M = np.asarray(M, dtype=np.float64)
    B, C, H, W = src.shape
    ho, wo = dsize
    out = np.zeros((B, C, ho, wo), dtype=np.float64)
    v, u = np.meshgrid(np.arange(ho, dtype=np.float64), np.arange(wo, dtype=np.float64), indexing="ij")
    pts = np.stack([u.ravel(), v.ravel(), np.ones(u.size)], axis=0)
    for b in range(B):
        p = np.linalg.inv(M[b]) @ pts
        z = p[2]
        ok = np.abs(z) > 1e-8
        x = np.where(ok, p[0] / np.where(ok, z, 1.0), np.nan)
        y = np.where(ok, p[1] / np.where(ok, z, 1.0), np.nan)
        x0 = np.floor(x)
        y0 = np.floor(y)
        fx = x - x0
        fy = y - y0
        acc = np.zeros((C, u.size), dtype=np.float64)
        for dy, wy in ((0, 1.0 - fy), (1, fy)):
            for dx, wx in ((0, 1.0 - fx), (1, fx)):
                xi = x0 + dx
                yi = y0 + dy
                inb = ok & (xi >= 0) & (xi <= W - 1) & (yi >= 0) & (yi <= H - 1)
                xs = np.where(inb, xi, 0).astype(np.int64)
                ys = np.where(inb, yi, 0).astype(np.int64)
                w = np.where(inb, wx * wy, 0.0)
                acc += src[b][:, ys, xs] * w[None, :]
        out[b] = acc.reshape(C, ho, wo)
    return out


def touched_footprint(M: np.ndarray, src_hw, dst_hw) -> int:
    """Number of distinct in-bounds source pixels that are a bilinear corner of
    at least one output sample (SURVEY §8(d) ``T_v``), from f64 ``M^-1``."""
    H, W = src_hw
    ho, wo = dst_hw
    v, u = np.meshgrid(np.arange(ho, dtype=np.float64), np.arange(wo, dtype=np.float64), indexing="ij")
    p = np.linalg.inv(np.asarray(M, np.float64)) @ np.stack([u.ravel(), v.ravel(), np.ones(u.size)])
    z = p[2]
    ok = np.abs(z) > 1e-8
    x = np.floor(np.where(ok, p[0] / np.where(ok, z, 1), -10))
    y = np.floor(np.where(ok, p[1] / np.where(ok, z, 1), -10))
    seen = np.zeros((H, W), dtype=bool)
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x + dx, y + dy
            inb = (xi >= 0) & (xi <= W - 1) & (yi >= 0) & (yi <= H - 1)
            seen[yi[inb].astype(np.int64), xi[inb].astype(np.int64)] = True
    return int(seen.sum())
