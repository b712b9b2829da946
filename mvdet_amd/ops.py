"""Tensor-level wrappers over the C ABI (``include/mvbev.h``).

Every function here launches HIP kernels from ``libmvbev.so`` on torch's
current stream; none has a CPU or stock-torch fallback — a CPU tensor, a
missing library or a bad argument raises.

* ``warp_perspective`` — kornia-0.6.11-compatible signature/errors
  (``kornia.geometry.transform.warp_perspective``, the op called at
  ``persp_trans_detector.py:69``).
* ``warp_into`` — the zero-copy form used by the detector: writes one view
  straight into its channel slice of the fused ground-plane tensor (``:77``).
* ``fill_coord_map`` — the two coord channels (``:21,77``).
* ``PackedConv3x3`` / ``conv3x3`` / ``conv3x3_cout1`` — the fusion head convs
  (``:51-54,81``).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import torch

from . import _native
from .geometry import kornia_src_norm_from_dst_norm

KC = _native.KC
BN = _native.BN


def _require_cuda(*tensors):
    for t in tensors:
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise RuntimeError("mvdet_amd ops run only on a ROCm GPU tensor (no CPU fallback)")


def _stream(t: torch.Tensor) -> int:
    return _native.stream_ptr(t.device)


# ----------------------------------------------------------------------------------------------
# warp

def warp_into(src: torch.Tensor, m_norm: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """Warp ``src`` [B,C,H,W] into ``dst`` [B,C,Ho,Wo] (a view, innermost stride 1).

    ``m_norm`` is the device fp32 [B,3,3] (or [1,3,3] broadcast is NOT allowed;
    pass B rows) src_norm <- dst_norm matrix from ``kornia_src_norm_from_dst_norm``.
    """
    _require_cuda(src, m_norm, dst)
    if src.dim() != 4 or dst.dim() != 4:
        raise ValueError("src and dst must be 4-D")
    B, C, H, W = src.shape
    if dst.shape[0] != B or dst.shape[1] != C:
        raise ValueError(f"dst {tuple(dst.shape)} does not match src {tuple(src.shape)}")
    if m_norm.shape != (B, 3, 3) or m_norm.dtype != torch.float32 or not m_norm.is_contiguous():
        raise ValueError("m_norm must be a contiguous float32 [B,3,3] device tensor")
    if src.dtype != dst.dtype:
        raise TypeError("src and dst dtypes differ")
    lib = _native.load()
    if src.dtype == torch.float32:
        fn, name = lib.mvbev_warp_perspective_f32, "mvbev_warp_perspective_f32"
    elif src.dtype == torch.float16:
        fn, name = lib.mvbev_warp_perspective_f16, "mvbev_warp_perspective_f16"
    else:
        raise TypeError(f"unsupported dtype {src.dtype}")
    st = fn(src.data_ptr(), B, C, H, W, _native.strides4(src), m_norm.data_ptr(), dst.data_ptr(),
            dst.shape[2], dst.shape[3], _native.strides4(dst), _stream(dst))
    _native.check(st, name)
    return dst


def split_shape(B: int, C: int, H: int, W: int) -> Tuple[int, ...]:
    """Shape of a [B, C, H, W] tensor in the split-bf16 blocked layout (bf16 storage)."""
    return (B, (C + KC - 1) // KC, H, W, 2, KC)


def split_pix_shape(B: int, C: int, H: int, W: int) -> Tuple[int, ...]:
    """Shape of a [B, C, H, W] tensor in the pixel-major split-bf16 layout (MVBEV_LAYOUT_SPLIT_BF16_PIX:
    per pixel its 8-channel groups side by side, each 16 B hi then 16 B lo)."""
    return (B, H, W, (C + KC - 1) // KC, 2, KC)


def _out_layout(out: torch.Tensor, B: int, C: int, H: int, W: int) -> int:
    """The MVBEV_LAYOUT_* of a conv output tensor: fp32 [B, C, H, W], split-bf16 or pixel-major split-bf16."""
    if out.dtype == torch.float32 and tuple(out.shape) == (B, C, H, W) and out.is_contiguous():
        return _native.LAYOUT_F32
    if out.dtype == torch.bfloat16 and out.is_contiguous():
        if tuple(out.shape) == split_shape(B, C, H, W):
            return _native.LAYOUT_SPLIT_BF16
        if tuple(out.shape) == split_pix_shape(B, C, H, W):
            return _native.LAYOUT_SPLIT_PIX
    raise ValueError(f"out must be a contiguous fp32 {(B, C, H, W)}, bf16 {split_shape(B, C, H, W)} (split) or "
                     f"bf16 {split_pix_shape(B, C, H, W)} (pixel-major split) tensor, got "
                     f"{out.dtype} {tuple(out.shape)}")


def split_decode(t: torch.Tensor, C: Optional[int] = None) -> torch.Tensor:
    """Split-bf16 blocked [B, G, H, W, 2, 8] -> fp32 [B, C, H, W] (hi + lo)."""
    B, G, H, W, _, _ = t.shape
    v = t[..., 0, :].float() + t[..., 1, :].float()        # [B, G, H, W, 8]
    v = v.permute(0, 1, 4, 2, 3).reshape(B, G * KC, H, W)
    return v[:, :C] if C is not None else v


def warp_views_upsampled_into(srcs, up_hw, m_norms, dsts, split: bool = False, dst_zeroed: bool = False) -> None:
    """Fused bilinear upsample + warp of several views in ONE launch.

    ``srcs[i]`` [B,C,h,w] backbone-resolution maps that the reference upsamples to ``up_hw``
    with ``F.interpolate(..., mode='bilinear')`` (``persp_trans_detector.py:65``) before the
    warp; ``m_norms[i]`` the kornia matrix for the upsampled size; ``dsts`` as in
    ``warp_views_into`` (fp32 [B,C,Ho,Wo] views, or split-bf16 blocked with ``split=True``);
    ``dst_zeroed`` as in ``warp_views_into``."""
    n = len(srcs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(dsts)) or n > 16:
        raise ValueError("need 1..16 matching srcs / m_norms / dsts")
    _require_cuda(*srcs, *dsts)
    B, C, h, w = srcs[0].shape
    H, W = int(up_hw[0]), int(up_hw[1])
    if H < h or W < w:
        raise ValueError(f"upsample size {up_hw} must not be smaller than the source {(h, w)}")
    dtype = srcs[0].dtype
    Ho, Wo = dsts[0].shape[2], dsts[0].shape[3]
    want = split_shape(B, C, Ho, Wo) if split else (B, C, Ho, Wo)
    arr = (_native.WarpView * n)()
    for i, (s, m, d) in enumerate(zip(srcs, m_norms, dsts)):
        if tuple(s.shape) != (B, C, h, w) or tuple(d.shape) != want or s.dtype != dtype:
            raise ValueError(f"all views must share shapes/dtype: src {tuple(s.shape)} dst {tuple(d.shape)}")
        if split:
            if d.dtype != torch.bfloat16 or d.stride(5) != 1 or d.stride(4) != KC or d.stride(3) != 2 * KC:
                raise ValueError("split dst must be a bf16 [B,G,Ho,Wo,2,8] tensor with contiguous pixels")
            dstr = (d.stride(0) // 16, d.stride(1) // 16, d.stride(2) // 16, 1)
        else:
            if d.dtype != torch.float32 or dtype != torch.float32:
                raise TypeError("the fp32-output fused warp takes fp32 sources and destinations")
            dstr = tuple(d.stride())
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i] = _native.WarpView(s.data_ptr(), (ctypes.c_int64 * 4)(*s.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(*dstr), (ctypes.c_float * 9)(*mm))
    if dtype not in (torch.float32, torch.float16):
        raise TypeError(f"unsupported dtype {dtype}")
    lib = _native.load()
    st = lib.mvbev_warp_views_upsampled_ex(arr, n, int(dtype == torch.float16), B, C, h, w, H, W, Ho, Wo,
                                           _native.LAYOUT_SPLIT_BF16 if split else _native.LAYOUT_F32,
                                           _native.WARP_DST_ZEROED if dst_zeroed else 0, _stream(dsts[0]))
    _native.check(st, "mvbev_warp_views_upsampled_ex")


def warp_views_into(srcs, m_norms, dsts, split: bool = False, C: Optional[int] = None,
                    dst_zeroed: bool = False) -> None:
    """Warp several views (same shapes) in ONE launch.

    ``srcs[i]`` [B,C,H,W], ``m_norms[i]`` a host [3,3] src_norm <- dst_norm matrix shared by
    the batch (``kornia_src_norm_from_dst_norm``).  ``dsts[i]``: [B,C,Ho,Wo] views (innermost
    stride 1, same dtype as the sources) or, with ``split=True``, contiguous split-bf16 blocked
    tensors [B, ceil(C/8), Ho, Wo, 2, 8] (``split_shape``).  ``dst_zeroed`` (split only): the
    caller guarantees the dsts already hold zeros wherever a sample falls outside its source
    (a persistent zero-initialised slab of this geometry), so those pixels are not rewritten
    (``MVBEV_WARP_DST_ZEROED``).
    """
    n = len(srcs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(dsts)) or n > 16:
        raise ValueError("need 1..16 matching srcs / m_norms / dsts")
    _require_cuda(*srcs, *dsts)
    B, C, H, W = srcs[0].shape
    dtype = srcs[0].dtype
    if split:
        Ho, Wo = dsts[0].shape[2], dsts[0].shape[3]
        want = split_shape(B, C, Ho, Wo)
    else:
        Ho, Wo = dsts[0].shape[2], dsts[0].shape[3]
        want = (B, C, Ho, Wo)
    arr = (_native.WarpView * n)()
    for i, (s, m, d) in enumerate(zip(srcs, m_norms, dsts)):
        if tuple(s.shape) != (B, C, H, W) or tuple(d.shape) != want:
            raise ValueError(f"all views must share shapes: src {tuple(s.shape)} dst {tuple(d.shape)} want {want}")
        if s.dtype != dtype:
            raise TypeError("all views must share one dtype")
        if split:
            if d.dtype != torch.bfloat16 or d.stride(5) != 1 or d.stride(4) != KC or d.stride(3) != 2 * KC:
                raise ValueError("split dst must be a bf16 [B,G,Ho,Wo,2,8] tensor with contiguous pixels")
            dstr = (d.stride(0) // 16, d.stride(1) // 16, d.stride(2) // 16, 1)  # 32-byte units
        else:
            if d.dtype != dtype:
                raise TypeError("dst dtype must match src")
            dstr = tuple(d.stride())
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i] = _native.WarpView(s.data_ptr(), (ctypes.c_int64 * 4)(*s.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(*dstr), (ctypes.c_float * 9)(*mm))
    lib = _native.load()
    if split:
        if dtype not in (torch.float32, torch.float16):
            raise TypeError(f"unsupported dtype {dtype}")
        st = lib.mvbev_warp_views_split_bf16_ex(arr, n, int(dtype == torch.float16), B, C, H, W, Ho, Wo,
                                                _native.WARP_DST_ZEROED if dst_zeroed else 0, _stream(dsts[0]))
        _native.check(st, "mvbev_warp_views_split_bf16_ex")
        return
    if dtype == torch.float32:
        fn, name = lib.mvbev_warp_views_f32, "mvbev_warp_views_f32"
    elif dtype == torch.float16:
        fn, name = lib.mvbev_warp_views_f16, "mvbev_warp_views_f16"
    else:
        raise TypeError(f"unsupported dtype {dtype}")
    _native.check(fn(arr, n, B, C, H, W, Ho, Wo, _stream(dsts[0])), name)


def warp_perspective(src: torch.Tensor, M: torch.Tensor, dsize: Tuple[int, int], mode: str = "bilinear",
                     padding_mode: str = "zeros", align_corners: bool = True,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Drop-in for kornia 0.6.11 ``warp_perspective`` (default-argument path).

    ``M`` (src pixel -> dst pixel, [B,3,3]) is normalised and inverted on the host in
    fp32 exactly as kornia does; the HIP kernel does transform + divide + bilinear
    gather.  Only bilinear / zeros / align_corners=True are implemented (the only
    combination the reference exercises, ``persp_trans_detector.py:69``).
    """
    if not isinstance(src, torch.Tensor):
        raise TypeError(f"Input src type is not a torch.Tensor. Got {type(src)}")
    if not isinstance(M, torch.Tensor):
        raise TypeError(f"Input M type is not a torch.Tensor. Got {type(M)}")
    if not len(src.shape) == 4:
        raise ValueError(f"Input src must be a BxCxHxW tensor. Got {src.shape}")
    if not (len(M.shape) == 3 and M.shape[-2:] == (3, 3)):
        raise ValueError(f"Input M must be a Bx3x3 tensor. Got {M.shape}")
    if mode != "bilinear" or padding_mode != "zeros" or not align_corners:
        raise NotImplementedError("only mode='bilinear', padding_mode='zeros', align_corners=True")
    B, C, H, W = src.shape
    ho, wo = int(dsize[0]), int(dsize[1])
    if M.shape[0] != B:
        raise ValueError(f"M batch {M.shape[0]} != src batch {B}")
    m_norm = kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo)).to(src.device).contiguous()
    if out is None:
        out = torch.empty((B, C, ho, wo), dtype=src.dtype, device=src.device)
    return warp_into(src, m_norm, out)


def fill_coord_map(dst: torch.Tensor) -> torch.Tensor:
    """Write the coord map (``create_coord_map``) into ``dst`` [B,2,Ho,Wo] (a view)."""
    _require_cuda(dst)
    if dst.dim() != 4 or dst.shape[1] != 2 or dst.dtype != torch.float32:
        raise ValueError("dst must be a float32 [B,2,Ho,Wo] view")
    B, _, ho, wo = dst.shape
    st = _native.load().mvbev_fill_coord_map_f32(dst.data_ptr(), B, ho, wo, _native.strides4(dst),
                                                 _stream(dst))
    _native.check(st, "mvbev_fill_coord_map_f32")
    return dst


def coord_term(weight: torch.Tensor, bias: Optional[torch.Tensor], coord_c0: int, hw,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv1's coord term [Cout, H, W] (``mvbev_coord_term_f32``): ``bias`` + conv2d of the coord map
    (``persp_trans_detector.py:103-112``, zero padding 1) with ``weight[:, coord_c0:coord_c0 + 2]`` —
    the input-independent part of conv1 (``:51`` over ``:77``'s concat)."""
    _require_cuda(weight)
    if weight.dim() != 4 or tuple(weight.shape[2:]) != (3, 3) or weight.dtype != torch.float32:
        raise ValueError("weight must be a float32 [Cout, Cin, 3, 3] tensor")
    w = weight.detach().contiguous()
    cout, cin = w.shape[:2]
    H, W = int(hw[0]), int(hw[1])
    b = None if bias is None else bias.detach().contiguous()
    if b is not None and (b.numel() != cout or b.dtype != torch.float32):
        raise ValueError(f"bias must be float32 [{cout}]")
    if out is None:
        out = torch.empty((cout, H, W), dtype=torch.float32, device=w.device)
    elif tuple(out.shape) != (cout, H, W) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 [{cout}, {H}, {W}] tensor")
    st = _native.load().mvbev_coord_term_f32(w.data_ptr(), cin, int(coord_c0), 0 if b is None else b.data_ptr(),
                                             cout, H, W, out.data_ptr(), _stream(w))
    _native.check(st, "mvbev_coord_term_f32")
    return out


def _gate(gate):
    """``(flag, tag)`` -> (device pointer, int32 tag) for the ABI (None -> NULL, 0)."""
    if gate is None:
        return None, 0
    flag, tag = gate
    _require_cuda(flag)
    if flag.dtype != torch.int32 or flag.numel() < 1:
        raise ValueError("the guard flag is a device int32 tensor")
    return flag.data_ptr(), int(tag)


def warp_views_exact_into(srcs, m_norms, dsts, up_hw=None, gate=None, row0s=None, grid_rows: Optional[int] = None) -> None:
    """The reference's own evaluation order of the warp (a5) — and, with ``up_hw``, of the 3x
    upsample feeding it (a4 + a5): ``mvbev_warp_views_exact_f32``.  Every product
    ``F.interpolate`` and ``grid_sample`` form is formed (zero weights included), so a NaN / inf in
    ``srcs`` reaches exactly the outputs it reaches in ``persp_trans_detector.py:65-69``.  fp32 (or,
    ABI 11900, fp16) ``srcs[i]`` [B,C,h,w] (the warp's source, or with ``up_hw`` the backbone map),
    ``dsts[i]`` fp32 [B,C,rows,Wo] views (innermost stride 1); ``gate`` as ``conv3x3_desc``'s (the
    non-finite guard).  ``row0s`` (ABI 11900, ``mvbev_warp_views_exact_rows``): ``dsts[i]`` holds the
    ``rows`` grid rows from ``row0s[i]`` of a ``grid_rows``-row grid (row windows: the exact path in
    bands, the band exchange's windows); default the whole grid."""
    n = len(srcs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(dsts)) or n > 16:
        raise ValueError("need 1..16 matching srcs / m_norms / dsts")
    _require_cuda(*srcs, *dsts)
    B, C, h, w = srcs[0].shape
    dtype = srcs[0].dtype
    H, W = (h, w) if up_hw is None else (int(up_hw[0]), int(up_hw[1]))
    rows, Wo = dsts[0].shape[2], dsts[0].shape[3]
    Ho = rows if grid_rows is None else int(grid_rows)
    if row0s is None and grid_rows is not None and grid_rows != rows:
        raise ValueError("a row window needs row0s")
    arr = (_native.WarpView * n)()
    for i, (s_, m, d) in enumerate(zip(srcs, m_norms, dsts)):
        if tuple(s_.shape) != (B, C, h, w) or s_.dtype != dtype or dtype not in (torch.float32, torch.float16):
            raise ValueError("all views must be fp32 (or fp16) [B,C,h,w] of one shape and dtype")
        if tuple(d.shape) != (B, C, rows, Wo) or d.dtype != torch.float32 or d.stride(3) != 1:
            raise ValueError(f"dst must be an fp32 [{B},{C},{rows},{Wo}] view with unit column stride")
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i] = _native.WarpView(s_.data_ptr(), (ctypes.c_int64 * 4)(*s_.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(*d.stride()), (ctypes.c_float * 9)(*mm))
    gp, gt = _gate(gate)
    lib = _native.load()
    if row0s is None and dtype == torch.float32:
        st = lib.mvbev_warp_views_exact_f32(arr, n, B, C, h, w, H, W, Ho, Wo, gp, gt, _stream(dsts[0]))
        _native.check(st, "mvbev_warp_views_exact_f32")
        return
    r0 = (ctypes.c_int32 * n)(*([0] * n if row0s is None else [int(r) for r in row0s]))
    st = lib.mvbev_warp_views_exact_rows(arr, r0, n, int(dtype == torch.float16), B, C, h, w, H, W, Ho, Wo, rows,
                                         gp, gt, _stream(dsts[0]))
    _native.check(st, "mvbev_warp_views_exact_rows")


def warp_views_split_rows_into(srcs, m_norms, dsts, row0s, grid_rows: int, dst_zeroed: bool = False,
                               nonfinite=None) -> None:
    """Row windows of the split-bf16 warp in ONE launch (``mvbev_warp_views_split_bf16_rows``):
    ``dsts[i]`` (split-bf16 blocked [B, ceil(C/8), rows, Wo, 2, 8], contiguous pixels) receives the
    ``rows`` grid rows from ``row0s[i]`` of source ``srcs[i]`` (fp32 or fp16 [B,C,H,W]) warped by the
    host kornia matrix ``m_norms[i]`` onto the ``grid_rows``-row grid.  Entries may share a source (the
    band exchange warps each view's window of every destination rank in one launch).  ``dst_zeroed``
    as ``warp_views_into``'s; ``nonfinite``: ``(flag, tag)`` — the non-finite report."""
    n = len(srcs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(dsts) == len(row0s)) or n > 16:
        raise ValueError("need 1..16 matching srcs / m_norms / dsts / row0s")
    _require_cuda(*srcs, *dsts)
    B, C, H, W = srcs[0].shape
    dtype = srcs[0].dtype
    if dtype not in (torch.float32, torch.float16):
        raise TypeError(f"unsupported dtype {dtype}")
    rows, Wo = dsts[0].shape[2], dsts[0].shape[3]
    want = split_shape(B, C, rows, Wo)
    arr = (_native.WarpView * n)()
    for i, (s_, m, d) in enumerate(zip(srcs, m_norms, dsts)):
        if tuple(s_.shape) != (B, C, H, W) or s_.dtype != dtype:
            raise ValueError("all views must share one shape and dtype")
        if tuple(d.shape) != want or d.dtype != torch.bfloat16 or d.stride(5) != 1 or d.stride(4) != KC or \
                d.stride(3) != 2 * KC:
            raise ValueError(f"split dst must be a bf16 {want} tensor with contiguous pixels")
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i] = _native.WarpView(s_.data_ptr(), (ctypes.c_int64 * 4)(*s_.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(d.stride(0) // 16, d.stride(1) // 16, d.stride(2) // 16, 1),
                                  (ctypes.c_float * 9)(*mm))
    r0 = (ctypes.c_int32 * n)(*[int(r) for r in row0s])
    fp, ft = _gate(nonfinite)
    st = _native.load().mvbev_warp_views_split_bf16_rows(arr, r0, n, int(dtype == torch.float16), B, C, H, W,
                                                         int(grid_rows), Wo, rows,
                                                         _native.WARP_DST_ZEROED if dst_zeroed else 0, fp, ft,
                                                         _stream(dsts[0]))
    _native.check(st, "mvbev_warp_views_split_bf16_rows")


def bias_relu_nonfinite_(y: torch.Tensor, init: torch.Tensor, row0: int, relu: bool = True, flag=None) -> torch.Tensor:
    """``y = relu(y + init[:, row0:row0 + rows])`` in place (NaN-preserving) for a contiguous fp32
    [B, C, rows, W] ``y`` and the contiguous [C, H, W] ``init``; ``flag``: ``(flag, tag)`` — tag is
    stored into the device int32 flag when a result is non-finite (``mvbev_bias_relu_nonfinite_f32``)."""
    _require_cuda(y, init)
    if y.dim() != 4 or y.dtype != torch.float32 or not y.is_contiguous():
        raise ValueError("y must be a contiguous fp32 [B,C,rows,W] tensor")
    B, C, rows, W = y.shape
    if init.dtype != torch.float32 or not init.is_contiguous() or init.dim() != 3 or init.shape[0] != C or \
            init.shape[2] != W:
        raise ValueError("init must be a contiguous fp32 [C,H,W] tensor")
    fp, ft = _gate(flag)
    st = _native.load().mvbev_bias_relu_nonfinite_f32(y.data_ptr(), init.data_ptr(), B, C, rows, W, init.shape[1],
                                                      int(row0), int(bool(relu)), fp, ft, _stream(y))
    _native.check(st, "mvbev_bias_relu_nonfinite_f32")
    return y


def store_gated_(src: torch.Tensor, dst: torch.Tensor, gate) -> torch.Tensor:
    """``mvbev_store_gated_f32``: the fp32 [B, C, H, W] view ``src`` into ``dst`` — an fp32 [B, C, H, W] view,
    or a split-bf16 blocked [B, G, H, W, 2, 8] view (a non-finite value kept in hi, lo = 0) — when the device
    flag of ``gate = (flag, tag)`` holds tag; no host sync either way."""
    _require_cuda(src, dst)
    if src.dtype != torch.float32 or src.dim() != 4 or src.stride(3) != 1:
        raise ValueError("src must be an fp32 [B, C, H, W] view with unit column stride")
    B, C, H, W = src.shape
    if dst.dtype == torch.bfloat16:
        if tuple(dst.shape) != split_shape(B, C, H, W) or dst.stride(5) != 1 or dst.stride(4) != KC or \
                dst.stride(3) != 2 * KC:
            raise ValueError(f"split dst must be a [B, G, H, W, 2, 8] view of {split_shape(B, C, H, W)} with "
                             "contiguous pixels")
        layout, dstr = _native.LAYOUT_SPLIT_BF16, (dst.stride(0) // 16, dst.stride(1) // 16, dst.stride(2) // 16, 1)
    elif dst.dtype == torch.float32 and tuple(dst.shape) == (B, C, H, W) and dst.stride(3) == 1:
        layout, dstr = _native.LAYOUT_F32, tuple(dst.stride())
    else:
        raise ValueError("dst must be an fp32 [B, C, H, W] view or a split-bf16 one")
    gp, gt = _gate(gate)
    st = _native.load().mvbev_store_gated_f32(src.data_ptr(), _native._i64x4(*src.stride()), dst.data_ptr(),
                                              _native._i64x4(*dstr), B, C, H, W, layout, gp, gt, _stream(src))
    _native.check(st, "mvbev_store_gated_f32")
    return dst


def zero_gated_(t: torch.Tensor, gate) -> torch.Tensor:
    """Zero the contiguous ``t`` when the device flag of ``gate = (flag, tag)`` holds tag
    (``mvbev_zero_gated``), else leave it: no host sync either way."""
    _require_cuda(t)
    if not t.is_contiguous():
        raise ValueError("t must be contiguous")
    gp, gt = _gate(gate)
    st = _native.load().mvbev_zero_gated(t.data_ptr(), t.numel() * t.element_size(), gp, gt, _stream(t))
    _native.check(st, "mvbev_zero_gated")
    return t


def is_channels_last_source(x: torch.Tensor) -> bool:
    """True when the fused warps take ``x`` [B,C,H,W] fp32 in their channels-last form (ABI 11700: unit
    channel stride, whole 32-channel groups, strides multiples of 4 floats, 16-B aligned)."""
    sB, sC, sH, sW = x.stride()
    C = x.shape[1]
    return (x.dtype == torch.float32 and C % 32 == 0 and sC == 1 and sW >= C and sH >= sW * x.shape[3]
            and sW % 4 == 0 and sH % 4 == 0 and sB % 4 == 0 and x.data_ptr() % 16 == 0)


def to_channels_last_into(srcs, dsts) -> list:
    """``mvbev_nchw_to_nhwc_f32``: copy fp32 ``srcs[i]`` [B,C,H,W] (any strides) into the contiguous
    [B,H,W,C] ``dsts[i]``, every view in one launch; returns the channels-last [B,C,H,W] views of
    ``dsts`` (the same logical tensors as ``srcs``)."""
    n = len(srcs)
    if n == 0:
        return []
    if len(dsts) != n or n > 16:
        raise ValueError("need 1..16 matching srcs / dsts")
    _require_cuda(*srcs, *dsts)
    B, C, H, W = srcs[0].shape
    arr = (_native.WarpView * n)()
    for i, (s_, d) in enumerate(zip(srcs, dsts)):
        if tuple(s_.shape) != (B, C, H, W) or s_.dtype != torch.float32:
            raise ValueError("all views must be fp32 [B,C,H,W] of one shape")
        if tuple(d.shape) != (B, H, W, C) or d.dtype != torch.float32 or not d.is_contiguous():
            raise ValueError(f"dst must be a contiguous fp32 [{B},{H},{W},{C}] tensor")
        arr[i] = _native.WarpView(s_.data_ptr(), (ctypes.c_int64 * 4)(*s_.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(0, 0, 0, 1), (ctypes.c_float * 9)())
    st = _native.load().mvbev_nchw_to_nhwc_f32(arr, n, B, C, H, W, _stream(dsts[0]))
    _native.check(st, "mvbev_nchw_to_nhwc_f32")
    return [d.permute(0, 3, 1, 2) for d in dsts]


# ----------------------------------------------------------------------------------------------
# convs

def padded_channels(cin: int) -> int:
    return (cin + KC - 1) // KC * KC


PRECISIONS = ("fp32", "bf16x3")


class PackedConv3x3:
    """MFMA-layout copy of an ``nn.Conv2d`` 3x3 weight (optionally with its input
    channels permuted by ``chan_map``), re-packed only when the parameter changes
    (keyed by ``(data_ptr, _version, shape)``).

    ``precision``: "fp32" (fp32 MFMA, exact fp32 products) or "bf16x3" (hi/lo bf16 split,
    three bf16 MFMA passes, fp32 accumulation)."""

    def __init__(self, chan_map: Optional[Sequence[int]] = None, precision: str = "fp32", wino: bool = False,
                 form: int = 3):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}")
        if wino and precision != "bf16x3":
            raise ValueError("the row-Winograd packing is bf16x3")
        if form not in (3, 4) or (form == 4 and not wino):
            raise ValueError("form 4 (F(4,3)) is a row-Winograd packing")
        self.precision = precision
        # wino: the row-Winograd weights G w of mvbev_pack_conv3x3_weight_wino (conv3x3_wino); form 4: F(4,3)'s
        # (mvbev_pack_conv3x3_weight_wino43, conv3x3_wino43)
        self.wino = wino
        self.form = form
        self._key = None
        self.packed: Optional[torch.Tensor] = None
        self.chan_map = None if chan_map is None else [int(c) for c in chan_map]
        self._map_dev: Optional[torch.Tensor] = None

    @property
    def K(self) -> Optional[int]:
        return None if self.chan_map is None else len(self.chan_map)

    def map_dev(self, device) -> Optional[torch.Tensor]:
        """The channel map as a device int32 tensor (None without a map), without packing anything."""
        if self.chan_map is not None and (self._map_dev is None or self._map_dev.device != torch.device(device)):
            self._map_dev = torch.tensor(self.chan_map, dtype=torch.int32, device=device)
        return self._map_dev

    def get_gated(self, weight: torch.Tensor, gate) -> torch.Tensor:
        """The fp32 pack, enqueued gated on ``gate = (flag, tag)`` on EVERY call (no cache: a skipped pack
        must not be taken for a current one — ``mvbev_pack_conv3x3_weight_f32_gated``); the buffer is reused."""
        _require_cuda(weight)
        if self.precision != "fp32" or self.wino:
            raise ValueError("gated packs are fp32 packs")
        cout, cin, kh, kw = weight.shape
        if (kh, kw) != (3, 3) or weight.dtype != torch.float32 or cout % BN:
            raise ValueError("expected a float32 [Cout,Cin,3,3] weight with Cout a multiple of 128")
        lib = _native.load()
        K = cin if self.chan_map is None else len(self.chan_map)
        if self.chan_map is not None and (self._map_dev is None or self._map_dev.device != weight.device):
            self._map_dev = torch.tensor(self.chan_map, dtype=torch.int32, device=weight.device)
        n = lib.mvbev_conv3x3_packed_floats(cout, K)
        if self.packed is None or self.packed.numel() != n or self.packed.device != weight.device:
            self.packed = torch.empty(n, dtype=torch.float32, device=weight.device)
        self._key = None
        w = weight.detach()
        if not w.is_contiguous():
            raise ValueError("the gated pack reads the weight in place: it must be contiguous")
        gp, gt = _gate(gate)
        st = lib.mvbev_pack_conv3x3_weight_f32_gated(w.data_ptr(), cout, cin, None if self._map_dev is None
                                                     else self._map_dev.data_ptr(), K, self.packed.data_ptr(),
                                                     gp, gt, _stream(self.packed))
        _native.check(st, "mvbev_pack_conv3x3_weight_f32_gated")
        return self.packed

    def get(self, weight: torch.Tensor) -> torch.Tensor:
        _require_cuda(weight)
        lib = _native.load()
        # the packed layout belongs to the library that packed it (A/B runs swap libraries)
        key = (weight.data_ptr(), weight._version, tuple(weight.shape), id(lib))
        if key != self._key:
            cout, cin, kh, kw = weight.shape
            if (kh, kw) != (3, 3) or weight.dtype != torch.float32:
                raise ValueError("expected a float32 [Cout,Cin,3,3] weight")
            if cout % BN:
                raise ValueError(f"Cout={cout} must be a multiple of {BN}")
            K = cin if self.chan_map is None else len(self.chan_map)
            if self.chan_map is not None and (self._map_dev is None or self._map_dev.device != weight.device):
                self._map_dev = torch.tensor(self.chan_map, dtype=torch.int32, device=weight.device)
            cmap = None if self._map_dev is None else self._map_dev.data_ptr()
            w = weight.detach().contiguous()
            if self.precision == "fp32":
                n = lib.mvbev_conv3x3_packed_floats(cout, K)
                packed = torch.empty(n, dtype=torch.float32, device=weight.device)
                st = lib.mvbev_pack_conv3x3_weight_f32(w.data_ptr(), cout, cin, cmap, K, packed.data_ptr(),
                                                       _stream(packed))
                _native.check(st, "mvbev_pack_conv3x3_weight_f32")
            elif self.wino and self.form == 4:
                n = lib.mvbev_conv3x3_packed_bytes_wino43(cout, K)
                packed = torch.empty(n // 2, dtype=torch.bfloat16, device=weight.device)
                st = lib.mvbev_pack_conv3x3_weight_wino43(w.data_ptr(), cout, cin, cmap, K, packed.data_ptr(),
                                                          _stream(packed))
                _native.check(st, "mvbev_pack_conv3x3_weight_wino43")
            elif self.wino:
                n = lib.mvbev_conv3x3_packed_bytes_wino(cout, K)
                packed = torch.empty(n // 2, dtype=torch.bfloat16, device=weight.device)
                st = lib.mvbev_pack_conv3x3_weight_wino(w.data_ptr(), cout, cin, cmap, K, packed.data_ptr(),
                                                        _stream(packed))
                _native.check(st, "mvbev_pack_conv3x3_weight_wino")
            else:
                n = lib.mvbev_conv3x3_packed_bytes_bf16x3(cout, K)
                packed = torch.empty(n // 2, dtype=torch.bfloat16, device=weight.device)
                st = lib.mvbev_pack_conv3x3_weight_bf16x3(w.data_ptr(), cout, cin, cmap, K, packed.data_ptr(),
                                                          _stream(packed))
                _native.check(st, "mvbev_pack_conv3x3_weight_bf16x3")
            self.packed, self._key = packed, key
        return self.packed


class PackedWinoDgrad3x3:
    """The row-Winograd weights of a data gradient (``conv3x3_wino_dgrad`` / ``conv3x3_wino_dil``)
    packed straight from the forward weight [Cout_f, Cin_f, 3, 3]: in / out channels swapped, taps
    reversed, the first ``cout`` forward input channels (``mvbev_pack_conv3x3_weight_wino_dgrad``);
    re-packed when the parameter changes (keyed as ``PackedConv3x3``)."""

    def __init__(self, cout: int):
        if cout <= 0 or cout % BN:
            raise ValueError(f"cout={cout} must be a positive multiple of {BN}")
        self.cout = int(cout)
        self._key = None
        self.packed: Optional[torch.Tensor] = None

    def get(self, weight: torch.Tensor) -> torch.Tensor:
        _require_cuda(weight)
        lib = _native.load()
        key = (weight.data_ptr(), weight._version, tuple(weight.shape), id(lib))
        if key != self._key:
            cout_f, cin_f, kh, kw = weight.shape
            if (kh, kw) != (3, 3) or weight.dtype != torch.float32 or cin_f < self.cout:
                raise ValueError(f"expected a float32 [Cout, >= {self.cout}, 3, 3] weight")
            w = weight.detach().contiguous()
            n = lib.mvbev_conv3x3_packed_bytes_wino(self.cout, cout_f)
            packed = torch.empty(n // 2, dtype=torch.bfloat16, device=weight.device)
            st = lib.mvbev_pack_conv3x3_weight_wino_dgrad(w.data_ptr(), cout_f, cin_f, self.cout, packed.data_ptr(),
                                                          _stream(packed))
            _native.check(st, "mvbev_pack_conv3x3_weight_wino_dgrad")
            self.packed, self._key = packed, key
        return self.packed


def conv_desc(B: int, K: int, H: int, W: int, group: int, group_stride: int, batch_stride: int,
              in_row0: int = 0, in_rows: Optional[int] = None, out_row0: int = 0,
              out_rows: Optional[int] = None) -> "_native.ConvDesc":
    return _native.ConvDesc(B, K, H, W, group, group_stride, batch_stride, in_row0,
                            H if in_rows is None else in_rows, out_row0, H if out_rows is None else out_rows)


def conv3x3_workspace_bytes(desc, cout: int) -> int:
    """Device workspace the bf16x3 conv's stream-K schedule wants for this shape (0 = none)."""
    return int(_native.load().mvbev_conv3x3_bf16x3_workspace_bytes(ctypes.byref(desc), cout))


def warp_tile_mask(m_norms, src_hw, grid_hw, row0: int, rows: int, halo: int, device,
                   tile_h: Optional[int] = None, tile_w: Optional[int] = None) -> torch.Tensor:
    """Frustum mask of the conv tiles (``mvbev_warp_tile_mask``): int32 [tiles] on ``device``,
    bit s set where slot s's warp can be non-zero in the tile + ``halo``.  ``m_norms[s]`` is a
    host [3,3] kornia matrix, or None for an empty slot (always zero).  ``tile_h``: tile rows
    (default ``_native.TILE_H``; the split-input conv's is ``_native.conv_tile_rows``)."""
    tile_h = _native.TILE_H if tile_h is None else int(tile_h)
    tile_w = _native.TILE_W if tile_w is None else int(tile_w)
    n = len(m_norms)
    if not 0 < n <= 16:
        raise ValueError("need 1..16 slots")
    arr = (_native.WarpView * n)()
    for i, m in enumerate(m_norms):
        # an empty slot: a finite map far outside the source (bit stays clear)
        mm = [0.0, 0.0, 1e6, 0.0, 0.0, 1e6, 0.0, 0.0, 1.0] if m is None else \
            torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i].m = (ctypes.c_float * 9)(*mm)
    H, W = src_hw
    Ho, Wo = grid_hw
    tiles = -(-rows // tile_h) * -(-Wo // tile_w)
    mask = torch.zeros(tiles, dtype=torch.int32, device=device)
    st = _native.load().mvbev_warp_tile_mask(arr, n, H, W, Ho, Wo, row0, rows, tile_h, tile_w,
                                             halo, mask.data_ptr(), _stream(mask))
    _native.check(st, "mvbev_warp_tile_mask")
    return mask


def warp_nonfinite_views(m_norms, src_hw, grid_hw, device) -> int:
    """``mvbev_warp_nonfinite_views``: bit s set when slot s's warp (host [3,3] kornia matrix
    ``m_norms[s]``, None = empty slot) has an output pixel with non-finite sample coordinates
    (a NaN output).  Geometry only; one small launch and one 4-byte copy to the host."""
    n = len(m_norms)
    if not 0 < n <= 16:
        raise ValueError("need 1..16 slots")
    arr = (_native.WarpView * n)()
    for i, m in enumerate(m_norms):
        mm = [0.0, 0.0, 1e6, 0.0, 0.0, 1e6, 0.0, 0.0, 1.0] if m is None else \
            torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i].m = (ctypes.c_float * 9)(*mm)
    H, W = src_hw
    Ho, Wo = grid_hw
    bits = torch.zeros(1, dtype=torch.int32, device=device)
    st = _native.load().mvbev_warp_nonfinite_views(arr, n, H, W, Ho, Wo, bits.data_ptr(), _stream(bits))
    _native.check(st, "mvbev_warp_nonfinite_views")
    return int(bits.item()) & 0xFFFFFFFF


def ring_tile_mask(m_norms, src_hw, grid_hw, row0: int, rows: int, device, space: int) -> Optional[torch.Tensor]:
    """Frustum mask (halo 1) of a dilation-1 ring conv's pixel tiles in tile space ``space``
    (``_native.TILES_*``) over grid rows [row0, row0+rows): the regular 12 x 32 tiles of the
    space's columns, then (edge strip) its edge_rows x EW tiles of the last columns.  None when
    the space does not apply to this grid width."""
    Wo = int(grid_hw[1])
    d = conv_desc(1, 8, int(grid_hw[0]), Wo, group=8, group_stride=0, batch_stride=0, in_row0=row0, in_rows=rows,
                  out_row0=row0, out_rows=rows)
    g = _native.ring_tile_space(d, space)
    if g is None:
        return None
    tiles_x, tiles_y, edge_tiles, ew, edge_rows = g
    th = _native.conv_tile_rows(_native.LAYOUT_SPLIT_BF16, 1)
    grid = warp_tile_mask(m_norms, src_hw, grid_hw, row0, rows, 1, device, tile_h=th)
    grid = grid.reshape(tiles_y, -(-Wo // _native.TILE_W))[:, :tiles_x].reshape(-1)
    if edge_tiles == 0:
        return grid.contiguous()
    strip = warp_tile_mask(m_norms, src_hw, grid_hw, row0, rows, 1, device, tile_h=edge_rows, tile_w=ew)
    strip = strip.reshape(edge_tiles, -(-Wo // ew))[:, -1]
    return torch.cat([grid, strip]).contiguous()


def heavy_first_order(mask: torch.Tensor, B: int) -> torch.Tensor:
    """Pixel tiles (b, tile) sorted by active channel groups, most first, equal view sets
    together: the run order that evens out a frustum-masked conv's per-tile work."""
    masks = [int(v) & 0xFFFFFFFF for v in mask.cpu().tolist()]
    bits = [bin(m).count("1") for m in masks]
    T = len(bits)
    # most work first; equal view sets adjacent (they share weight chunks when run together)
    order = sorted(range(B * T), key=lambda i: (-bits[i % T], masks[i % T], i))
    return torch.tensor(order, dtype=torch.int32, device=mask.device)


def conv3x3_desc(x: torch.Tensor, desc, packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor] = None,
                 init: Optional[torch.Tensor] = None, dilation: int = 1, relu: bool = False,
                 out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                 group_mask: Optional[torch.Tensor] = None, tile_order: Optional[torch.Tensor] = None,
                 tile_space: int = _native.TILES_GRID, gate=None, band_rows: int = 0) -> torch.Tensor:
    """Low-level form: ``x`` addressed through ``desc`` (``mvbev_conv_desc``).  ``gate`` (fp32
    conv only): ``(flag, tag)`` — the kernel runs only when the device int32 ``flag[0] == tag``
    (the non-finite guard's path; ``warp_views_wino_rows_into``'s report).  ``band_rows`` (fp32 conv
    only, ABI 11900): ``out`` is the row-banded [bands, B, cout, band_rows, W] of ``conv3x3_wino``
    (global output row g at band g // band_rows).  bf16x3 only,
    optional: ``workspace`` — device scratch for the split-K tail
    (``conv3x3_workspace_bytes``); ``group_mask`` — per-tile active channel groups
    (``warp_tile_mask``), whose cleared groups are skipped; ``tile_order`` — with a mask,
    the B x tiles pixel tiles in run order (``heavy_first_order``); ``tile_space`` — ``_native.TILES_EDGE_STRIP``: the ring kernel's edge-strip tiles
    (``mvbev_conv3x3_bf16x3_ex3``; the mask and order then index that space, ``ring_tile_mask``)."""
    _require_cuda(x, packed)
    bf16x3 = packed.dtype == torch.bfloat16
    if x.dtype not in ((torch.float32, torch.float16, torch.bfloat16) if bf16x3 else (torch.float32,)):
        raise TypeError(f"x dtype {x.dtype} not supported by the {'bf16x3' if bf16x3 else 'fp32'} conv")
    # bf16 storage means the split-bf16 blocked layout (4 bytes per logical element)
    layout = {torch.float32: _native.LAYOUT_F32, torch.float16: _native.LAYOUT_F16,
              torch.bfloat16: _native.LAYOUT_SPLIT_BF16}[x.dtype]
    unit = 2 if x.dtype == torch.float16 else 4
    B, H, W, out_rows = desc.B, desc.H, desc.W, desc.out_rows
    need = (desc.K // desc.group - 1) * desc.group_stride + (B - 1) * desc.batch_stride + \
        desc.group * desc.in_rows * W
    if (x.untyped_storage().nbytes() - x.storage_offset() * x.element_size()) // unit < need:
        raise ValueError("x's storage is too small for the conv descriptor")
    y_split = out is not None and out.dtype == torch.bfloat16  # split-bf16 blocked output
    if band_rows:
        nb = -(-(desc.out_row0 + out_rows) // band_rows)
        if bf16x3 or out is None or out.dim() != 5 or out.shape[0] < nb or \
                tuple(out.shape[1:]) != (B, cout, band_rows, W) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"a banded out must be a contiguous fp32 [>={nb},{B},{cout},{band_rows},{W}] tensor "
                             "of the fp32 conv")
    elif out is None:
        out = torch.empty((B, cout, out_rows, W), dtype=torch.float32, device=x.device)
    elif y_split:
        if not bf16x3 or tuple(out.shape) != split_shape(B, cout, out_rows, W) or not out.is_contiguous():
            raise ValueError(f"a split out must be a contiguous bf16 {split_shape(B, cout, out_rows, W)} tensor "
                             "of the bf16x3 conv")
    elif tuple(out.shape) != (B, cout, out_rows, W) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"out must be a contiguous fp32 [{B},{cout},{out_rows},{W}] tensor")
    if bias is not None:
        _require_cuda(bias)
        bias = bias.detach().contiguous()
    if init is not None:
        _require_cuda(init)
        if init.numel() != cout * H * W or not init.is_contiguous():
            raise ValueError("init must be a contiguous [Cout,H,W] tensor")
    lib = _native.load()
    need_packed = (lib.mvbev_conv3x3_packed_bytes_bf16x3(cout, desc.K) if bf16x3
                   else 4 * lib.mvbev_conv3x3_packed_floats(cout, desc.K))
    if packed.numel() * packed.element_size() < need_packed:
        raise ValueError("packed weights are smaller than the conv needs (packed for another K/Cout or library)")
    bp = bias.data_ptr() if bias is not None else None
    ip = init.data_ptr() if init is not None else None
    if bf16x3:
        if gate is not None:
            raise ValueError("gate applies to the fp32 conv")
        wsp, wsn, gmp = None, 0, None
        if workspace is not None:
            _require_cuda(workspace)
            wsp, wsn = workspace.data_ptr(), workspace.numel() * workspace.element_size()
        if tile_space != _native.TILES_GRID:
            g = _native.ring_tile_space(desc, tile_space) if layout == _native.LAYOUT_SPLIT_BF16 else None
            if g is None or workspace is not None:
                raise ValueError(f"tile space {tile_space} does not apply to this conv")
            tiles = g[0] * g[1] + g[2]
        else:
            tiles = -(-desc.out_rows // _native.conv_tile_rows(layout, dilation)) * -(-W // _native.TILE_W)
        if group_mask is not None:
            _require_cuda(group_mask)
            if group_mask.dtype != torch.int32 or group_mask.numel() < tiles or not group_mask.is_contiguous():
                raise ValueError(f"group_mask must be a contiguous int32 tensor of >= {tiles} tiles")
            gmp = group_mask.data_ptr()
        top = None
        if tile_order is not None:
            _require_cuda(tile_order)
            if group_mask is None or tile_order.dtype != torch.int32 or tile_order.numel() != B * tiles:
                raise ValueError("tile_order must be an int32 permutation of the B x tiles pixel tiles")
            top = tile_order.data_ptr()
        if tile_space != _native.TILES_GRID:
            st = lib.mvbev_conv3x3_bf16x3_ex3(x.data_ptr(), layout, ctypes.byref(desc), packed.data_ptr(), bp, ip,
                                              cout, int(dilation), int(bool(relu)), out.data_ptr(),
                                              _native.LAYOUT_SPLIT_BF16 if y_split else _native.LAYOUT_F32,
                                              gmp, top, int(tile_space), _stream(x))
            _native.check(st, "mvbev_conv3x3_bf16x3_ex3")
            return out
        st = lib.mvbev_conv3x3_bf16x3_ex(x.data_ptr(), layout, ctypes.byref(desc),
                                         packed.data_ptr(), bp, ip, cout, int(dilation), int(bool(relu)),
                                         out.data_ptr(), _native.LAYOUT_SPLIT_BF16 if y_split else _native.LAYOUT_F32,
                                         gmp, top, wsp, wsn, _stream(x))
        _native.check(st, "mvbev_conv3x3_bf16x3_ex")
    elif group_mask is not None:
        raise ValueError("group_mask needs the bf16x3 conv")
    else:
        gp, gt = _gate(gate)
        st = lib.mvbev_conv3x3_f32_ex(x.data_ptr(), ctypes.byref(desc), packed.data_ptr(), bp, ip, cout,
                                      int(dilation), int(bool(relu)), out.data_ptr(), int(band_rows), gp, gt, _stream(x))
        _native.check(st, "mvbev_conv3x3_f32_ex")
    return out


def wino_rows_bytes(desc) -> int:
    """Bytes of the row-Winograd transform T of a conv1 input (``mvbev_wino_rows_bytes``)."""
    return int(_native.load().mvbev_wino_rows_bytes(ctypes.byref(desc)))


def wino_rows(x: torch.Tensor, desc, t: torch.Tensor, group_mask: Optional[torch.Tensor] = None,
              dilation: int = 1, gate=None) -> torch.Tensor:
    """B^T over every 3-row output tile's 5 input rows of the split-bf16 ``x`` (addressed through
    ``desc`` as ``conv3x3_desc``) into ``t`` (bf16, >= ``wino_rows_bytes`` bytes; with
    ``group_mask`` zero-filled once and only written by this call with that mask):
    ``mvbev_wino_rows_split_bf16``; ``dilation`` 2: conv2's interleaved row tiles, input rows
    2 apart (``mvbev_wino_rows_split_bf16_dil``); ``gate`` = (flag, tag): only when the device flag holds
    the tag (``mvbev_wino_rows_split_bf16_gated``)."""
    _require_cuda(x, t)
    if x.dtype != torch.bfloat16 or t.dtype != torch.bfloat16 or not t.is_contiguous():
        raise TypeError("wino_rows reads the split-bf16 slab and writes a contiguous bf16 T")
    gmp = None
    if group_mask is not None:
        _require_cuda(group_mask)
        tiles = -(-desc.out_rows // 12) * -(-desc.W // _native.TILE_W)
        if group_mask.dtype != torch.int32 or group_mask.numel() < tiles or not group_mask.is_contiguous():
            raise ValueError(f"group_mask must be a contiguous int32 tensor of >= {tiles} tiles")
        gmp = group_mask.data_ptr()
    if gate is not None:
        gp, gt = _gate(gate)
        st = _native.load().mvbev_wino_rows_split_bf16_gated(x.data_ptr(), ctypes.byref(desc), int(dilation), gmp,
                                                             t.data_ptr(), t.numel() * t.element_size(), gp, gt,
                                                             _stream(x))
        _native.check(st, "mvbev_wino_rows_split_bf16_gated")
        return t
    st = _native.load().mvbev_wino_rows_split_bf16_dil(x.data_ptr(), ctypes.byref(desc), int(dilation), gmp,
                                                       t.data_ptr(), t.numel() * t.element_size(), _stream(x))
    _native.check(st, "mvbev_wino_rows_split_bf16_dil")
    return t


def wino_tile_rows(Ho: int, form: int = 3) -> int:
    """Row tiles of a whole-grid row-Winograd transform: 4 ceil(Ho / 12) three-row tiles (F(3,3)), or
    4 ceil(Ho / 16) four-row tiles (``form`` 4, F(4,3))."""
    return 4 * (-(-int(Ho) // (12 if form == 3 else 16)))


def warp_wino_boxes(m_norms, src_hw, grid_hw, device, backbone_hw=None, form: int = 3) -> torch.Tensor:
    """``mvbev_warp_wino_boxes``: the per-(view, block) staging boxes of the NCHW fused warp + B^T for the
    whole-grid T (r3 rows 4 * ceil(Ho / 12)) — geometry only, computed once and reused every frame.
    ``backbone_hw``: the channels-last fused upsample warp's boxes of its 3x3 windows in the backbone maps
    (``mvbev_warp_upsampled_wino_boxes``; ``src_hw`` = the upsampled size).  ``form`` 4: the blocks of the
    F(4,3) fused warp (the same 12-row blocks, ceil(r4 / 3) of them: r3 = 4 ceil(r4 / 3))."""
    Ho, Wo = int(grid_hw[0]), int(grid_hw[1])
    r3 = 4 * (-(-wino_tile_rows(Ho, 4) // 3)) if form == 4 else wino_tile_rows(Ho)
    n = len(m_norms)
    if not 0 < n <= 16:
        raise ValueError("need 1..16 views")
    lib = _native.load()
    boxes = torch.empty((n, int(lib.mvbev_warp_wino_boxes_count(Wo, r3)), 4), dtype=torch.int32, device=device)
    arr = (_native.WarpView * n)()
    for i, m in enumerate(m_norms):
        arr[i].m = (ctypes.c_float * 9)(*torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist())
    if backbone_hw is not None:
        st = lib.mvbev_warp_upsampled_wino_boxes(arr, n, int(backbone_hw[0]), int(backbone_hw[1]), int(src_hw[0]),
                                                 int(src_hw[1]), Ho, Wo, r3, boxes.data_ptr(), _stream(boxes))
        _native.check(st, "mvbev_warp_upsampled_wino_boxes")
        return boxes
    st = lib.mvbev_warp_wino_boxes(arr, n, int(src_hw[0]), int(src_hw[1]), Ho, Wo, r3, boxes.data_ptr(),
                                   _stream(boxes))
    _native.check(st, "mvbev_warp_wino_boxes")
    return boxes


def warp_views_wino_rows_into(srcs, m_norms, t: torch.Tensor, slots, Cs: int, K: int, Ho: int, Wo: int,
                              dst_zeroed: bool = False, up_hw=None, nonfinite=None, boxes=None,
                              form: int = 3) -> None:
    """Warp + row-Winograd transform in ONE launch (``mvbev_warp_views_wino_rows``): view i
    (fp32 ``srcs[i]`` [B,C,H,W], host kornia matrix ``m_norms[i]``) lands in channels
    [slots[i] * Cs, + C) of ``t``, the T buffer of ``wino_rows`` for a K-channel slab of
    Ho x Wo (whole grid, out_row0 = 0); the slab itself is not written.  ``up_hw``: the sources
    are backbone-resolution maps upsampled 3x to ``up_hw`` inside the warp
    (``mvbev_warp_views_upsampled_wino_rows``; ``m_norms`` for the upsampled size).  ``nonfinite``:
    ``(flag, tag)`` — ``tag`` is stored into the device int32 ``flag[0]`` when a sample reads a NaN /
    inf feature (the fused form cannot keep the reference's NaN pattern; ``warp_views_exact_into``
    and the gated fp32 convs can).  ``form`` 4: ``t`` is the F(4,3) transform T43 of ``wino43_rows``
    (``MVBEV_WARP_WINO43``; ``boxes`` from ``warp_wino_boxes(..., form=4)``)."""
    n = len(srcs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(slots)) or n > 16:
        raise ValueError("need 1..16 matching srcs / m_norms / slots")
    _require_cuda(t, *srcs)
    B, C, H, W = srcs[0].shape
    if form not in (3, 4):
        raise ValueError("form must be 3 (F(3,3)) or 4 (F(4,3))")
    r3, nx = wino_tile_rows(Ho, form), form + 2  # row tiles, transformed rows per tile
    K8 = K // KC
    if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.numel() < B * K8 * nx * r3 * Wo * 16:
        raise ValueError("t must be a contiguous bf16 buffer of wino_rows_bytes (form 4: wino43_rows_bytes)")
    if Cs % KC or C > Cs:
        raise ValueError("Cs must be a multiple of 8 holding C")
    arr = (_native.WarpView * n)()
    dtype = srcs[0].dtype
    if dtype == torch.float16 and up_hw is not None:
        raise TypeError("the fused upsample warp takes fp32 backbone maps")
    for i, (s_, m, slot) in enumerate(zip(srcs, m_norms, slots)):
        if tuple(s_.shape) != (B, C, H, W) or s_.dtype != dtype or dtype not in (torch.float32, torch.float16):
            raise ValueError("all views must be fp32 (or fp16: ABI 11900) [B,C,H,W] of one shape and dtype")
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i].src = s_.data_ptr()
        arr[i].src_strides = _native._i64x4(*s_.stride())
        arr[i].dst = t.data_ptr() + 32 * (int(slot) * (Cs // KC)) * nx * r3 * Wo
        arr[i].dst_strides = _native._i64x4(K8 * nx * r3 * Wo, nx * r3 * Wo, Wo, 1)  # 32-byte units
        arr[i].m = (ctypes.c_float * 9)(*mm)
    flags = ((_native.WARP_DST_ZEROED if dst_zeroed else 0) | (_native.WARP_SRC_F16 if dtype == torch.float16 else 0)
             | (_native.WARP_WINO43 if form == 4 else 0))
    fp, ft = _gate(nonfinite)
    if boxes is not None:  # (from warp_wino_boxes with the same matrices, in the same view order)
        _require_cuda(boxes)
        if boxes.dtype != torch.int32 or tuple(boxes.shape[:1]) != (n,) or not boxes.is_contiguous():
            raise ValueError("boxes must be warp_wino_boxes' int32 [views, tiles, 4] table of these views")
    bp = None if boxes is None else boxes.data_ptr()
    if up_hw is not None:
        st = _native.load().mvbev_warp_views_upsampled_wino_rows_ex(arr, n, B, C, H, W, int(up_hw[0]), int(up_hw[1]),
                                                                    Ho, Wo, r3, flags, fp, ft, bp, _stream(t))
        _native.check(st, "mvbev_warp_views_upsampled_wino_rows_ex")
        return
    st = _native.load().mvbev_warp_views_wino_rows_ex(arr, n, B, C, H, W, Ho, Wo, r3, flags, fp, ft, bp, _stream(t))
    _native.check(st, "mvbev_warp_views_wino_rows_ex")


def conv3x3_wino(t: torch.Tensor, desc, packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor] = None,
                 init: Optional[torch.Tensor] = None, relu: bool = False, out: Optional[torch.Tensor] = None,
                 group_mask: Optional[torch.Tensor] = None,
                 tile_order: Optional[torch.Tensor] = None, band_rows: int = 0) -> torch.Tensor:
    """The dilation-1 3x3 conv of ``conv3x3_desc`` from its row-Winograd transform ``t``
    (``wino_rows``) with ``PackedConv3x3(..., wino=True)`` weights: ``mvbev_conv3x3_wino_bf16x3``.
    ``out``: fp32 [B, cout, out_rows, W] or split-bf16 (``split_shape``); mask / order as the
    12 x 32 grid tiles of ``conv3x3_desc``.  ``band_rows`` > 0: ``out`` is fp32 in row bands,
    contiguous [bands, B, cout, band_rows, W] with bands * band_rows >= out_rows (computed row r at
    band r // band_rows) — the partial-sum mode's reduce-scatter input, written in place."""
    _require_cuda(t, packed)
    B, W, out_rows = desc.B, desc.W, desc.out_rows
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino(cout, desc.K):
        raise ValueError("packed weights are smaller than the Winograd conv needs")
    if t.numel() * t.element_size() < wino_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's row-Winograd transform")
    y_split = out is not None and out.dtype == torch.bfloat16
    if band_rows:
        nb = -(-out_rows // band_rows)
        if (out is None or out.dim() != 5 or out.shape[0] < nb or tuple(out.shape[1:]) != (B, cout, band_rows, W)
                or out.dtype != torch.float32 or not out.is_contiguous()):
            raise ValueError(f"a banded out must be a contiguous fp32 [>={nb},{B},{cout},{band_rows},{W}] tensor")
    elif out is None:
        out = torch.empty((B, cout, out_rows, W), dtype=torch.float32, device=t.device)
    elif y_split:
        if tuple(out.shape) != split_shape(B, cout, out_rows, W) or not out.is_contiguous():
            raise ValueError(f"a split out must be a contiguous bf16 {split_shape(B, cout, out_rows, W)} tensor")
    elif tuple(out.shape) != (B, cout, out_rows, W) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"out must be a contiguous fp32 [{B},{cout},{out_rows},{W}] tensor")
    if init is not None:
        _require_cuda(init)
        if init.numel() != cout * desc.H * W or not init.is_contiguous():
            raise ValueError("init must be a contiguous [Cout,H,W] tensor")
    tiles = -(-out_rows // 12) * -(-W // _native.TILE_W)
    gmp = top = None
    if group_mask is not None:
        _require_cuda(group_mask)
        if group_mask.dtype != torch.int32 or group_mask.numel() < tiles or not group_mask.is_contiguous():
            raise ValueError(f"group_mask must be a contiguous int32 tensor of >= {tiles} tiles")
        gmp = group_mask.data_ptr()
    if tile_order is not None:
        if group_mask is None or tile_order.dtype != torch.int32 or tile_order.numel() != B * tiles:
            raise ValueError("tile_order must be an int32 permutation of the B x tiles pixel tiles")
        top = tile_order.data_ptr()
    b = bias.detach().contiguous() if bias is not None else None
    bp = b.data_ptr() if b is not None else None
    st = lib.mvbev_conv3x3_wino_bf16x3(t.data_ptr(), ctypes.byref(desc), packed.data_ptr(), bp,
                                       init.data_ptr() if init is not None else None, cout, int(bool(relu)),
                                       out.data_ptr(), _native.LAYOUT_SPLIT_BF16 if y_split else _native.LAYOUT_F32,
                                       int(band_rows), gmp, top, _stream(t))
    _native.check(st, "mvbev_conv3x3_wino_bf16x3")
    return out


def conv3x3(x: torch.Tensor, packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor] = None,
            dilation: int = 1, relu: bool = False, init: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``relu?(conv2d(x, w, bias, padding=d, dilation=d) [+ init])`` for a contiguous
    [B, K, H, W] fp32 tensor (K = the packed channel count, a multiple of 8)."""
    _require_cuda(x)
    if x.dim() != 4 or not x.is_contiguous():
        raise ValueError("x must be a contiguous [B,K,H,W] tensor")
    B, K, H, W = x.shape
    if K % KC:
        raise ValueError(f"K={K} must be a multiple of {KC}")
    d = conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    return conv3x3_desc(x, d, packed, cout, bias, init, dilation, relu, out)


def conv3x3_cout1(x: torch.Tensor, weight: torch.Tensor, dilation: int, H: Optional[int] = None,
                  in_row0: int = 0, out_row0: int = 0, out_rows: Optional[int] = None,
                  out: Optional[torch.Tensor] = None, gate=None) -> torch.Tensor:
    """``conv2d(x, weight[1,C,3,3], padding=d, dilation=d)`` (no bias).

    ``x`` [B,C,rows,W] holds global rows ``[in_row0, in_row0+rows)`` of an ``H``-row image
    (default: the whole image); returns rows ``[out_row0, out_row0+out_rows)`` → [B,1,out_rows,W].
    ``gate``: as ``conv3x3_desc``'s.
    """
    _require_cuda(x, weight)
    if x.dim() != 4 or x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("x must be a contiguous float32 [B,C,rows,W] tensor")
    B, C, rows, W = x.shape
    H = rows if H is None else H
    out_rows = H - out_row0 if out_rows is None else out_rows
    if tuple(weight.shape) != (1, C, 3, 3):
        raise ValueError(f"weight must be [1,{C},3,3], got {tuple(weight.shape)}")
    w = weight.detach().contiguous()
    if out is None:
        out = torch.empty((B, 1, out_rows, W), dtype=torch.float32, device=x.device)
    elif tuple(out.shape) != (B, 1, out_rows, W) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous fp32 [{B},1,{out_rows},{W}] tensor")
    gp, gt = _gate(gate)
    st = _native.load().mvbev_conv3x3_cout1_f32(x.data_ptr(), B, C, H, W, in_row0, rows, out_row0, out_rows,
                                                w.data_ptr(), int(dilation), out.data_ptr(), gp, gt, _stream(x))
    _native.check(st, "mvbev_conv3x3_cout1_f32")
    return out


def conv3x3_cout1_partials_bytes(desc, cout: int) -> int:
    """Bytes of the partial-sum buffer ``conv3x3_then_cout1_partials`` needs for this conv."""
    return int(_native.load().mvbev_conv3x3_bf16x3_cout1_partials_bytes(ctypes.byref(desc), int(cout)))


def conv3x3_then_cout1_partials(x: torch.Tensor, desc, packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor],
                                dilation: int, relu: bool, weight3: torch.Tensor, partials: torch.Tensor) -> None:
    """The split-bf16-input conv of ``conv3x3_desc`` (bf16x3, no init / mask) without its
    output in HBM: its epilogue writes, for the following single-output conv ``weight3``
    [1, cout, 3, 3], one partial per (64-channel set, tap, pixel) into ``partials`` (fp32,
    ``conv3x3_cout1_partials_bytes``); ``cout1_from_partials`` finishes that conv.
    (``persp_trans_detector.py:53-54``: map_classifier[2:5] without y2 in memory.)"""
    _require_cuda(x, packed, weight3, partials)
    if x.dtype != torch.bfloat16 or packed.dtype != torch.bfloat16:
        raise TypeError("the fused conv -> cout1 path takes the split-bf16 layout and bf16x3 packed weights")
    if tuple(weight3.shape) != (1, cout, 3, 3):
        raise ValueError(f"weight3 must be [1,{cout},3,3], got {tuple(weight3.shape)}")
    if partials.dtype != torch.float32 or not partials.is_contiguous():
        raise ValueError("partials must be a contiguous float32 tensor")
    w3 = weight3.detach().contiguous()
    b = bias.detach().contiguous() if bias is not None else None
    st = _native.load().mvbev_conv3x3_bf16x3_cout1_partials(
        x.data_ptr(), ctypes.byref(desc), packed.data_ptr(), b.data_ptr() if b is not None else None, int(cout),
        int(dilation), int(bool(relu)), w3.data_ptr(), partials.data_ptr(),
        partials.numel() * partials.element_size(), _stream(x))
    _native.check(st, "mvbev_conv3x3_bf16x3_cout1_partials")


def conv3x3_wino_dil(t: torch.Tensor, desc, packed: torch.Tensor, cout: int, dilation: int,
                     bias: Optional[torch.Tensor] = None, relu: bool = False,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The dense 3x3 conv of ``conv3x3_desc`` with ``dilation`` (1 or 2) from its row-Winograd
    transform ``t`` (``wino_rows(..., dilation=dilation)``) and ``PackedConv3x3(..., wino=True)``
    weights, no init / mask: ``mvbev_conv3x3_wino_bf16x3_dil``.  ``out`` fp32 or split-bf16."""
    _require_cuda(t, packed)
    B, W, out_rows = desc.B, desc.W, desc.out_rows
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino(cout, desc.K):
        raise ValueError("packed weights are smaller than the Winograd conv needs")
    if t.numel() * t.element_size() < wino_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's row-Winograd transform")
    y_split = out is not None and out.dtype == torch.bfloat16
    if out is None:
        out = torch.empty((B, cout, out_rows, W), dtype=torch.float32, device=t.device)
    elif y_split:
        if tuple(out.shape) != split_shape(B, cout, out_rows, W) or not out.is_contiguous():
            raise ValueError(f"a split out must be a contiguous bf16 {split_shape(B, cout, out_rows, W)} tensor")
    elif tuple(out.shape) != (B, cout, out_rows, W) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"out must be a contiguous fp32 [{B},{cout},{out_rows},{W}] tensor")
    b = bias.detach().contiguous() if bias is not None else None
    st = lib.mvbev_conv3x3_wino_bf16x3_dil(t.data_ptr(), ctypes.byref(desc), packed.data_ptr(),
                                           b.data_ptr() if b is not None else None, cout, int(dilation),
                                           int(bool(relu)), out.data_ptr(),
                                           _native.LAYOUT_SPLIT_BF16 if y_split else _native.LAYOUT_F32, _stream(t))
    _native.check(st, "mvbev_conv3x3_wino_bf16x3_dil")
    return out


def conv3x3_wino_dgrad(t: torch.Tensor, desc, packed: torch.Tensor, cout: int, out: torch.Tensor,
                       out_mask: Optional[torch.Tensor] = None, cot_per_group: int = 1) -> torch.Tensor:
    """A dilation-1 data gradient from the row-Winograd transform ``t`` of the split-bf16 dy
    (``wino_rows``) and ``PackedConv3x3(..., wino=True)`` weights of the forward weight with its in /
    out channels swapped and taps reversed: ``mvbev_conv3x3_wino_bf16x3_dgrad``.  ``out``: fp32
    [B, cout, out_rows, W], split-bf16 or pixel-major split-bf16 (``split_pix_shape``); ``out_mask`` as ``conv3x3_dgrad``'s (12 x 32 tiles,
    ``cot_per_group`` 128-channel Cout tiles per bit): cleared tiles are not written."""
    _require_cuda(t, packed, out)
    B, W, out_rows = desc.B, desc.W, desc.out_rows
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino(cout, desc.K):
        raise ValueError("packed weights are smaller than the Winograd conv needs")
    if t.numel() * t.element_size() < wino_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's row-Winograd transform")
    layout = _out_layout(out, B, cout, out_rows, W)
    mp = None
    if out_mask is not None:
        _require_cuda(out_mask)
        tiles = -(-out_rows // 12) * -(-W // _native.TILE_W)
        if out_mask.dtype != torch.int32 or out_mask.numel() < tiles or not out_mask.is_contiguous():
            raise ValueError(f"out_mask must be a contiguous int32 tensor of >= {tiles} tiles")
        mp = out_mask.data_ptr()
    st = lib.mvbev_conv3x3_wino_bf16x3_dgrad(t.data_ptr(), ctypes.byref(desc), packed.data_ptr(), cout, out.data_ptr(),
                                             layout, mp, int(cot_per_group), _stream(t))
    _native.check(st, "mvbev_conv3x3_wino_bf16x3_dgrad")
    return out


def conv3x3_wino_then_cout1_partials(t: torch.Tensor, desc, packed: torch.Tensor, cout: int,
                                     bias: Optional[torch.Tensor], dilation: int, relu: bool,
                                     weight3: torch.Tensor, partials: torch.Tensor) -> None:
    """``conv3x3_then_cout1_partials`` from the row-Winograd transform ``t`` of its input
    (``wino_rows(..., dilation=dilation)``) and ``PackedConv3x3(..., wino=True)`` weights:
    ``mvbev_conv3x3_wino_bf16x3_cout1_partials`` (dilation 2, relu; the same partials)."""
    _require_cuda(t, packed, weight3, partials)
    if t.dtype != torch.bfloat16 or packed.dtype != torch.bfloat16:
        raise TypeError("the Winograd conv -> cout1 path takes a bf16 T and bf16x3 Winograd weights")
    if tuple(weight3.shape) != (1, cout, 3, 3):
        raise ValueError(f"weight3 must be [1,{cout},3,3], got {tuple(weight3.shape)}")
    if partials.dtype != torch.float32 or not partials.is_contiguous():
        raise ValueError("partials must be a contiguous float32 tensor")
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino(cout, desc.K):
        raise ValueError("packed weights are smaller than the Winograd conv needs")
    if t.numel() * t.element_size() < wino_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's row-Winograd transform")
    w3 = weight3.detach().contiguous()
    b = bias.detach().contiguous() if bias is not None else None
    st = lib.mvbev_conv3x3_wino_bf16x3_cout1_partials(
        t.data_ptr(), ctypes.byref(desc), packed.data_ptr(), b.data_ptr() if b is not None else None, int(cout),
        int(dilation), int(bool(relu)), w3.data_ptr(), partials.data_ptr(),
        partials.numel() * partials.element_size(), _stream(t))
    _native.check(st, "mvbev_conv3x3_wino_bf16x3_cout1_partials")


# -- row-Winograd F(4,3) (ABI 12400: mvbev_*wino43*) ------------------------------------------------
WINO43_TILE_ROWS = 16  # output rows per F(4,3) conv tile (its frustum-mask / order granule)


def wino43_rows_bytes(desc) -> int:
    """Bytes of the F(4,3) row transform T43 of a conv input (``mvbev_wino43_rows_bytes``)."""
    return int(_native.load().mvbev_wino43_rows_bytes(ctypes.byref(desc)))


def _mask43(mask, desc, what: str):
    if mask is None:
        return None
    _require_cuda(mask)
    tiles = -(-desc.out_rows // WINO43_TILE_ROWS) * -(-desc.W // _native.TILE_W)
    if mask.dtype != torch.int32 or mask.numel() < tiles or not mask.is_contiguous():
        raise ValueError(f"{what} must be a contiguous int32 tensor of >= {tiles} tiles (16 x 32)")
    return mask.data_ptr()


def wino43_rows(x: torch.Tensor, desc, t: torch.Tensor, group_mask: Optional[torch.Tensor] = None,
                dilation: int = 1) -> torch.Tensor:
    """B^T of F(4,3) over every 4-row output tile's 6 input rows of the split-bf16 ``x`` into ``t``
    (``mvbev_wino43_rows_split_bf16``; ``group_mask`` over 16 x 32 tiles, ``t`` zero-filled once)."""
    _require_cuda(x, t)
    if x.dtype != torch.bfloat16 or t.dtype != torch.bfloat16 or not t.is_contiguous():
        raise TypeError("wino43_rows reads the split-bf16 slab and writes a contiguous bf16 T")
    st = _native.load().mvbev_wino43_rows_split_bf16(x.data_ptr(), ctypes.byref(desc), int(dilation),
                                                     _mask43(group_mask, desc, "group_mask"), t.data_ptr(),
                                                     t.numel() * t.element_size(), _stream(x))
    _native.check(st, "mvbev_wino43_rows_split_bf16")
    return t


def pack_wino43(weight: torch.Tensor, chan_map: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """G w of F(4,3), split hi / lo, in the F(4,3) conv's layout (``mvbev_pack_conv3x3_weight_wino43``);
    ``chan_map``: device int32 map of the conv input channel k to the weight's input channel."""
    _require_cuda(weight)
    cout, cin, kh, kw = weight.shape
    if (kh, kw) != (3, 3) or weight.dtype != torch.float32 or cout % BN:
        raise ValueError("expected a float32 [Cout,Cin,3,3] weight with Cout a multiple of 128")
    K = cin if chan_map is None else chan_map.numel()
    lib = _native.load()
    n = int(lib.mvbev_conv3x3_packed_bytes_wino43(cout, K)) // 2
    if out is None or out.numel() < n:
        out = torch.empty(n, dtype=torch.bfloat16, device=weight.device)
    w = weight.detach().contiguous()
    st = lib.mvbev_pack_conv3x3_weight_wino43(w.data_ptr(), cout, cin, None if chan_map is None else
                                              chan_map.data_ptr(), K, out.data_ptr(), _stream(out))
    _native.check(st, "mvbev_pack_conv3x3_weight_wino43")
    return out


def conv3x3_wino43(t: torch.Tensor, desc, packed: torch.Tensor, cout: int, bias: Optional[torch.Tensor] = None,
                   init: Optional[torch.Tensor] = None, relu: bool = False, out: Optional[torch.Tensor] = None,
                   group_mask: Optional[torch.Tensor] = None, tile_order: Optional[torch.Tensor] = None,
                   dilation: int = 1) -> torch.Tensor:
    """``conv3x3_wino`` in the F(4,3) form: from ``wino43_rows``' T and ``pack_wino43`` weights
    (``mvbev_conv3x3_wino43_bf16x3``; mask / order over 16 x 32 tiles; ``out`` fp32 or split-bf16)."""
    _require_cuda(t, packed)
    B, W, out_rows = desc.B, desc.W, desc.out_rows
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino43(cout, desc.K):
        raise ValueError("packed weights are smaller than the F(4,3) conv needs")
    if t.numel() * t.element_size() < wino43_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's F(4,3) transform")
    y_split = out is not None and out.dtype == torch.bfloat16
    if out is None:
        out = torch.empty((B, cout, out_rows, W), dtype=torch.float32, device=t.device)
    elif y_split:
        if tuple(out.shape) != split_shape(B, cout, out_rows, W) or not out.is_contiguous():
            raise ValueError(f"a split out must be a contiguous bf16 {split_shape(B, cout, out_rows, W)} tensor")
    elif tuple(out.shape) != (B, cout, out_rows, W) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"out must be a contiguous fp32 [{B},{cout},{out_rows},{W}] tensor")
    if init is not None:
        _require_cuda(init)
        if init.numel() != cout * desc.H * W or not init.is_contiguous():
            raise ValueError("init must be a contiguous [Cout,H,W] tensor")
    gmp = _mask43(group_mask, desc, "group_mask")
    top = None
    if tile_order is not None:
        tiles = -(-out_rows // WINO43_TILE_ROWS) * -(-W // _native.TILE_W)
        if group_mask is None or tile_order.dtype != torch.int32 or tile_order.numel() != B * tiles:
            raise ValueError("tile_order must be an int32 permutation of the B x tiles pixel tiles")
        top = tile_order.data_ptr()
    b = bias.detach().contiguous() if bias is not None else None
    st = lib.mvbev_conv3x3_wino43_bf16x3(t.data_ptr(), ctypes.byref(desc), packed.data_ptr(),
                                         b.data_ptr() if b is not None else None,
                                         init.data_ptr() if init is not None else None, cout, int(dilation),
                                         int(bool(relu)), out.data_ptr(),
                                         _native.LAYOUT_SPLIT_BF16 if y_split else _native.LAYOUT_F32, gmp, top,
                                         _stream(t))
    _native.check(st, "mvbev_conv3x3_wino43_bf16x3")
    return out


def conv3x3_wino43_then_cout1_partials(t: torch.Tensor, desc, packed: torch.Tensor, cout: int,
                                       bias: Optional[torch.Tensor], relu: bool, weight3: torch.Tensor,
                                       partials: torch.Tensor) -> None:
    """``conv3x3_wino_then_cout1_partials`` (dilation 2) in the F(4,3) form: the same partials
    (``mvbev_conv3x3_wino43_bf16x3_cout1_partials``)."""
    _require_cuda(t, packed, weight3, partials)
    if tuple(weight3.shape) != (1, cout, 3, 3):
        raise ValueError(f"weight3 must be [1,{cout},3,3], got {tuple(weight3.shape)}")
    if partials.dtype != torch.float32 or not partials.is_contiguous():
        raise ValueError("partials must be a contiguous float32 tensor")
    lib = _native.load()
    if packed.numel() * packed.element_size() < lib.mvbev_conv3x3_packed_bytes_wino43(cout, desc.K):
        raise ValueError("packed weights are smaller than the F(4,3) conv needs")
    if t.numel() * t.element_size() < wino43_rows_bytes(desc):
        raise ValueError("t is smaller than the descriptor's F(4,3) transform")
    w3 = weight3.detach().contiguous()
    b = bias.detach().contiguous() if bias is not None else None
    st = lib.mvbev_conv3x3_wino43_bf16x3_cout1_partials(
        t.data_ptr(), ctypes.byref(desc), packed.data_ptr(), b.data_ptr() if b is not None else None, int(cout), 2,
        int(bool(relu)), w3.data_ptr(), partials.data_ptr(), partials.numel() * partials.element_size(), _stream(t))
    _native.check(st, "mvbev_conv3x3_wino43_bf16x3_cout1_partials")


def cout1_from_partials(partials: torch.Tensor, desc, cout: int, dilation3: int, map_row0: int, map_rows: int,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``conv2d(act(y), weight3, padding=d3, dilation=d3)`` rows ``[map_row0, map_row0+map_rows)``
    → [B,1,map_rows,W] from ``conv3x3_then_cout1_partials``' partials (fixed summation order)."""
    _require_cuda(partials)
    B, W = desc.B, desc.W
    if out is None:
        out = torch.empty((B, 1, map_rows, W), dtype=torch.float32, device=partials.device)
    st = _native.load().mvbev_cout1_reduce_partials(partials.data_ptr(), ctypes.byref(desc), int(cout), int(dilation3),
                                                     out.data_ptr(), int(map_row0), int(map_rows), _stream(partials))
    _native.check(st, "mvbev_cout1_reduce_partials")
    return out


# ----------------------------------------------------------------------------------------------
# backward: the adjoints autograd needs to train through the hot path

def warp_views_backward(grad_outs, m_norms, grad_srcs) -> None:
    """Adjoint of ``warp_views_into`` (fp32): ``grad_srcs[i]`` [B,C,H,W] (innermost stride 1)
    ACCUMULATES w_corner * ``grad_outs[i]`` [B,C,Ho,Wo] for every in-bounds bilinear corner of
    every finite inside sample (grid_sample's backward under kornia.warp_perspective,
    ``persp_trans_detector.py:69``).  ``m_norms[i]``: host [3,3] src_norm <- dst_norm."""
    n = len(grad_outs)
    if n == 0:
        return
    if not (len(m_norms) == n == len(grad_srcs)) or n > 16:
        raise ValueError("need 1..16 matching grad_outs / m_norms / grad_srcs")
    _require_cuda(*grad_outs, *grad_srcs)
    B, C, Ho, Wo = grad_outs[0].shape
    _, _, H, W = grad_srcs[0].shape
    arr = (_native.WarpView * n)()
    for i, (g, m, d) in enumerate(zip(grad_outs, m_norms, grad_srcs)):
        if tuple(g.shape) != (B, C, Ho, Wo) or tuple(d.shape) != (B, C, H, W):
            raise ValueError(f"all views must share shapes: grad_out {tuple(g.shape)} grad_src {tuple(d.shape)}")
        if g.dtype != torch.float32 or d.dtype != torch.float32:
            raise TypeError("the warp backward is fp32")
        if d.stride(3) != 1:
            raise ValueError("grad_src needs contiguous rows (innermost stride 1)")
        mm = torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist()
        arr[i] = _native.WarpView(g.data_ptr(), (ctypes.c_int64 * 4)(*g.stride()), d.data_ptr(),
                                  (ctypes.c_int64 * 4)(*d.stride()), (ctypes.c_float * 9)(*mm))
    st = _native.load().mvbev_warp_views_backward_f32(arr, n, B, C, H, W, Ho, Wo, _stream(grad_srcs[0]))
    _native.check(st, "mvbev_warp_views_backward_f32")


class WarpAdjointPlan:
    """CSR transpose of one view's bilinear sampling matrix (``mvbev_warp_adjoint_plan``):
    geometry only, built once per (matrix, sizes, device) on the GPU."""

    def __init__(self, m_norm, src_hw, grid_hw, device, backbone_hw=None):
        """``backbone_hw`` (h, w): the plan of the fused 3x-upsample + warp
        (``warp_views_upsampled_into``) from the h x w map upsampled to ``src_hw``; its
        ``src_hw`` is then (h, w), the pixels the adjoint writes."""
        H, W = int(src_hw[0]), int(src_hw[1])
        Ho, Wo = int(grid_hw[0]), int(grid_hw[1])
        device = torch.device(device)
        mm = (ctypes.c_float * 9)(*torch.as_tensor(m_norm, dtype=torch.float32).reshape(9).tolist())
        lib = _native.load()
        if backbone_hw is None:
            self.src_hw, self.grid_hw, per = (H, W), (Ho, Wo), 4
        else:
            h, w = int(backbone_hw[0]), int(backbone_hw[1])
            self.src_hw, self.grid_hw, per = (h, w), (Ho, Wo), 9
        P = self.src_hw[0] * self.src_hw[1]
        self.row_ptr = torch.empty(P + 1, dtype=torch.int32, device=device)
        self.col = torch.empty(per * Ho * Wo, dtype=torch.int32, device=device)
        self.val = torch.empty(per * Ho * Wo, dtype=torch.float32, device=device)
        scratch = torch.empty(P, dtype=torch.int32, device=device)
        if backbone_hw is None:
            st = lib.mvbev_warp_adjoint_plan(mm, H, W, Ho, Wo, self.row_ptr.data_ptr(), self.col.data_ptr(),
                                             self.val.data_ptr(), scratch.data_ptr(), _stream(self.row_ptr))
        else:
            st = lib.mvbev_warp_upsampled_adjoint_plan(mm, h, w, H, W, Ho, Wo, self.row_ptr.data_ptr(),
                                                       self.col.data_ptr(), self.val.data_ptr(), scratch.data_ptr(),
                                                       _stream(self.row_ptr))
        _native.check(st, "warp adjoint plan")
        self._scratch = scratch  # freed with the plan (kept until the stream has used it)

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1].item())


def warp_views_adjoint(grad_outs, plans, grad_srcs, accumulate: bool = False, pixel_major: bool = False) -> None:
    """Deterministic gather form of ``warp_views_backward``: ``grad_srcs[i]`` [B,C,H,W] =
    (or += with ``accumulate``) the adjoint of view i's warp applied to ``grad_outs[i]``;
    ``plans[i]`` its ``WarpAdjointPlan``.  ``grad_outs[i]``: fp32 [B,C,Ho,Wo] with dense rows,
    or a bf16 split-bf16 blocked [B, C/8, Ho, Wo, 2, 8] view (``split_shape``; C % 8 == 0), or with
    ``pixel_major`` a [B, Ho, Wo, C/8, 2, 8] view of a pixel-major split tensor (``split_pix_shape``, the
    view's groups a slice of the pixel's: MVBEV_LAYOUT_SPLIT_BF16_PIX) — the same grad_srcs, which may then
    also be channels-last tensors (all of them or none)."""
    n = len(grad_outs)
    if n == 0:
        return
    if not (len(plans) == n == len(grad_srcs)) or n > 16:
        raise ValueError("need 1..16 matching grad_outs / plans / grad_srcs")
    _require_cuda(*grad_outs, *grad_srcs)
    split = grad_outs[0].dtype == torch.bfloat16
    B, C, H, W = grad_srcs[0].shape
    # pixel-major split: [B, Ho, Wo, C/8, 2, 8] slices (of a [B, Ho, Wo, G, 2, 8] tensor)
    pixm = bool(pixel_major)
    if pixm and not split:
        raise ValueError("pixel_major needs bf16 split grad_outs")
    if split:
        if C % KC:
            raise ValueError("a split grad_out needs C % 8 == 0")
        if pixm:
            Ho, Wo = grad_outs[0].shape[1], grad_outs[0].shape[2]
            want = split_pix_shape(B, C, Ho, Wo)
        else:
            Ho, Wo = grad_outs[0].shape[2], grad_outs[0].shape[3]
            want = split_shape(B, C, Ho, Wo)
    else:
        Ho, Wo = grad_outs[0].shape[2], grad_outs[0].shape[3]
        want = (B, C, Ho, Wo)
    arr = (_native.WarpAdjointView * n)()
    for i, (g, pl, d) in enumerate(zip(grad_outs, plans, grad_srcs)):
        if tuple(g.shape) != want or tuple(d.shape) != (B, C, H, W):
            raise ValueError(f"all views must share shapes: grad_out {tuple(g.shape)} (want {want}) "
                             f"grad_src {tuple(d.shape)}")
        if pl.src_hw != (H, W) or pl.grid_hw != (Ho, Wo):
            raise ValueError("plan built for other sizes")
        if d.dtype != torch.float32 or g.dtype != (torch.bfloat16 if split else torch.float32):
            raise TypeError("grad_src is fp32; grad_out fp32 or split-bf16 (bf16 storage)")
        if pixm:
            if g.stride(5) != 1 or g.stride(4) != KC or g.stride(3) != 2 * KC or g.stride(1) != g.stride(2) * Wo:
                raise ValueError("pixel-major split grad_out needs adjacent groups and dense pixels")
            gstr = (g.stride(0) // 16, 1, g.stride(1) // 16, g.stride(2) // 16)  # 32-byte units
        elif split:
            if g.stride(5) != 1 or g.stride(4) != KC or g.stride(3) != 2 * KC or g.stride(2) != 2 * KC * Wo:
                raise ValueError("split grad_out needs dense pixels")
            gstr = (g.stride(0) // 16, g.stride(1) // 16, Wo, 1)  # 32-byte units
        else:
            if g.stride(3) != 1 or g.stride(2) != Wo:
                raise ValueError("grad_out planes must be dense (row stride = width, column stride 1)")
            gstr = tuple(g.stride())
        cl = pixm and d.stride(1) == 1 and d.stride(3) == C and d.stride(2) == W * C  # channels-last grad_src
        if not cl and (d.stride(3) != 1 or d.stride(2) != W):
            raise ValueError("grad_src planes must be dense (row stride = width, column stride 1), or "
                             "channels-last with a pixel-major grad_out")
        arr[i] = _native.WarpAdjointView(g.data_ptr(), (ctypes.c_int64 * 4)(*gstr), d.data_ptr(),
                                         (ctypes.c_int64 * 4)(*d.stride()), pl.row_ptr.data_ptr(),
                                         pl.col.data_ptr(), pl.val.data_ptr())
    layout = _native.LAYOUT_SPLIT_PIX if pixm else _native.LAYOUT_SPLIT_BF16 if split else _native.LAYOUT_F32
    st = _native.load().mvbev_warp_views_adjoint(arr, n, layout, B, C, H, W, Ho, Wo, int(bool(accumulate)),
                                                 _stream(grad_srcs[0]))
    _native.check(st, "mvbev_warp_views_adjoint")


class PackedDgrad3x3:
    """bf16x3-packed weights of a 3x3 conv's DATA gradient (transposed, flipped taps:
    ``mvbev_pack_conv3x3_dgrad_bf16x3``).  Output channel o of the dgrad conv = forward input
    channel ``chan_map[o]`` (None: identity over ``k_out`` channels).  Re-packed only when the
    parameter changes."""

    def __init__(self, k_out: int, chan_map: Optional[Sequence[int]] = None):
        self.k_out = int(k_out)
        if chan_map is not None and len(chan_map) != self.k_out:
            raise ValueError("chan_map must have k_out entries")
        self.chan_map = None if chan_map is None else [int(c) for c in chan_map]
        self.cout_p = -(-self.k_out // BN) * BN   # dgrad conv output channels (padded)
        self._key = None
        self.packed: Optional[torch.Tensor] = None
        self._map_dev: Optional[torch.Tensor] = None

    def get(self, weight: torch.Tensor) -> torch.Tensor:
        _require_cuda(weight)
        lib = _native.load()
        key = (weight.data_ptr(), weight._version, tuple(weight.shape), id(lib))
        if key != self._key:
            cout_w, cin_w, kh, kw = weight.shape
            if (kh, kw) != (3, 3) or weight.dtype != torch.float32:
                raise ValueError("expected a float32 [Cout,Cin,3,3] weight")
            if cout_w % KC:
                raise ValueError(f"forward Cout={cout_w} must be a multiple of {KC} (the dgrad conv's K)")
            if self.chan_map is None and self.k_out > cin_w:
                raise ValueError(f"k_out={self.k_out} exceeds the weight's {cin_w} input channels")
            if self.chan_map is not None and (self._map_dev is None or self._map_dev.device != weight.device):
                self._map_dev = torch.tensor(self.chan_map, dtype=torch.int32, device=weight.device)
            cmap = None if self._map_dev is None else self._map_dev.data_ptr()
            w = weight.detach().contiguous()
            n = lib.mvbev_conv3x3_packed_bytes_bf16x3(self.cout_p, cout_w)
            packed = torch.empty(n // 2, dtype=torch.bfloat16, device=weight.device)
            st = lib.mvbev_pack_conv3x3_dgrad_bf16x3(w.data_ptr(), cout_w, cin_w, cmap, self.k_out,
                                                     packed.data_ptr(), _stream(packed))
            _native.check(st, "mvbev_pack_conv3x3_dgrad_bf16x3")
            self.packed, self._key = packed, key
        return self.packed


def dgrad_schedule(B: int, cout_p: int, H: int, W: int, K: int, out_mask: Optional[torch.Tensor],
                   cot_per_group: int, device, split: bool = True):
    """The balanced ring-kernel schedule (``schedule.plan``) of ``conv3x3_dgrad`` from a
    split-bf16 dy (12-row tiles, all K chunks per block, the output-side mask's blocks)."""
    from . import schedule
    th = dgrad_tile_rows(True, 1)
    ty, tx = -(-H // th), -(-W // _native.TILE_W)
    om = None if out_mask is None else [int(v) for v in out_mask.cpu().tolist()]
    blocks = schedule.ring_blocks(B, ty, tx, cout_p // BN, -(-K // (2 * KC)), out_mask=om,
                                  cot_per_group=cot_per_group)
    cus = torch.cuda.get_device_properties(torch.device(device)).multi_processor_count
    return schedule.plan(blocks, cus, device, split=split)


def conv3x3_dgrad(dy: torch.Tensor, packed: PackedDgrad3x3, weight: torch.Tensor, dilation: int,
                  out: Optional[torch.Tensor] = None, out_mask: Optional[torch.Tensor] = None,
                  cot_per_group: int = 1, sched=None) -> torch.Tensor:
    """Data gradient of a 3x3 stride-1 conv (padding = dilation): dy [B,Cout_w,H,W] fp32
    contiguous (or its split-bf16 layout, a bf16 ``split_shape`` tensor: the LDS-DMA ring
    kernel) -> [B, cout_p, H, W] fp32, or the split-bf16 layout when ``out`` is a bf16
    ``split_shape`` tensor (channel o = forward input channel chan_map[o]; channels past
    k_out are zero).  ``out_mask`` (int32 per conv output tile, ``warp_tile_mask`` at
    ``dgrad_tile_rows`` rows): tiles of output channel group g (``cot_per_group`` 128-channel
    tiles) whose bit is clear are NOT written (for a consumer that never reads them).
    ``sched``: a ``dgrad_schedule`` of the same sizes and mask (split-bf16 dy only)."""
    _require_cuda(dy)
    dy_split = dy.dtype == torch.bfloat16
    if dy.dim() != (6 if dy_split else 4) or dy.dtype not in (torch.float32, torch.bfloat16) or not dy.is_contiguous():
        raise ValueError("dy must be a contiguous float32 [B,Cout,H,W] tensor or its split-bf16 layout")
    if dy_split:
        B, G, H, W = dy.shape[:4]
        K = 8 * G
    else:
        B, K, H, W = dy.shape
    if K != weight.shape[0]:
        raise ValueError(f"dy has {K} channels, the weight {weight.shape[0]} outputs")
    cp = packed.cout_p
    if out is None:
        out = torch.empty((B, cp, H, W), dtype=torch.float32, device=dy.device)
    layout = _out_layout(out, B, cp, H, W)
    if layout == _native.LAYOUT_SPLIT_PIX and not dy_split:
        raise ValueError("a pixel-major split out needs the ring kernel (a split-bf16 dy)")
    mp = None
    if out_mask is not None:
        _require_cuda(out_mask)
        tiles = -(-H // dgrad_tile_rows(dy_split, dilation)) * -(-W // _native.TILE_W)
        if out_mask.dtype != torch.int32 or out_mask.numel() < tiles or not out_mask.is_contiguous():
            raise ValueError(f"out_mask must be a contiguous int32 tensor of >= {tiles} tiles")
        mp = out_mask.data_ptr()
    d = conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    if sched is not None:
        if not dy_split:
            raise ValueError("a ring-kernel schedule needs a split-bf16 dy")
        st = _native.load().mvbev_conv3x3_dgrad_bf16x3_sched(
            dy.data_ptr(), _native.LAYOUT_SPLIT_BF16, ctypes.byref(d), packed.get(weight).data_ptr(), cp,
            int(dilation), out.data_ptr(), layout, mp, int(cot_per_group), ctypes.byref(sched.c), _stream(dy))
        _native.check(st, "mvbev_conv3x3_dgrad_bf16x3_sched")
        return out
    st = _native.load().mvbev_conv3x3_dgrad_bf16x3_ex(
        dy.data_ptr(), _native.LAYOUT_SPLIT_BF16 if dy_split else _native.LAYOUT_F32, ctypes.byref(d),
        packed.get(weight).data_ptr(), cp, int(dilation), out.data_ptr(), layout, mp, int(cot_per_group), _stream(dy))
    _native.check(st, "mvbev_conv3x3_dgrad_bf16x3_ex")
    return out


def dgrad_tile_rows(dy_split: bool, dilation: int = 1) -> int:
    """Output-tile rows of ``conv3x3_dgrad`` (its ``out_mask`` granule) for this dy layout."""
    return _native.conv_tile_rows(_native.LAYOUT_SPLIT_BF16 if dy_split else _native.LAYOUT_F32, dilation)


def _chunk_lists(mask: torch.Tensor, groups: int, B: int, rows: int, rows_per_tile: int, W: int):
    """Per channel group, the (b, row, 32-px segment) chunks whose mask tile (row // rows_per_tile,
    segment) has the group's bit -> (chunk_list, chunk_off) int32 device tensors (chunk id
    (b * rows + row) * segments + segment, in that order)."""
    import numpy as np
    tx = -(-W // _native.TILE_W)
    segs = -(-W // 32)
    assert segs == tx, "wgrad chunks are 32 px = one conv tile column"
    m = np.asarray(mask.cpu().numpy(), dtype=np.int64) & 0xFFFFFFFF
    tile = np.repeat(np.arange(rows) // rows_per_tile, segs) * tx + np.tile(np.arange(segs), rows)  # per (row, seg)
    per_img = m[tile]
    lists, off = [], [0]
    for g in range(groups):
        act = np.nonzero((per_img >> g) & 1)[0]
        full = (np.arange(B)[:, None] * (rows * segs) + act[None, :]).reshape(-1)
        lists.append(full)
        off.append(off[-1] + full.size)
    lst = np.concatenate(lists) if lists else np.zeros(0, np.int64)
    dev = mask.device
    return (torch.tensor(lst, dtype=torch.int32, device=dev) if lst.size else torch.zeros(1, dtype=torch.int32,
                                                                                          device=dev),
            torch.tensor(off, dtype=torch.int32, device=dev))


def wgrad_chunk_lists(mask: torch.Tensor, groups: int, B: int, H: int, W: int):
    """Per channel group, the wgrad pixel chunks (row segments of 32 px) whose window the
    frustum ``mask`` (``warp_tile_mask`` over rows [0, H), halo >= the conv's dilation) marks
    as possibly non-zero -> (chunk_list, chunk_off) int32 device tensors."""
    return _chunk_lists(mask, groups, B, H, _native.TILE_H, W)


def split_rows_shape(B: int, C: int, H: int, W: int):
    """Shape of the row-split bf16 layout (MVBEV_LAYOUT_SPLIT_ROWS) of a [B,C,H,W] tensor:
    per (channel, row, 8-pixel run) bf16 hi[8] then lo[8]."""
    return (B, C, H, W // 8, 2, 8)


def split_rows(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 [B,C,H,W] (contiguous, W % 8 == 0) -> its row-split bf16 form (``split_rows_shape``),
    hi = bf16(x), lo = bf16(x - hi): the conv weight gradient's pre-split dy."""
    _require_cuda(x)
    if x.dim() != 4 or x.dtype != torch.float32 or not x.is_contiguous() or x.shape[3] % 8:
        raise ValueError("split_rows needs a contiguous float32 [B,C,H,W] tensor with W % 8 == 0")
    B, C, H, W = x.shape
    if out is None:
        out = torch.empty(split_rows_shape(B, C, H, W), dtype=torch.bfloat16, device=x.device)
    elif tuple(out.shape) != split_rows_shape(B, C, H, W) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError("out must be a contiguous bf16 tensor of split_rows_shape")
    st = _native.load().mvbev_split_rows_bf16(x.data_ptr(), B * C * H, W, out.data_ptr(), _stream(x))
    _native.check(st, "mvbev_split_rows_bf16")
    return out


def conv3x3_wgrad(x: torch.Tensor, desc, dy: torch.Tensor, dilation: int, cin_w: int,
                  chan_map: Optional[torch.Tensor] = None, dw: Optional[torch.Tensor] = None,
                  workspace: Optional[torch.Tensor] = None, chunk_lists=None,
                  dy_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Weight gradient of a 3x3 conv whose input ``x`` is addressed by ``desc`` (fp32, or the
    split-bf16 layout when ``x`` is bf16) and whose output gradient is ``dy`` [B,Cout,H,W] fp32:
    writes dw[co][chan_map[k]][:] (identity without a map) of a [Cout, cin_w, 3, 3] tensor
    (allocated zeroed when ``dw`` is None; unmapped channels are left as they are).
    ``dy_rows``: optionally dy's ``split_rows`` form, which the LDS-DMA kernel reads instead
    of splitting dy itself (bitwise the same dw; used where that kernel applies, else dy)."""
    _require_cuda(x, dy)
    if dy.dim() != 4 or dy.dtype != torch.float32 or not dy.is_contiguous():
        raise ValueError("dy must be a contiguous float32 [B,Cout,H,W] tensor")
    B, cout, H, W = dy.shape
    if dy_rows is not None:
        _require_cuda(dy_rows)
        if (tuple(dy_rows.shape) != split_rows_shape(B, cout, H, W) or dy_rows.dtype != torch.bfloat16
                or not dy_rows.is_contiguous()):
            raise ValueError("dy_rows must be dy's split_rows form")
    if (desc.B, desc.H, desc.W) != (B, H, W):
        raise ValueError("dy does not match the conv descriptor")
    if x.dtype == torch.float32:
        layout = _native.LAYOUT_F32
    elif x.dtype == torch.bfloat16:
        layout = _native.LAYOUT_SPLIT_BF16
    else:
        raise TypeError(f"x dtype {x.dtype} not supported by the wgrad kernel")
    if chan_map is not None:
        _require_cuda(chan_map)
        if chan_map.dtype != torch.int32 or chan_map.numel() != desc.K:
            raise ValueError("chan_map must be an int32 device tensor of K entries")
    if dw is None:
        dw = torch.zeros((cout, cin_w, 3, 3), dtype=torch.float32, device=dy.device)
    elif tuple(dw.shape) != (cout, cin_w, 3, 3) or not dw.is_contiguous() or dw.dtype != torch.float32:
        raise ValueError(f"dw must be a contiguous fp32 [{cout},{cin_w},3,3] tensor")
    lib = _native.load()
    need = int(lib.mvbev_conv3x3_wgrad_workspace_bytes(ctypes.byref(desc), cout))
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty((need + 3) // 4, dtype=torch.float32, device=dy.device)
    cl, co = (None, None) if chunk_lists is None else (chunk_lists[0].data_ptr(), chunk_lists[1].data_ptr())
    for d, dl in ((dy_rows, _native.LAYOUT_SPLIT_ROWS), (dy, _native.LAYOUT_F32)):
        if d is None:
            continue
        st = lib.mvbev_conv3x3_wgrad_bf16x3_ex2(x.data_ptr(), layout, ctypes.byref(desc), d.data_ptr(), dl, cout,
                                                int(dilation), None if chan_map is None else chan_map.data_ptr(),
                                                cin_w, dw.data_ptr(), cl, co, workspace.data_ptr(),
                                                workspace.numel() * workspace.element_size(), _stream(dy))
        if st == _native.ERR_SHAPE and dl == _native.LAYOUT_SPLIT_ROWS:
            continue  # not the LDS-DMA path (nothing was launched): the fp32 dy
        _native.check(st, "mvbev_conv3x3_wgrad_bf16x3_ex2")
        break
    return dw


def wino_dy_rows(dy: torch.Tensor, out: Optional[torch.Tensor] = None, dilation: int = 1) -> torch.Tensor:
    """fp32 dy [B,Cout,H,W] (contiguous, W % 8 == 0) -> D_xi = sum_j AT[j][xi] dy[base(r3) + dilation j] in
    the row-split bf16 layout, [B, 5, Cout, R3, W/8, 2, 8] (``mvbev_wino_dy_rows_f32``; R3 = ceil(H/3) for
    dilation 1, 4 ceil(H/12) over conv2's interleaved row tiles for dilation 2): the output-gradient side
    of ``conv3x3_wgrad_wino``."""
    _require_cuda(dy)
    if dy.dim() != 4 or dy.dtype != torch.float32 or not dy.is_contiguous() or dy.shape[3] % 8:
        raise ValueError("wino_dy_rows needs a contiguous float32 [B,C,H,W] tensor with W % 8 == 0")
    B, C, H, W = dy.shape
    if dilation not in (1, 2):
        raise ValueError("dilation must be 1 or 2")
    shape = (B, 5, C, wino_r3(H, dilation), W // 8, 2, 8)
    if out is None:
        out = torch.empty(shape, dtype=torch.bfloat16, device=dy.device)
    elif tuple(out.shape) != shape or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous bf16 tensor of shape {shape}")
    st = _native.load().mvbev_wino_dy_rows_f32(dy.data_ptr(), B, C, H, W, int(dilation), out.data_ptr(),
                                               out.numel() * out.element_size(), _stream(dy))
    _native.check(st, "mvbev_wino_dy_rows_f32")
    return out


def wino_r3(H: int, dilation: int = 1) -> int:
    """3-row tiles of a row-Winograd transform over H rows: ceil(H/3), or 4 per 12-row tile (dilation 2)."""
    return -(-H // 3) if dilation == 1 else 4 * (-(-H // 12))


def wgrad_wino_chunk_lists(mask: torch.Tensor, groups: int, B: int, H: int, W: int):
    """Per channel group, the Winograd wgrad chunks (b, r3 < ceil(H/3), 32-px segment) whose T row
    can be non-zero: the forward's 12-row frustum ``mask`` (``conv1_mask(tile_h=12)``, the mask T was
    written under) at tile (r3 // 4, segment) -> (chunk_list, chunk_off) int32 device tensors."""
    if mask.numel() != -(-H // 12) * (-(-W // _native.TILE_W)):
        raise ValueError("the mask must be over 12-row conv tiles (the rows T was written in)")
    return _chunk_lists(mask, groups, B, wino_r3(H), 4, W)


def conv3x3_wgrad_wino(t: torch.Tensor, desc, dy_wino: torch.Tensor, cin_w: int,
                       chan_map: Optional[torch.Tensor] = None, dw: Optional[torch.Tensor] = None,
                       workspace: Optional[torch.Tensor] = None, chunk_lists=None, dilation: int = 1) -> torch.Tensor:
    """Weight gradient of a dilation-1 3x3 conv from its forward's row-Winograd transform ``t``
    (``wino_rows`` of the input ``desc`` addresses, or the fused warp's) and ``dy_wino`` =
    ``wino_dy_rows(dy)`` (``mvbev_conv3x3_wgrad_wino_bf16x3``): the same dw as ``conv3x3_wgrad``
    within the 3xbf16 error.  ``chunk_lists``: ``wgrad_wino_chunk_lists`` of the mask T was written
    under.  Writes dw[co][chan_map[k]][:] of a [Cout, cin_w, 3, 3] tensor (allocated zeroed when None)."""
    _require_cuda(t, dy_wino)
    B, cout = dy_wino.shape[0], dy_wino.shape[2]
    if dy_wino.dim() != 7 or dy_wino.dtype != torch.bfloat16 or not dy_wino.is_contiguous() or dy_wino.shape[1] != 5:
        raise ValueError("dy_wino must be wino_dy_rows' output")
    if (desc.B, wino_r3(desc.H, dilation), desc.W // 8) != (B, dy_wino.shape[3], dy_wino.shape[4]):
        raise ValueError("dy_wino does not match the conv descriptor")
    if chan_map is not None:
        _require_cuda(chan_map)
        if chan_map.dtype != torch.int32 or chan_map.numel() != desc.K:
            raise ValueError("chan_map must be an int32 device tensor of K entries")
    if dw is None:
        dw = torch.zeros((cout, cin_w, 3, 3), dtype=torch.float32, device=t.device)
    elif tuple(dw.shape) != (cout, cin_w, 3, 3) or not dw.is_contiguous() or dw.dtype != torch.float32:
        raise ValueError(f"dw must be a contiguous fp32 [{cout},{cin_w},3,3] tensor")
    lib = _native.load()
    need = int(lib.mvbev_conv3x3_wgrad_wino_workspace_bytes(ctypes.byref(desc), cout, int(dilation)))
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty((need + 3) // 4, dtype=torch.float32, device=t.device)
    cl, co = (None, None) if chunk_lists is None else (chunk_lists[0].data_ptr(), chunk_lists[1].data_ptr())
    st = lib.mvbev_conv3x3_wgrad_wino_bf16x3(t.data_ptr(), t.numel() * t.element_size(), ctypes.byref(desc),
                                             dy_wino.data_ptr(), dy_wino.numel() * dy_wino.element_size(), cout,
                                             int(dilation), None if chan_map is None else chan_map.data_ptr(), cin_w,
                                             dw.data_ptr(),
                                             cl, co, workspace.data_ptr(),
                                             workspace.numel() * workspace.element_size(), _stream(t))
    _native.check(st, "mvbev_conv3x3_wgrad_wino_bf16x3")
    return dw


def conv3x3_bias_coord_grad(dy: torch.Tensor, dilation: int, db: Optional[torch.Tensor] = None,
                            dw: Optional[torch.Tensor] = None, coord_ch: int = 0) -> None:
    """db[co] = sum dy[:, co]; with ``dw`` [Cout, Cin_w, 3, 3], also the weight gradient of the
    two coord-map channels ``coord_ch, coord_ch + 1`` (``create_coord_map``)."""
    _require_cuda(dy)
    if dy.dim() != 4 or dy.dtype != torch.float32 or not dy.is_contiguous():
        raise ValueError("dy must be a contiguous float32 [B,Cout,H,W] tensor")
    B, cout, H, W = dy.shape
    cin_w = 0
    for t in (db, dw):
        if t is not None:
            _require_cuda(t)
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("db / dw must be contiguous fp32 tensors")
    if db is not None and db.numel() != cout:
        raise ValueError("db must have Cout entries")
    if dw is not None:
        if dw.dim() != 4 or dw.shape[0] != cout or tuple(dw.shape[2:]) != (3, 3):
            raise ValueError("dw must be [Cout, Cin_w, 3, 3]")
        cin_w = dw.shape[1]
    st = _native.load().mvbev_conv3x3_bias_coord_grad_f32(
        dy.data_ptr(), B, cout, H, W, int(dilation), None if db is None else db.data_ptr(),
        None if dw is None else dw.data_ptr(), cin_w, int(coord_ch), _stream(dy))
    _native.check(st, "mvbev_conv3x3_bias_coord_grad_f32")


def relu_backward_(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """In place: dy = dy where y > 0 else 0 (``y`` = the ReLU's output)."""
    _require_cuda(dy, y)
    if dy.shape != y.shape or dy.dtype != torch.float32 or y.dtype != torch.float32 or \
            not dy.is_contiguous() or not y.is_contiguous():
        raise ValueError("dy and y must be contiguous fp32 tensors of one shape")
    st = _native.load().mvbev_relu_backward_f32(dy.data_ptr(), y.data_ptr(), dy.numel(), _stream(dy))
    _native.check(st, "mvbev_relu_backward_f32")
    return dy


def relu_backward_split_(dy: torch.Tensor, y_split: torch.Tensor, dy_split: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In place: dy [B,C,H,W] fp32 = dy where y > 0 else 0, with the ReLU output ``y_split`` in
    the split-bf16 layout (``split_shape(B, C, H, W)``, y = hi + lo); ``dy_split`` (optional,
    same split shape) also receives the masked dy in the split layout."""
    _require_cuda(dy, y_split)
    B, C, H, W = dy.shape
    if dy.dtype != torch.float32 or not dy.is_contiguous():
        raise ValueError("dy must be a contiguous fp32 [B,C,H,W] tensor")
    for t in (y_split, dy_split):
        if t is not None and (t.dtype != torch.bfloat16 or tuple(t.shape) != split_shape(B, C, H, W)
                              or not t.is_contiguous()):
            raise ValueError(f"split tensors must be contiguous bf16 {split_shape(B, C, H, W)}")
    st = _native.load().mvbev_relu_backward_split_f32(dy.data_ptr(), y_split.data_ptr(), B, C, H, W,
                                                       None if dy_split is None else dy_split.data_ptr(), _stream(dy))
    _native.check(st, "mvbev_relu_backward_split_f32")
    return dy


def conv3x3_cout1_backward(x: torch.Tensor, weight: torch.Tensor, dmap: torch.Tensor, dilation: int,
                           relu_mask: bool = False, need_dx: bool = True, need_dw: bool = True,
                           dx_split: Optional[torch.Tensor] = None):
    """Backward of ``conv3x3_cout1`` over a whole image: returns (dx [B,C,H,W] or None,
    dw [1,C,3,3] or None).  ``relu_mask``: zero dx where x <= 0 (x = the previous ReLU's output,
    its backward fused).  ``dx_split`` (optional, bf16 ``split_shape(B,C,H,W)``) also receives
    dx in the split-bf16 layout (the next data-gradient conv's input)."""
    _require_cuda(x, weight, dmap)
    if x.dim() != 4 or x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("x must be a contiguous float32 [B,C,H,W] tensor")
    B, C, H, W = x.shape
    if tuple(weight.shape) != (1, C, 3, 3):
        raise ValueError(f"weight must be [1,{C},3,3]")
    if tuple(dmap.shape) != (B, 1, H, W) or dmap.dtype != torch.float32:
        raise ValueError(f"dmap must be fp32 [{B},1,{H},{W}]")
    dmap = dmap.contiguous()
    w = weight.detach().contiguous()
    dx = torch.empty_like(x) if need_dx else None
    dw = torch.empty((1, C, 3, 3), dtype=torch.float32, device=x.device) if need_dw else None
    if dx is None and dw is None:
        return None, None
    if dx_split is not None and (dx is None or dx_split.dtype != torch.bfloat16 or not dx_split.is_contiguous()
                                 or tuple(dx_split.shape) != split_shape(B, C, H, W)):
        raise ValueError(f"dx_split must be a contiguous bf16 {split_shape(B, C, H, W)} tensor (with dx)")
    st = _native.load().mvbev_conv3x3_cout1_backward_ex(
        x.data_ptr(), w.data_ptr(), dmap.data_ptr(), B, C, H, W, int(dilation), int(bool(relu_mask)),
        None if dx is None else dx.data_ptr(), None if dx_split is None else dx_split.data_ptr(),
        None if dw is None else dw.data_ptr(), _stream(x))
    _native.check(st, "mvbev_conv3x3_cout1_backward_ex")
    return dx, dw


class BevFuse:
    """The one-call C ABI of the inference hot path (``mvbev_bev_plan_init`` /
    ``mvbev_bev_fuse_prepare`` / ``mvbev_bev_fuse``, include/mvbev.h): what a non-Python caller
    binds instead of orchestrating the entry points.  ``m_norms``: per view the
    host kornia src_norm <- dst_norm matrix; ``src_kind``: ``_native.BEV_SRC_*`` (fp32 kinds may carry
    ``_native.BEV_SRC_CHANNELS_LAST``: the views are passed channels_last; ``_native.BEV_NO_GUARD``: no
    non-finite guard, no guard regions in the workspace)."""

    def __init__(self, m_norms, C: int, src_hw, grid_hw, B: int = 1, src_kind: int = 0, backbone_hw=None):
        g = _native.BevGeometry()
        g.num_views = len(m_norms)
        g.src_kind = int(src_kind)
        g.B, g.C = int(B), int(C)
        g.H, g.W = (int(x) for x in src_hw)
        g.Ho, g.Wo = (int(x) for x in grid_hw)
        if backbone_hw is not None:
            g.h, g.w = (int(x) for x in backbone_hw)
        for v, m in enumerate(m_norms):
            g.m[v] = (ctypes.c_float * 9)(*torch.as_tensor(m, dtype=torch.float32).reshape(9).tolist())
        self.plan = _native.BevPlan()
        _native.check(_native.load().mvbev_bev_plan_init(ctypes.byref(g), ctypes.byref(self.plan)),
                      "mvbev_bev_plan_init")
        self.ws: Optional[torch.Tensor] = None
        self._keep = ()

    @property
    def wino(self) -> bool:
        return bool(self.plan.wino)

    @property
    def wino2(self) -> bool:
        """conv2 -> conv3 partials run row-Winograd (finite geometry; after prepare)."""
        return bool(self.plan.wino2)

    def _check_weights(self, w) -> None:
        g = self.plan.g
        want = [(512, g.num_views * g.C + 2, 3, 3), (512,), (512, 512, 3, 3), (512,), (1, 512, 3, 3)]
        names = ["map_classifier[0].weight", "map_classifier[0].bias", "map_classifier[2].weight",
                 "map_classifier[2].bias", "map_classifier[4].weight"]
        for t, shape, name in zip(w, want, names):
            if t is None and name.endswith("bias"):
                continue
            if not isinstance(t, torch.Tensor) or tuple(t.shape) != shape or t.dtype != torch.float32:
                got = (tuple(t.shape), t.dtype) if isinstance(t, torch.Tensor) else type(t)
                raise ValueError(f"{name} must be float32 {list(shape)}, got {got}")

    def prepare(self, map_classifier, device) -> None:
        """Once per weight version: ``map_classifier`` the reference's nn.Sequential (:51-54).  The
        C ABI cannot check raw pointers, so the weights' shapes and dtypes are checked here."""
        w = [map_classifier[0].weight, map_classifier[0].bias, map_classifier[2].weight, map_classifier[2].bias,
             map_classifier[4].weight]
        self._check_weights(w)
        n = int(self.plan.workspace_bytes)
        if self.ws is None or self.ws.numel() < n + 256:
            self.ws = torch.empty(n + 256, dtype=torch.uint8, device=device)
        base = self.ws.data_ptr()
        self._base = base + (-base) % 256  # the ABI wants a 256-B aligned workspace
        self._keep = tuple(None if t is None else t.detach().contiguous() for t in w)  # b2 / w3 read per frame
        _require_cuda(*[t for t in self._keep if t is not None])
        st = _native.load().mvbev_bev_fuse_prepare(ctypes.byref(self.plan),
                                                   *[None if t is None else t.data_ptr() for t in self._keep],
                                                   self._base, n, _stream(self.ws))
        _native.check(st, "mvbev_bev_fuse_prepare")
        self._device = self.ws.device

    def __call__(self, views, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One frame: ``views[v]`` per ``src_kind`` (fp32 / fp16 [B,C,H,W], or fp32 backbone maps
        [B,C,h,w]).  Every shape, dtype and device is checked here: the kernels behind the C ABI
        trust the plan's geometry, so a mismatched tensor would be read or written out of bounds."""
        g = self.plan.g
        if not self.plan.prepared:
            raise RuntimeError("BevFuse.prepare(map_classifier, device) must run before the first frame")
        if len(views) != g.num_views:
            raise ValueError(f"need {g.num_views} views")
        kind = g.src_kind & ~(_native.BEV_SRC_CHANNELS_LAST | _native.BEV_NO_GUARD)
        cl = bool(g.src_kind & _native.BEV_SRC_CHANNELS_LAST)
        backbone = kind == _native.BEV_SRC_BACKBONE_F32
        shape = (g.B, g.C, g.h, g.w) if backbone else (g.B, g.C, g.H, g.W)
        dtype = torch.float16 if kind == _native.BEV_SRC_F16 else torch.float32
        for i, v in enumerate(views):
            if not isinstance(v, torch.Tensor) or tuple(v.shape) != shape or v.dtype != dtype:
                got = (tuple(v.shape), v.dtype) if isinstance(v, torch.Tensor) else type(v)
                raise ValueError(f"view {i} must be {dtype} {list(shape)}, got {got}")
        # the plan's layout: NCHW, or (BEV_SRC_CHANNELS_LAST) the same tensors channels_last
        views = [v.contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format) for v in views]
        _require_cuda(*views)
        if any(v.device != self._device for v in views):
            raise ValueError(f"every view must be on {self._device} (the workspace's device)")
        if out is None:
            out = torch.empty((g.B, 1, g.Ho, g.Wo), dtype=torch.float32, device=views[0].device)
        elif (tuple(out.shape) != (g.B, 1, g.Ho, g.Wo) or out.dtype != torch.float32 or not out.is_contiguous()
              or not out.is_cuda or out.device != self._device):
            raise ValueError(f"out must be a contiguous float32 [{g.B}, 1, {g.Ho}, {g.Wo}] tensor on {self._device}")
        arr = (ctypes.c_void_p * g.num_views)(*[v.data_ptr() for v in views])
        st = _native.load().mvbev_bev_fuse(ctypes.byref(self.plan), arr, out.data_ptr(), self._base,
                                           int(self.plan.workspace_bytes), _stream(out))
        _native.check(st, "mvbev_bev_fuse")
        return out
