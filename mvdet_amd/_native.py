"""ctypes binding of libmvbev.so (the C ABI declared in ``include/mvbev.h``).

The product path has no CPU fallback: if the library is missing or a call
returns an error, this module raises.  Tensors cross the boundary as raw device
pointers, sizes and element strides; the stream is torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libmvbev.so"

# Every symbol include/mvbev.h declares (tests check the library exports them all).
EXPORTS = (
    "mvbev_status_string",
    "mvbev_version",
    "mvbev_warp_perspective_f32",
    "mvbev_warp_perspective_f16",
    "mvbev_warp_views_f32",
    "mvbev_warp_views_f16",
    "mvbev_warp_views_upsampled",
    "mvbev_fill_coord_map_f32",
    "mvbev_conv3x3_packed_floats",
    "mvbev_pack_conv3x3_weight_f32",
    "mvbev_conv3x3_f32",
    "mvbev_conv3x3_cout1_f32",
    "mvbev_conv3x3_packed_bytes_bf16x3",
    "mvbev_pack_conv3x3_weight_bf16x3",
    "mvbev_conv3x3_bf16x3_workspace_bytes",
    "mvbev_conv3x3_bf16x3_ex",
    "mvbev_warp_tile_mask",
    "mvbev_threshold_points",
    "mvbev_point_nms_workspace_bytes",
    "mvbev_point_nms_ws",
    "mvbev_warp_views_backward_f32",
    "mvbev_pack_conv3x3_dgrad_bf16x3",
    "mvbev_conv3x3_wgrad_workspace_bytes",
    "mvbev_conv3x3_bias_coord_grad_f32",
    "mvbev_relu_backward_f32",
    "mvbev_warp_adjoint_plan",
    "mvbev_warp_views_adjoint",
    "mvbev_conv3x3_bf16x3_tile_rows",
    "mvbev_warp_views_split_bf16_ex",
    "mvbev_warp_views_upsampled_ex",
    "mvbev_conv3x3_bf16x3_cout1_partials_bytes",
    "mvbev_conv3x3_bf16x3_cout1_partials",
    "mvbev_cout1_reduce_partials",
    "mvbev_conv3x3_dgrad_bf16x3_ex",
    "mvbev_relu_backward_split_f32",
    "mvbev_conv3x3_cout1_backward_ex",
    "mvbev_warp_upsampled_adjoint_plan",
    "mvbev_conv3x3_wgrad_bf16x3_ex2",
    "mvbev_split_rows_bf16",
    "mvbev_conv_schedule_slot_bytes",
    "mvbev_conv3x3_dgrad_bf16x3_sched",
    "mvbev_conv_ring_tile_space",
    "mvbev_conv3x3_bf16x3_ex3",
    "mvbev_conv3x3_packed_bytes_wino",
    "mvbev_pack_conv3x3_weight_wino",
    "mvbev_wino_rows_bytes",
    "mvbev_wino_rows_split_bf16",
    "mvbev_conv3x3_wino_bf16x3",
    "mvbev_wino_rows_split_bf16_dil",
    "mvbev_conv3x3_wino_bf16x3_dil",
    "mvbev_conv3x3_wino_bf16x3_cout1_partials",
    "mvbev_conv3x3_wino_bf16x3_dgrad",
    "mvbev_pack_conv3x3_weight_wino_dgrad",
    "mvbev_warp_views_wino_rows",
    "mvbev_warp_views_upsampled_wino_rows",
    "mvbev_warp_nonfinite_views",
    "mvbev_bev_plan_init",
    "mvbev_bev_fuse_workspace_bytes",
    "mvbev_bev_fuse_prepare",
    "mvbev_bev_fuse",
    "mvbev_warp_views_exact_f32",
    "mvbev_nchw_to_nhwc_f32",
    "mvbev_warp_views_split_bf16_rows",
    "mvbev_warp_views_exact_rows",
    "mvbev_conv3x3_f32_ex",
    "mvbev_bias_relu_nonfinite_f32",
    "mvbev_coord_term_f32",
    "mvbev_zero_gated",
    "mvbev_wino_dy_rows_bytes",
    "mvbev_wino_dy_rows_f32",
    "mvbev_conv3x3_wgrad_wino_workspace_bytes",
    "mvbev_conv3x3_wgrad_wino_bf16x3",
    "mvbev_store_gated_f32",
    "mvbev_pack_conv3x3_weight_f32_gated",
    "mvbev_wino_rows_split_bf16_gated",
    "mvbev_warp_wino_boxes_count",
    "mvbev_warp_wino_boxes",
    "mvbev_warp_views_wino_rows_ex",
    "mvbev_warp_upsampled_wino_boxes",
    "mvbev_warp_views_upsampled_wino_rows_ex",
    "mvbev_conv3x3_packed_bytes_wino43",
    "mvbev_pack_conv3x3_weight_wino43",
    "mvbev_wino43_rows_bytes",
    "mvbev_wino43_rows_split_bf16",
    "mvbev_conv3x3_wino43_bf16x3",
    "mvbev_conv3x3_wino43_bf16x3_cout1_partials",
)
BEV_SRC_F32, BEV_SRC_F16, BEV_SRC_BACKBONE_F32 = 0, 1, 2  # MVBEV_BEV_SRC_*
BEV_SRC_CHANNELS_LAST = 16  # MVBEV_BEV_SRC_CHANNELS_LAST (flag)
BEV_NO_GUARD = 32  # MVBEV_BEV_NO_GUARD (flag, ABI 11900)
WARP_DST_ZEROED = 1  # MVBEV_WARP_DST_ZEROED
WARP_SRC_F16 = 2  # MVBEV_WARP_SRC_F16 (mvbev_warp_views_wino_rows, ABI 11900)
WARP_WINO43 = 4  # MVBEV_WARP_WINO43 (the fused warps write the F(4,3) transform, ABI 12400)
TILES_GRID, TILES_EDGE_STRIP = 0, 1  # MVBEV_TILES_*
ERR_SHAPE = -2  # MVBEV_ERR_SHAPE
ERR_DILATION = -6  # MVBEV_ERR_DILATION

KC = 8    # MVBEV_CONV_KC
LAYOUT_F32, LAYOUT_F16, LAYOUT_SPLIT_BF16, LAYOUT_SPLIT_ROWS, LAYOUT_SPLIT_PIX = 0, 1, 2, 3, 4  # MVBEV_LAYOUT_*
BN = 128  # MVBEV_CONV_BN
TILE_H, TILE_W = 8, 32  # MVBEV_CONV_TILE_H / _W (fp32/fp16 input; split input: conv_tile_rows())

_i64 = ctypes.c_int64
_p = ctypes.c_void_p
_i64x4 = ctypes.c_int64 * 4

_lib = None


class ConvDesc(ctypes.Structure):
    """``mvbev_conv_desc`` (include/mvbev.h)."""
    _fields_ = [(n, ctypes.c_int64) for n in ("B", "K", "H", "W", "group", "group_stride", "batch_stride",
                                               "in_row0", "in_rows", "out_row0", "out_rows")]


class WarpView(ctypes.Structure):
    """``mvbev_warp_view`` (include/mvbev.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("src_strides", ctypes.c_int64 * 4), ("dst", ctypes.c_void_p),
                ("dst_strides", ctypes.c_int64 * 4), ("m", ctypes.c_float * 9)]


class WarpAdjointView(ctypes.Structure):
    """``mvbev_warp_adjoint_view`` (include/mvbev.h)."""
    _fields_ = [("grad_out", ctypes.c_void_p), ("grad_out_strides", ctypes.c_int64 * 4),
                ("grad_src", ctypes.c_void_p), ("grad_src_strides", ctypes.c_int64 * 4),
                ("row_ptr", ctypes.c_void_p), ("col", ctypes.c_void_p), ("val", ctypes.c_void_p)]


class ConvSchedule(ctypes.Structure):
    """``mvbev_conv_schedule`` (include/mvbev.h)."""
    _fields_ = [("items", ctypes.c_void_p), ("nitems", ctypes.c_int32), ("fixups", ctypes.c_void_p),
                ("nfix", ctypes.c_int32), ("nslots", ctypes.c_int32), ("partials", ctypes.c_void_p),
                ("partial_bytes", ctypes.c_size_t)]


class BevGeometry(ctypes.Structure):
    """``mvbev_bev_geometry`` (include/mvbev.h)."""
    _fields_ = [("num_views", ctypes.c_int32), ("src_kind", ctypes.c_int32)] + \
        [(n, ctypes.c_int64) for n in ("B", "C", "h", "w", "H", "W", "Ho", "Wo")] + \
        [("m", (ctypes.c_float * 9) * 16)]


class BevPlan(ctypes.Structure):
    """``mvbev_bev_plan`` (include/mvbev.h)."""
    _fields_ = [("g", BevGeometry), ("wino", ctypes.c_int32), ("frustum", ctypes.c_int32),
                ("prepared", ctypes.c_int32), ("wino2", ctypes.c_int32), ("guard", ctypes.c_int32),
                ("Cs", ctypes.c_int64), ("tiles", ctypes.c_int64), ("off", ctypes.c_size_t * 24),
                ("workspace_bytes", ctypes.c_size_t),
                ("b2", ctypes.c_void_p), ("w3", ctypes.c_void_p)]


class NativeError(RuntimeError):
    pass


def _declare(lib):
    lib.mvbev_status_string.restype = ctypes.c_char_p
    lib.mvbev_status_string.argtypes = [ctypes.c_int]
    lib.mvbev_version.restype = ctypes.c_int
    lib.mvbev_version.argtypes = []
    for name in ("mvbev_warp_perspective_f32", "mvbev_warp_perspective_f16"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [_p, _i64, _i64, _i64, _i64, _i64x4, _p, _p, _i64, _i64, _i64x4, _p]
    for name in ("mvbev_warp_views_f32", "mvbev_warp_views_f16"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _i64, _i64, _p]
    lib.mvbev_warp_views_upsampled.restype = ctypes.c_int
    lib.mvbev_warp_views_upsampled.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, ctypes.c_int, _i64, _i64,
                                               _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_int, _p]
    lib.mvbev_fill_coord_map_f32.restype = ctypes.c_int
    lib.mvbev_fill_coord_map_f32.argtypes = [_p, _i64, _i64, _i64, _i64x4, _p]
    lib.mvbev_conv3x3_packed_floats.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_packed_floats.argtypes = [_i64, _i64]
    lib.mvbev_pack_conv3x3_weight_f32.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_f32.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p]
    lib.mvbev_conv3x3_f32.restype = ctypes.c_int
    lib.mvbev_conv3x3_f32.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64, ctypes.c_int,
                                      ctypes.c_int, _p, _p, ctypes.c_int32, _p]
    lib.mvbev_conv3x3_packed_bytes_bf16x3.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_packed_bytes_bf16x3.argtypes = [_i64, _i64]
    lib.mvbev_pack_conv3x3_weight_bf16x3.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_bf16x3.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p]
    lib.mvbev_conv3x3_bf16x3_workspace_bytes.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_bf16x3_workspace_bytes.argtypes = [ctypes.POINTER(ConvDesc), _i64]
    lib.mvbev_conv3x3_bf16x3_ex.restype = ctypes.c_int
    lib.mvbev_conv3x3_bf16x3_ex.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64,
                                            ctypes.c_int, ctypes.c_int, _p, ctypes.c_int, _p, _p, _p,
                                            ctypes.c_size_t, _p]
    lib.mvbev_conv_ring_tile_space.restype = ctypes.c_int
    lib.mvbev_conv_ring_tile_space.argtypes = [ctypes.POINTER(ConvDesc), ctypes.c_int, ctypes.POINTER(_i64)]
    lib.mvbev_conv3x3_bf16x3_ex3.restype = ctypes.c_int
    lib.mvbev_conv3x3_bf16x3_ex3.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64,
                                             ctypes.c_int, ctypes.c_int, _p, ctypes.c_int, _p, _p, ctypes.c_int, _p]
    lib.mvbev_conv3x3_packed_bytes_wino.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_packed_bytes_wino.argtypes = [_i64, _i64]
    lib.mvbev_pack_conv3x3_weight_wino.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_wino.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p]
    lib.mvbev_wino_rows_bytes.restype = ctypes.c_size_t
    lib.mvbev_wino_rows_bytes.argtypes = [ctypes.POINTER(ConvDesc)]
    lib.mvbev_wino_rows_split_bf16.restype = ctypes.c_int
    lib.mvbev_wino_rows_split_bf16.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_conv3x3_wino_bf16x3.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino_bf16x3.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64, ctypes.c_int, _p,
                                              ctypes.c_int, _i64, _p, _p, _p]
    lib.mvbev_wino_rows_split_bf16_dil.restype = ctypes.c_int
    lib.mvbev_wino_rows_split_bf16_dil.argtypes = [_p, ctypes.POINTER(ConvDesc), ctypes.c_int, _p, _p, ctypes.c_size_t,
                                                   _p]
    lib.mvbev_conv3x3_wino_bf16x3_dil.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino_bf16x3_dil.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _i64, ctypes.c_int,
                                                  ctypes.c_int, _p, ctypes.c_int, _p]
    lib.mvbev_pack_conv3x3_weight_wino_dgrad.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_wino_dgrad.argtypes = [_p, _i64, _i64, _i64, _p, _p]
    lib.mvbev_conv3x3_wino_bf16x3_dgrad.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino_bf16x3_dgrad.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _i64, _p, ctypes.c_int, _p,
                                                    _i64, _p]
    lib.mvbev_conv3x3_wino_bf16x3_cout1_partials.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino_bf16x3_cout1_partials.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _i64, ctypes.c_int,
                                                             ctypes.c_int, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_conv3x3_packed_bytes_wino43.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_packed_bytes_wino43.argtypes = [_i64, _i64]
    lib.mvbev_pack_conv3x3_weight_wino43.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_wino43.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p]
    lib.mvbev_wino43_rows_bytes.restype = ctypes.c_size_t
    lib.mvbev_wino43_rows_bytes.argtypes = [ctypes.POINTER(ConvDesc)]
    lib.mvbev_wino43_rows_split_bf16.restype = ctypes.c_int
    lib.mvbev_wino43_rows_split_bf16.argtypes = [_p, ctypes.POINTER(ConvDesc), ctypes.c_int, _p, _p, ctypes.c_size_t,
                                                 _p]
    lib.mvbev_conv3x3_wino43_bf16x3.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino43_bf16x3.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64, ctypes.c_int,
                                                ctypes.c_int, _p, ctypes.c_int, _p, _p, _p]
    lib.mvbev_conv3x3_wino43_bf16x3_cout1_partials.restype = ctypes.c_int
    lib.mvbev_conv3x3_wino43_bf16x3_cout1_partials.argtypes = \
        lib.mvbev_conv3x3_wino_bf16x3_cout1_partials.argtypes
    lib.mvbev_warp_views_wino_rows.restype = ctypes.c_int
    lib.mvbev_warp_views_wino_rows.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _i64,
                                               _i64, _i64, ctypes.c_int, _p, ctypes.c_int32, _p]
    lib.mvbev_warp_views_wino_rows_ex.restype = ctypes.c_int
    lib.mvbev_warp_views_wino_rows_ex.argtypes = lib.mvbev_warp_views_wino_rows.argtypes[:-1] + [_p, _p]
    lib.mvbev_warp_wino_boxes_count.restype = _i64
    lib.mvbev_warp_wino_boxes_count.argtypes = [_i64, _i64]
    lib.mvbev_warp_wino_boxes.restype = ctypes.c_int
    lib.mvbev_warp_wino_boxes.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _i64, _p,
                                          _p]
    lib.mvbev_warp_views_upsampled_wino_rows.restype = ctypes.c_int
    lib.mvbev_warp_views_upsampled_wino_rows.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64,
                                                         _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_int, _p,
                                                         ctypes.c_int32, _p]
    lib.mvbev_warp_views_upsampled_wino_rows_ex.restype = ctypes.c_int
    lib.mvbev_warp_views_upsampled_wino_rows_ex.argtypes = lib.mvbev_warp_views_upsampled_wino_rows.argtypes[:-1] + [
        _p, _p]
    lib.mvbev_warp_upsampled_wino_boxes.restype = ctypes.c_int
    lib.mvbev_warp_upsampled_wino_boxes.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64,
                                                    _i64, _i64, _i64, _p, _p]
    lib.mvbev_warp_views_exact_f32.restype = ctypes.c_int
    lib.mvbev_warp_views_exact_f32.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _i64,
                                               _i64, _i64, _i64, _p, ctypes.c_int32, _p]
    lib.mvbev_warp_views_split_bf16_rows.restype = ctypes.c_int
    lib.mvbev_warp_views_split_bf16_rows.argtypes = [ctypes.POINTER(WarpView), _p, ctypes.c_int, ctypes.c_int, _i64,
                                                     _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_int, _p,
                                                     ctypes.c_int32, _p]
    lib.mvbev_warp_views_exact_rows.restype = ctypes.c_int
    lib.mvbev_warp_views_exact_rows.argtypes = [ctypes.POINTER(WarpView), _p, ctypes.c_int, ctypes.c_int, _i64, _i64,
                                                _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p, ctypes.c_int32, _p]
    lib.mvbev_conv3x3_f32_ex.restype = ctypes.c_int
    lib.mvbev_conv3x3_f32_ex.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _p, _i64, ctypes.c_int,
                                         ctypes.c_int, _p, _i64, _p, ctypes.c_int32, _p]
    lib.mvbev_coord_term_f32.restype = ctypes.c_int
    lib.mvbev_coord_term_f32.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _i64, _p, _p]
    lib.mvbev_bias_relu_nonfinite_f32.restype = ctypes.c_int
    lib.mvbev_bias_relu_nonfinite_f32.argtypes = [_p, _p, _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_int, _p,
                                                  ctypes.c_int32, _p]
    lib.mvbev_zero_gated.restype = ctypes.c_int
    lib.mvbev_zero_gated.argtypes = [_p, _i64, _p, ctypes.c_int32, _p]
    lib.mvbev_store_gated_f32.restype = ctypes.c_int
    lib.mvbev_store_gated_f32.argtypes = [_p, _i64x4, _p, _i64x4, _i64, _i64, _i64, _i64, ctypes.c_int, _p,
                                          ctypes.c_int32, _p]
    lib.mvbev_pack_conv3x3_weight_f32_gated.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_weight_f32_gated.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p, ctypes.c_int32, _p]
    lib.mvbev_wino_rows_split_bf16_gated.restype = ctypes.c_int
    lib.mvbev_wino_rows_split_bf16_gated.argtypes = [_p, ctypes.POINTER(ConvDesc), ctypes.c_int, _p, _p,
                                                     ctypes.c_size_t, _p, ctypes.c_int32, _p]
    lib.mvbev_nchw_to_nhwc_f32.restype = ctypes.c_int
    lib.mvbev_nchw_to_nhwc_f32.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _p]
    lib.mvbev_warp_tile_mask.restype = ctypes.c_int
    lib.mvbev_warp_tile_mask.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _i64,
                                         _i64, _i64, _i64, _i64, _p, _p]
    lib.mvbev_warp_nonfinite_views.restype = ctypes.c_int
    lib.mvbev_warp_nonfinite_views.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64, _p, _p]
    lib.mvbev_bev_plan_init.restype = ctypes.c_int
    lib.mvbev_bev_plan_init.argtypes = [ctypes.POINTER(BevGeometry), ctypes.POINTER(BevPlan)]
    lib.mvbev_bev_fuse_workspace_bytes.restype = ctypes.c_size_t
    lib.mvbev_bev_fuse_workspace_bytes.argtypes = [ctypes.POINTER(BevGeometry)]
    lib.mvbev_bev_fuse_prepare.restype = ctypes.c_int
    lib.mvbev_bev_fuse_prepare.argtypes = [ctypes.POINTER(BevPlan), _p, _p, _p, _p, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_bev_fuse.restype = ctypes.c_int
    lib.mvbev_bev_fuse.argtypes = [ctypes.POINTER(BevPlan), ctypes.POINTER(ctypes.c_void_p), _p, _p, ctypes.c_size_t,
                                   _p]
    lib.mvbev_threshold_points.restype = ctypes.c_int
    lib.mvbev_threshold_points.argtypes = [_p, _i64, _i64, ctypes.c_float, _p, _p, _p, _i64, _p]
    lib.mvbev_point_nms_workspace_bytes.restype = ctypes.c_size_t
    lib.mvbev_point_nms_workspace_bytes.argtypes = [_i64, _i64]
    lib.mvbev_point_nms_ws.restype = ctypes.c_int
    lib.mvbev_point_nms_ws.argtypes = [_p, _p, _i64, ctypes.c_float, _i64, _p, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_warp_views_backward_f32.restype = ctypes.c_int
    lib.mvbev_warp_views_backward_f32.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, _i64, _i64, _i64, _i64,
                                                  _i64, _i64, _p]
    lib.mvbev_pack_conv3x3_dgrad_bf16x3.restype = ctypes.c_int
    lib.mvbev_pack_conv3x3_dgrad_bf16x3.argtypes = [_p, _i64, _i64, _p, _i64, _p, _p]
    lib.mvbev_conv3x3_wgrad_workspace_bytes.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_wgrad_workspace_bytes.argtypes = [ctypes.POINTER(ConvDesc), _i64]
    lib.mvbev_conv3x3_bias_coord_grad_f32.restype = ctypes.c_int
    lib.mvbev_conv3x3_bias_coord_grad_f32.argtypes = [_p, _i64, _i64, _i64, _i64, ctypes.c_int, _p, _p, _i64,
                                                      _i64, _p]
    lib.mvbev_relu_backward_f32.restype = ctypes.c_int
    lib.mvbev_relu_backward_f32.argtypes = [_p, _p, _i64, _p]
    lib.mvbev_conv3x3_wgrad_bf16x3_ex2.restype = ctypes.c_int
    lib.mvbev_conv3x3_wgrad_bf16x3_ex2.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ConvDesc), _p, ctypes.c_int,
                                                   _i64, ctypes.c_int, _p, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_split_rows_bf16.restype = ctypes.c_int
    lib.mvbev_split_rows_bf16.argtypes = [_p, _i64, _i64, _p, _p]
    lib.mvbev_wino_dy_rows_bytes.restype = ctypes.c_size_t
    lib.mvbev_wino_dy_rows_bytes.argtypes = [_i64, _i64, _i64, _i64, ctypes.c_int]
    lib.mvbev_wino_dy_rows_f32.restype = ctypes.c_int
    lib.mvbev_wino_dy_rows_f32.argtypes = [_p, _i64, _i64, _i64, _i64, ctypes.c_int, _p, ctypes.c_size_t, _p]
    lib.mvbev_conv3x3_wgrad_wino_workspace_bytes.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_wgrad_wino_workspace_bytes.argtypes = [ctypes.POINTER(ConvDesc), _i64, ctypes.c_int]
    lib.mvbev_conv3x3_wgrad_wino_bf16x3.restype = ctypes.c_int
    lib.mvbev_conv3x3_wgrad_wino_bf16x3.argtypes = [_p, ctypes.c_size_t, ctypes.POINTER(ConvDesc), _p, ctypes.c_size_t,
                                                    _i64, ctypes.c_int, _p, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_conv_schedule_slot_bytes.restype = ctypes.c_size_t
    lib.mvbev_conv_schedule_slot_bytes.argtypes = []
    lib.mvbev_conv3x3_dgrad_bf16x3_sched.restype = ctypes.c_int
    lib.mvbev_conv3x3_dgrad_bf16x3_sched.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ConvDesc), _p, _i64,
                                                     ctypes.c_int, _p, ctypes.c_int, _p, _i64,
                                                     ctypes.POINTER(ConvSchedule), _p]
    lib.mvbev_warp_adjoint_plan.restype = ctypes.c_int
    lib.mvbev_warp_adjoint_plan.argtypes = [ctypes.POINTER(ctypes.c_float), _i64, _i64, _i64, _i64, _p, _p, _p, _p,
                                            _p]
    lib.mvbev_warp_upsampled_adjoint_plan.restype = ctypes.c_int
    lib.mvbev_warp_upsampled_adjoint_plan.argtypes = [ctypes.POINTER(ctypes.c_float), _i64, _i64, _i64, _i64, _i64,
                                                      _i64, _p, _p, _p, _p, _p]
    lib.mvbev_warp_views_adjoint.restype = ctypes.c_int
    lib.mvbev_warp_views_adjoint.argtypes = [ctypes.POINTER(WarpAdjointView), ctypes.c_int, ctypes.c_int, _i64,
                                             _i64, _i64, _i64, _i64, _i64, ctypes.c_int, _p]
    lib.mvbev_conv3x3_cout1_f32.restype = ctypes.c_int
    lib.mvbev_conv3x3_cout1_f32.argtypes = [_p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p,
                                            ctypes.c_int, _p, _p, ctypes.c_int32, _p]
    lib.mvbev_warp_views_split_bf16_ex.restype = ctypes.c_int
    lib.mvbev_warp_views_split_bf16_ex.argtypes = [ctypes.POINTER(WarpView), ctypes.c_int, ctypes.c_int, _i64, _i64,
                                                   _i64, _i64, _i64, _i64, ctypes.c_int, _p]
    lib.mvbev_warp_views_upsampled_ex.restype = ctypes.c_int
    lib.mvbev_warp_views_upsampled_ex.argtypes = (lib.mvbev_warp_views_upsampled.argtypes[:-1] +
                                                  [ctypes.c_int, _p])
    lib.mvbev_conv3x3_bf16x3_tile_rows.restype = ctypes.c_int
    lib.mvbev_conv3x3_bf16x3_tile_rows.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.mvbev_conv3x3_bf16x3_cout1_partials_bytes.restype = ctypes.c_size_t
    lib.mvbev_conv3x3_bf16x3_cout1_partials_bytes.argtypes = [ctypes.POINTER(ConvDesc), _i64]
    lib.mvbev_conv3x3_bf16x3_cout1_partials.restype = ctypes.c_int
    lib.mvbev_conv3x3_bf16x3_cout1_partials.argtypes = [_p, ctypes.POINTER(ConvDesc), _p, _p, _i64, ctypes.c_int,
                                                        ctypes.c_int, _p, _p, ctypes.c_size_t, _p]
    lib.mvbev_conv3x3_dgrad_bf16x3_ex.restype = ctypes.c_int
    lib.mvbev_conv3x3_dgrad_bf16x3_ex.argtypes = [_p, ctypes.c_int, ctypes.POINTER(ConvDesc), _p, _i64, ctypes.c_int,
                                                  _p, ctypes.c_int, _p, _i64, _p]
    lib.mvbev_conv3x3_cout1_backward_ex.restype = ctypes.c_int
    lib.mvbev_conv3x3_cout1_backward_ex.argtypes = [_p, _p, _p, _i64, _i64, _i64, _i64, ctypes.c_int, ctypes.c_int,
                                                    _p, _p, _p, _p]
    lib.mvbev_relu_backward_split_f32.restype = ctypes.c_int
    lib.mvbev_relu_backward_split_f32.argtypes = [_p, _p, _i64, _i64, _i64, _i64, _p, _p]
    lib.mvbev_cout1_reduce_partials.restype = ctypes.c_int
    lib.mvbev_cout1_reduce_partials.argtypes = [_p, ctypes.POINTER(ConvDesc), _i64, ctypes.c_int, _p, _i64, _i64, _p]


def load(path: os.PathLike | str | None = None):
    """Load (once) and return the library handle; raises if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # MVBEV_LIB overrides the library path (A/B runs of experimental builds)
    p = Path(path) if path else Path(os.environ.get("MVBEV_LIB", LIB_PATH))
    if not p.exists():
        raise NativeError(
            f"libmvbev.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C mvdet_amd/csrc` (there is no CPU fallback)")
    lib = ctypes.CDLL(str(p))
    _declare(lib)
    if path is None:
        _lib = lib
    return lib


def ring_tile_space(desc: ConvDesc, space: int):
    """``mvbev_conv_ring_tile_space``: (tiles_x, tiles_y, edge_tiles, edge width, edge rows) of
    the ring conv's pixel-tile space ``space`` for ``desc``, or None when it does not apply."""
    g = (_i64 * 5)()
    st = load().mvbev_conv_ring_tile_space(ctypes.byref(desc), int(space), g)
    return tuple(int(v) for v in g) if st == 0 else None


def conv_tile_rows(layout: int, dilation: int = 1) -> int:
    """Output rows per tile of the bf16x3 conv for this input layout (the granule of its
    frustum mask / tile order): 12 for split-bf16 input (LDS-DMA ring kernel), else TILE_H."""
    return int(load().mvbev_conv3x3_bf16x3_tile_rows(int(layout), int(dilation)))


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().mvbev_status_string(status).decode()
        raise NativeError(f"{what} failed: {msg} (status {status})")


def strides4(t) -> "ctypes.Array":
    s = t.stride()
    if len(s) != 4:
        raise ValueError(f"expected a 4-D tensor, got {len(s)}-D")
    return _i64x4(*s)


def stream_ptr(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
