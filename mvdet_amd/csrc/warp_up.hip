// Fused 3x bilinear upsample + homography warp for gfx950.
//
// The reference feeds the warp an upsampled copy of the backbone map:
//   img_feature = F.interpolate(feat, upsample_shape, mode='bilinear')   persp_trans_detector.py:65
//   world_feature = kornia...warp_perspective(img_feature, proj_mat, ...)                     :69
// (align_corners=False for the upsample, True for the warp's grid_sample).  Here the [B,C,H,W]
// upsampled tensor (265 MB per view at config 2) is never materialised: every bilinear corner
// of the warp is the upsample evaluated on the fly from the [B,C,h,w] map.
//
// Per output pixel (channel-independent, once): the warp's corner positions and weights in
// the upsampled grid exactly as warp_tile_kernel computes them; for each in-bounds corner
// (ux, uy) the upsample's source taps (PyTorch area_pixel_compute_source_index:
// s = max(0, (u + 0.5) * (in/out) - 0.5), i0 = floor(s), i1 = min(i0 + 1, in - 1),
// l1 = s - i0, l0 = 1 - l1).  Two adjacent upsampled rows (columns) reach at most three
// consecutive source rows (columns) when out >= in, so the whole sample is one 3x3 window of
// the source with 9 combined weights.  Per channel: 9 loads (L1/L2-resident: the source is
// 1/9 of the upsampled size) and 9 FMAs.
#include "warp_common.h"


namespace mvbev {

struct UpArgs {
  WarpArgs w;     // views, sizes of the UPSAMPLED image in w.H/w.W, grid, tiling
  int h, sw;      // source (backbone-resolution) height and width
  float sy, sx;   // upsample source scales in/out (h/H, w/W) as PyTorch computes them
  // (ABI 12200) warp_up_wino_cl_kernel: the per-(view, block tile) box of the blocks' 3x3 backbone windows,
  // int32 [nviews][tiles][4] {r0, r1, c0, c1 | nonfinite << 30} (r1 < 0: no sample inside), computed once per
  // geometry by mvbev_warp_upsampled_wino_boxes; NULL: each block reduces its own box
  const int32_t* boxes;
};

// a window row of 4 fp32 source pixels: 16 bytes, 4-byte aligned
typedef float f32x4u_t __attribute__((ext_vector_type(4), aligned(4)));

template <typename T, bool SPLIT, bool QUAD>
__global__ __launch_bounds__(kUpTH * kUpTW) void warp_up_kernel(const UpArgs ua) {
  const WarpArgs& a = ua.w;
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int tile = lb % a.tiles;
  const int chunk = (lb / a.tiles) % a.chunks;
  const int bv = lb / (a.tiles * a.chunks);
  const int view = bv % a.nviews;
  const int b = bv / a.nviews;
  const WarpView& vw = a.v[view];
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  constexpr int WC = 64 / kUpWR, WAVES_X = kUpTW / WC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = ty * kUpTH + (wave / WAVES_X) * kUpWR + lane / WC;
  const int u = tx * kUpTW + (wave % WAVES_X) * WC + lane % WC;
  if (v >= a.Ho || u >= a.Wo) return;
  const int c_begin = chunk * kUpCPB;
  const int c_end = min(a.C, c_begin + kUpCPB);
  const int H = a.H, W = a.W, h = ua.h, w = ua.sw;

  float m[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = vw.m[i];
  // the sample's 3x3 backbone window (warp corners in the upsampled grid by the same
  // warp_coord as warp_tile_kernel, each corner's upsample taps folded per axis)
  const UpWindow uw = up_window(m, u, v, a.Ho, a.Wo, H, W, h, w, ua.sy, ua.sx);
  const bool finite = uw.finite, inside = uw.inside;
  const float fill = finite ? 0.f : __builtin_nanf("");
  const int cb = uw.cb, rb = uw.rb;
  const float(&ax)[3] = uw.ax;
  const float(&ay)[3] = uw.ay;
  // one 16-B load per window row: shift the window left to fit 4 columns inside the row
  // (the shifted-in column gets weight 0); rows are clamped (their weights are 0 past h-1)
  const bool wide = QUAD && w >= 4;
  const int c4 = wide ? min(cb, w - 4) : cb;
  const int sh = cb - c4;  // 0 .. 2
  float bx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = j - sh;
    bx[j] = (k == 0 ? ax[0] : 0.f) + (k == 1 ? ax[1] : 0.f) + (k == 2 ? ax[2] : 0.f);
  }
  int col[3], row[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    col[j] = min(cb + j, w - 1);
    row[j] = min(rb + j, h - 1);
  }
  const int64_t sH = vw.sH, sW = vw.sW, sC = vw.sC;
  int64_t off[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) off[i][j] = row[i] * sH + (wide ? c4 + j : col[j]) * sW;
  const T* base = static_cast<const T*>(vw.src) + (int64_t)b * vw.sB;
  auto sample = [&](int c) __attribute__((always_inline)) {
    const T* pc = base + (int64_t)c * sC;
    float acc = 0.f;
    if (wide) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const f32x4u_t q = *reinterpret_cast<const f32x4u_t*>(pc + off[i][0]);
        acc += ay[i] * (bx[0] * q.x + bx[1] * q.y + bx[2] * q.z + bx[3] * q.w);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        float r = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) r += ax[j] * to_f32<T>(pc[off[i][j]]);
        acc += ay[i] * r;
      }
    }
    return acc;
  };

  if (a.skip_zero && !inside && finite) return;  // dst already zero there (MVBEV_WARP_DST_ZEROED)
  if constexpr (SPLIT) {
    u32x4_t* out = static_cast<u32x4_t*>(vw.dst) + 2 * ((int64_t)b * vw.dB + (int64_t)v * vw.dH + u);
    const int64_t dG = 2 * vw.dC;
    for (int g = c_begin / 8; g * 8 < c_end; ++g) {
      float vals[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = g * 8 + j;
        vals[j] = c < c_end ? (inside ? sample(c) : fill) : 0.f;
      }
      store_split8(out + g * dG, vals);
    }
  } else {
    T* out = static_cast<T*>(vw.dst) + (int64_t)b * vw.dB + (int64_t)v * vw.dH + u;
    const int64_t dC = vw.dC;
    for (int c = c_begin; c < c_end; c += 4) {
      float r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = (c + k < c_end) ? (inside ? sample(c + k) : fill) : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < c_end) out[(int64_t)(c + k) * dC] = from_f32<T>(r[k]);
    }
  }
}

// Fused 3x upsample + warp + row-Winograd transform (inference conv1 from backbone-resolution
// maps, the detector's path): phase 1 warps the block's 14 input rows as warp_up_kernel samples
// them (fp32 source, 16-B window rows), phase 2 is wino_rows_phase2 (warp_common.h).
// LDS staging (round 3): the TA/TD load path bound the first version (77-80 % busy at cfg2): every
// thread gathered its 3 window rows of 16 B per channel through L1, although a block's 14 x 16
// output pixels sample a source box of only ~85 backbone pixels (median at cfg2; <= 512 for 94 %
// of the work).  Now the block first reduces its pixels' windows to that box and, when the box
// holds at most kUpStage pixels, loads it once per channel with contiguous row loads into LDS;
// the windows are then read from LDS (the 3 columns of the window, ds reads).  Larger boxes (the
// near field) keep the direct 16-B window loads.  Same weights, same summation order per tap.
#ifndef MVBEV_UPW_STAGE
#define MVBEV_UPW_STAGE 384  // max staged box pixels per channel (8 channels x 384 x 4 B = 12 KiB); 0 = off
#endif
// (Pixel-major staging — a 3x3 window tap as two 16-B LDS reads for the 8 channels — measured 2.2x
// slower: 0.86 vs 0.39 ms at cfg2.)
constexpr int kUpStage = MVBEV_UPW_STAGE;

// Round 4 (the round-3 form was VALU / LDS-issue bound, 9 ds_read_b32 + 12 FMAs
// per channel and sample): the staged box is stored channel-pair interleaved, stage2[pair][row][col]
// = {channel 2p, channel 2p + 1}, so one ds_read_b64 serves two channels of a window tap and the
// separable 3x3 window is evaluated on f32x2 (v_pk_fma_f32): per sample 36 ds_read_b64 + 48 packed
// FMAs instead of 72 ds_read_b32 + 96 FMAs, the same fp32 operations per channel in the same order.
// cfg2: 0.39-0.42 ms vs 0.42-0.44 (profiles/r04a_kbench.jsonl).  (Several 8-channel groups per block,
// the sample geometry computed once for them, spilled and ran 0.64-0.85 ms: removed.)
constexpr int G = 1;
template <int FORM = 3>
__global__ __launch_bounds__(kWwThreads) MVBEV_WARP_OCC void warp_up_wino2_kernel(const UpArgs ua, int r3_rows,
                                                                                  int cgroups) {
  __shared__ __attribute__((aligned(16))) float ds[kWwRows][kWwCols][8];
  __shared__ unsigned char nz[kWwRows][kWwCols];
  __shared__ __attribute__((aligned(16))) f32x2_t stage2[4 * (kUpStage > 0 ? kUpStage : 1)];
  __shared__ int box[4];
  const WarpArgs& a = ua.w;
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int tile = lb % a.tiles;
  const int cg = (lb / a.tiles) % cgroups;
  const int bv = lb / (a.tiles * cgroups);
  const int view = bv % a.nviews;
  const int b = bv / a.nviews;
  const WarpView& vw = a.v[view];
  const int k = tile / a.tiles_x, tx = tile - k * a.tiles_x;
  const int H = a.H, W = a.W, h = ua.h, w = ua.sw;
  const int tid = threadIdx.x;
  const int i = tid / kWwCols, c = tid % kWwCols;
  const int v = 12 * k - 1 + i, u = tx * kWwCols + c;
  const bool live = i < kWwRows && v >= 0 && v < a.Ho && u < a.Wo;
  if (tid == 0) {
    box[0] = INT32_MAX;
    box[1] = -1;
    box[2] = INT32_MAX;
    box[3] = -1;
  }
  UpWindow uw;
  uw.inside = false;
  uw.finite = true;
  if (live) {
    float m[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
    uw = up_window(m, u, v, a.Ho, a.Wo, H, W, h, w, ua.sy, ua.sx);
  }
  __syncthreads();
  if (kUpStage > 0) {
    int r0 = uw.inside ? uw.rb : INT32_MAX, r1 = uw.inside ? min(uw.rb + 2, h - 1) : -1;
    int q0 = uw.inside ? uw.cb : INT32_MAX, q1 = uw.inside ? min(uw.cb + 2, w - 1) : -1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r0 = min(r0, __shfl_xor(r0, o));
      r1 = max(r1, __shfl_xor(r1, o));
      q0 = min(q0, __shfl_xor(q0, o));
      q1 = max(q1, __shfl_xor(q1, o));
    }
    if ((tid & 63) == 0 && r1 >= 0) {
      atomicMin(&box[0], r0);
      atomicMax(&box[1], r1);
      atomicMin(&box[2], q0);
      atomicMax(&box[3], q1);
    }
  }
  __syncthreads();
  const float* base = static_cast<const float*>(vw.src) + (int64_t)b * vw.sB;
  const bool quad_ok = (w & 3) == 0 && (vw.sH & 3) == 0 && (vw.sC & 3) == 0 &&
                       (reinterpret_cast<uintptr_t>(base) & 15) == 0;
  const StageBox sb = stage_box_shape(box, w, quad_ok);
  const int R = sb.R, Cb = sb.pitch, n = R * Cb;
  const bool staged = kUpStage > 0 && box[1] >= 0 && n <= kUpStage;  // uniform per block
  // the window's LDS base offset (staged): rows / columns clamped like the window's
  const int rb0 = uw.rb - box[0], cb0 = uw.cb - sb.c0;
  const bool any = live && (uw.inside || !uw.finite);
#pragma unroll 1
  for (int gi = 0; gi < G; ++gi) {
    const int chunk = cg * G + gi;
    const int c_begin = chunk * kUpCPB;
    if (c_begin >= a.C) break;  // uniform
    const int c_end = min(a.C, c_begin + kUpCPB);
    if (gi > 0) __syncthreads();  // the previous group's phase 2 is done with ds / stage2
    if (staged) {  // the box of the group's 8 channels, channel-pair interleaved
      if (sb.quad) {
        const int Q = sb.pitch >> 2, items = R * Q;
        for (int it = tid; it < items; it += kWwThreads) {
          const int r = it / Q, q = it - r * Q;
          const float* src = base + (int64_t)(sb.r0 + r) * vw.sH + sb.c0 + 4 * q;
          f32x4a_t t[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            t[j] = *reinterpret_cast<const f32x4a_t*>(src + (int64_t)min(c_begin + j, c_end - 1) * vw.sC);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            f32x4a_t* dst = reinterpret_cast<f32x4a_t*>(stage2 + p * n + r * Cb + 4 * q);
            dst[0] = f32x4a_t{t[2 * p][0], t[2 * p + 1][0], t[2 * p][1], t[2 * p + 1][1]};
            dst[1] = f32x4a_t{t[2 * p][2], t[2 * p + 1][2], t[2 * p][3], t[2 * p + 1][3]};
          }
        }
      } else {
        for (int r = tid / 32; r < R; r += kWwThreads / 32)
          for (int cc = tid % 32; cc < sb.pitch; cc += 32) {
            float t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
              t[j] = base[(int64_t)min(c_begin + j, c_end - 1) * vw.sC + (int64_t)(sb.r0 + r) * vw.sH + sb.c0 + cc];
#pragma unroll
            for (int p = 0; p < 4; ++p) stage2[p * n + r * Cb + cc] = f32x2_t{t[2 * p], t[2 * p + 1]};
          }
      }
      __syncthreads();
    }
    if (i < kWwRows) {
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = 0.f;
      if (live) {
        if (!uw.inside) {
          if (!uw.finite) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = c_begin + j < c_end ? __builtin_nanf("") : 0.f;
          }
        } else if (staged) {
          int idx[3][3];
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q)
              idx[r][q] = (min(uw.rb + r, h - 1) - uw.rb + rb0) * Cb + (min(uw.cb + q, w - 1) - uw.cb + cb0);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x2_t* sp = stage2 + p * n;
            f32x2_t acc = {0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              f32x2_t rr = {0.f, 0.f};
#pragma unroll
              for (int q = 0; q < 3; ++q) rr += uw.ax[q] * sp[idx[r][q]];
              acc += uw.ay[r] * rr;
            }
            d[2 * p] = c_begin + 2 * p < c_end ? acc.x : 0.f;
            d[2 * p + 1] = c_begin + 2 * p + 1 < c_end ? acc.y : 0.f;
          }
        } else {
          const int cb = uw.cb, rb = uw.rb;
          const int c4 = min(cb, w - 4), sh = cb - c4;
          float bx[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kk = j - sh;
            bx[j] = (kk == 0 ? uw.ax[0] : 0.f) + (kk == 1 ? uw.ax[1] : 0.f) + (kk == 2 ? uw.ax[2] : 0.f);
          }
          int64_t off[3];
#pragma unroll
          for (int r = 0; r < 3; ++r) off[r] = min(rb + r, h - 1) * vw.sH + c4;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int ch = min(c_begin + j, c_end - 1);
            const float* pc = base + (int64_t)ch * vw.sC;
            float acc = 0.f;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              const f32x4u_t q = *reinterpret_cast<const f32x4u_t*>(pc + off[r]);
              acc += uw.ay[r] * (bx[0] * q.x + bx[1] * q.y + bx[2] * q.z + bx[3] * q.w);
            }
            d[j] = c_begin + j < c_end ? acc : 0.f;
          }
        }
      }
      *reinterpret_cast<f32x4a_t*>(&ds[i][c][0]) = f32x4a_t{d[0], d[1], d[2], d[3]};
      *reinterpret_cast<f32x4a_t*>(&ds[i][c][4]) = f32x4a_t{d[4], d[5], d[6], d[7]};
      if (gi == 0) nz[i][c] = any;
    }
    __syncthreads();
    wino_rows_phase2<FORM>(ds, nz, vw, a, b, chunk, k, tx, r3_rows);
  }
}

// Fused 3x upsample + warp + B^T for channels-last backbone maps (round 4: sC == 1, the [B, C, h, w]
// tensor in channels_last memory format, or the NCHW map transposed once by mvbev_nchw_to_nhwc_f32).
// The NCHW form stages one 8-channel plane box per block and reads each window tap per channel pair
// from LDS (issue-bound: 37 % of wave cycles waiting on instructions, 0.38-0.41 ms at cfg2).  Here a
// staged box pixel is one 128-B line of 32 channels, so a lane's 16-B LDS read serves 4 channels of a
// tap, and the transform runs in registers:
//   phase 0: the block's 14 x 16 pixels' windows (up_window, once per pixel) -> LDS, the box reduced;
//   stage:   the box (<= kUcStage backbone pixels) with 16-B loads, 8 lanes per pixel line;
//   phase 1: thread = (column, channel quad) walks the 14 rows of its column: per row 9 ds_read_b128
//            taps, the separable window sum on f32x4 (same order per channel as the NCHW kernels);
//   phase 2: B^T of each 3-row tile's 5 rows from the thread's own registers, 8 B of hi and lo per
//            T row (no LDS round trip).
// A block whose box exceeds kUcStage (the near field) reads its taps straight from global memory.
#ifndef MVBEV_UPCL_STAGE
#define MVBEV_UPCL_STAGE 128
#endif
constexpr int kUcCh = 32, kUcThreads = 128, kUcStage = MVBEV_UPCL_STAGE, kWcPixUp = kWwRows * kWcCols;
static_assert(kWcCols * 8 == kUcThreads, "thread = (column, channel quad)");

template <int FORM = 3>
__global__ __launch_bounds__(kUcThreads) void warp_up_wino_cl_kernel(const UpArgs ua, int r3_rows) {
  __shared__ __attribute__((aligned(16))) f32x4a_t box_px[kUcStage * 8];  // [pixel][quad]
  __shared__ __attribute__((aligned(16))) f32x4a_t pax[kWcPixUp];  // ax0, ax1, ax2, ay0
  __shared__ __attribute__((aligned(8))) f32x2_t pay[kWcPixUp];     // ay1, ay2
  __shared__ int pint[kWcPixUp];  // rb << 16 | cb << 2 | class (0 zero, 1 inside, 2 NaN)
  __shared__ int box[4];
  const WarpArgs& a = ua.w;
  const WarpBlock wb = warp_block_index(a);
  const int tile = wb.tile, grp = wb.chunk, view = wb.view, b = wb.b, k = wb.k, tx = wb.tx;  // grp: 32-channel group
  const WarpView& vw = a.v[view];
  const int H = a.H, W = a.W, h = ua.h, w = ua.sw;
  const int tid = threadIdx.x;
  // (round 6) with the per-geometry table the 16 channel-group blocks of a (view, tile) take its box
  // instead of reducing it, and a block with no sample inside the source returns at once (before any barrier)
  int bxv[4];
  if (ua.boxes) {
    const int32_t* e = ua.boxes + 4 * ((int64_t)view * a.tiles + tile);
    bxv[0] = e[0];
    bxv[1] = e[1];
    bxv[2] = e[2];
    const int c1f = e[3];
    bxv[3] = c1f & 0x3FFFFFFF;
    if (a.skip_zero && bxv[1] < 0 && !(c1f >> 30)) return;
  } else if (tid == 0) {
    box[0] = INT32_MAX;
    box[1] = -1;
    box[2] = INT32_MAX;
    box[3] = -1;
  }
  if (!ua.boxes) __syncthreads();
  float m[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
  int r0 = INT32_MAX, r1 = -1, q0 = INT32_MAX, q1 = -1;
  for (int p = tid; p < kWcPixUp; p += kUcThreads) {  // phase 0
    const int i = p / kWcCols, c = p % kWcCols;
    const int v = 12 * k - 1 + i, u = tx * kWcCols + c;
    UpWindow uw;
    uw.inside = false;
    uw.finite = true;
    uw.rb = uw.cb = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) uw.ax[j] = uw.ay[j] = 0.f;
    if (v >= 0 && v < a.Ho && u < a.Wo) uw = up_window(m, u, v, a.Ho, a.Wo, H, W, h, w, ua.sy, ua.sx);
    const int cl = uw.inside ? 1 : (uw.finite ? 0 : 2);
    pax[p] = f32x4a_t{uw.ax[0], uw.ax[1], uw.ax[2], uw.ay[0]};
    pay[p] = f32x2_t{uw.ay[1], uw.ay[2]};
    pint[p] = (uw.rb << 16) | (uw.cb << 2) | cl;
    if (cl == 1) {
      r0 = min(r0, uw.rb);
      r1 = max(r1, min(uw.rb + 2, h - 1));
      q0 = min(q0, uw.cb);
      q1 = max(q1, min(uw.cb + 2, w - 1));
    }
  }
  if (!ua.boxes) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r0 = min(r0, __shfl_xor(r0, o));
      r1 = max(r1, __shfl_xor(r1, o));
      q0 = min(q0, __shfl_xor(q0, o));
      q1 = max(q1, __shfl_xor(q1, o));
    }
    if ((tid & 63) == 0 && r1 >= 0) {
      atomicMin(&box[0], r0);
      atomicMax(&box[1], r1);
      atomicMin(&box[2], q0);
      atomicMax(&box[3], q1);
    }
  }
  __syncthreads();  // (the windows in LDS; and the reduced box)
  if (!ua.boxes) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bxv[q] = box[q];
  }
  const int br0 = bxv[0], bc0 = bxv[2];
  const int R = bxv[1] - br0 + 1, Cb = bxv[3] - bc0 + 1;  // (an all-outside block: R, Cb <= 0)
  const bool staged = bxv[1] >= 0 && R * Cb <= kUcStage;  // uniform per block
  // the batch item's 32-channel group (16-B aligned: host check)
  const float* gbase = static_cast<const float*>(vw.src) + (int64_t)b * vw.sB + (int64_t)grp * kUcCh;
  if (staged) {
    for (int it = tid; it < R * Cb * 8; it += kUcThreads) {
      const int px = it >> 3, q = it & 7;
      const int r = px / Cb, c = px - r * Cb;
      box_px[it] = *reinterpret_cast<const f32x4a_t*>(gbase + (int64_t)(br0 + r) * vw.sH + (int64_t)(bc0 + c) * vw.sW + 4 * q);
    }
    __syncthreads();
  }
  const int c = tid >> 3, q = tid & 7;  // column, channel quad
  const int u = tx * kWcCols + c;
  f32x4a_t d[kWwRows];
  bool nzr[kWwRows];
#pragma unroll
  for (int i = 0; i < kWwRows; ++i) {  // phase 1
    const int p = i * kWcCols + c;
    const int pk = pint[p], cls = pk & 3, prb = pk >> 16, pcb = (pk >> 2) & 0x3fff;
    const f32x4a_t ax = pax[p];
    const f32x2_t ay12 = pay[p];
    const f32x4a_t ay = {ax.w, ay12.x, ay12.y, 0.f};
    f32x4a_t acc = {0.f, 0.f, 0.f, 0.f};
    if (cls == 1) {
      int ro[3], co[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        ro[j] = min(prb + j, h - 1);
        co[j] = min(pcb + j, w - 1);
      }
      f32x4a_t s[3][3];
      if (staged) {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int j = 0; j < 3; ++j) s[r][j] = box_px[((ro[r] - br0) * Cb + (co[j] - bc0)) * 8 + q];
      } else {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            s[r][j] = *reinterpret_cast<const f32x4a_t*>(gbase + (int64_t)ro[r] * vw.sH + (int64_t)co[j] * vw.sW + 4 * q);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        f32x4a_t rr = {0.f, 0.f, 0.f, 0.f};
        rr += ax.x * s[r][0];
        rr += ax.y * s[r][1];
        rr += ax.z * s[r][2];
        acc += (r == 0 ? ay.x : r == 1 ? ay.y : ay.z) * rr;
      }
    } else if (cls == 2) {
      acc = f32x4a_t{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    }
    d[i] = acc;
    nzr[i] = cls != 0;
  }
  if (u >= a.Wo) return;
  const int chunk = grp * (kUcCh / 8) + (q >> 1), half = q & 1;
  // phase 2: tile qt = rows FORM qt .. FORM qt + FORM + 1 (FORM 4: 3 four-row tiles, T43 rows 6 r4 + xi)
  constexpr int NT = FORM == 3 ? 4 : 3, NX = FORM + 2;
#pragma unroll
  for (int qt = 0; qt < NT; ++qt) {
    const int r3 = NT * k + qt, i0 = FORM * qt;
    if (r3 >= r3_rows) break;
    int any = 0;
#pragma unroll
    for (int m = 0; m < NX; ++m) any |= nzr[i0 + m];
    if (a.skip_zero && !any) continue;
    f32x4a_t dd[NX], t[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) dd[m] = d[i0 + m];
    wino_bt<FORM>(dd, t);
    if (a.nonfinite) {  // as wino_rows_phase2
      const f32x4a_t sum = wino_bt_sum<FORM>(t);
      if (!isfinite((sum.x + sum.y) + (sum.z + sum.w))) *a.nonfinite = a.nf_tag;
    }
    unsigned* out = reinterpret_cast<unsigned*>(static_cast<u32x4_t*>(vw.dst) +
                                                (2 * ((int64_t)b * vw.dB + (int64_t)chunk * vw.dC +
                                                      (int64_t)(NX * r3) * vw.dH) + u)) + 2 * half;
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      const float h0 = (float)(__bf16)t[xi].x, h1 = (float)(__bf16)t[xi].y;
      const float h2 = (float)(__bf16)t[xi].z, h3 = (float)(__bf16)t[xi].w;
      unsigned* o = out + (int64_t)xi * vw.dH * 8;
      *reinterpret_cast<u32x2_t*>(o) = u32x2_t{pack_bf16x2(h0, h1), pack_bf16x2(h2, h3)};
      *reinterpret_cast<u32x2_t*>(o + vw.dH * 4) =
          u32x2_t{pack_bf16x2(t[xi].x - h0, t[xi].y - h1), pack_bf16x2(t[xi].z - h2, t[xi].w - h3)};
    }
  }
}

// The per-(view, tile) backbone-window boxes of warp_up_wino_cl_kernel (ABI 12200), once per geometry: the
// same pixels and up_window as its phase 0, {r0, r1, c0, c1 | nonfinite << 30} (r1 = -1: no sample inside).
__global__ __launch_bounds__(kUcThreads) void up_box_kernel(const UpArgs ua, int32_t* __restrict__ boxes) {
  __shared__ int box[5];
  const WarpArgs& a = ua.w;
  const int tile = blockIdx.x % a.tiles, view = blockIdx.x / a.tiles;
  const WarpView& vw = a.v[view];
  const int k = tile / a.tiles_x, tx = tile - k * a.tiles_x;
  const int h = ua.h, w = ua.sw;
  const int tid = threadIdx.x;
  if (tid == 0) {
    box[0] = INT32_MAX;
    box[1] = -1;
    box[2] = INT32_MAX;
    box[3] = -1;
    box[4] = 0;
  }
  __syncthreads();
  float m[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
  for (int p = tid; p < kWcPixUp; p += kUcThreads) {
    const int i = p / kWcCols, c = p % kWcCols;
    const int v = 12 * k - 1 + i, u = tx * kWcCols + c;
    if (v < 0 || v >= a.Ho || u >= a.Wo) continue;
    const UpWindow uw = up_window(m, u, v, a.Ho, a.Wo, a.H, a.W, h, w, ua.sy, ua.sx);
    if (uw.inside) {
      atomicMin(&box[0], uw.rb);
      atomicMax(&box[1], min(uw.rb + 2, h - 1));
      atomicMin(&box[2], uw.cb);
      atomicMax(&box[3], min(uw.cb + 2, w - 1));
    } else if (!uw.finite) {
      atomicOr(&box[4], 1);
    }
  }
  __syncthreads();
  if (tid == 0) {
    const int empty = box[1] < 0;
    const int4 out = make_int4(empty ? 0 : box[0], box[1], empty ? 0 : box[2], (empty ? 0 : box[3]) | (box[4] << 30));
    *reinterpret_cast<int4*>(boxes + 4 * ((int64_t)view * a.tiles + tile)) = out;
  }
}

// The exact-order warp (a5) and upsample + warp (a4 + a5): the non-finite guard's path
// (mvbev_warp_views_exact_f32).  Per output pixel the kornia coordinates (warp_coord), then, per
// in-bounds corner, the source value — with UP, PyTorch's bilinear upsample of that upsampled pixel
// evaluated as the reference's CPU F.interpolate does (two taps per axis, both multiplied even at
// weight 0: t = (x00 l0x + x01 l1x) l0y + (x10 l0x + x11 l1x) l1y) — times its grid_sample weight,
// out-of-bounds corners selected to 0 (never multiplied).  So every product the reference forms is
// formed here, and a NaN / inf in the features reaches exactly the outputs it reaches in
// persp_trans_detector.py:65-69 (the fused kernels fold the taps into one 3x3 window and cannot).
// Plain fp32 out [B][C][Ho][Wo] at element strides; one thread per output pixel, 8 channels per
// block; runs only when *gate == gate_tag (the fused warp's report), else exits at once.  Row windows
// (ABI 11900): dst row v is grid row vw.row0 + v, a.out_rows rows (0 = Ho) — the exact path runs in row
// bands (bounded memory) and the band exchange's windows.  T: fp32 or fp16 sources (fp32 math).
template <bool UP, typename T>
__global__ __launch_bounds__(256) void warp_exact_kernel(const UpArgs ua, int pix_blocks, int units) {
  const WarpArgs& a = ua.w;
  if (a.gate && *a.gate != a.gate_tag) return;  // the usual case: a few thousand workgroups exit here
  const int orows = a.out_rows ? a.out_rows : a.Ho;
  // grid-stride over units = (b * nviews + view, 256-pixel block): one thread per output pixel, all
  // channels (the taps computed once per pixel)
  for (int unit = blockIdx.x; unit < units; unit += gridDim.x) {
    const int bv = unit / pix_blocks, p = (unit - bv * pix_blocks) * 256 + threadIdx.x;
    if (p >= orows * a.Wo) continue;
    const int view = bv % a.nviews, b = bv / a.nviews;
    const WarpView& vw = a.v[view];
    const int v = p / a.Wo, u = p - v * a.Wo;
    float m[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) m[i] = vw.m[i];
    const WarpCoord wc = warp_coord(m, u, v + vw.row0, a.Ho, a.Wo, a.H, a.W);
    float* out = static_cast<float*>(vw.dst) + (int64_t)b * vw.dB + (int64_t)v * vw.dH + u;
    if (!wc.inside) {
      const float fill = wc.finite ? 0.f : __builtin_nanf("");
      for (int c = 0; c < a.C; ++c) out[(int64_t)c * vw.dC] = fill;
      continue;
    }
    const float ix = wc.ix, iy = wc.iy;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
    const float wt[4] = {(fx1 - ix) * (fy1 - iy), (ix - fx0) * (fy1 - iy), (fx1 - ix) * (iy - fy0),
                         (ix - fx0) * (iy - fy0)};  // nw, ne, sw, se (GridSampler.h)
    const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= a.W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= a.H - 1;
    const bool ok[4] = {vx0 && vy0, vx1 && vy0, vx0 && vy1, vx1 && vy1};
    // per corner: the source offsets (UP: its 2 x 2 upsample taps) and their weights
    int64_t off[4][4];
    float lx[4][2], ly[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cx = min(max(x0 + (k & 1), 0), a.W - 1), cy = min(max(y0 + (k >> 1), 0), a.H - 1);
      if constexpr (UP) {
        const UpTaps tx = up_taps(cx, ua.sx, ua.sw), ty = up_taps(cy, ua.sy, ua.h);
        off[k][0] = ty.i0 * vw.sH + tx.i0 * vw.sW;
        off[k][1] = ty.i0 * vw.sH + tx.i1 * vw.sW;
        off[k][2] = ty.i1 * vw.sH + tx.i0 * vw.sW;
        off[k][3] = ty.i1 * vw.sH + tx.i1 * vw.sW;
        lx[k][0] = tx.l0, lx[k][1] = tx.l1, ly[k][0] = ty.l0, ly[k][1] = ty.l1;
      } else {
        off[k][0] = off[k][1] = off[k][2] = off[k][3] = cy * vw.sH + cx * vw.sW;
        lx[k][0] = lx[k][1] = ly[k][0] = ly[k][1] = 0.f;
      }
    }
    const T* base = static_cast<const T*>(vw.src) + (int64_t)b * vw.sB;
    for (int c = 0; c < a.C; ++c) {
      const T* pc = base + (int64_t)c * vw.sC;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float val;
        if constexpr (UP) {
          val = (to_f32<T>(pc[off[k][0]]) * lx[k][0] + to_f32<T>(pc[off[k][1]]) * lx[k][1]) * ly[k][0] +
                (to_f32<T>(pc[off[k][2]]) * lx[k][0] + to_f32<T>(pc[off[k][3]]) * lx[k][1]) * ly[k][1];
        } else {
          val = to_f32<T>(pc[off[k][0]]);
        }
        acc += (ok[k] ? val : 0.f) * wt[k];
      }
      out[(int64_t)c * vw.dC] = acc;
    }
  }
}

}  // namespace mvbev

static int warp_exact(const mvbev_warp_view* views, const int32_t* row0s, int nviews, int src_is_f16, int64_t B,
                      int64_t C, int64_t h, int64_t w, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t out_rows,
                      const int32_t* gate, int32_t gate_tag, void* stream) {
  using namespace mvbev;
  if (!views) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || nviews <= 0 || out_rows < 0)
    return MVBEV_ERR_RANK;
  const int64_t orows = out_rows ? out_rows : Ho;
  if (nviews > kWarpMaxViews || B * nviews > 65535 || C > INT32_MAX || H > INT32_MAX / 2 || W > INT32_MAX / 2 ||
      Ho > INT32_MAX / 2 || orows > Ho || orows * Wo > INT32_MAX - 256 ||
      ceil_div(orows * Wo, 256) * B * nviews > INT32_MAX || H < h || W < w)
    return MVBEV_ERR_SHAPE;
  UpArgs ua = {};
  WarpArgs& a = ua.w;
  for (int i = 0; i < nviews; ++i) {
    const mvbev_warp_view& s = views[i];
    if (!s.src || !s.dst) return MVBEV_ERR_NULL;
    if (s.dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
    WarpView& d = a.v[i];
    d.src = s.src; d.sB = s.src_strides[0]; d.sC = s.src_strides[1];
    d.sH = s.src_strides[2]; d.sW = s.src_strides[3];
    d.dst = s.dst; d.dB = s.dst_strides[0]; d.dC = s.dst_strides[1]; d.dH = s.dst_strides[2];
    d.m_dev = nullptr;
    for (int k = 0; k < 9; ++k) d.m[k] = s.m[k];
    d.row0 = row0s ? row0s[i] : 0;
    if (d.row0 < 0 || d.row0 + orows > Ho) return MVBEV_ERR_SHAPE;
  }
  a.nviews = nviews;
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.out_rows = (int)out_rows;
  a.gate = gate;
  a.gate_tag = gate_tag;
  ua.h = (int)h; ua.sw = (int)w;
  ua.sy = (float)h / (float)H;
  ua.sx = (float)w / (float)W;
  const int pix_blocks = (int)ceil_div(orows * Wo, 256), units = pix_blocks * (int)(B * nviews);
  const dim3 grid((unsigned)std::min(units, 2048));
  const bool up = !(h == H && w == W);
#define MVBEV_EXACT_LAUNCH(UP, T) \
  hipLaunchKernelGGL((warp_exact_kernel<UP, T>), grid, dim3(256), 0, as_stream(stream), ua, pix_blocks, units)
  if (src_is_f16) {
    if (up) MVBEV_EXACT_LAUNCH(true, __half); else MVBEV_EXACT_LAUNCH(false, __half);
  } else {
    if (up) MVBEV_EXACT_LAUNCH(true, float); else MVBEV_EXACT_LAUNCH(false, float);
  }
#undef MVBEV_EXACT_LAUNCH
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

extern "C" int mvbev_warp_views_exact_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t h,
                                          int64_t w, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                          const int32_t* gate, int32_t gate_tag, void* stream) {
  return warp_exact(views, nullptr, nviews, 0, B, C, h, w, H, W, Ho, Wo, 0, gate, gate_tag, stream);
}

extern "C" int mvbev_warp_views_exact_rows(const mvbev_warp_view* views, const int32_t* row0s, int nviews,
                                           int src_is_f16, int64_t B, int64_t C, int64_t h, int64_t w, int64_t H,
                                           int64_t W, int64_t Ho, int64_t Wo, int64_t out_rows,
                                           const int32_t* gate, int32_t gate_tag, void* stream) {
  if (!row0s) return MVBEV_ERR_NULL;
  if (out_rows <= 0) return MVBEV_ERR_RANK;
  return warp_exact(views, row0s, nviews, src_is_f16, B, C, h, w, H, W, Ho, Wo, out_rows, gate, gate_tag, stream);
}

extern "C" int mvbev_warp_views_upsampled_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B,
                                                       int64_t C, int64_t h, int64_t w, int64_t H, int64_t W,
                                                       int64_t Ho, int64_t Wo, int64_t r3_rows, int flags,
                                                       int32_t* nonfinite, int32_t nf_tag, const int32_t* boxes,
                                                       void* stream);

extern "C" int mvbev_warp_views_upsampled_wino_rows(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                                                    int64_t h, int64_t w, int64_t H, int64_t W, int64_t Ho,
                                                    int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                                                    int32_t nf_tag, void* stream) {
  return mvbev_warp_views_upsampled_wino_rows_ex(views, nviews, B, C, h, w, H, W, Ho, Wo, r3_rows, flags, nonfinite,
                                                 nf_tag, nullptr, stream);
}

extern "C" int mvbev_warp_upsampled_wino_boxes(const mvbev_warp_view* views, int nviews, int64_t h, int64_t w,
                                               int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows,
                                               int32_t* boxes, void* stream) {
  using namespace mvbev;
  if (!views || !boxes) return MVBEV_ERR_NULL;
  if (nviews <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || r3_rows <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || 3 * r3_rows < Ho || H < h || W < w || h >= 32768 || w >= 16384) return MVBEV_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(boxes) & 15) return MVBEV_ERR_ALIGN;
  UpArgs ua = {};
  WarpArgs& a = ua.w;
  for (int i = 0; i < nviews; ++i)
    for (int q = 0; q < 9; ++q) a.v[i].m[q] = views[i].m[q];
  a.nviews = nviews;
  a.H = (int)H, a.W = (int)W, a.Ho = (int)Ho, a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kWcCols);
  a.tiles = a.tiles_x * (int)ceil_div(r3_rows, 4);
  ua.h = (int)h, ua.sw = (int)w;
  ua.sy = (float)h / (float)H;
  ua.sx = (float)w / (float)W;
  hipLaunchKernelGGL(up_box_kernel, dim3((unsigned)(a.tiles * nviews)), dim3(kUcThreads), 0, as_stream(stream), ua,
                     boxes);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

extern "C" int mvbev_warp_views_upsampled_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B,
                                                       int64_t C, int64_t h, int64_t w, int64_t H, int64_t W,
                                                       int64_t Ho, int64_t Wo, int64_t r3_rows, int flags,
                                                       int32_t* nonfinite, int32_t nf_tag, const int32_t* boxes,
                                                       void* stream) {
  using namespace mvbev;
  if (flags & ~(MVBEV_WARP_DST_ZEROED | MVBEV_WARP_WINO43)) return MVBEV_ERR_SHAPE;
  const bool w43 = (flags & MVBEV_WARP_WINO43) != 0;  // T43: r3_rows counts four-row tiles, 3 per block
  const int form = w43 ? 4 : 3, tpb = w43 ? 3 : 4;
  if (!views) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || nviews <= 0 || r3_rows <= 0)
    return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || B * nviews > 65535 || C > INT32_MAX || H > INT32_MAX / 2 || W > INT32_MAX / 2 ||
      Ho > INT32_MAX / 2 || Wo > INT32_MAX / 2 || H < h || W < w || w < 4 || form * r3_rows < Ho ||
      ceil_div(r3_rows, tpb) * ceil_div(Wo, kWwCols) * ceil_div(C, kUpCPB) * B * nviews > INT32_MAX)
    return MVBEV_ERR_SHAPE;
  UpArgs ua = {};
  WarpArgs& a = ua.w;
  for (int i = 0; i < nviews; ++i) {
    const mvbev_warp_view& s = views[i];
    if (!s.src || !s.dst) return MVBEV_ERR_NULL;
    if (s.dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
    WarpView& d = a.v[i];
    d.src = s.src; d.sB = s.src_strides[0]; d.sC = s.src_strides[1];
    d.sH = s.src_strides[2]; d.sW = s.src_strides[3];
    d.dst = s.dst; d.dB = s.dst_strides[0]; d.dC = s.dst_strides[1]; d.dH = s.dst_strides[2];
    d.m_dev = nullptr;
    for (int k = 0; k < 9; ++k) d.m[k] = s.m[k];
  }
  a.nviews = nviews;
  a.skip_zero = (flags & MVBEV_WARP_DST_ZEROED) != 0;
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kWwCols);
  a.tiles = a.tiles_x * (int)ceil_div(r3_rows, tpb);
  a.chunks = (int)ceil_div(C, kUpCPB);
  a.nwg = a.tiles * a.chunks * a.B * a.nviews;
  a.nonfinite = nonfinite;
  a.nf_tag = nf_tag;
  ua.h = (int)h; ua.sw = (int)w;
  ua.sy = (float)h / (float)H;
  ua.sx = (float)w / (float)W;
  // channels-last maps (every view: unit channel stride, 16-B aligned whole 32-channel groups) take the
  // line-per-pixel kernel; NCHW maps need unit column stride (16-B window rows)
  bool cl = C % kUcCh == 0 && h < 32768 && w < 16384;  // (the packed window origin of the kernel)
  for (int i = 0; i < nviews; ++i) {
    const WarpView& d = a.v[i];
    cl = cl && d.sC == 1 && d.sW >= C && d.sH >= d.sW * w && d.sB >= 0 && d.sW % 4 == 0 && d.sH % 4 == 0 &&
         d.sB % 4 == 0 && (reinterpret_cast<uintptr_t>(d.src) & 15) == 0;
  }
  if (cl) {
    a.tiles_x = (int)ceil_div(Wo, kWcCols);
    a.tiles = a.tiles_x * (int)ceil_div(r3_rows, tpb);
    a.chunks = (int)(C / kUcCh);
    a.nwg = a.tiles * a.chunks * a.B * a.nviews;
    set_fastdiv(a);
    ua.boxes = boxes;
    if (w43)
      hipLaunchKernelGGL((warp_up_wino_cl_kernel<4>), dim3((unsigned)a.nwg), dim3(kUcThreads), 0, as_stream(stream),
                         ua, (int)r3_rows);
    else
      hipLaunchKernelGGL((warp_up_wino_cl_kernel<3>), dim3((unsigned)a.nwg), dim3(kUcThreads), 0, as_stream(stream),
                         ua, (int)r3_rows);
    MVBEV_CHECK_LAUNCH();
    return MVBEV_OK;
  }
  for (int i = 0; i < nviews; ++i)
    if (a.v[i].sW != 1) return MVBEV_ERR_STRIDE;  // 16-B window rows
  if (w43)
    hipLaunchKernelGGL((warp_up_wino2_kernel<4>), dim3((unsigned)a.nwg), dim3(kWwThreads), 0, as_stream(stream), ua,
                       (int)r3_rows, a.chunks);
  else
    hipLaunchKernelGGL((warp_up_wino2_kernel<3>), dim3((unsigned)a.nwg), dim3(kWwThreads), 0, as_stream(stream), ua,
                       (int)r3_rows, a.chunks);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

extern "C" int mvbev_warp_views_upsampled_ex(const mvbev_warp_view* views, int nviews, int src_is_f16,
                                             int64_t B, int64_t C, int64_t h, int64_t w, int64_t H,
                                             int64_t W, int64_t Ho, int64_t Wo, int out_layout, int flags,
                                             void* stream) {
  using namespace mvbev;
  if (flags & ~MVBEV_WARP_DST_ZEROED) return MVBEV_ERR_SHAPE;
  if (!views) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 ||
      nviews <= 0)
    return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || B * nviews > 65535 || C > INT32_MAX || H > INT32_MAX / 2 ||
      W > INT32_MAX / 2 || Ho > INT32_MAX / 2 || Wo > INT32_MAX / 2 || H < h || W < w ||
      ceil_div(Ho, kUpTH) * ceil_div(Wo, kUpTW) * ceil_div(C, kUpCPB) * B * nviews > INT32_MAX)
    return MVBEV_ERR_SHAPE;  // upsampling only (H >= h, W >= w): the 3x3 window bound
  if (out_layout != MVBEV_LAYOUT_F32 && out_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;
  if (out_layout == MVBEV_LAYOUT_F32 && src_is_f16) return MVBEV_ERR_SHAPE;
  UpArgs ua = {};
  WarpArgs& a = ua.w;
  for (int i = 0; i < nviews; ++i) {
    const mvbev_warp_view& s = views[i];
    if (!s.src || !s.dst) return MVBEV_ERR_NULL;
    if (s.dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
    if (s.dst_strides[2] != Wo) return MVBEV_ERR_STRIDE;  // a T row = its hi plane [Wo] then its lo plane
    WarpView& d = a.v[i];
    d.src = s.src; d.sB = s.src_strides[0]; d.sC = s.src_strides[1];
    d.sH = s.src_strides[2]; d.sW = s.src_strides[3];
    d.dst = s.dst; d.dB = s.dst_strides[0]; d.dC = s.dst_strides[1]; d.dH = s.dst_strides[2];
    d.m_dev = nullptr;
    for (int k = 0; k < 9; ++k) d.m[k] = s.m[k];
  }
  a.nviews = nviews;
  a.skip_zero = (flags & MVBEV_WARP_DST_ZEROED) != 0;
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kUpTW);
  a.tiles = a.tiles_x * (int)ceil_div(Ho, kUpTH);
  a.chunks = (int)ceil_div(C, kUpCPB);
  a.nwg = a.tiles * a.chunks * a.B * a.nviews;
  ua.h = (int)h; ua.sw = (int)w;
  ua.sy = (float)h / (float)H;  // area_pixel_compute_scale(align_corners=false, no scale)
  ua.sx = (float)w / (float)W;
  hipStream_t st = as_stream(stream);
  // fp32 rows with unit column stride: 16-B row loads (QUAD); otherwise 9 scalar loads
  bool quad = !src_is_f16;
  for (int i = 0; i < nviews; ++i) quad = quad && views[i].src_strides[3] == 1;
  if (out_layout == MVBEV_LAYOUT_SPLIT_BF16) {
    if (src_is_f16)
      hipLaunchKernelGGL((warp_up_kernel<__half, true, false>), dim3((unsigned)a.nwg), dim3(kUpTH * kUpTW), 0, st, ua);
    else if (quad)
      hipLaunchKernelGGL((warp_up_kernel<float, true, true>), dim3((unsigned)a.nwg), dim3(kUpTH * kUpTW), 0, st, ua);
    else
      hipLaunchKernelGGL((warp_up_kernel<float, true, false>), dim3((unsigned)a.nwg), dim3(kUpTH * kUpTW), 0, st, ua);
  } else if (quad) {
    hipLaunchKernelGGL((warp_up_kernel<float, false, true>), dim3((unsigned)a.nwg), dim3(kUpTH * kUpTW), 0, st, ua);
  } else {
    hipLaunchKernelGGL((warp_up_kernel<float, false, false>), dim3((unsigned)a.nwg), dim3(kUpTH * kUpTW), 0, st, ua);
  }
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

extern "C" int mvbev_warp_views_upsampled(const mvbev_warp_view* views, int nviews, int src_is_f16,
                                          int64_t B, int64_t C, int64_t h, int64_t w, int64_t H,
                                          int64_t W, int64_t Ho, int64_t Wo, int out_layout,
                                          void* stream) {
  return mvbev_warp_views_upsampled_ex(views, nviews, src_is_f16, B, C, h, w, H, W, Ho, Wo, out_layout, 0,
                                       stream);
}

// NCHW -> NHWC (channels-last) copy of the views' backbone maps, one launch for every view: the input
// of warp_up_wino_cl_kernel for producers that emit NCHW (the maps are 1/9 of the upsampled size:
// 0.13 GB read + written at cfg2).  Block = (view, batch item, 32 channels, 64 pixels) through an LDS
// tile (pitch 65: conflict-free column reads); reads 256-B channel rows, writes 128-B pixel lines.
namespace mvbev {
struct TransArgs {
  const float* src[kWarpMaxViews];
  int64_t sB[kWarpMaxViews], sC[kWarpMaxViews], sH[kWarpMaxViews], sW[kWarpMaxViews];
  float* dst[kWarpMaxViews];
  int B, C, H, W, ctiles, ptiles;
};
// VEC (every view: contiguous planes, sC / sB / H * W multiples of 4, 16-B aligned, C % 32 == 0):
// 16-B loads of 4 pixels of a channel and 16-B stores of 4 channels of a pixel
template <bool VEC>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const TransArgs a) {
  __shared__ float t[32][65];
  const int HW = a.H * a.W;
  int blk = blockIdx.x;
  const int pt = blk % a.ptiles;
  blk /= a.ptiles;
  const int ct = blk % a.ctiles;
  blk /= a.ctiles;
  const int b = blk % a.B, v = blk / a.B;
  const int tid = threadIdx.x;
  const float* src = a.src[v] + (int64_t)b * a.sB[v];
  float* dst = a.dst[v] + (int64_t)b * HW * a.C;
  if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // thread = (channel, pixel quad)
      const int cc = (tid >> 4) + 16 * k, pq = tid & 15, p = pt * 64 + 4 * pq;
      if (p < HW) {
        const f32x4a_t q = *reinterpret_cast<const f32x4a_t*>(src + (int64_t)(ct * 32 + cc) * a.sC[v] + p);
        t[cc][4 * pq] = q.x;
        t[cc][4 * pq + 1] = q.y;
        t[cc][4 * pq + 2] = q.z;
        t[cc][4 * pq + 3] = q.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // thread = (pixel, channel quad)
      const int pp = (tid >> 3) + 32 * k, cq = tid & 7, p = pt * 64 + pp;
      if (p < HW)
        *reinterpret_cast<f32x4a_t*>(dst + (int64_t)p * a.C + ct * 32 + 4 * cq) =
            f32x4a_t{t[4 * cq][pp], t[4 * cq + 1][pp], t[4 * cq + 2][pp], t[4 * cq + 3][pp]};
    }
    return;
  }
  for (int cc = tid >> 6; cc < 32; cc += 4) {
    const int c = ct * 32 + cc, p = pt * 64 + (tid & 63);
    if (c < a.C && p < HW) {
      const int y = p / a.W, x = p - y * a.W;
      t[cc][tid & 63] = src[(int64_t)c * a.sC[v] + (int64_t)y * a.sH[v] + (int64_t)x * a.sW[v]];
    }
  }
  __syncthreads();
  for (int pp = tid >> 5; pp < 64; pp += 8) {
    const int p = pt * 64 + pp, c = ct * 32 + (tid & 31);
    if (p < HW && c < a.C) dst[(int64_t)p * a.C + c] = t[tid & 31][pp];
  }
}
}  // namespace mvbev

extern "C" int mvbev_nchw_to_nhwc_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                                      int64_t W, void* stream) {
  using namespace mvbev;
  if (!views) return MVBEV_ERR_NULL;
  if (nviews <= 0 || B <= 0 || C <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || C > INT32_MAX || H * W > INT32_MAX - 64) return MVBEV_ERR_SHAPE;
  TransArgs a = {};
  for (int i = 0; i < nviews; ++i) {
    if (!views[i].src || !views[i].dst) return MVBEV_ERR_NULL;
    a.src[i] = static_cast<const float*>(views[i].src);
    a.sB[i] = views[i].src_strides[0];
    a.sC[i] = views[i].src_strides[1];
    a.sH[i] = views[i].src_strides[2];
    a.sW[i] = views[i].src_strides[3];
    a.dst[i] = static_cast<float*>(views[i].dst);
  }
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W;
  a.ctiles = (int)ceil_div(C, 32);
  a.ptiles = (int)ceil_div(H * W, 64);
  const int64_t nwg = (int64_t)a.ptiles * a.ctiles * B * nviews;
  if (nwg > INT32_MAX) return MVBEV_ERR_SHAPE;
  bool vec = C % 32 == 0 && (H * W) % 4 == 0 && (reinterpret_cast<uintptr_t>(views[0].dst) & 15) == 0;
  for (int i = 0; i < nviews; ++i)
    vec = vec && a.sW[i] == 1 && a.sH[i] == W && a.sC[i] % 4 == 0 && a.sB[i] % 4 == 0 &&
          (reinterpret_cast<uintptr_t>(a.src[i]) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.dst[i]) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<true>, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<false>, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}
