// Definitions shared by the warp kernels (warp.hip, warp_up.hip); gfx950 only.
#pragma once

#include <type_traits>

#include "common.h"

namespace mvbev {

// Gather warp (warp_tile_kernel) tiling.  A/B on cfg2 (7 views, 1 launch, split-bf16 out):
// 64 ch/block with 4x16 waves 0.51 ms; 32 ch 0.47; 16 ch 0.44; 8 ch 0.416; 8 ch with 8x8
// waves 0.391 (square wave footprints; a block's few planes keep the XCD's L2 working set
// small, so neighbouring tiles still find their shared source lines there).  Block tile
// (round 2, same box, 8 ch, 8x8 waves): 32x32 0.492 ms, 16x32 0.452, 16x16 0.350-0.366,
// 8x16 0.358, 8x8 0.360, 16x8 0.356 (two waves stacked vertically)
#ifndef MVBEV_WARP_TH
#define MVBEV_WARP_TH 16
#define MVBEV_WARP_TW 8
#define MVBEV_WARP_WR 8
#endif
#ifndef MVBEV_WARP_CPB
#define MVBEV_WARP_CPB 8
#endif
#ifndef MVBEV_WARP_GU
#define MVBEV_WARP_GU 1  // 8-channel groups sampled before their stores are issued
#endif
constexpr int kWarpTH = MVBEV_WARP_TH;    // output rows per block
constexpr int kWarpTW = MVBEV_WARP_TW;    // output cols per block
constexpr int kWarpWR = MVBEV_WARP_WR;    // output rows per wave (wave tile WR x 64/WR)
constexpr int kWarpCPB = MVBEV_WARP_CPB;  // channels per block
// fused upsample+warp (warp_up_kernel): cfg2 +a4 A/B 64 ch/block, 4x16 waves 0.478 ms;
// 32 ch 0.476; 16 ch 8x8 waves 0.476; 8 ch 8x8 waves 0.372; block tile (round 2, same box):
// 16x16 0.338, 16x8 0.335, 8x8 (one wave) 0.330
#ifndef MVBEV_WARPUP_TH
#define MVBEV_WARPUP_TH 8
#define MVBEV_WARPUP_TW 8
#define MVBEV_WARPUP_WR 8
#endif
#ifndef MVBEV_WARPUP_CPB
#define MVBEV_WARPUP_CPB 8
#endif
constexpr int kUpTH = MVBEV_WARPUP_TH;
constexpr int kUpTW = MVBEV_WARPUP_TW;
constexpr int kUpWR = MVBEV_WARPUP_WR;
constexpr int kUpCPB = MVBEV_WARPUP_CPB;
constexpr int kWarpMaxViews = 16;

struct WarpView {
  const void* src;
  int64_t sB, sC, sH, sW;
  void* dst;
  int64_t dB, dC, dH;
  const float* m_dev;  // device [B][9] (per batch item) or nullptr -> m below
  float m[9];          // src_norm <- dst_norm, shared by every batch item
  int row0;            // grid row of dst row 0 (a row window of the grid: warp_tile_kernel, the exact warp)
};

// n / d for 0 <= n < 2^31 as (umulhi(n, m) + n) >> s (round 6: the fused warps' block decomposition took four
// runtime divisions, ~100 scalar instructions of the ~295 each wave issued at cfg3); m == 0: not set (plain division)
struct FastDiv {
  uint32_t m, s;
};
inline FastDiv make_fastdiv(int d) {  // host, d >= 1
  uint32_t s = 0;
  while ((1ull << s) < (unsigned long long)d) ++s;
  return FastDiv{(uint32_t)(((1ull << 32) * ((1ull << s) - (unsigned long long)d)) / (unsigned long long)d + 1), s};
}
__device__ inline int fdiv(int n, int d, FastDiv f) {
  return f.m ? (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s) : n / d;
}

struct WarpArgs {
  WarpView v[kWarpMaxViews];
  int nviews, B, C, H, W, Ho, Wo, tiles_x, tiles, chunks, nwg;
  bool pair;  // fp32 rows with unit column stride and W >= 2: corner pairs as 8-B loads
  bool skip_zero;  // MVBEV_WARP_DST_ZEROED: outside samples (exact zeros) are not written
  // non-finite guard (ABI 11600): the fused warps store nf_tag into *nonfinite when a sample they
  // produce is non-finite (a NaN / inf in the features it reads); the exact warp runs only when
  // *gate == gate_tag (NULL: always)
  int32_t* nonfinite;
  int32_t nf_tag;
  const int32_t* gate;
  int32_t gate_tag;
  // rows of each dst (a row window of the Ho-row grid starting at its view's row0; 0 = Ho):
  // warp_tile_kernel and the exact warp (ABI 11900)
  int out_rows;
  // (ABI 12200) warp_wino_kernel: the per-(view, block tile) source box of the block's bilinear corners,
  // int32 [nviews][tiles][4] {r0, r1, c0, c1 | nonfinite << 30} (r1 < 0: no sample inside the source),
  // computed once per geometry by mvbev_warp_wino_boxes; NULL: each block reduces its own box
  const int32_t* boxes;
  // (round 6) fast divisors of tiles, chunks, nviews and tiles_x for warp_block_index (set_fastdiv; zero: unset)
  FastDiv fd_tiles, fd_chunks, fd_nviews, fd_tiles_x;
};

inline void set_fastdiv(WarpArgs& a) {  // host, after the tiling fields are final
  a.fd_tiles = make_fastdiv(a.tiles);
  a.fd_chunks = make_fastdiv(a.chunks);
  a.fd_nviews = make_fastdiv(a.nviews);
  a.fd_tiles_x = make_fastdiv(a.tiles_x);
}

// a fused-warp block's coordinates: lb = xcd_remap(block) = ((b * nviews + view) * chunks + chunk) * tiles + tile,
// tile = k * tiles_x + tx
struct WarpBlock {
  int tile, chunk, view, b, k, tx;
};
__device__ inline WarpBlock warp_block_index(const WarpArgs& a) {
  WarpBlock r;
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int q1 = fdiv(lb, a.tiles, a.fd_tiles);
  r.tile = lb - q1 * a.tiles;
  const int q2 = fdiv(q1, a.chunks, a.fd_chunks);
  r.chunk = q1 - q2 * a.chunks;
  r.b = fdiv(q2, a.nviews, a.fd_nviews);
  r.view = q2 - r.b * a.nviews;
  r.k = fdiv(r.tile, a.tiles_x, a.fd_tiles_x);
  r.tx = r.tile - r.k * a.tiles_x;
  return r;
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
// a horizontally adjacent corner pair (nw,ne) / (sw,se) of an fp32 row: 8 bytes, 4-byte aligned
typedef float f32x2u_t __attribute__((ext_vector_type(2), aligned(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// SPLIT output: the "split-bf16 blocked" layout consumed by the 3xbf16 conv (see
// mvbev.h MVBEV_LAYOUT_SPLIT_BF16): per (batch, group of 8 channels, row, col) 32 bytes =
// bf16 hi[8] then bf16 lo[8] with x = hi + lo (+ ~2^-17 relative); dst strides in 32-B units.
__device__ inline void store_split8(u32x4_t* dst, const float (&v)[8]) {
  bf16x8_t hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)v[j];
    hi[j] = h;
    lo[j] = (__bf16)(v[j] - (float)h);
  }
  dst[0] = __builtin_bit_cast(u32x4_t, hi);  // (non-temporal stores measured no faster)
  dst[1] = __builtin_bit_cast(u32x4_t, lo);
}

// kornia 0.6.11 warp coordinates of output pixel (u, v): create_meshgrid(normalized) ->
// transform_points ([gx gy 1] @ M^T, convert_points_from_homogeneous eps=1e-8) ->
// grid_sampler_unnormalize(align_corners=True).  One definition for every warp kernel and
// the conv tile mask, so "this output pixel is exactly zero" is decided by the same fp32 ops
// that produce the pixel.
struct WarpCoord {
  float ix, iy;
  bool finite, inside;  // !finite -> NaN output; finite && !inside -> exactly 0 (zero padding)
};
__device__ inline WarpCoord warp_coord(const float (&m)[9], int u, int v, int Ho, int Wo, int H, int W) {
  // no fma contraction: every kernel (and the tile mask) must get the same ix / iy bit for bit — an
  // ulp of ix (~3e-5 at a few hundred pixels) moves the bilinear weights by as much, and fma
  // contraction is a per-call-site compiler choice
#pragma clang fp contract(off)
  const float gx = ((float)u / (float)(Wo - 1) - 0.5f) * 2.0f;
  const float gy = ((float)v / (float)(Ho - 1) - 0.5f) * 2.0f;
  float x = gx * m[0] + gy * m[1] + m[2];
  float y = gx * m[3] + gy * m[4] + m[5];
  const float z = gx * m[6] + gy * m[7] + m[8];
  const float scale = fabsf(z) > 1e-8f ? 1.0f / (z + 1e-8f) : 1.0f;
  x = scale * x;
  y = scale * y;
  WarpCoord c;
  c.ix = ((x + 1.f) / 2.f) * (float)(W - 1);
  c.iy = ((y + 1.f) / 2.f) * (float)(H - 1);
  c.finite = isfinite(c.ix) && isfinite(c.iy);
  c.inside = c.finite && c.ix > -1.f && c.ix < (float)W && c.iy > -1.f && c.iy < (float)H;
  return c;
}

// PyTorch's bilinear upsample taps of upsampled index X along an axis of n backbone pixels
// (align_corners=False, scale = n / N): s = max(0, (X + 0.5) * scale - 0.5), i0 = min(floor(s),
// n - 1), i1 = i0 + (i0 < n - 1), weights l0 = 1 - (s - i0) on i0 and l1 = s - i0 on i1.
struct UpTaps {
  int i0, i1;
  float l0, l1;
};
__device__ inline UpTaps up_taps(int X, float scale, int n) {
  // no fma contraction: PyTorch's CPU upsample rounds the product before the subtraction, so an
  // upsampled index 3k + 1 lands exactly on source pixel k (l1 = 0, a zero-weight tap that turns
  // an inf source value into NaN, as the reference does)
#pragma clang fp contract(off)
  UpTaps t;
  float s = scale * ((float)X + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  t.i0 = min((int)s, n - 1);
  t.i1 = t.i0 + (t.i0 < n - 1 ? 1 : 0);
  t.l1 = s - (float)t.i0;
  t.l0 = 1.f - t.l1;
  return t;
}

// The fused 3x-upsample + warp sample of output pixel (u, v) as one 3x3 window of the
// backbone-resolution map (warp_up_kernel, and the plan of its adjoint): the warp's corners in
// the upsampled H x W grid (warp_coord), each corner's PyTorch bilinear upsample taps
// (align_corners=False: s = max(0, (i + 0.5) * scale - 0.5), i0 = floor(s), i1 = min(i0 + 1,
// n - 1)), summed per axis into 3 window weights (the 2-D corner weights factor, so the 3x3
// weights are the outer product ay[i] * ax[j] at backbone pixel (rb + i, cb + j); a window
// row / column past the map carries weight 0).
struct UpWindow {
  int rb, cb;
  float ay[3], ax[3];
  bool finite, inside;
};
__device__ inline UpWindow up_window(const float (&m)[9], int u, int v, int Ho, int Wo, int H, int W, int h, int w,
                                     float sy, float sx) {
#pragma clang fp contract(off)  // (as warp_coord: the same window weights in every kernel)
  UpWindow r;
  const WarpCoord wc = warp_coord(m, u, v, Ho, Wo, H, W);
  const float ix = wc.ix, iy = wc.iy;
  r.finite = wc.finite;
  r.inside = wc.inside;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = r.inside ? (int)fx0 : 0, y0 = r.inside ? (int)fy0 : 0;
  const float wx[2] = {fx0 + 1.f - ix, ix - fx0};  // warp weights of columns x0, x0+1
  const float wy[2] = {fy0 + 1.f - iy, iy - fy0};  // ... of rows y0, y0+1
  int cxi[2][2], cyi[2][2];
  float lxv[2][2], lyv[2][2];
  bool okx[2], oky[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ux = x0 + k, uy = y0 + k;
    okx[k] = r.inside && ux >= 0 && ux <= W - 1;
    oky[k] = r.inside && uy >= 0 && uy <= H - 1;
    const UpTaps tx = up_taps(ux, sx, w), ty = up_taps(uy, sy, h);
    cxi[k][0] = tx.i0;
    cxi[k][1] = tx.i1;
    lxv[k][0] = tx.l0;
    lxv[k][1] = tx.l1;
    cyi[k][0] = ty.i0;
    cyi[k][1] = ty.i1;
    lyv[k][0] = ty.l0;
    lyv[k][1] = ty.l1;
  }
  r.cb = okx[0] ? cxi[0][0] : cxi[1][0];
  r.rb = oky[0] ? cyi[0][0] : cyi[1][0];
#pragma unroll
  for (int j = 0; j < 3; ++j) r.ax[j] = 0.f, r.ay[j] = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        r.ax[j] += (okx[k] && cxi[k][t] - r.cb == j) ? wx[k] * lxv[k][t] : 0.f;
        r.ay[j] += (oky[k] && cyi[k][t] - r.rb == j) ? wy[k] * lyv[k][t] : 0.f;
      }
    }
  return r;
}

// Warp + row-Winograd transform kernels (warp_wino_kernel, warp_up_wino_kernel): a block warps
// the kWwRows input rows 12 k - 1 + i of 4 three-row output tiles x kWwCols columns of one
// view's 8-channel group into LDS (ds[row][col][channel], nz = some sample non-zero), then this
// phase stores the transformed rows B^T d (points 0, 1, -1, 2, inf; the rows of wino_rows_kernel
// in conv_bf16x3.hip) split-bf16 at T rows 5 r3 + xi (vw.dst strides in 32-B units: dB per item,
// dC per 8-channel group, dH per T row).  One thread per (tile, column, channel pair) computes
// all 5 rows of its 2 channels (the 5 input rows read once, no per-row branching) and writes
// its 4 bytes of each row's hi[8] and lo[8] (the 4 threads of a column fill the 32-B entry; a
// wave covers 16 consecutive columns: 512 contiguous bytes per row).  skip_zero: a (tile,
// column) whose 5 samples are all outside the source is not written (T zero-filled, written only
// by this geometry).
#ifndef MVBEV_WW_COLS
#define MVBEV_WW_COLS 16  // columns per fused-warp block (threads = 16 x columns; cfg2: 8 0.52-0.56 ms, 16 0.51)
#endif
constexpr int kWwRows = 14, kWwCols = MVBEV_WW_COLS, kWwThreads = 16 * kWwCols;
// the channels-last fused warps' block: 14 rows x 16 columns, 256 (plain) / 128 (upsample) threads
constexpr int kWcCols = 16, kWcThreads = 256;
// (several 8-channel groups per block, the sample geometry computed once for all of them, measured
// no faster at cfg2: 1 group 0.463 / 0.521 ms up / plain, 2 groups 0.462 / 0.538, 4 0.466 / 0.544 —
// the geometry's VALU work is not what binds these kernels; the TA/TD load path is: 77-84 % busy)
static_assert(kWarpCPB == 8 && kUpCPB == 8, "one 8-channel group per warp block");
static_assert(4 * kWwCols * 4 == kWwThreads, "phase 2: one (tile, column, channel pair) per thread");
// 8 waves per SIMD asked of the compiler (VGPRs capped at 64: 72 -> 64 measured -4 % on both fused warps)
#define MVBEV_WARP_OCC __attribute__((amdgpu_waves_per_eu(8, 8)))
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ inline unsigned pack_bf16x2(float x, float y) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)x) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)y) << 16);
}

typedef float f32x4a_t __attribute__((ext_vector_type(4)));  // 16-B aligned

// The staging box of a fused-warp block: source rows [r0, r0 + R) x columns [c0, c0 + pitch)
// of its 8 channels (fp32, unit column stride), staged as stage[j][r][col - c0].  With quad
// (uniform: the row / channel pitches, the source base and W multiples of 4 floats, 16-B
// aligned) the box is widened to whole aligned 16-B quads — one 16-B load per (row, quad,
// channel) and a 16-B LDS store, a quarter of the load instructions of one float per lane
// (the load path, TA/TD, binds these kernels); else one float per lane, 32 lanes a row.
struct StageBox {
  int r0, R, c0, pitch;  // pitch = staged columns per row
  bool quad;
};
__device__ inline StageBox stage_box_shape(const int (&box)[4], int W, bool quad_ok) {
  StageBox sb;
  sb.r0 = box[0];
  sb.R = box[1] - box[0] + 1;
  sb.quad = quad_ok;
  sb.c0 = quad_ok ? (box[2] & ~3) : box[2];
  const int c1 = quad_ok ? min((box[3] | 3) + 1, W) : box[3] + 1;  // W % 4 == 0 when quad_ok
  sb.pitch = c1 - sb.c0;
  return sb;
}
// channel-pair staging (round 6): stage2[p][r][col] = {channel 2p, channel 2p + 1} (fp32 pairs; T = float or
// __half sources; quad: 16-B fp32 / 8-B fp16 loads of 4 columns where the source's strides and alignment allow,
// interleaved by pair into two 16-B LDS stores) — a warped sample then reads each corner of two channels with
// one ds_read_b64 (16 per pixel and 8-channel group instead of 32 ds_read_b32)
template <int NT, typename T = float>
__device__ inline void stage_box_load(const T* __restrict__ base, int64_t sC, int64_t sH, int c_begin, int c_end,
                                      const StageBox& sb, f32x2_t* __restrict__ stage2, int tid) {
  const int n = sb.R * sb.pitch;
  // the 8 channels' planes: pointers stepped by sC from channel c_begin (a short last group repeats its last
  // channel) — the 64-bit min / multiply per channel this replaces was ~160 scalar instructions per wave
  // (32-bit offsets from one pointer instead: 1-2 % slower at cfg2 / cfg4 / cfg5, 2 % faster at cfg3)
  const T* pl[8];
  pl[0] = base + (int64_t)c_begin * sC;
#pragma unroll
  for (int j = 1; j < 8; ++j) pl[j] = c_begin + j < c_end ? pl[j - 1] + sC : pl[j - 1];
  if (sb.quad) {
    const int Q = sb.pitch >> 2, items = sb.R * Q;
    for (int it = tid; it < items; it += NT) {
      const int r = it / Q, q = it - r * Q;
      const int64_t o = (int64_t)(sb.r0 + r) * sH + sb.c0 + 4 * q;
      f32x4a_t t[8];
      if constexpr (std::is_same<T, float>::value) {
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = *reinterpret_cast<const f32x4a_t*>(pl[j] + o);
      } else {  // 4 halves (8 B) per lane and channel
        uint2 u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = *reinterpret_cast<const uint2*>(pl[j] + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const T* h = reinterpret_cast<const T*>(&u[j]);
          t[j] = f32x4a_t{to_f32<T>(h[0]), to_f32<T>(h[1]), to_f32<T>(h[2]), to_f32<T>(h[3])};
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const f32x4a_t x = t[2 * p], y = t[2 * p + 1];
        f32x4a_t* dst = reinterpret_cast<f32x4a_t*>(stage2 + p * n + r * sb.pitch + 4 * q);
        dst[0] = f32x4a_t{x[0], y[0], x[1], y[1]};
        dst[1] = f32x4a_t{x[2], y[2], x[3], y[3]};
      }
    }
    return;
  }
  for (int r = tid / 32; r < sb.R; r += NT / 32)
    for (int cc = tid % 32; cc < sb.pitch; cc += 32) {
      float t[8];
      const int64_t o = (int64_t)(sb.r0 + r) * sH + sb.c0 + cc;
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = to_f32<T>(pl[j][o]);
#pragma unroll
      for (int p = 0; p < 4; ++p) stage2[p * n + r * sb.pitch + cc] = f32x2_t{t[2 * p], t[2 * p + 1]};
    }
}

// FORM 3: the F(3,3) transform above.  FORM 4 (ABI 12400): the F(4,3) transform of the xi-major F(4,3) conv
// (conv_bf16x3.hip "Row-Winograd F(4,3)": B^T rows of points 0, +-1, +-2, inf) — the block's 12 output rows are 3
// four-row tiles r4 = 3 k + q (q < 3), input rows i0 = 4 q .. 4 q + 5 of the same 14-row block, T43 rows 6 r4 + xi
// (the last thread quarter idles); the same phase 1, boxes and skip rules.
template <int FORM, typename V>
__device__ inline void wino_bt(const V (&d)[FORM + 2], V (&t)[FORM + 2]) {
  if constexpr (FORM == 3) {
    t[0] = 2.f * d[0] - d[1] - 2.f * d[2] + d[3];
    t[1] = -2.f * d[1] - d[2] + d[3];
    t[2] = 2.f * d[1] - 3.f * d[2] + d[3];
    t[3] = d[3] - d[1];
    t[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
  } else {  // as wino43_rows_kernel (conv_bf16x3.hip), the same fp32 expressions
    t[0] = 4.f * d[0] - 5.f * d[2] + d[4];
    t[1] = -4.f * d[1] - 4.f * d[2] + d[3] + d[4];
    t[2] = 4.f * d[1] - 4.f * d[2] - d[3] + d[4];
    t[3] = -2.f * d[1] - d[2] + 2.f * d[3] + d[4];
    t[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
    t[5] = 4.f * d[1] - 5.f * d[3] + d[5];
  }
}
// the non-finite report's sum of a thread's T values (F(3,3): the order of rounds 3-6)
template <int FORM, typename V>
__device__ inline V wino_bt_sum(const V (&t)[FORM + 2]) {
  if constexpr (FORM == 3) return (t[0] + t[1]) + (t[2] + t[3]) + t[4];
  else return ((t[0] + t[1]) + (t[2] + t[3])) + (t[4] + t[5]);
}

template <int FORM = 3>
__device__ inline void wino_rows_phase2(const float (&ds)[kWwRows][kWwCols][8], const unsigned char (&nz)[kWwRows][kWwCols],
                                        const WarpView& vw, const WarpArgs& a, int b, int chunk, int k, int tx,
                                        int r3_rows) {
  static_assert(FORM == 3 || FORM == 4, "row-Winograd form");
  constexpr int NT = FORM == 3 ? 4 : 3, NX = FORM + 2;  // row tiles per block, transformed rows per tile
  const int it = threadIdx.x;
  const int cp = it & 3, c = (it >> 2) % kWwCols, q = it / (4 * kWwCols);
  const int r3 = NT * k + q, u = tx * kWwCols + c;
  if (q >= NT || r3 >= r3_rows || u >= a.Wo) return;
  const int i0 = FORM * q;  // rows i0 .. i0 + NX - 1 of the block
  bool any = false;
#pragma unroll
  for (int m = 0; m < NX; ++m) any |= nz[i0 + m][c] != 0;
  if (a.skip_zero && !any) return;
  f32x2_t d[NX];
#pragma unroll
  for (int m = 0; m < NX; ++m) d[m] = *reinterpret_cast<const f32x2_t*>(&ds[i0 + m][c][2 * cp]);
  f32x2_t t[NX];
  wino_bt<FORM>(d, t);
  if (a.nonfinite) {
    // every d row enters some T row with a non-zero coefficient, and a sample is non-finite when a
    // value it reads is (every read value is multiplied by its weight, zero weights included), so
    // the sum of the T values is non-finite whenever a feature this thread's samples read is
    // (or, conservatively, when finite values overflow): the caller's exact path then runs
    const f32x2_t sum = wino_bt_sum<FORM>(t);
    if (!isfinite(sum.x + sum.y)) *a.nonfinite = a.nf_tag;
  }
  // a T row of dH (= Wo) columns is its hi plane [dH][8 bf16] then its lo plane (16-B units)
  unsigned* out = reinterpret_cast<unsigned*>(static_cast<u32x4_t*>(vw.dst) +
                                              (2 * ((int64_t)b * vw.dB + (int64_t)chunk * vw.dC +
                                                    (int64_t)(NX * r3) * vw.dH) + u)) + cp;
#pragma unroll
  for (int xi = 0; xi < NX; ++xi) {
    const float h0 = (float)(__bf16)t[xi].x, h1 = (float)(__bf16)t[xi].y;
    unsigned* o = out + (int64_t)xi * vw.dH * 8;  // 8 dwords per 32-B unit
    o[0] = pack_bf16x2(h0, h1);
    o[vw.dH * 4] = pack_bf16x2(t[xi].x - h0, t[xi].y - h1);
  }
}

}  // namespace mvbev
