// Homography warp (kornia 0.6.11 warp_perspective semantics) for gfx950.
//
// Replaces kornia.geometry.transform.warp_perspective at
// multiview_detector/models/persp_trans_detector.py:69 and, through the dst
// strides, the torch.cat at :77 (each view writes straight into its slot of the fused
// ground-plane slab).
//
// Per output pixel (u = col, v = row) of batch item b:
//   g   = kornia create_meshgrid (normalised):  gx = (u/(Wo-1) - 0.5)*2, gy likewise
//   p   = M @ [gx, gy, 1]            (M = src_norm <- dst_norm, fp32, computed on the host)
//   s   = |p.z| > 1e-8 ? 1/(p.z + 1e-8) : 1;  (x, y) = s * (p.x, p.y)   (no z>0 mask)
//   ix  = ((x+1)/2)*(W-1), iy = ((y+1)/2)*(H-1)          (GridSampler.h:31, align_corners)
//   out = sum over the 4 in-bounds corners of src * bilinear weight    (zeros padding;
//         a non-finite ix/iy gives NaN in every channel, like torch's CPU grid_sample)
//
// Kernel shape (HBM-bound gather): a block is a 2-D output tile of TH x TW pixels
// (one thread per pixel; each wave a WR x 64/WR sub-tile) and a slice of 64 channels.  The pixel's transform, corner offsets and weights are computed
// once and reused over the channel slice; 4 channels x 4 corners of loads are in flight
// per thread.  The compact 2-D tile keeps each source footprint inside one block (the
// corners of neighbouring pixels share 128-B lines in L1/L2) instead of being re-fetched
// by the blocks of neighbouring output rows on other XCDs.  One launch covers every view
// of a frame (grid.z = batch x view) so the 7-view warp is a single dispatch.
#include "warp_common.h"

#include <type_traits>

namespace mvbev {

template <typename T, int UNROLL, bool SPLIT, bool PAIR>
__global__ __launch_bounds__(kWarpTH * kWarpTW) void warp_tile_kernel(const WarpArgs a) {
  // Logical block order (batch*view, channel chunk, tile) with tile fastest, dealt to the
  // XCDs in contiguous ranges: neighbouring tiles of one plane share an L2 (their source
  // footprints overlap in the far field, where many grid cells map into one source line).
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int tile = lb % a.tiles;
  const int chunk = (lb / a.tiles) % a.chunks;
  const int bv = lb / (a.tiles * a.chunks);
  const int view = bv % a.nviews;
  const int b = bv / a.nviews;
  const WarpView& vw = a.v[view];
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  constexpr int WC = 64 / kWarpWR, WAVES_X = kWarpTW / WC;
  static_assert(kWarpTH * kWarpTW % 64 == 0 && kWarpTH * kWarpTW <= 1024 && kWarpTW % WC == 0 && kWarpTH % kWarpWR == 0, "tile");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = ty * kWarpTH + (wave / WAVES_X) * kWarpWR + lane / WC;
  const int u = tx * kWarpTW + (wave % WAVES_X) * WC + lane % WC;
  if (v >= (a.out_rows ? a.out_rows : a.Ho) || u >= a.Wo) return;  // dst row v = grid row v + vw.row0
  const int c_begin = chunk * kWarpCPB;
  const int c_end = min(a.C, c_begin + kWarpCPB);
  const int H = a.H, W = a.W;

  float m[9];
  if (vw.m_dev) {
#pragma unroll
    for (int i = 0; i < 9; ++i) m[i] = vw.m_dev[9 * b + i];
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) m[i] = vw.m[i];
  }
  const WarpCoord wc = warp_coord(m, u, v + vw.row0, a.Ho, a.Wo, H, W);
  const float ix = wc.ix, iy = wc.iy;
  const bool finite = wc.finite, inside = wc.inside;
  const float fill = finite ? 0.f : __builtin_nanf("");
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = inside ? (int)fx0 : 0, y0 = inside ? (int)fy0 : 0;
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  // torch GridSampler bilinear weights (nw, ne, sw, se)
  const float w_nw = (fx1 - ix) * (fy1 - iy);
  const float w_ne = (ix - fx0) * (fy1 - iy);
  const float w_sw = (fx1 - ix) * (iy - fy0);
  const float w_se = (ix - fx0) * (iy - fy0);
  const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= H - 1;
  const bool ok_nw = vx0 && vy0, ok_ne = vx1 && vy0, ok_sw = vx0 && vy1, ok_se = vx1 && vy1;
  // Invalid corners read a safe in-bounds pixel and are replaced by 0 (select, not a
  // multiply by a zero weight: keeps inf/NaN semantics of the reference).
  const int cx0 = max(x0, 0), cy0 = max(y0, 0);
  const int cx1 = min(x0 + 1, W - 1), cy1 = min(y0 + 1, H - 1);
  const int64_t sH = vw.sH, sW = vw.sW, sC = vw.sC;
  const int64_t o_nw = cy0 * sH + cx0 * sW, o_ne = cy0 * sH + cx1 * sW;
  const int64_t o_sw = cy1 * sH + cx0 * sW, o_se = cy1 * sH + cx1 * sW;
  // PAIR: one 8-B load per row covers both x-corners (columns bx, bx+1, bx clamped into
  // [0, W-2]); nw/ne pick their half (x0 = -1 or W-1 leave the other corner invalid)
  const int bx = min(max(x0, 0), W - 2);
  const int64_t o_top = cy0 * sH + bx, o_bot = cy1 * sH + bx;
  const bool nw_lo = x0 == bx, ne_lo = x0 + 1 == bx;
  const T* base = static_cast<const T*>(vw.src) + (int64_t)b * vw.sB;
  auto sample = [&](int c) __attribute__((always_inline)) {
    const T* pc = base + (int64_t)c * sC;
    float vnw, vne, vsw, vse;
    if constexpr (PAIR) {
      const f32x2u_t top = *reinterpret_cast<const f32x2u_t*>(pc + o_top);
      const f32x2u_t bot = *reinterpret_cast<const f32x2u_t*>(pc + o_bot);
      vnw = nw_lo ? top.x : top.y;
      vne = ne_lo ? top.x : top.y;
      vsw = nw_lo ? bot.x : bot.y;
      vse = ne_lo ? bot.x : bot.y;
    } else {
      vnw = to_f32<T>(pc[o_nw]); vne = to_f32<T>(pc[o_ne]);
      vsw = to_f32<T>(pc[o_sw]); vse = to_f32<T>(pc[o_se]);
    }
    float acc = 0.f;
    acc += (ok_nw ? vnw : 0.f) * w_nw;
    acc += (ok_ne ? vne : 0.f) * w_ne;
    acc += (ok_sw ? vsw : 0.f) * w_sw;
    acc += (ok_se ? vse : 0.f) * w_se;
    return acc;
  };

  // the caller's dst already holds zeros wherever the sample falls outside the source
  if (a.skip_zero && !inside && finite) return;
  if constexpr (SPLIT) {
    u32x4_t* out = static_cast<u32x4_t*>(vw.dst) + 2 * ((int64_t)b * vw.dB + (int64_t)v * vw.dH + u);
    const int64_t dG = 2 * vw.dC;
    constexpr int GU = MVBEV_WARP_GU;
    for (int g0 = c_begin / 8; g0 * 8 < c_end; g0 += GU) {
      float vals[GU][8];
#pragma unroll
      for (int k = 0; k < GU; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = (g0 + k) * 8 + j;
          vals[k][j] = c < c_end ? (inside ? sample(c) : fill) : 0.f;
        }
      if (a.nonfinite) {  // the non-finite report (ABI 11900; as the fused warps', wino_rows_phase2)
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < GU; ++k)
#pragma unroll
          for (int j = 0; j < 8; ++j) sum += vals[k][j];
        if (!isfinite(sum)) *a.nonfinite = a.nf_tag;
      }
#pragma unroll
      for (int k = 0; k < GU; ++k)
        if ((g0 + k) * 8 < c_end) store_split8(out + (g0 + k) * dG, vals[k]);
    }
    return;
  } else {
    T* out = static_cast<T*>(vw.dst) + (int64_t)b * vw.dB + (int64_t)v * vw.dH + u;
    const int64_t dC = vw.dC;
    if (!inside) {
      for (int c = c_begin; c < c_end; ++c) out[(int64_t)c * dC] = from_f32<T>(fill);
      return;
    }
    int c = c_begin;
    for (; c + UNROLL <= c_end; c += UNROLL) {
      float r[UNROLL];
#pragma unroll
      for (int k = 0; k < UNROLL; ++k) r[k] = sample(c + k);
#pragma unroll
      for (int k = 0; k < UNROLL; ++k) out[(int64_t)(c + k) * dC] = from_f32<T>(r[k]);
    }
    for (; c < c_end; ++c) out[(int64_t)c * dC] = from_f32<T>(sample(c));
  }
}

// Warp + row-Winograd input transform in one pass (inference conv1, csrc/conv_bf16x3.hip
// "Row-Winograd conv1"): a block = 4 three-row output tiles (12 rows) x 16 columns of one view's
// kWwGroups consecutive 8-channel groups, one after the other (round 6: the block decode, box, sample geometry
// and address setup once per 2 groups; cfg3 4.09 -> 3.43-3.50 ms, cfg5 3.51 -> 3.12-3.14, cfg2 0.441 -> 0.421-0.428;
// 4 groups spill at any occupancy).  Phase 1: thread (row i < 14, column) warps input row 12 k - 1 + i like
// warp_tile_kernel (zero outside the grid) into LDS; phase 2: each (tile, column, xi) applies
// B^T to its 5 rows and stores the transformed row split-bf16 at T row 5 r3 + xi (dst strides
// in 32-B units: dB per item, dC per 8-channel group, dH per T row).  The slab itself is never
// written.  skip_zero: a (tile, column) whose 5 samples all fall outside the source is not
// written (T is zero-filled once and only ever written by this geometry).
// LDS staging (round 3), as warp_up_wino_kernel: the block's bilinear corners span a source box
// of ~330 upsampled pixels at cfg2 (median; the TA/TD load path was 84 % busy gathering them as
// two 8-B corner pairs per channel and pixel); when the box holds at most kWwStage pixels it is
// loaded once per channel with contiguous row loads into LDS and the corners are read from there.
#ifndef MVBEV_WW_STAGE
#define MVBEV_WW_STAGE 384  // max staged box pixels per channel (8 channels x 384 x 4 B = 12 KiB); 0 = off
#endif
constexpr int kWwStage = MVBEV_WW_STAGE;
#ifndef MVBEV_WW_GROUPS
#define MVBEV_WW_GROUPS 2  // 8-channel groups per block of warp_wino_kernel (A/B below)
#endif
constexpr int kWwGroups = MVBEV_WW_GROUPS;

#ifndef MVBEV_WW_WAVES
#define MVBEV_WW_WAVES 7  // waves per SIMD asked of the compiler (7: at most 72 VGPRs; 2 groups fit without spills)
#endif
template <bool PAIR, typename T = float, int FORM = 3>
__global__ __launch_bounds__(kWwThreads) __attribute__((amdgpu_waves_per_eu(MVBEV_WW_WAVES, 8)))
void warp_wino_kernel(const WarpArgs a, int r3_rows) {
  static_assert(!PAIR || std::is_same<T, float>::value, "corner pairs are fp32 8-B loads");
  __shared__ __attribute__((aligned(16))) float ds[kWwRows][kWwCols][8];  // [row][col][channel]
  __shared__ unsigned char nz[kWwRows][kWwCols];
  __shared__ __attribute__((aligned(16))) f32x2_t stage2[kWarpCPB / 2 * (kWwStage > 0 ? kWwStage : 1)];
  __shared__ int box[4];  // source rows [box0, box1], columns [box2, box3] of the block's corners
  const WarpBlock wb = warp_block_index(a);
  const int tile = wb.tile, view = wb.view, b = wb.b, k = wb.k, tx = wb.tx;
  const WarpView& vw = a.v[view];
  // (round 6) kWwGroups consecutive 8-channel groups per block: the block index, box, sample geometry and
  // address setup are done once for all of them (a.chunks counts group blocks)
  const int chunk0 = wb.chunk * kWwGroups;
  const int H = a.H, W = a.W;
  const int tid = threadIdx.x;
  const int i = tid / kWwCols, c = tid % kWwCols;  // 16 x kWwCols threads, rows >= 14 idle
  const int v = 12 * k - 1 + i, u = tx * kWwCols + c;
  const bool live = i < kWwRows && v >= 0 && v < a.Ho && u < a.Wo;
  // (ABI 12200) the block's source box from the per-geometry table: the 64 channel-group blocks of a
  // (view, tile) no longer each reduce the same box (24 ds_bpermute + 4 LDS atomics per wave and a
  // barrier: ~47 % of this kernel's LDS instructions at cfg2), and a block with no sample inside the
  // source (32 % of cfg2's blocks) leaves before doing anything
  int bx[4];
  if (a.boxes) {
    const int32_t* e = a.boxes + 4 * ((int64_t)view * a.tiles + tile);
    bx[0] = e[0];
    bx[1] = e[1];
    bx[2] = e[2];
    const int c1f = e[3];
    bx[3] = c1f & 0x3FFFFFFF;
    if (a.skip_zero && bx[1] < 0 && !(c1f >> 30)) return;  // whole block, before any barrier
  } else if (tid == 0) {
    box[0] = INT32_MAX;
    box[1] = -1;
    box[2] = INT32_MAX;
    box[3] = -1;
  }
  WarpCoord wc;
  wc.inside = false;
  wc.finite = true;
  wc.ix = wc.iy = 0.f;
  if (live) {
    float m[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
    wc = warp_coord(m, u, v, a.Ho, a.Wo, H, W);
  }
  const float ix = wc.ix, iy = wc.iy;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = wc.inside ? (int)fx0 : 0, y0 = wc.inside ? (int)fy0 : 0;
  const int cx0 = max(x0, 0), cy0 = max(y0, 0);
  const int cx1 = min(x0 + 1, W - 1), cy1 = min(y0 + 1, H - 1);
  if (!a.boxes) {
    __syncthreads();
    if (kWwStage > 0) {  // the box: a shuffle reduction per wave, then one LDS atomic per wave and bound
      int r0 = wc.inside ? cy0 : INT32_MAX, r1 = wc.inside ? cy1 : -1;
      int q0 = wc.inside ? cx0 : INT32_MAX, q1 = wc.inside ? cx1 : -1;
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
#pragma unroll
    for (int q = 0; q < 4; ++q) bx[q] = box[q];
  }
  const T* base = static_cast<const T*>(vw.src) + (int64_t)b * vw.sB;
  const bool quad_ok = vw.sW == 1 && (W & 3) == 0 && (vw.sH & 3) == 0 && (vw.sC & 3) == 0 &&
                       (reinterpret_cast<uintptr_t>(base) & (4 * sizeof(T) - 1)) == 0;
  const StageBox sb = stage_box_shape(bx, W, quad_ok);  // 16-B staging loads where the source allows
  const int R = sb.R, Cb = sb.pitch;
  // uniform per block (the staged path needs unit column stride: the non-quad loads assume it too)
  const bool staged = kWwStage > 0 && bx[1] >= 0 && vw.sW == 1 && R * Cb <= kWwStage;
  // the sample's geometry, shared by every group (same products, in the same order, as before)
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  const float w_nw = (fx1 - ix) * (fy1 - iy), w_ne = (ix - fx0) * (fy1 - iy);
  const float w_sw = (fx1 - ix) * (iy - fy0), w_se = (ix - fx0) * (iy - fy0);
  const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= H - 1;
  const bool ok_nw = vx0 && vy0, ok_ne = vx1 && vy0, ok_sw = vx0 && vy1, ok_se = vx1 && vy1;
  const int n = R * Cb;
  const int t0 = (cy0 - bx[0]) * Cb, t1 = (cy1 - bx[0]) * Cb;
  const int l0 = cx0 - sb.c0, l1 = cx1 - sb.c0;
  for (int g = 0; g < kWwGroups; ++g) {  // uniform (unrolled by the compiler: the rolled loop spills)
    const int chunk = chunk0 + g;
    const int c_begin = chunk * kWarpCPB;
    if (c_begin >= a.C) break;
    const int c_end = min(a.C, c_begin + kWarpCPB);
    // before this group's phase 1 writes ds, the previous group's phase 2 must have read it: the staging barrier
    // below serves (stage2's last readers, the previous phase 1, finished before that group's second barrier)
    if (g && !staged) __syncthreads();
    if (staged) {
      stage_box_load<kWwThreads, T>(base, vw.sC, vw.sH, c_begin, c_end, sb, stage2, tid);
      __syncthreads();
    }
    if (i < kWwRows) {  // phase 1: one warped pixel (8 channels) per thread
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = 0.f;
      bool any = false;
      if (live) {
        if (!wc.inside) {
          if (!wc.finite) {
            any = true;
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = c_begin + j < c_end ? __builtin_nanf("") : 0.f;
          }
        } else {
          any = true;
          if (staged) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {  // a channel pair per ds_read_b64 (the same products per channel)
              const f32x2_t* sp = stage2 + p * n;
              const f32x2_t vnw = sp[t0 + l0], vne = sp[t0 + l1], vsw = sp[t1 + l0], vse = sp[t1 + l1];
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                float acc = 0.f;
                acc += (ok_nw ? vnw[e] : 0.f) * w_nw;
                acc += (ok_ne ? vne[e] : 0.f) * w_ne;
                acc += (ok_sw ? vsw[e] : 0.f) * w_sw;
                acc += (ok_se ? vse[e] : 0.f) * w_se;
                d[2 * p + e] = c_begin + 2 * p + e < c_end ? acc : 0.f;
              }
            }
          } else {
            const int64_t sH = vw.sH, sW = vw.sW, sC = vw.sC;
            const int bxc = min(max(x0, 0), W - 2);
            const int64_t o_top = cy0 * sH + bxc, o_bot = cy1 * sH + bxc;
            const bool nw_lo = x0 == bxc, ne_lo = x0 + 1 == bxc;
            const int64_t o_nw = cy0 * sH + cx0 * sW, o_ne = cy0 * sH + cx1 * sW;
            const int64_t o_sw = cy1 * sH + cx0 * sW, o_se = cy1 * sH + cx1 * sW;
            const T* pc = base + (int64_t)c_begin * sC;  // stepped per channel (no 64-bit multiply per channel)
#pragma unroll
            for (int j = 0; j < 8; ++j) {  // straight-line (a short last group re-reads its last channel)
              if (j > 0 && c_begin + j < c_end) pc += sC;
              float vnw, vne, vsw, vse;
              if constexpr (PAIR) {
                const f32x2u_t top = *reinterpret_cast<const f32x2u_t*>(pc + o_top);
                const f32x2u_t bot = *reinterpret_cast<const f32x2u_t*>(pc + o_bot);
                vnw = nw_lo ? top.x : top.y;
                vne = ne_lo ? top.x : top.y;
                vsw = nw_lo ? bot.x : bot.y;
                vse = ne_lo ? bot.x : bot.y;
              } else {
                vnw = to_f32<T>(pc[o_nw]); vne = to_f32<T>(pc[o_ne]); vsw = to_f32<T>(pc[o_sw]); vse = to_f32<T>(pc[o_se]);
              }
              float acc = 0.f;
              acc += (ok_nw ? vnw : 0.f) * w_nw;
              acc += (ok_ne ? vne : 0.f) * w_ne;
              acc += (ok_sw ? vsw : 0.f) * w_sw;
              acc += (ok_se ? vse : 0.f) * w_se;
              d[j] = c_begin + j < c_end ? acc : 0.f;
            }
          }
        }
      }
      // two 16-B stores (the element-wise form compiled to 8 ds_write_b32)
      *reinterpret_cast<f32x4a_t*>(&ds[i][c][0]) = f32x4a_t{d[0], d[1], d[2], d[3]};
      *reinterpret_cast<f32x4a_t*>(&ds[i][c][4]) = f32x4a_t{d[4], d[5], d[6], d[7]};
      nz[i][c] = any;
    }
    __syncthreads();
    wino_rows_phase2<FORM>(ds, nz, vw, a, b, chunk, k, tx, r3_rows);
  }
}

// The per-(view, tile) source boxes of warp_wino_kernel (ABI 12200), once per geometry: a block per (view,
// tile) evaluates the same pixels, coordinates (warp_coord) and clamped corners as the fused warp's block
// and stores {r0, r1, c0, c1 | nonfinite << 30} (r1 = -1: no sample inside the source; nonfinite: some live
// pixel has non-finite coordinates — its NaN output must still be written).
__global__ __launch_bounds__(kWwThreads) void wino_box_kernel(const WarpArgs a, int32_t* __restrict__ boxes) {
  __shared__ int box[5];
  const int tile = blockIdx.x % a.tiles, view = blockIdx.x / a.tiles;
  const WarpView& vw = a.v[view];
  const int k = tile / a.tiles_x, tx = tile - k * a.tiles_x;
  const int tid = threadIdx.x;
  const int i = tid / kWwCols, c = tid % kWwCols;
  const int v = 12 * k - 1 + i, u = tx * kWwCols + c;
  const bool live = i < kWwRows && v >= 0 && v < a.Ho && u < a.Wo;
  if (tid == 0) {
    box[0] = INT32_MAX;
    box[1] = -1;
    box[2] = INT32_MAX;
    box[3] = -1;
    box[4] = 0;
  }
  __syncthreads();
  WarpCoord wc;
  wc.inside = false;
  wc.finite = true;
  wc.ix = wc.iy = 0.f;
  if (live) {
    float m[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
    wc = warp_coord(m, u, v, a.Ho, a.Wo, a.H, a.W);
  }
  if (wc.inside) {
    const int x0 = (int)floorf(wc.ix), y0 = (int)floorf(wc.iy);
    atomicMin(&box[0], max(y0, 0));
    atomicMax(&box[1], min(y0 + 1, a.H - 1));
    atomicMin(&box[2], max(x0, 0));
    atomicMax(&box[3], min(x0 + 1, a.W - 1));
  }
  if (live && !wc.finite) atomicOr(&box[4], 1);
  __syncthreads();
  if (tid == 0) {  // one 16-B vector store
    const int empty = box[1] < 0;
    const int4 out = make_int4(empty ? 0 : box[0], box[1], empty ? 0 : box[2], (empty ? 0 : box[3]) | (box[4] << 30));
    *reinterpret_cast<int4*>(boxes + 4 * ((int64_t)view * a.tiles + tile)) = out;
  }
}

// warp_wino_kernel for channels-last sources (round 4: sC == 1, the [B, C, H, W] tensor in torch's
// channels_last memory format).  An NCHW source puts each channel's bilinear corners in its own
// plane: a block of 8 channels fetches 8 boxes of ~20-column rows, whose 128-B lines it reads only
// partly (2.2x read amplification at cfg2).  Channels-last puts a pixel's channels side by side, so
// a block takes 32 channels (one 128-B line per source pixel): 8 lanes load a corner's line as
// 16-B pieces, every fetched byte is used, and the gather needs no staging box.
// Phase 0: one thread per warped pixel (14 rows x 16 columns) computes its coordinates once (LDS).
// Phase 1: 8 lanes per pixel, 7 pixels per thread: 4 corner loads each as bounds-checked buffer
// loads (a corner outside the source reads 0 without a fetch, so the loads are unconditional and
// the 28 of a thread are in flight together), the bilinear sum into ds[pixel][40] (pitch 40
// floats: conflict-free 16-B reads in phase 2).  Phase 2: one thread per (tile, column, 8-channel
// chunk, 4-channel half) applies B^T and stores 8 B of each T row's hi and lo planes.  Same T
// (same fp32 ops per channel as warp_wino_kernel) for the same logical source.
// kWcPitch 40 floats: a ds_read_b128 lane group of phase 2 (8 columns x 2 halves) then covers 16 distinct
// 4-bank slots, (10 c + h) mod 16 (36 left 2-way conflicts: 2.6 M conflict cycles per 3.8 M LDS instructions)
constexpr int kWcCh = 32, kWcPitch = 40, kWcPix = kWwRows * kWcCols;
constexpr int kWcOutside = 0x7fff0000;  // byte offset of "no corner" (sources must stay below it)
static_assert(kWcCols == 16 && kWcThreads == 256, "channels-last fused warp: 256 threads, 16 columns");
static_assert(kWcPix % 32 == 0, "phase 1: 32 pixels per pass");

template <int FORM = 3>
__global__ __launch_bounds__(kWcThreads) __attribute__((amdgpu_waves_per_eu(4, 8)))
void warp_wino_cl_kernel(const WarpArgs a, int r3_rows) {
  __shared__ __attribute__((aligned(16))) float ds[kWcPix * kWcPitch];
  __shared__ float2 crd[kWcPix];
  __shared__ unsigned char cls[kWcPix];  // 0: exact zero (outside / off the grid), 1: inside, 2: non-finite
  const WarpBlock wb = warp_block_index(a);
  const int tile = wb.tile, grp = wb.chunk, view = wb.view, b = wb.b, k = wb.k, tx = wb.tx;  // grp: 32-channel group
  const WarpView& vw = a.v[view];
  const int tid = threadIdx.x;
  // (round 6) the per-geometry box table (the same 14 x 16 block tiles as warp_wino_kernel): a block with no
  // sample inside the source and none non-finite returns at once (T zero-filled, skip_zero)
  if (a.boxes && a.skip_zero) {
    const int32_t* e = a.boxes + 4 * ((int64_t)view * a.tiles + tile);
    if (e[1] < 0 && !(e[3] >> 30)) return;
  }
  const int H = a.H, W = a.W;
  if (tid < kWcPix) {
    const int i = tid / kWcCols, c = tid % kWcCols;
    const int v = 12 * k - 1 + i, u = tx * kWcCols + c;
    unsigned char cl = 0;
    float ix = 0.f, iy = 0.f;
    if (v >= 0 && v < a.Ho && u < a.Wo) {
      float m[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) m[q] = vw.m[q];
      const WarpCoord wc = warp_coord(m, u, v, a.Ho, a.Wo, H, W);
      cl = wc.inside ? 1 : (wc.finite ? 0 : 2);
      ix = wc.ix;
      iy = wc.iy;
    }
    crd[tid] = make_float2(ix, iy);
    cls[tid] = cl;
  }
  __syncthreads();
  // the batch item's 32-channel group; offsets past its extent read as 0 (no fetch)
  // (the host checked that the extent is below kOff)
  const char* gbase = static_cast<const char*>(vw.src) + ((int64_t)b * vw.sB + (int64_t)grp * kWcCh) * 4;
  const int extent = (int)(((int64_t)(H - 1) * vw.sH + (int64_t)(W - 1) * vw.sW + kWcCh) * 4);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(gbase), (short)0, extent, 0x00020000);
  const int qd = tid & 7;
  const int sH4 = (int)vw.sH * 4, sW4 = (int)vw.sW * 4, q4 = 16 * qd;
  constexpr int kOff = kWcOutside;  // past the extent: the load returns 0
#pragma unroll
  for (int s = 0; s < kWcPix / 32; ++s) {
    const int p = (tid >> 3) + 32 * s;
    const int cl = cls[p];
    const float2 q = crd[p];
    const float fx0 = floorf(q.x), fy0 = floorf(q.y);
    const int x0 = cl == 1 ? (int)fx0 : -2, y0 = cl == 1 ? (int)fy0 : -2;
    const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
    const float w_nw = (fx1 - q.x) * (fy1 - q.y), w_ne = (q.x - fx0) * (fy1 - q.y);
    const float w_sw = (fx1 - q.x) * (q.y - fy0), w_se = (q.x - fx0) * (q.y - fy0);
    const bool vx0 = x0 >= 0, vx1 = x0 + 1 >= 0 && x0 + 1 <= W - 1;
    const bool vy0 = y0 >= 0, vy1 = y0 + 1 >= 0 && y0 + 1 <= H - 1;
    const int r0 = y0 * sH4, r1 = r0 + sH4, c0 = x0 * sW4, c1 = c0 + sW4;
    const f32x4a_t vnw = __builtin_bit_cast(f32x4a_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, vx0 && vy0 ? r0 + c0 + q4 : kOff, 0, 0));
    const f32x4a_t vne = __builtin_bit_cast(f32x4a_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, vx1 && vy0 ? r0 + c1 + q4 : kOff, 0, 0));
    const f32x4a_t vsw = __builtin_bit_cast(f32x4a_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, vx0 && vy1 ? r1 + c0 + q4 : kOff, 0, 0));
    const f32x4a_t vse = __builtin_bit_cast(f32x4a_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, vx1 && vy1 ? r1 + c1 + q4 : kOff, 0, 0));
    f32x4a_t acc = {0.f, 0.f, 0.f, 0.f};
    acc += vnw * w_nw;
    acc += vne * w_ne;
    acc += vsw * w_sw;
    acc += vse * w_se;
    if (cl != 1) acc = cl == 2 ? f32x4a_t{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                                          __builtin_nanf("")}
                               : f32x4a_t{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4a_t*>(ds + p * kWcPitch + 4 * qd) = acc;
  }
  __syncthreads();
  // phase 2 (FORM 4: 3 four-row tiles per block, rows i0 = 4 q .. 4 q + 5, T43 rows 6 r4 + xi; q = 3 idles)
  constexpr int NT = FORM == 3 ? 4 : 3, NX = FORM + 2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int it = tid + kWcThreads * h;
    const int half = it & 1, c = (it >> 1) & 15, ch8 = (it >> 5) & 3, q = it >> 7;
    const int r3 = NT * k + q, u = tx * kWcCols + c;
    if (q >= NT || r3 >= r3_rows || u >= a.Wo) continue;
    const int i0 = FORM * q;
    int any = 0;
#pragma unroll
    for (int m = 0; m < NX; ++m) any |= cls[(i0 + m) * 16 + c];
    if (a.skip_zero && !any) continue;
    f32x4a_t d[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m)
      d[m] = *reinterpret_cast<const f32x4a_t*>(ds + ((i0 + m) * 16 + c) * kWcPitch + 8 * ch8 + 4 * half);
    f32x4a_t t[NX];
    wino_bt<FORM>(d, t);
    if (a.nonfinite) {  // as wino_rows_phase2
      const f32x4a_t sum = wino_bt_sum<FORM>(t);
      if (!isfinite((sum.x + sum.y) + (sum.z + sum.w))) *a.nonfinite = a.nf_tag;
    }
    const int chunk = grp * (kWcCh / 8) + ch8;
    unsigned* out = reinterpret_cast<unsigned*>(static_cast<u32x4_t*>(vw.dst) +
                                                (2 * ((int64_t)b * vw.dB + (int64_t)chunk * vw.dC +
                                                      (int64_t)(NX * r3) * vw.dH) + u)) + 2 * half;
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      const float h0 = (float)(__bf16)t[xi].x, h1 = (float)(__bf16)t[xi].y;
      const float h2 = (float)(__bf16)t[xi].z, h3 = (float)(__bf16)t[xi].w;
      unsigned* o = out + (int64_t)xi * vw.dH * 8;
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2_t*>(o) = u32x2_t{pack_bf16x2(h0, h1), pack_bf16x2(h2, h3)};
      *reinterpret_cast<u32x2_t*>(o + vw.dH * 4) =
          u32x2_t{pack_bf16x2(t[xi].x - h0, t[xi].y - h1), pack_bf16x2(t[xi].z - h2, t[xi].w - h3)};
    }
  }
}

template <typename T, bool SPLIT>
static void launch_warp_t(const WarpArgs& a, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {
    if (a.pair) {
      hipLaunchKernelGGL((warp_tile_kernel<T, 4, SPLIT, true>), dim3((unsigned)a.nwg), dim3(kWarpTH * kWarpTW), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((warp_tile_kernel<T, 4, SPLIT, false>), dim3((unsigned)a.nwg), dim3(kWarpTH * kWarpTW), 0, s, a);
}

template <typename T>
static int launch_warp(const WarpArgs& a, void* stream, bool split = false) {
  if (split)
    launch_warp_t<T, true>(a, as_stream(stream));
  else
    launch_warp_t<T, false>(a, as_stream(stream));
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

template <typename T>
static int finish_args_and_launch(WarpArgs& a, int64_t B, int64_t C, int64_t H, int64_t W,
                                  int64_t Ho, int64_t Wo, void* stream, bool split = false) {
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kWarpTW);
  a.tiles = a.tiles_x * (int)ceil_div(a.out_rows ? a.out_rows : Ho, kWarpTH);
  a.chunks = (int)ceil_div(C, kWarpCPB);
  a.nwg = a.tiles * a.chunks * a.B * a.nviews;
#ifndef MVBEV_WARP_PAIR
#define MVBEV_WARP_PAIR 1
#endif
  a.pair = MVBEV_WARP_PAIR && W >= 2;
  for (int i = 0; i < a.nviews; ++i) a.pair = a.pair && a.v[i].sW == 1;
  return launch_warp<T>(a, stream, split);
}

static int check_sizes(int64_t B, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int nviews) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || nviews <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || B * nviews > 65535 || C > INT32_MAX || H > INT32_MAX / 2 ||
      W > INT32_MAX / 2 || Ho > INT32_MAX / 2 || Wo > INT32_MAX / 2 ||
      ceil_div(Ho, kWarpTH) * ceil_div(Wo, kWarpTW) * ceil_div(C, kWarpCPB) * B * nviews > INT32_MAX)
    return MVBEV_ERR_SHAPE;
  return MVBEV_OK;
}

template <typename T>
static int warp_single(const void* src, int64_t B, int64_t C, int64_t H, int64_t W,
                       const int64_t* ss, const float* m, void* dst, int64_t Ho, int64_t Wo,
                       const int64_t* ds, void* stream) {
  if (!src || !m || !dst || !ss || !ds) return MVBEV_ERR_NULL;
  const int st = check_sizes(B, C, H, W, Ho, Wo, 1);
  if (st != MVBEV_OK) return st;
  if (ds[3] != 1) return MVBEV_ERR_STRIDE;
  WarpArgs a = {};
  a.v[0] = WarpView{src, ss[0], ss[1], ss[2], ss[3], dst, ds[0], ds[1], ds[2], m, {}};
  a.nviews = 1;
  return finish_args_and_launch<T>(a, B, C, H, W, Ho, Wo, stream);
}

template <typename T>
static int warp_views(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                      int64_t W, int64_t Ho, int64_t Wo, void* stream, bool split = false, int flags = 0,
                      const int32_t* row0s = nullptr, int64_t out_rows = 0, int32_t* nonfinite = nullptr,
                      int32_t nf_tag = 0) {
  if (!views) return MVBEV_ERR_NULL;
  const int st = check_sizes(B, C, H, W, Ho, Wo, nviews);
  if (st != MVBEV_OK) return st;
  if (out_rows < 0 || out_rows > Ho) return MVBEV_ERR_SHAPE;
  WarpArgs a = {};
  a.out_rows = (int)out_rows;
  a.nonfinite = nonfinite;
  a.nf_tag = nf_tag;
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
    if (d.row0 < 0 || d.row0 + (out_rows ? out_rows : Ho) > Ho) return MVBEV_ERR_SHAPE;
  }
  a.nviews = nviews;
  a.skip_zero = (flags & MVBEV_WARP_DST_ZEROED) != 0;
  return finish_args_and_launch<T>(a, B, C, H, W, Ho, Wo, stream, split);
}

// Per conv tile (tile_h x tile_w output pixels of rows [row0, row0 + rows), plus `halo`
// pixels around it, clipped to the grid): bit s of mask[tile] is set when view s's warp
// output can be non-zero anywhere in that region (some pixel is in-bounds, or non-finite ->
// NaN).  A clear bit means every channel of that view is exactly 0 there, so the conv may
// skip those input channels for the tile without changing a single output bit.
__global__ void tile_mask_kernel(WarpArgs a, int row0, int rows, int tile_h, int tile_w, int halo,
                                 int tiles_x, uint32_t* mask) {
  __shared__ uint32_t bits;
  if (threadIdx.x == 0) bits = 0;
  __syncthreads();
  const int tile = blockIdx.x;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int r0 = max(0, row0 + ty * tile_h - halo), r1 = min(a.Ho, row0 + min(rows, (ty + 1) * tile_h) + halo);
  const int c0 = max(0, tx * tile_w - halo), c1 = min(a.Wo, (tx + 1) * tile_w + halo);
  const int w = c1 - c0, npix = (r1 - r0) * w;
  uint32_t mine = 0;
  for (int p = threadIdx.x; p < npix; p += blockDim.x) {
    const int v = r0 + p / w, u = c0 + p % w;
    for (int s = 0; s < a.nviews; ++s) {
      float m[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) m[i] = a.v[s].m[i];
      const WarpCoord c = warp_coord(m, u, v, a.Ho, a.Wo, a.H, a.W);
      if (c.inside || !c.finite) mine |= 1u << s;
    }
  }
  if (mine) atomicOr(&bits, mine);
  __syncthreads();
  if (threadIdx.x == 0) mask[tile] = bits;
}

// bit s of *bits: some output pixel of view s has non-finite warp coordinates (NaN output).
// One workgroup (run once per geometry), LDS reduction, one plain store.
__global__ void nonfinite_views_kernel(WarpArgs a, uint32_t* bits) {
  __shared__ uint32_t blk;
  if (threadIdx.x == 0) blk = 0;
  __syncthreads();
  uint32_t mine = 0;
  const int npix = a.Ho * a.Wo;
  for (int p = threadIdx.x; p < npix; p += blockDim.x) {
    const int v = p / a.Wo, u = p - v * a.Wo;
    for (int s = 0; s < a.nviews; ++s) {
      float m[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) m[i] = a.v[s].m[i];
      if (!warp_coord(m, u, v, a.Ho, a.Wo, a.H, a.W).finite) mine |= 1u << s;
    }
  }
  if (mine) atomicOr(&blk, mine);
  __syncthreads();
  if (threadIdx.x == 0) *bits = blk;
}

// coord_map (persp_trans_detector.py:103-112): grid / (n-1) * 2 - 1 in float64, then .float()
__global__ void coord_map_kernel(float* dst, int64_t dB, int64_t dC, int64_t dH, int Ho, int Wo) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Ho * Wo) return;
  const int v = p / Wo, u = p - v * Wo;
  float* o = dst + (int64_t)blockIdx.y * dB + (int64_t)v * dH + u;
  o[0] = (float)((double)u / (double)(Wo - 1) * 2.0 - 1.0);
  o[dC] = (float)((double)v / (double)(Ho - 1) * 2.0 - 1.0);
}

// a gated zero fill (ABI 11900): 16-B stores over n16 units when *gate == tag, else nothing — the band
// exchange's send chunks after a frame whose exact path overwrote them (they are zero-filled once and
// then written only by the window warps with MVBEV_WARP_DST_ZEROED)
__global__ __launch_bounds__(256) void zero_gated_kernel(u32x4_t* dst, int64_t n16, const int32_t* gate, int32_t tag) {
  if (*gate != tag) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = u32x4_t{0u, 0u, 0u, 0u};
}

// a gated store (ABI 12200): fp32 src [B][C][H][W] (element strides) into dst as fp32 (element strides) or
// as the split-bf16 blocked layout (32-B units: batch, channel group, row; 8 channels of a pixel per entry),
// when *gate == tag — the training forward's exact path puts its activations where the native backward
// reads them.  The split keeps a non-finite value in hi with lo = 0 (hi + lo is the value: inf stays inf,
// so the backward's ReLU mask hi + lo > 0 is torch's), unlike the fast path's split (lo = v - hi).
struct StoreArgs {
  const float* src;
  int64_t sB, sC, sH;
  void* dst;
  int64_t dB, dC, dH;
  int B, C, H, W, split;
  const int32_t* gate;
  int32_t gate_tag;
};
__global__ __launch_bounds__(256) void store_gated_kernel(const StoreArgs a) {
  if (*a.gate != a.gate_tag) return;
  const int G = a.split ? (a.C + 7) / 8 : a.C;
  const int64_t n = (int64_t)a.B * G * a.H * a.W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % a.W);
    int64_t r = i / a.W;
    const int y = (int)(r % a.H);
    r /= a.H;
    const int g = (int)(r % G);
    const int b = (int)(r / G);
    const float* s = a.src + (int64_t)b * a.sB + (int64_t)y * a.sH + x;
    if (!a.split) {
      static_cast<float*>(a.dst)[(int64_t)b * a.dB + (int64_t)g * a.dC + (int64_t)y * a.dH + x] = s[(int64_t)g * a.sC];
      continue;
    }
    bf16x8_t hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * g + j;
      const float v = c < a.C ? s[(int64_t)c * a.sC] : 0.f;
      const __bf16 h = (__bf16)v;
      hi[j] = h;
      lo[j] = (__bf16)(isfinite(v) ? v - (float)h : 0.f);
    }
    u32x4_t* o = static_cast<u32x4_t*>(a.dst) + 2 * ((int64_t)b * a.dB + (int64_t)g * a.dC + (int64_t)y * a.dH + x);
    o[0] = __builtin_bit_cast(u32x4_t, hi);
    o[1] = __builtin_bit_cast(u32x4_t, lo);
  }
}

}  // namespace mvbev

extern "C" {

int mvbev_store_gated_f32(const float* src, const int64_t src_strides[4], void* dst, const int64_t dst_strides[4],
                          int64_t B, int64_t C, int64_t H, int64_t W, int dst_layout, const int32_t* gate,
                          int32_t gate_tag, void* stream) {
  using namespace mvbev;
  if (!src || !dst || !gate || !src_strides || !dst_strides) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (dst_layout != MVBEV_LAYOUT_F32 && dst_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;
  if (src_strides[3] != 1 || dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
  if (dst_layout == MVBEV_LAYOUT_SPLIT_BF16 && (reinterpret_cast<uintptr_t>(dst) & 15)) return MVBEV_ERR_ALIGN;
  StoreArgs a;
  a.src = src;
  a.sB = src_strides[0], a.sC = src_strides[1], a.sH = src_strides[2];
  a.dst = dst;
  a.dB = dst_strides[0], a.dC = dst_strides[1], a.dH = dst_strides[2];
  a.B = (int)B, a.C = (int)C, a.H = (int)H, a.W = (int)W, a.split = dst_layout == MVBEV_LAYOUT_SPLIT_BF16;
  a.gate = gate, a.gate_tag = gate_tag;
  const int64_t n = B * (a.split ? ceil_div(C, 8) : C) * H * W;
  hipLaunchKernelGGL(store_gated_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, 256), 8192)), dim3(256), 0,
                     as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_zero_gated(void* dst, int64_t bytes, const int32_t* gate, int32_t gate_tag, void* stream) {
  using namespace mvbev;
  if (!dst || !gate) return MVBEV_ERR_NULL;
  if (bytes <= 0) return MVBEV_ERR_RANK;
  if (bytes % 16 || (reinterpret_cast<uintptr_t>(dst) & 15)) return MVBEV_ERR_ALIGN;
  const int64_t n16 = bytes / 16;
  hipLaunchKernelGGL(zero_gated_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n16, 256), 4096)), dim3(256), 0,
                     as_stream(stream), static_cast<u32x4_t*>(dst), n16, gate, gate_tag);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

const char* mvbev_status_string(int s) {
  switch (s) {
    case MVBEV_OK: return "ok";
    case MVBEV_ERR_RANK: return "non-positive size";
    case MVBEV_ERR_SHAPE: return "inconsistent or unsupported shape";
    case MVBEV_ERR_STRIDE: return "unsupported stride";
    case MVBEV_ERR_ALIGN: return "misaligned pointer";
    case MVBEV_ERR_NULL: return "null pointer";
    case MVBEV_ERR_DILATION: return "unsupported dilation";
    case MVBEV_ERR_HIP: return "HIP launch failed";
    default: return "unknown status";
  }
}

int mvbev_version(void) { return 12400; }

int mvbev_warp_perspective_f32(const float* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m, float* dst,
                               int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream) {
  return mvbev::warp_single<float>(src, B, C, H, W, src_strides, m, dst, Ho, Wo, dst_strides,
                                   stream);
}

int mvbev_warp_perspective_f16(const void* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m, void* dst,
                               int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream) {
  return mvbev::warp_single<__half>(src, B, C, H, W, src_strides, m, dst, Ho, Wo, dst_strides,
                                    stream);
}

int mvbev_warp_views_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                         int64_t H, int64_t W, int64_t Ho, int64_t Wo, void* stream) {
  return mvbev::warp_views<float>(views, nviews, B, C, H, W, Ho, Wo, stream);
}

int mvbev_warp_views_split_bf16_ex(const mvbev_warp_view* views, int nviews, int src_is_f16,
                                   int64_t B, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                   int flags, void* stream) {
  if (flags & ~MVBEV_WARP_DST_ZEROED) return MVBEV_ERR_SHAPE;
  if (src_is_f16)
    return mvbev::warp_views<__half>(views, nviews, B, C, H, W, Ho, Wo, stream, true, flags);
  return mvbev::warp_views<float>(views, nviews, B, C, H, W, Ho, Wo, stream, true, flags);
}

int mvbev_warp_views_split_bf16_rows(const mvbev_warp_view* views, const int32_t* row0s, int nviews, int src_is_f16,
                                     int64_t B, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                     int64_t out_rows, int flags, int32_t* nonfinite, int32_t nf_tag, void* stream) {
  if (flags & ~MVBEV_WARP_DST_ZEROED) return MVBEV_ERR_SHAPE;
  if (!row0s) return MVBEV_ERR_NULL;
  if (out_rows <= 0) return MVBEV_ERR_RANK;
  if (src_is_f16)
    return mvbev::warp_views<__half>(views, nviews, B, C, H, W, Ho, Wo, stream, true, flags, row0s, out_rows,
                                     nonfinite, nf_tag);
  return mvbev::warp_views<float>(views, nviews, B, C, H, W, Ho, Wo, stream, true, flags, row0s, out_rows,
                                  nonfinite, nf_tag);
}

int mvbev_warp_views_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                                  int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                                  int32_t nf_tag, const int32_t* boxes, void* stream);

int mvbev_warp_views_wino_rows(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                               int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                               int32_t nf_tag, void* stream) {
  return mvbev_warp_views_wino_rows_ex(views, nviews, B, C, H, W, Ho, Wo, r3_rows, flags, nonfinite, nf_tag, nullptr,
                                       stream);
}

int64_t mvbev_warp_wino_boxes_count(int64_t Wo, int64_t r3_rows) {
  if (Wo <= 0 || r3_rows <= 0) return 0;
  return mvbev::ceil_div(Wo, (int64_t)mvbev::kWwCols) * mvbev::ceil_div(r3_rows, (int64_t)4);
}

int mvbev_warp_wino_boxes(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                          int64_t r3_rows, int32_t* boxes, void* stream) {
  using namespace mvbev;
  if (!views || !boxes) return MVBEV_ERR_NULL;
  if (nviews <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || r3_rows <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || 3 * r3_rows < Ho || H >= (1 << 29) || W >= (1 << 29)) return MVBEV_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(boxes) & 15) return MVBEV_ERR_ALIGN;
  WarpArgs a = {};
  for (int i = 0; i < nviews; ++i)
    for (int q = 0; q < 9; ++q) a.v[i].m[q] = views[i].m[q];
  a.nviews = nviews;
  a.H = (int)H, a.W = (int)W, a.Ho = (int)Ho, a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kWwCols);
  a.tiles = a.tiles_x * (int)ceil_div(r3_rows, 4);
  hipLaunchKernelGGL(wino_box_kernel, dim3((unsigned)(a.tiles * nviews)), dim3(kWwThreads), 0, as_stream(stream), a,
                     boxes);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_warp_views_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                                  int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                                  int32_t nf_tag, const int32_t* boxes, void* stream) {
  using namespace mvbev;
  if (!views) return MVBEV_ERR_NULL;
  if (flags & ~(MVBEV_WARP_DST_ZEROED | MVBEV_WARP_SRC_F16 | MVBEV_WARP_WINO43)) return MVBEV_ERR_SHAPE;
  const bool f16 = (flags & MVBEV_WARP_SRC_F16) != 0;
  const bool w43 = (flags & MVBEV_WARP_WINO43) != 0;  // T43: r3_rows counts four-row tiles, 3 per block
  const int form = w43 ? 4 : 3, tpb = w43 ? 3 : 4;
  int st = check_sizes(B, C, H, W, r3_rows, Wo, nviews);
  if (st != MVBEV_OK) return st;
  st = check_sizes(B, C, H, W, Ho, Wo, nviews);
  if (st != MVBEV_OK) return st;
  if (form * r3_rows < Ho || W < 2) return MVBEV_ERR_SHAPE;
  WarpArgs a = {};
  bool pair = true;
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
    pair = pair && d.sW == 1;
  }
  a.nviews = nviews;
  a.skip_zero = (flags & MVBEV_WARP_DST_ZEROED) != 0;
  a.nonfinite = nonfinite;
  a.nf_tag = nf_tag;
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, kWwCols);
  a.tiles = a.tiles_x * (int)ceil_div(r3_rows, tpb);  // 4 three-row (3 four-row) tiles per block
  // channels-last sources (every view: unit channel stride, 16-B aligned pixels of whole 32-channel
  // groups, offsets within 31 bits) take the line-per-pixel kernel
  bool cl = C % kWcCh == 0 && !f16;
  for (int i = 0; i < nviews && cl; ++i) {
    const WarpView& d = a.v[i];
    cl = d.sC == 1 && d.sW >= C && d.sH > 0 && d.sB >= 0 && d.sW % 4 == 0 && d.sH % 4 == 0 && d.sB % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(d.src) & 15) == 0 &&
         ((H - 1) * d.sH + (W - 1) * d.sW + C) * 4 < kWcOutside;
  }
  if (cl) {
    a.tiles_x = (int)ceil_div(Wo, kWcCols);
    a.tiles = a.tiles_x * (int)ceil_div(r3_rows, tpb);
  }
  a.chunks = (int)ceil_div(C, cl ? kWcCh : kWarpCPB * kWwGroups);  // (NCHW: blocks of kWwGroups 8-channel groups)
  a.nwg = a.tiles * a.chunks * a.B * a.nviews;
  set_fastdiv(a);
  a.boxes = boxes;  // (the line-per-pixel kernel's 14 x 16 block tiles are warp_wino_kernel's: same table)
  const dim3 grid((unsigned)a.nwg), block(cl ? kWcThreads : kWwThreads);
  hipStream_t s = as_stream(stream);
  const int r = (int)r3_rows;
  if (w43) {
    if (cl) hipLaunchKernelGGL((warp_wino_cl_kernel<4>), grid, block, 0, s, a, r);
    else if (f16) hipLaunchKernelGGL((warp_wino_kernel<false, __half, 4>), grid, block, 0, s, a, r);
    else if (pair) hipLaunchKernelGGL((warp_wino_kernel<true, float, 4>), grid, block, 0, s, a, r);
    else hipLaunchKernelGGL((warp_wino_kernel<false, float, 4>), grid, block, 0, s, a, r);
  } else if (cl) {
    hipLaunchKernelGGL((warp_wino_cl_kernel<3>), grid, block, 0, s, a, r);
  } else if (f16) {
    hipLaunchKernelGGL((warp_wino_kernel<false, __half>), grid, block, 0, s, a, r);
  } else if (pair) {
    hipLaunchKernelGGL((warp_wino_kernel<true>), grid, block, 0, s, a, r);
  } else {
    hipLaunchKernelGGL((warp_wino_kernel<false>), grid, block, 0, s, a, r);
  }
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_warp_views_f16(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                         int64_t H, int64_t W, int64_t Ho, int64_t Wo, void* stream) {
  return mvbev::warp_views<__half>(views, nviews, B, C, H, W, Ho, Wo, stream);
}

int mvbev_warp_tile_mask(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W,
                         int64_t Ho, int64_t Wo, int64_t row0, int64_t rows, int64_t tile_h,
                         int64_t tile_w, int64_t halo, uint32_t* mask, void* stream) {
  using namespace mvbev;
  if (!views || !mask) return MVBEV_ERR_NULL;
  if (nviews <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || rows <= 0 || tile_h <= 0 ||
      tile_w <= 0 || halo < 0)
    return MVBEV_ERR_RANK;
  if (nviews > 32 || nviews > kWarpMaxViews || row0 < 0 || row0 + rows > Ho) return MVBEV_ERR_SHAPE;
  WarpArgs a = {};
  for (int i = 0; i < nviews; ++i)
    for (int k = 0; k < 9; ++k) a.v[i].m[k] = views[i].m[k];
  a.nviews = nviews;
  a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  const int tiles_x = (int)ceil_div(Wo, tile_w);
  const int64_t tiles = tiles_x * ceil_div(rows, tile_h);
  if (tiles > INT32_MAX) return MVBEV_ERR_SHAPE;
  hipLaunchKernelGGL(tile_mask_kernel, dim3((unsigned)tiles), dim3(256), 0, as_stream(stream), a,
                     (int)row0, (int)rows, (int)tile_h, (int)tile_w, (int)halo, tiles_x, mask);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_warp_nonfinite_views(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W, int64_t Ho,
                               int64_t Wo, uint32_t* bits, void* stream) {
  using namespace mvbev;
  if (!views || !bits) return MVBEV_ERR_NULL;
  if (nviews <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || Ho * Wo > INT32_MAX) return MVBEV_ERR_SHAPE;
  WarpArgs a = {};
  for (int i = 0; i < nviews; ++i)
    for (int k = 0; k < 9; ++k) a.v[i].m[k] = views[i].m[k];
  a.nviews = nviews;
  a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  hipLaunchKernelGGL(nonfinite_views_kernel, dim3(1), dim3(1024), 0, as_stream(stream), a, bits);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_fill_coord_map_f32(float* dst, int64_t B, int64_t Ho, int64_t Wo,
                             const int64_t dst_strides[4], void* stream) {
  if (!dst || !dst_strides) return MVBEV_ERR_NULL;
  if (B <= 0 || Ho <= 0 || Wo <= 0) return MVBEV_ERR_RANK;
  if (dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
  dim3 grid((unsigned)mvbev::ceil_div(Ho * Wo, 256), (unsigned)B);
  hipLaunchKernelGGL(mvbev::coord_map_kernel, grid, dim3(256), 0, mvbev::as_stream(stream), dst,
                     dst_strides[0], dst_strides[1], dst_strides[2], (int)Ho, (int)Wo);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

}  // extern "C"
