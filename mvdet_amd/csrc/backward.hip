// Native backward of the project+fuse hot path for gfx950: what
// autograd needs to train through PerspTransDetector.forward (trainer.py:38-49) without the
// stock-torch fallback.
//
//   warp (a5, persp_trans_detector.py:69)   adjoint of the bilinear gather: grad_src +=
//                                            w_corner * grad_out (fp32 atomic adds), the
//                                            kornia/grid_sample weights of the forward
//   conv1 / conv2 (map_classifier[0], [2])  weight gradient: wgrad_kernel below (3xbf16 MFMA);
//                                            data gradient: the forward conv kernel with the
//                                            weights packed transposed + flipped
//                                            (mvbev_pack_conv3x3_dgrad_bf16x3, conv_bf16x3.hip);
//                                            bias + coord-channel gradients: bias_coord_grad_kernel
//   ReLUs (map_classifier[1], [3])          relu_backward_kernel (torch threshold_backward:
//                                            grad where the ReLU output > 0)
//   conv3 (map_classifier[4], Cout = 1)     cout1_dgrad_kernel (fused with conv2's ReLU mask),
//                                            cout1_wgrad_kernel
//
// Weight gradient as a GEMM: dW_t[co][k] = sum over pixels p of dy[co][p] * x[k][p + s_t]
// (s_t = the tap's dilated offset).  M = Cout, N = input channels x 9 taps, K = pixels.  A
// workgroup (8 waves) owns 128 output channels x 64 input channels x all 9 taps and walks its
// share of the pixels in chunks of one 32-pixel row segment (2 MFMA K-steps of 16):
//   A image  dy[128 co][32 px] bf16 hi / lo, 80-B rows (conflict-free ds_read_b128 of 8 px);
//   B image  x[3 rows][32 + 2d px][32 ch] bf16 hi / lo per 32-channel half, 64 B per pixel;
//            the B fragment (8 consecutive pixels of one channel per lane) is read with the
//            gfx950 transposing ds_read_b64_tr_b16 from this channel-innermost image (the
//            slab's own split-bf16 layout copied 16 B at a time), so every tap is just a
//            different pixel offset: no im2col, no shifted copies, 4 rows x 64 B = 256 B per
//            32-lane half = conflict-free.
// Wave = 32 co x 32 ch x 9 taps (9 accumulators); per K-step 2 A + 36 transposed B reads for
// 27 MFMAs (3 passes: lo*hi, hi*lo, hi*hi as in the forward).  The pixels are split into P
// partitions (row bands) so the launch fills the CUs; partial sums land in a workspace and
// wgrad_reduce_kernel adds them in partition order (deterministic) while scattering the
// channels into the module's weight layout through chan_map.
#include "warp_common.h"

#include <climits>
#include <type_traits>
#include <utility>

namespace mvbev {
namespace bwd {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#ifndef MVBEV_WGRAD_CPW
#define MVBEV_WGRAD_CPW 1  // 32-channel output blocks per wave (1: 8 waves; 2: 4 waves, one per SIMD, 512
                           // registers: conv1 wgrad 4.35 vs 3.10 ms, measured slower)
#endif
constexpr int CPW = MVBEV_WGRAD_CPW;
#ifndef MVBEV_WGRAD_DMA
#define MVBEV_WGRAD_DMA 1  // split-bf16 x + aligned dy: wgrad_dma_kernel (LDS-DMA staging)
#endif
constexpr int NWV = 8 / CPW;  // waves per workgroup: (4 / CPW) (output channels) x 2 (input channels)
constexpr int NTH = 64 * NWV;
constexpr int MT = 128;       // output channels per workgroup
constexpr int NT = 64;        // input channels per workgroup (the Winograd form: 2 NT)
constexpr int PX = 32;        // pixels per chunk (one row segment) = 2 K-steps
constexpr int AP = PX + 8;    // bf16 per A-image row (80 B)

struct WArgs {
  const void* x;
  const float* dy;
  float* ws;
  int64_t group_stride, batch_stride;
  int group, K, Cout, B, H, W;
  int segs, nchunks, P, n_ct, n_kt, ntiles;
  bool vec_dy;  // W % 4 == 0 and dy 16-B aligned: dy rows as 16-B loads
  bool dy_rows;  // dy in MVBEV_LAYOUT_SPLIT_ROWS (pre-split bf16 hi / lo; wgrad_dma_kernel only)
  // frustum (optional): per input-channel group (desc group = one camera's slot), the pixel
  // chunks whose x window can be non-zero, clist[coff[g] .. coff[g+1]); a tile's partitions
  // split its group's list instead of all chunks (skipped chunks contribute exactly 0)
  const int32_t* clist;
  const int32_t* coff;
};

struct SplitIn {};

__device__ inline bf16x8 tr_read8(const __bf16* p) {
  // two transposed 4x16 reads: pixels 0..3 then 4..7 of the lane's 8-pixel K run
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p + 4 * 32));
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ inline void split4(const floatx4 v, u32x2& hi, u32x2& lo) {
  bf16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 t = (__bf16)v[j];
    h[j] = t;
    l[j] = (__bf16)(v[j] - (float)t);
  }
  hi = __builtin_bit_cast(u32x2, h);
  lo = __builtin_bit_cast(u32x2, l);
}

template <typename TIn, int DIL>
__global__ __launch_bounds__(NTH, 1) void wgrad_kernel(const WArgs a) {
  constexpr int XW = PX + 2 * DIL;       // window columns
  constexpr int BPIX = 3 * XW;           // window pixels (3 tap rows)
  constexpr int BIMG = BPIX * 32;        // bf16 per (channel half, part) image
  constexpr int AIMG = MT * AP;          // bf16 per A part
  constexpr int BUF = 2 * AIMG + 4 * BIMG;
  constexpr int BENT = BPIX * 8;         // staging entries (window pixel, 8-channel group)
  constexpr int BPT = (BENT + NTH - 1) / NTH;
  constexpr bool SPLIT = std::is_same<TIn, SplitIn>::value;
  constexpr int AIT = MT * 8 / NTH;      // dy staging: 8 threads per 32-pixel row, AIT rows each
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;
  // (partition, tile) with partitions slowest, dealt to the XCDs in contiguous ranges: the
  // workgroups that run together on one XCD sweep the same pixels (dy / x lines shared in L2)
  const int lb = xcd_remap(blockIdx.x, a.P * a.ntiles);
  const int p = lb / a.ntiles, tile = lb - p * a.ntiles;
  const int ct = tile % a.n_ct, kt = tile / a.n_ct;
  const int32_t* list = nullptr;
  int nact = a.nchunks;
  if (a.clist) {
    const int grp = (kt * NT) / a.group;
    list = a.clist + a.coff[grp];
    nact = a.coff[grp + 1] - a.coff[grp];
  }
  const int c0 = (int)((int64_t)nact * p / a.P);
  const int c1 = (int)((int64_t)nact * (p + 1) / a.P);
  const int W = a.W, H = a.H;
  const int64_t plane = (int64_t)H * W;

  floatx4 areg[AIT];
  u32x4 bsp[BPT][SPLIT ? 2 : 1];
  float bfl[BPT][SPLIT ? 1 : 8];
  bool bok[BPT];

  auto load = [&](int ci) __attribute__((always_inline)) {
    const int c = list ? list[ci] : ci;
    const int R = c / a.segs, seg = c - R * a.segs;
    const int b = R / H, y = R - b * H;
    const int x0 = seg * PX;
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int co = ct * MT + (tid >> 3) + (NTH / 8) * i;
      const int px = x0 + 4 * (tid & 7);
      const float* src = a.dy + (((int64_t)b * a.Cout + co) * H + y) * W;
      if (a.vec_dy) {
        areg[i] = px < W ? *reinterpret_cast<const floatx4*>(src + px) : floatx4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) areg[i][j] = px + j < W ? src[px + j] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = tid + NTH * i;
      const int g8 = e / BPIX, pix = e - g8 * BPIX;
      const int r = pix / XW, cc = pix - r * XW;
      const int gy = y + (r - 1) * DIL, gx = x0 - DIL + cc;
      const int k0 = kt * NT + g8 * 8;
      const bool ok = e < BENT && gy >= 0 && gy < H && gx >= 0 && gx < W && k0 < a.K;
      bok[i] = ok;
      int64_t base = 0;
      if (ok) {
        const int g_ = k0 / a.group;
        base = (int64_t)b * a.batch_stride + g_ * a.group_stride + (int64_t)(k0 - g_ * a.group) * plane;
      }
      const int64_t pofs = ok ? (int64_t)gy * W + gx : 0;
      if constexpr (SPLIT) {
        const u32x4* xc = static_cast<const u32x4*>(a.x) + base / 4 + 2 * pofs;
        bsp[i][0] = xc[0];
        bsp[i][1] = xc[1];
      } else {
        const float* xc = static_cast<const float*>(a.x) + base + pofs;
#pragma unroll
        for (int j = 0; j < 8; ++j) bfl[i][j] = xc[j * plane];
      }
    }
  };

  auto store = [&](int bb) __attribute__((always_inline)) {
    __bf16* L = lds + bb * BUF;
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int row = (tid >> 3) + (NTH / 8) * i, q = tid & 7;
      u32x2 hi, lo;
      split4(areg[i], hi, lo);
      *reinterpret_cast<u32x2*>(L + row * AP + 4 * q) = hi;
      *reinterpret_cast<u32x2*>(L + AIMG + row * AP + 4 * q) = lo;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = tid + NTH * i;
      if (BENT % NTH != 0 && e >= BENT) continue;
      const int g8 = e / BPIX, pix = e - g8 * BPIX;
      __bf16* Bh = L + 2 * AIMG + ((g8 >> 2) * 2) * BIMG + pix * 32 + (g8 & 3) * 8;
      const u32x4 z = {0u, 0u, 0u, 0u};
      if constexpr (SPLIT) {
        *reinterpret_cast<u32x4*>(Bh) = bok[i] ? bsp[i][0] : z;
        *reinterpret_cast<u32x4*>(Bh + BIMG) = bok[i] ? bsp[i][1] : z;
      } else {
        bf16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bok[i] ? bfl[i][j] : 0.f;
          const __bf16 t = (__bf16)v;
          hi[j] = t;
          lo[j] = (__bf16)(v - (float)t);
        }
        *reinterpret_cast<u32x4*>(Bh) = __builtin_bit_cast(u32x4, hi);
        *reinterpret_cast<u32x4*>(Bh + BIMG) = __builtin_bit_cast(u32x4, lo);
      }
    }
  };

  const int cw = wave % (4 / CPW), cb = wave / (4 / CPW);  // output block group, channel half
  const int gi = (lane >> 4) & 1, li = lane & 15;
  // transposed-read address of the lane: pixel 8kh + (li>>2) (+4 in the second read),
  // channels 16gi + 4(li&3) .. +3 of the wave's 32-channel half
  const int tr0 = (8 * kh + (li >> 2)) * 32 + 16 * gi + 4 * (li & 3);
  floatx16 acc[CPW][9];
#pragma unroll
  for (int m = 0; m < CPW; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = floatx16{0};

  auto compute = [&](int bb) __attribute__((always_inline)) {
    const __bf16* L = lds + bb * BUF;
    const __bf16* Ah = L + (32 * CPW * cw + l32) * AP + 8 * kh;
    const __bf16* Bh = L + 2 * AIMG + (cb * 2) * BIMG + tr0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ahi[CPW], alo[CPW];
#pragma unroll
      for (int m = 0; m < CPW; ++m) {
        ahi[m] = *reinterpret_cast<const bf16x8*>(Ah + 32 * m * AP + 16 * s);
        alo[m] = *reinterpret_cast<const bf16x8*>(Ah + 32 * m * AP + AIMG + 16 * s);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = ((t / 3) * XW + 16 * s + (t % 3) * DIL) * 32;
        const bf16x8 bhi = tr_read8(Bh + off);
        const bf16x8 blo = tr_read8(Bh + BIMG + off);
#pragma unroll
        for (int m = 0; m < CPW; ++m) {
          acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[m], bhi, acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[m], blo, acc[m][t], 0, 0, 0);
          acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[m], bhi, acc[m][t], 0, 0, 0);
        }
      }
    }
  };

  if (c0 < c1) {
    load(c0);
    store(0);
    if (c0 + 1 < c1) load(c0 + 1);
    __syncthreads();
    int i = 0;
    for (int c = c0; c < c1; ++c, ++i) {
      compute(i & 1);
      if (c + 1 < c1) store((i + 1) & 1);
      if (c + 2 < c1) load(c + 2);
      __syncthreads();
    }
  }

  // partial sums of this partition: ws[p][tap][co][k] (lanes along k: coalesced)
  const int k = kt * NT + 32 * cb + l32;
  if (k < a.K) {
#pragma unroll
    for (int m = 0; m < CPW; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = ct * MT + 32 * (CPW * cw + m) + (r & 3) + 8 * (r >> 2) + 4 * kh;
          a.ws[(((int64_t)p * 9 + t) * a.Cout + co) * a.K + k] = acc[m][t][r];
        }
  }
}

// The same GEMM with LDS-DMA staging (split-bf16 x, 16-B aligned dy, W % 4 == 0): no staging
// registers, no split pass through VGPRs before the barrier.  Per chunk (32-pixel row
// segment) a buffer holds
//   A  dy[128 co][32 px] fp32 as DMA'd (8 x 16-B pieces per row, piece q of row r stored at
//      slot q ^ ((r >> 1) & 7): the fragment reads of 16 consecutive rows hit 64 distinct
//      banks); split into bf16 hi / lo at fragment-read time (the same rounding as split4) —
//      or, with dy pre-split by mvbev_split_rows_bf16 (MVBEV_LAYOUT_SPLIT_ROWS: per 8-pixel
//      run 16 B hi, 16 B lo, the same bytes per row), read as the fragments themselves: the
//      DMA and the reads are unchanged, the per-segment split is gone (conv1 at cfg2: 2.33 ->
//      2.22 ms + 35 us for the split pass; an ablation feeding unsplit bits ran 12 % faster, most
//      of which was the clock those operands allow, not the split's VALU);
//   B  the 3-row x window in the split slab's own order: per (32-channel half h, 8-channel
//      group g) a run [row][px][hi, lo] of 16-B pieces, so one DMA instruction copies ~1 KiB
//      of contiguous slab (16 pixels' hi + lo); run (h, g) starts at entry (4h + g) * GS +
//      (g & 1) + 8 (g >> 1), which puts the transposed reads of the 4 groups on distinct banks.
// Three buffers, one barrier per chunk: the wait before it retires this chunk's DMA (the next
// chunk's may stay in flight), the DMA after it refills the buffer read two chunks ago.
constexpr int WG_AENT = MT * PX / 4;  // A entries (16 B) per buffer: 1024
// Waves that issue the DMAs (8: all; 4: one per SIMD, the other wave of each SIMD starting its
// MFMAs at once while its partner queues the DMA pieces)
#ifndef MVBEV_WGRAD_DMAW
#define MVBEV_WGRAD_DMAW 8  // 4 measured equal (2.41 vs 2.42 ms) at 16 more VGPRs; 2: 3.45 ms
#endif
constexpr int WG_MAXC = 2048;         // chunk ids of a workgroup's partition, staged in LDS
template <int DIL, int ROWS = 3, int NH = 2> struct WgGeo {  // NH: 32-channel blocks of the window
  static constexpr int XW = PX + 2 * DIL, BPIX = ROWS * XW;
  static constexpr int RUN = 2 * BPIX;                      // entries of one (h, g) run
  static constexpr int GS = (RUN + 9 + 15) / 16 * 16;       // run stride (entries, 0 mod 16)
  static constexpr int BENT = 4 * NH * GS;
  static constexpr int DT = 64 * MVBEV_WGRAD_DMAW;         // DMA lanes (the first DMAW waves)
  static constexpr int NA = WG_AENT / DT;                   // A DMA instructions per DMA lane
  static constexpr int NB = (BENT + DT - 1) / DT;           // B DMA instructions per DMA lane
  static constexpr int BUFE = WG_AENT + NB * DT;            // entries per buffer (incl. tail)
  static_assert(WG_AENT % DT == 0, "A image must split evenly over the DMA lanes");
  static_assert(3 * BUFE * 16 + WG_MAXC * 4 <= 160 * 1024, "LDS");
};
__device__ u32x4 g_wg_zero[1];  // zero-initialised source of out-of-range entries

__device__ inline void wg_glds16(const void* src, u32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// LDS reads of a DMA-filled buffer as inline asm: for the builtins / plain loads the compiler
// drains every LDS-DMA in flight (vmcnt(0)) first, which would serialise the next chunks' DMA
// with this one's MFMAs.  The reads are ordered by explicit lgkmcnt(0) waits tied to the
// fragment registers (wg_lgkm_wait); the buffer's own DMA was retired before the barrier.
template <int OFF>
__device__ inline v4i16 wg_tr(uint32_t addr) {
  v4i16 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
// fragment registers tied after a wait: kept live (a read still in flight owns them) until it, and
// read only after it
template <int CB_> __device__ inline void wg_tie(v4i16 (&f)[CB_][4]) {
#pragma unroll
  for (int j = 0; j < CB_; ++j) asm volatile("" : "+v"(f[j][0]), "+v"(f[j][1]), "+v"(f[j][2]), "+v"(f[j][3]));
}
template <int CNT, int CB_> __device__ inline void wg_lgkm_wait(v4i16 (&f)[CB_][4]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(CNT));
  wg_tie(f);
}
__device__ inline bf16x8 wg_cat(v4i16 lo, v4i16 hi) {
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  const v8i16 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <typename F, int... U>
__device__ __attribute__((always_inline)) inline void wg_static_for(F& f, std::integer_sequence<int, U...>) {
  (f(std::integral_constant<int, U>{}), ...);
}
template <int B, int... U>
constexpr std::integer_sequence<int, (B + U)...> offset_seq(std::integer_sequence<int, U...>) {
  return {};
}

// WINO (conv1's weight gradient from the forward's row-Winograd transform, dilation 1): the same
// kernel over the transformed rows.  With the forward's y[3 r3 + j] = sum_xi AT[j][xi] (G w)_xi .
// T_xi[r3] (conv_bf16x3.hip, "Row-Winograd conv1"), per kernel column kw
//   dW[kh][kw] = sum_xi G[xi][kh] M_xi[kw],   M_xi[kw][co][ci] = sum_{b,r3,x} D_xi[co][r3][x] T_xi[ci][r3][x + kw - 1],
//   D_xi = sum_j AT[j][xi] dy[base(r3) + DIL j]   (wino_dy_rows_kernel, pre-split rows [B][5][Cout][R3][W];
//   base(r3) the forward's row tiles: 3 r3 for dilation 1, conv2's interleaved 12 (r3 / 4) + ring_base_row<2>
//   for dilation 2 — conv2's weight gradient from its T).
// A workgroup owns one xi and 128 input channels (desc group a multiple of 128 with chunk lists) (a wave: 32 Cout x 2 blocks of 32 channels, so
// each A fragment feeds both and a chunk carries twice the direct form's MFMAs per input channel
// block); its chunk is (b, r3, 32-px segment), the B window one T row (34 px of 128 channels, both
// split parts), 3 taps (kw), 6 steps of 2 x 3 MFMAs; a.H is R3 and a.x is T.  Per output row 5/3
// chunks of 1/3 the MFMAs: x0.556 of the direct form's.  wgrad_wino_reduce_kernel applies G while
// adding the partitions.
struct WinoT {
  int r5;         // T rows per (b, 8-channel block): 5 x 4 x tiles_y
};

template <int DIL, bool WINO = false>
__global__ __launch_bounds__(NTH, 1) void wgrad_dma_kernel(const WArgs a, const WinoT wt) {
  static_assert(NWV == 8, "wave layout: 4 output blocks x 2 channel halves");
  static_assert(!WINO || DIL == 1 || DIL == 2, "Winograd wgrad: dilation 1 or 2");
  constexpr int ROWS = WINO ? 1 : 3;      // window rows (taps kh)
  constexpr int NTAPS = 3 * ROWS;         // accumulators (kh, kw) / (kw)
  constexpr int NSTEP = 2 * NTAPS;        // (pixel step, tap) steps per chunk
  constexpr int CB = WINO ? 2 : 1;        // 32-channel blocks per wave
  constexpr int NTW = 64 * CB;            // input channels per workgroup
  using G = WgGeo<DIL, ROWS, 2 * CB>;
  constexpr int XW = G::XW, NA = G::NA, NB = G::NB, BUFE = G::BUFE, DT = G::DT;
  constexpr int DMAW = MVBEV_WGRAD_DMAW;
  __shared__ __attribute__((aligned(16))) u32x4 lds[3 * BUFE];
  __shared__ int cids[WG_MAXC];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, kh = lane >> 5;
  const int nt_all = a.ntiles * (WINO ? 5 : 1);
  const int lb = xcd_remap(blockIdx.x, a.P * nt_all);
  const int p = lb / nt_all, rem = lb - p * nt_all;
  const int xi = WINO ? rem / a.ntiles : 0, tile = rem - xi * a.ntiles;
  const int ct = tile % a.n_ct, kt = tile / a.n_ct;
  const int32_t* list = nullptr;
  int nact = a.nchunks;
  if (a.clist) {
    const int grp = (kt * NTW) / a.group;
    list = a.clist + a.coff[grp];
    nact = a.coff[grp + 1] - a.coff[grp];
  }
  const int c0 = (int)((int64_t)nact * p / a.P);
  const int c1 = (int)((int64_t)nact * (p + 1) / a.P);
  const int W = a.W, H = a.H;
  const int64_t plane = (int64_t)H * W;
  const u32x4* xs = static_cast<const u32x4*>(a.x);

  // LDS-DMA sources.  DMA lane's j-th instruction covers entry (j * DMAW + wave) * 64 + lane; the
  // chunk-invariant part of each source (channel / Cout row, window pixel) is an offset from the
  // chunk's origin, formed once, so an issue is a few adds, two range checks and a select per
  // instruction (formed per chunk, the divisions and 64-bit products cost about as many
  // cycles as the chunk's MFMAs).  A entry: dy row `row` (Cout), piece q (4 px, swizzled slot).
  int aofs[NA], acol[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int e = (j * DMAW + wave) * 64 + lane;
    const int row = e >> 3, q = (e & 7) ^ ((row >> 1) & 7);
    aofs[j] = (ct * MT + row) * (int)plane + 4 * q;
    acol[j] = 4 * q;
  }
  // B entry: run (h, g4), then (row r, window pixel cc, part); bdx = INT_MIN / 2 marks a zero
  // entry (run padding, channel past K): x0 + bdx then fails the column check
  int bofs[NB], bdy[NB], bdx[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int e = (j * DMAW + wave) * 64 + lane;
    const int hg = e / G::GS, g4 = hg & 3;
    const int q = e - hg * G::GS - ((g4 & 1) + 8 * (g4 >> 1));
    const int k0 = kt * NTW + (hg >> 2) * 32 + g4 * 8;
    const bool ok = hg < 8 * CB && q >= 0 && q < G::RUN && k0 < a.K;
    const int qc = ok ? q : 0, kc = ok ? k0 : 0;
    const int pix = qc >> 1, r = pix / XW, cc = pix - r * XW;
    bdx[j] = ok ? cc - DIL : INT_MIN / 2;
    if constexpr (WINO) {  // T block kc / 8: its row's hi plane [W], then its lo plane
      bdy[j] = 0;
      bofs[j] = (kc / 8) * (2 * wt.r5 * W) + (qc & 1) * W + cc - DIL;
    } else {
      const int g_ = kc / a.group;
      const int64_t cbase = g_ * a.group_stride + (int64_t)(kc - g_ * a.group) * plane;
      bdy[j] = (r - 1) * DIL;
      bofs[j] = (int)(cbase / 4) + 2 * (bdy[j] * W + cc - DIL) + (qc & 1);
    }
  }
  // chunk pk (packed b << 24 | y << 12 | seg, see the staging below) into buffer bb
  struct IssueCtx {
    const float* abase;
    const u32x4* bbase;
    u32x4* dst;
    int y, x0;
  };
  auto issue_prep = [&](int pk, int bb) __attribute__((always_inline)) {
    IssueCtx c;
    const int b = pk >> 24;
    c.y = (pk >> 12) & 4095;
    c.x0 = (pk & 4095) * PX;
    if constexpr (WINO) {  // D_xi rows [b][xi][co][r3]; T row 5 r3 + xi of batch b
      c.abase = a.dy + (((int64_t)b * 5 + xi) * a.Cout * H + c.y) * W + c.x0;
      c.bbase = xs + (int64_t)b * (a.K / 8) * (2 * (int64_t)wt.r5 * W) + 2 * (5 * c.y + xi) * W + c.x0;
    } else {
      c.abase = a.dy + ((int64_t)b * a.Cout * H + c.y) * W + c.x0;
      c.bbase = xs + (int64_t)b * (a.batch_stride / 4) + 2 * (c.y * W + c.x0);
    }
    c.dst = lds + bb * BUFE + wave * 64;
    return c;
  };
  auto issue_one = [&](const IssueCtx& c, auto j_) __attribute__((always_inline)) {
    constexpr int j = decltype(j_)::value;
    if (DMAW < NWV && wave >= DMAW) return;
    if constexpr (j < NA) {
      const bool ok = c.x0 + acol[j] < W;
      wg_glds16(ok ? (const void*)(c.abase + aofs[j]) : (const void*)g_wg_zero, c.dst + j * DT);
    } else {
      constexpr int jb = j - NA;
      const bool ok = (unsigned)(c.y + bdy[jb]) < (unsigned)H && (unsigned)(c.x0 + bdx[jb]) < (unsigned)W;
      const u32x4* bsrc = c.bbase + bofs[jb];
      wg_glds16(ok ? (const void*)bsrc : (const void*)g_wg_zero, c.dst + WG_AENT + jb * DT);
    }
  };
  auto issue = [&](int pk, int bb) __attribute__((always_inline)) {
    const IssueCtx c = issue_prep(pk, bb);
    auto one = [&](auto j_) __attribute__((always_inline)) { issue_one(c, j_); };
    wg_static_for(one, std::make_integer_sequence<int, NA + NB>{});
  };

  const int cw = wave & 3, cb = wave >> 2;
  const int gi = (lane >> 4) & 1, li = lane & 15;
  // transposed-read lane: pixel 8 kh + li / 4 (+ 4 for the second read), channels 16 gi + 4 (li & 3)
  // .. + 3 of the wave's half = group g = 2 gi + (li & 3) / 2, offset 4 (li & 1) in the piece
  const int trg = 2 * gi + ((li & 3) >> 1);
  const int tr0 = 16 * ((cb * CB * 4 + trg) * G::GS + (trg & 1) + 8 * (trg >> 1) + 2 * (8 * kh + (li >> 2))) +
                  8 * (li & 1);  // bytes; the wave's block j at + 64 j GS bytes
  const int arow = 32 * cw + l32, asw = (arow >> 1) & 7;
  floatx16 acc[CB][NTAPS];
#pragma unroll
  for (int j = 0; j < CB; ++j)
#pragma unroll
    for (int t = 0; t < NTAPS; ++t) acc[j][t] = floatx16{0};

  // Per chunk 18 (pixel step s, tap t) steps of 3 MFMAs.  Step u+2's 4 transposed reads go out
  // under step u's MFMAs and lgkmcnt(4) then retires step u+1's (in-order LDS returns; no
  // scalar loads are in flight inside the loop; one step ahead measured slower, 3.03 vs 2.93
  // ms).  Measured no faster: running a chunk's last two steps after the next barrier, under
  // the next chunk's first reads (2.47 vs 2.45 ms).
  // full = false: a last row segment with at most 16 pixels left; its second pixel step would
  // multiply zeros and is skipped (the reads it prefetched are drained by the next wait).
  floatx4 av[4];
  bf16x8 ahi[2], alo[2];
  v4i16 fr[3][CB][4];
  uint32_t bb0 = 0;
  auto read = [&](auto u_) __attribute__((always_inline)) {
    constexpr int u = decltype(u_)::value, s = u / NTAPS, t = u % NTAPS;
    constexpr int set = u % 3;
    constexpr int off = ((t / 3) * XW + 16 * s + (t % 3) * DIL) * 32;  // bytes (32 per pixel)
    constexpr int jb = 64 * G::GS;                                      // bytes between 32-channel blocks
    fr[set][0][0] = wg_tr<off>(bb0);
    fr[set][0][1] = wg_tr<off + 128>(bb0);
    fr[set][0][2] = wg_tr<off + 16>(bb0);
    fr[set][0][3] = wg_tr<off + 16 + 128>(bb0);
    if constexpr (CB == 2) {
      fr[set][1][0] = wg_tr<jb + off>(bb0);
      fr[set][1][1] = wg_tr<jb + off + 128>(bb0);
      fr[set][1][2] = wg_tr<jb + off + 16>(bb0);
      fr[set][1][3] = wg_tr<jb + off + 16 + 128>(bb0);
    }
  };
  auto mfma3 = [&](int t, bf16x8 ah, bf16x8 al, const v4i16 (&f)[CB][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const bf16x8 bhi = wg_cat(f[j][0], f[j][1]), blo = wg_cat(f[j][2], f[j][3]);
      acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bhi, acc[j][t], 0, 0, 0);
      acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, blo, acc[j][t], 0, 0, 0);
      acc[j][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bhi, acc[j][t], 0, 0, 0);
    }
  };
  // chunk in buffer bb: the A fragments and steps 0, 1's B fragments
  auto head_reads = [&](int bb) __attribute__((always_inline)) {
    const u32x4* L = lds + bb * BUFE;
    bb0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(L + WG_AENT) + (uint32_t)tr0;
    const uint32_t ab = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(
        reinterpret_cast<const floatx4*>(L) + arow * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t addr = ab + 16u * (uint32_t)((4 * (q >> 1) + 2 * kh + (q & 1)) ^ asw);
      asm volatile("ds_read_b128 %0, %1" : "=v"(av[q]) : "v"(addr));
    }
    read(std::integral_constant<int, 0>{});
    read(std::integral_constant<int, 1>{});
  };
  auto body = [&](bool full) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]));
    wg_tie(fr[0]);
    wg_tie(fr[1]);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const floatx4 v0 = av[2 * s], v1 = av[2 * s + 1];
      if (a.dy_rows) {  // pre-split rows: the 8-pixel run's hi piece, then its lo piece
        ahi[s] = __builtin_bit_cast(bf16x8, v0);
        alo[s] = __builtin_bit_cast(bf16x8, v1);
        continue;
      }
      u32x2 h0, l0, h1, l1;
      split4(v0, h0, l0);
      split4(v1, h1, l1);
      const u32x4 hh = {h0[0], h0[1], h1[0], h1[1]}, ll = {l0[0], l0[1], l1[0], l1[1]};
      ahi[s] = __builtin_bit_cast(bf16x8, hh);
      alo[s] = __builtin_bit_cast(bf16x8, ll);
    }
    auto step = [&](auto u_) __attribute__((always_inline)) {
      constexpr int u = decltype(u_)::value, s = u / NTAPS, t = u % NTAPS;
      constexpr int set = u % 3, nset = (u + 1) % 3;
      if constexpr (u + 2 < NSTEP) read(std::integral_constant<int, u + 2>{});
      mfma3(t, ahi[s], alo[s], fr[set]);
      if constexpr (u + 2 < NSTEP) {
        wg_lgkm_wait<4 * CB>(fr[nset]);
      } else if constexpr (u + 1 < NSTEP) {
        wg_lgkm_wait<0>(fr[nset]);
      }
    };
    wg_static_for(step, std::make_integer_sequence<int, NTAPS>{});
    if (full) wg_static_for(step, offset_seq<NTAPS>(std::make_integer_sequence<int, NTAPS>{}));
  };

  // the partition's chunk ids, staged in LDS before any DMA (a global load of the list inside
  // the loop would be waited for with vmcnt(0), draining the DMAs in flight)
  const int n = c1 - c0;
  for (int j = tid; j < n; j += NTH) {
    const int c = list ? list[c0 + j] : c0 + j;
    const int R = c / a.segs, seg = c - R * a.segs;
    const int b = R / H;
    cids[j] = (b << 24) | ((R - b * H) << 12) | seg;  // host: B < 128, H, segs <= 4096
  }
  __syncthreads();
  if (n > 0) {
    issue(cids[0], 0);
    if (n > 1) issue(cids[1], 1);
    for (int i = 0; i < n; ++i) {
      // retire chunk i's DMA (chunk i+1's may stay in flight) and every LDS read of chunk i-1
      // (fragment registers tied: a partial chunk's skipped reads must land before reuse)
      if (i + 1 < n) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NA + NB) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      wg_tie(fr[0]);
      wg_tie(fr[1]);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // (measured no faster: the pieces one after each of the first steps' MFMAs, 2.30 ms both)
      if (i + 2 < n) issue(cids[i + 2], (i + 2) % 3);
      const bool full = (cids[i] & 4095) * PX + 16 < W;
      head_reads(i % 3);
      body(full);
    }
  }

  constexpr int NOUT = WINO ? 15 : 9;  // ws taps: (xi, kw) / (kh, kw)
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int k = kt * NTW + 32 * (cb * CB + j) + l32;
    if (k >= a.K) continue;
#pragma unroll
    for (int t = 0; t < NTAPS; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = ct * MT + 32 * cw + (r & 3) + 8 * (r >> 2) + 4 * kh;
        a.ws[(((int64_t)p * NOUT + xi * 3 + t) * a.Cout + co) * a.K + k] = acc[j][t][r];
      }
  }
}

// dw[co][map(k)][t] = sum_p ws[p][t][co][k]  (partition order: deterministic).  One block per
// (co, 64 channels): the 9 x 64 sums are read along k (coalesced), transposed through LDS and
// written along (k, t), the weight's own order (contiguous wherever the channel map is).
constexpr int kWrK = 64, kWrThreads = 192;  // 9 * 64 = 3 * 192 sums per block
__global__ __launch_bounds__(kWrThreads) void wgrad_reduce_kernel(const float* __restrict__ ws, int P, int Cout, int K,
                                                              const int32_t* __restrict__ chan_map, int Cin_w,
                                                              float* __restrict__ dw) {
  __shared__ float sums[9 * kWrK];
  const int co = blockIdx.y, k0 = blockIdx.x * kWrK;
  const int64_t pstride = (int64_t)9 * Cout * K;
  float v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int i = threadIdx.x + j * kWrThreads, t = i / kWrK, k = k0 + i % kWrK;
    float s = 0.f;
    if (k < K) {
      const float* src = ws + ((int64_t)t * Cout + co) * K + k;
      int q = 0;
      for (; q + 8 <= P; q += 8) {  // loads issued together, added in partition order
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = src[(q + u) * pstride];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += x[u];
      }
      for (; q < P; ++q) s += src[q * pstride];
    }
    v[j] = s;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int i = threadIdx.x + j * kWrThreads;
    sums[(i % kWrK) * 9 + i / kWrK] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int i = threadIdx.x + j * kWrThreads, kk = i / 9, t = i - kk * 9, k = k0 + kk;
    if (k >= K) continue;
    const int cm = chan_map ? chan_map[k] : k;
    if (cm < 0 || cm >= Cin_w) continue;
    dw[((int64_t)co * Cin_w + cm) * 9 + t] = sums[i];
  }
}

// Winograd form: M[xi][kw] = sum_p ws[p][3 xi + kw][co][k] (partition order), then
// dw[co][map(k)][kh][kw] = sum_xi G[xi][kh] M[xi][kw] in double (G of pack_wino_kernel), rounded once.
constexpr int kWinoRedThreads = 320;  // 15 * 64 = 3 * 320 sums per block
__global__ __launch_bounds__(kWinoRedThreads) void wgrad_wino_reduce_kernel(const float* __restrict__ ws, int P, int Cout,
                                                                   int K, const int32_t* __restrict__ chan_map,
                                                                   int Cin_w, float* __restrict__ dw) {
  __shared__ float sums[15 * kWrK];
  const int co = blockIdx.y, k0 = blockIdx.x * kWrK;
  const int64_t pstride = (int64_t)15 * Cout * K;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int i = threadIdx.x + j * kWinoRedThreads, t = i / kWrK, k = k0 + i % kWrK;
    float s = 0.f;
    if (k < K) {
      const float* src = ws + ((int64_t)t * Cout + co) * K + k;
      int q = 0;
      for (; q + 4 <= P; q += 4) {
        float x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = src[(q + u) * pstride];
#pragma unroll
        for (int u = 0; u < 4; ++u) s += x[u];
      }
      for (; q < P; ++q) s += src[q * pstride];
    }
    sums[(i % kWrK) * 15 + t] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 9 * kWrK; i += kWinoRedThreads) {
    const int kk = i / 9, tap = i - kk * 9, kh = tap / 3, kw = tap - kh * 3, k = k0 + kk;
    if (k >= K) continue;
    const int cm = chan_map ? chan_map[k] : k;
    if (cm < 0 || cm >= Cin_w) continue;
    const float* m = sums + kk * 15 + kw;  // m[3 xi]
    const double m0 = m[0], m1 = m[3], m2 = m[6], m3 = m[9], m4 = m[12];
    const double v = kh == 0 ? 0.5 * (m0 - m1) + (m3 - m2) / 6.0
                   : kh == 1 ? -0.5 * m1 + (m2 + 2.0 * m3) / 6.0
                             : -0.5 * m1 + (4.0 * m3 - m2) / 6.0 + m4;
    dw[((int64_t)co * Cin_w + cm) * 9 + tap] = (float)v;
  }
}

// D[b][xi][co][r3] = split(sum_j AT[j][xi] dy[b][co][base(r3) + dil j]) in MVBEV_LAYOUT_SPLIT_ROWS (rows
// past H are zero), AT = [1 1 1 1 0; 0 1 -1 2 0; 0 1 1 4 1]: a thread per (b, co, r3, 8-pixel run).
__global__ __launch_bounds__(256) void wino_dy_rows_kernel(const floatx4* __restrict__ dy, int B, int Cout, int H,
                                                           int W, int R3, int dil, u32x4_t* __restrict__ out) {
  const int runs = W / 8;
  const int64_t n = (int64_t)B * Cout * R3 * runs;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int run = (int)(i % runs);
  int64_t r = i / runs;
  const int r3 = (int)(r % R3);
  r /= R3;
  const int co = (int)(r % Cout), b = (int)(r / Cout);
  float d[3][8];
  const int q = r3 & 3, base = dil == 1 ? 3 * r3 : 12 * (r3 >> 2) + (q >> 1) * 6 + (q & 1);  // ring_base_row<2>
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int y = base + dil * j;
    floatx4 v0 = floatx4{0.f, 0.f, 0.f, 0.f}, v1 = v0;
    if (y < H) {
      const floatx4* src = dy + ((((int64_t)b * Cout + co) * H + y) * W) / 4 + 2 * run;
      v0 = src[0];
      v1 = src[1];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) d[j][e] = v0[e], d[j][4 + e] = v1[e];
  }
  const int64_t plane = (int64_t)Cout * R3 * runs;  // runs per xi of one batch
  u32x4_t* o = out + 2 * (((int64_t)b * 5 * Cout + co) * R3 * runs + (int64_t)r3 * runs + run);
#pragma unroll
  for (int x = 0; x < 5; ++x) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a0 = d[0][e], a1 = d[1][e], a2 = d[2][e];
      v[e] = x == 0 ? a0 : x == 1 ? a0 + a1 + a2 : x == 2 ? a0 - a1 + a2 : x == 3 ? a0 + 2.f * a1 + 4.f * a2 : a2;
    }
    store_split8(o + 2 * (int64_t)x * plane, v);
  }
}

// ---------------------------------------------------------------------------------------------
// block-wide sum of NV values per thread (NWV waves), result valid in thread 0; fixed order
template <int NV, int NWV_>
__device__ inline void block_sum(float (&v)[NV], float* red /* LDS [NWV_][NV] */) {
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[j] += __shfl_xor(v[j], o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) red[wave * NV + j] = v[j];
  __syncthreads();
  // thread j < NV sums column j over the waves (thread 0 summing all NV x NWV_ values had the
  // compiler hoist every LDS load: 300+ registers and scratch spills at NV = 19)
  if (threadIdx.x < NV) {
    float t = 0.f;
    for (int w = 0; w < NWV_; ++w) t += red[w * NV + threadIdx.x];
    red[threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = red[j];
}

// The per-channel reductions below (one workgroup per output channel, 512 of them at the
// reference's widths) use 1024-thread workgroups so each CU holds 16+ waves of independent
// streaming loads; the coord values come from LDS tables (create_coord_map's float64
// formula, cast to fp32, evaluated once per row / column instead of per tap).
constexpr int kRedThreads = 1024;
constexpr int kRedWaves = kRedThreads / 64;
constexpr int kCoordTab = 4096;  // max H, W for the coord tables (larger grids: no dw)

// db[co] = sum dy[b][co][:]; with dw, the two coord channels (create_coord_map,
// persp_trans_detector.py:103-112, channels coord_ch and coord_ch + 1 of the conv input):
// dw[co][coord_ch + j][t] = sum_p dy[co][p] * coord_j(p + s_t), zero outside the grid.
__global__ __launch_bounds__(kRedThreads) void bias_coord_grad_kernel(const float* __restrict__ dy, int B, int Cout,
                                                                      int H, int W, int dil, float* db, float* dw,
                                                                      int Cin_w, int coord_ch) {
  __shared__ float red[kRedWaves * 19];
  __shared__ float tcx[kCoordTab], tcy[kCoordTab];
  const int co = blockIdx.x;
  if (dw) {
    for (int i = threadIdx.x; i < W; i += kRedThreads) tcx[i] = (float)((double)i / (double)(W - 1) * 2.0 - 1.0);
    for (int i = threadIdx.x; i < H; i += kRedThreads) tcy[i] = (float)((double)i / (double)(H - 1) * 2.0 - 1.0);
    __syncthreads();
  }
  float v[19];
#pragma unroll
  for (int j = 0; j < 19; ++j) v[j] = 0.f;
  const int HW = H * W;
  for (int b = 0; b < B; ++b) {
    const float* g = dy + ((int64_t)b * Cout + co) * HW;
    if (!dw) {
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
      int q = threadIdx.x;
      for (; q + 3 * kRedThreads < HW; q += 4 * kRedThreads)
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] += g[q + u * kRedThreads];
      for (; q < HW; q += kRedThreads) a4[0] += g[q];
      v[0] += (a4[0] + a4[1]) + (a4[2] + a4[3]);
      continue;
    }
    // separable form: per row y, Rx[kx] = sum_x dy cx(x + (kx - 1) dil) and Sx[kx] = sum_x dy [x + (kx - 1)
    // dil inside] (a wave per row, lanes along x, 4 loads in flight per lane), then
    //   dw_x[ky][kx] += [y + (ky - 1) dil inside] Rx[kx],  dw_y[ky][kx] += cy(y + (ky - 1) dil) Sx[kx]
    // (a thread per pixel accumulating the 19 sums with their bounds took 0.13 ms at cfg2)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll 1
    for (int y = wave; y < H; y += kRedWaves) {
      const float* row = g + (int64_t)y * W;
      float rx[3] = {0.f, 0.f, 0.f}, sx[3] = {0.f, 0.f, 0.f};
#pragma unroll 1
      for (int x0 = 0; x0 < W; x0 += 4 * 64) {
        float gv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int x = x0 + 64 * u + lane;
          gv[u] = x < W ? row[x] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int x = x0 + 64 * u + lane;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int xx = x + (k - 1) * dil;
            const bool okx = xx >= 0 && xx < W;
            rx[k] += okx ? gv[u] * tcx[okx ? xx : 0] : 0.f;
            sx[k] += okx ? gv[u] : 0.f;
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          rx[k] += __shfl_xor(rx[k], o);
          sx[k] += __shfl_xor(sx[k], o);
        }
      v[0] += sx[1];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int yy = y + (ky - 1) * dil;
        const bool oky = yy >= 0 && yy < H;
        const float cy = oky ? tcy[oky ? yy : 0] : 0.f;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          v[1 + 3 * ky + kx] += oky ? rx[kx] : 0.f;
          v[10 + 3 * ky + kx] += cy * sx[kx];
        }
      }
    }
  }
  if (dw && (threadIdx.x & 63) != 0) {  // every lane of a wave holds its sums: count them once
#pragma unroll
    for (int j = 0; j < 19; ++j) v[j] = 0.f;
  }
  block_sum<19, kRedWaves>(v, red);
  if (threadIdx.x == 0) {
    if (db) db[co] = v[0];
    if (dw)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        dw[((int64_t)co * Cin_w + coord_ch) * 9 + t] = v[1 + t];
        dw[((int64_t)co * Cin_w + coord_ch + 1) * 9 + t] = v[10 + t];
      }
  }
}

// torch threshold_backward(grad, relu_output, 0): grad where the ReLU output > 0, else 0
__global__ void relu_backward_kernel(float* __restrict__ dy, const float* __restrict__ y, int64_t n) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    floatx4 g = *reinterpret_cast<const floatx4*>(dy + i);
    const floatx4 v = *reinterpret_cast<const floatx4*>(y + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = v[j] > 0.f ? g[j] : 0.f;
    *reinterpret_cast<floatx4*>(dy + i) = g;
  } else {
    for (int64_t j = i; j < n; ++j) dy[j] = y[j] > 0.f ? dy[j] : 0.f;
  }
}

// dy (fp32 [B][C][HW]) *= [y > 0] with the ReLU output y in the split-bf16 layout
// ([B][C/8][HW] pieces of bf16 hi[8], lo[8]; y = hi + lo); dys (optional) also receives the
// masked dy in the split layout, the input of the next data-gradient conv (ring kernel).
__global__ void relu_backward_split_kernel(float* __restrict__ dy, const u32x4_t* __restrict__ y, int C, int64_t HW,
                                           u32x4_t* __restrict__ dys) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int g = blockIdx.y, b = blockIdx.z, G = C / 8;
  if (p >= HW) return;
  const int64_t e = ((int64_t)b * G + g) * HW + p;
  const bf16x8_t hi = __builtin_bit_cast(bf16x8_t, y[2 * e]), lo = __builtin_bit_cast(bf16x8_t, y[2 * e + 1]);
  float* d = dy + ((int64_t)b * C + 8 * g) * HW + p;
  float v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float yv = (float)hi[c] + (float)lo[c];
    v[c] = yv > 0.f ? d[c * HW] : 0.f;
    d[c * HW] = v[c];
  }
  if (dys) store_split8(dys + 2 * e, v);
}

// conv3 (Cout = 1, no bias) data gradient, times conv2's ReLU mask when relu_mask:
// dx[b][c][y][x] = sum_t w[c][t] * dmap[b][y - (ky-1)d][x - (kx-1)d]
constexpr int kCout1Cpb = 32;  // channels per block
// dxs (optional, C % 8 == 0): dx also in the split-bf16 layout (the next dgrad conv's input)
__global__ __launch_bounds__(256) void cout1_dgrad_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ dmap, int C, int H, int W,
                                                          int dil, int relu_mask, float* __restrict__ dx,
                                                          u32x4_t* __restrict__ dxs) {
  const int HW = H * W;
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.z;
  if (q >= HW) return;
  const int y = q / W, xx = q - y * W;
  float dm[9];
  const float* d = dmap + (int64_t)b * HW;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = y - (t / 3 - 1) * dil, xc = xx - (t % 3 - 1) * dil;
    dm[t] = (yy >= 0 && yy < H && xc >= 0 && xc < W) ? d[yy * W + xc] : 0.f;
  }
  const int cbeg = blockIdx.y * kCout1Cpb, cend = min(C, cbeg + kCout1Cpb);
  if (dxs) {  // groups of 8 channels (kCout1Cpb and C are multiples of 8)
    for (int c0 = cbeg; c0 < cend; c0 += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) s += w[c * 9 + t] * dm[t];
        const int64_t o = ((int64_t)b * C + c) * HW + q;
        v[j] = (!relu_mask || x[o] > 0.f) ? s : 0.f;
        dx[o] = v[j];
      }
      store_split8(dxs + 2 * (((int64_t)b * (C / 8) + c0 / 8) * HW + q), v);
    }
    return;
  }
  for (int c = cbeg; c < cend; ++c) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) s += w[c * 9 + t] * dm[t];
    const int64_t o = ((int64_t)b * C + c) * HW + q;
    dx[o] = (!relu_mask || x[o] > 0.f) ? s : 0.f;
  }
}

// conv3 weight gradient: dw[c][t] = sum_b sum_q x[b][c][q] * dmap[b][q - s_t]
__global__ __launch_bounds__(kRedThreads) void cout1_wgrad_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ dmap, int B, int C, int H,
                                                                  int W, int dil, float* __restrict__ dw) {
  __shared__ float red[kRedWaves * 9];
  const int c = blockIdx.x;
  const int HW = H * W;
  float v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) v[t] = 0.f;
  // pixels in batches of kC1U per thread: the batch's x and shifted-dmap loads are all issued
  // before the first product (one load in flight per thread and tap measured 0.25 ms at cfg2:
  // latency-bound at 2 workgroups per CU)
  constexpr int kC1U = 4;
  for (int b = 0; b < B; ++b) {
    const float* xc = x + ((int64_t)b * C + c) * HW;
    const float* d = dmap + (int64_t)b * HW;
    for (int q0 = threadIdx.x; q0 < HW; q0 += kC1U * kRedThreads) {
      float xv[kC1U], dv[kC1U][9];
#pragma unroll
      for (int u = 0; u < kC1U; ++u) {
        const int q = q0 + u * kRedThreads;
        const bool ok = q < HW;
        const int y = ok ? q / W : -H - 8 * dil, xx = ok ? q - y * W : 0;
        xv[u] = ok ? xc[q] : 0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int yy = y - (t / 3 - 1) * dil, xs = xx - (t % 3 - 1) * dil;
          dv[u][t] = (yy >= 0 && yy < H && xs >= 0 && xs < W) ? d[yy * W + xs] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kC1U; ++u)
#pragma unroll
        for (int t = 0; t < 9; ++t) v[t] += xv[u] * dv[u][t];
    }
  }
  block_sum<9, kRedWaves>(v, red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int t = 0; t < 9; ++t) dw[c * 9 + t] = v[t];
}

// ---------------------------------------------------------------------------------------------
// Warp adjoint: per output pixel (one thread) the forward's coordinates, corners and weights,
// then for every channel of the block's slice 4 atomic adds into the source gradient.  No
// gradient flows from a pixel whose sample point is outside (zero padding) or non-finite.
// WarpView here: src = grad_out ([B][C][Ho][Wo], strides sB..sW), dst = grad_src (dB, dC, dH, 1).
constexpr int kBwTH = 16, kBwTW = 16, kBwWR = 4, kBwCPB = 64;  // tiling of the atomic adjoint
__global__ __launch_bounds__(256) void warp_backward_kernel(const WarpArgs a) {
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int tile = lb % a.tiles;
  const int chunk = (lb / a.tiles) % a.chunks;
  const int bv = lb / (a.tiles * a.chunks);
  const int view = bv % a.nviews;
  const int b = bv / a.nviews;
  const WarpView& vw = a.v[view];
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  constexpr int WC = 64 / kBwWR, WAVES_X = kBwTW / WC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = ty * kBwTH + (wave / WAVES_X) * kBwWR + lane / WC;
  const int u = tx * kBwTW + (wave % WAVES_X) * WC + lane % WC;
  if (v >= a.Ho || u >= a.Wo) return;
  const int H = a.H, W = a.W;
  float m[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = vw.m[i];
  const WarpCoord wc = warp_coord(m, u, v, a.Ho, a.Wo, H, W);
  if (!wc.inside) return;
  const float ix = wc.ix, iy = wc.iy;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  const float w_nw = (fx1 - ix) * (fy1 - iy);
  const float w_ne = (ix - fx0) * (fy1 - iy);
  const float w_sw = (fx1 - ix) * (iy - fy0);
  const float w_se = (ix - fx0) * (iy - fy0);
  const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= H - 1;
  const bool ok_nw = vx0 && vy0, ok_ne = vx1 && vy0, ok_sw = vx0 && vy1, ok_se = vx1 && vy1;
  const int64_t o_nw = (int64_t)y0 * vw.dH + x0;
  const int64_t o_sw = o_nw + vw.dH;
  const float* go = static_cast<const float*>(vw.src) + (int64_t)b * vw.sB + (int64_t)v * vw.sH +
                    (int64_t)u * vw.sW;
  float* gs = static_cast<float*>(vw.dst) + (int64_t)b * vw.dB;
  const int c_begin = chunk * kBwCPB;
  const int c_end = min(a.C, c_begin + kBwCPB);
  constexpr int U = 4;
  int c = c_begin;
  auto scatter = [&](int ch, float g) __attribute__((always_inline)) {
    if (g == 0.f) return;  // adds nothing (a NaN/inf gradient still propagates)
    float* pc = gs + (int64_t)ch * vw.dC;
    if (ok_nw) unsafeAtomicAdd(pc + o_nw, w_nw * g);
    if (ok_ne) unsafeAtomicAdd(pc + o_nw + 1, w_ne * g);
    if (ok_sw) unsafeAtomicAdd(pc + o_sw, w_sw * g);
    if (ok_se) unsafeAtomicAdd(pc + o_sw + 1, w_se * g);
  };
  for (; c + U <= c_end; c += U) {
    float g[U];
#pragma unroll
    for (int k = 0; k < U; ++k) g[k] = go[(int64_t)(c + k) * vw.sC];
#pragma unroll
    for (int k = 0; k < U; ++k) scatter(c + k, g[k]);
  }
  for (; c < c_end; ++c) scatter(c, go[(int64_t)c * vw.sC]);
}


// ---------------------------------------------------------------------------------------------
// Warp adjoint as a gather (no atomics in the hot loop).  The bilinear warp is a sparse matrix
// S (Ho*Wo x H*W, <= 4 entries per row: the in-bounds corners of the sample, weights from the
// forward's own fp32 coordinate code); its adjoint grad_src = S^T grad_out is a CSR gather
// over S^T built once per geometry (the plan):
//   row_ptr[H*W + 1], col[] = output pixel, val[] = corner weight, entries of one source pixel
//   in increasing output-pixel order (deterministic summation order).
// Build: count (int atomics) -> single-workgroup exclusive scan -> fill (atomic cursor) ->
// per-segment insertion sort by output pixel.  Geometry only, so it runs once per view.

struct Corners {
  int idx[4];    // source pixel (y * W + x) or -1
  float w[4];
};
__device__ inline Corners warp_corners(const float (&m)[9], int u, int v, int Ho, int Wo, int H, int W) {
  Corners k;
  const WarpCoord wc = warp_coord(m, u, v, Ho, Wo, H, W);
#pragma unroll
  for (int i = 0; i < 4; ++i) k.idx[i] = -1, k.w[i] = 0.f;
  if (!wc.inside) return k;
  const float ix = wc.ix, iy = wc.iy;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  k.w[0] = (fx1 - ix) * (fy1 - iy);
  k.w[1] = (ix - fx0) * (fy1 - iy);
  k.w[2] = (fx1 - ix) * (iy - fy0);
  k.w[3] = (ix - fx0) * (iy - fy0);
  const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= H - 1;
  if (vx0 && vy0) k.idx[0] = y0 * W + x0;
  if (vx1 && vy0) k.idx[1] = y0 * W + x0 + 1;
  if (vx0 && vy1) k.idx[2] = (y0 + 1) * W + x0;
  if (vx1 && vy1) k.idx[3] = (y0 + 1) * W + x0 + 1;
  return k;
}

struct PlanArgs {
  float m[9];
  int H, W, Ho, Wo;
};

__global__ __launch_bounds__(256) void adj_count_kernel(const PlanArgs a, int32_t* __restrict__ counts) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= a.Ho * a.Wo) return;
  const Corners k = warp_corners(a.m, o % a.Wo, o / a.Wo, a.Ho, a.Wo, a.H, a.W);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (k.idx[i] >= 0) atomicAdd(counts + k.idx[i], 1);
}

// row_ptr[i] = sum counts[0..i), row_ptr[n] = total; also cursor[i] = row_ptr[i].  One
// workgroup of 1024 threads walks the array in 1024-element pieces (setup-time only).
__global__ __launch_bounds__(1024) void adj_scan_kernel(const int32_t* __restrict__ counts, int n,
                                                        int32_t* __restrict__ row_ptr, int32_t* __restrict__ cursor) {
  __shared__ int32_t part[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const int32_t c = i < n ? counts[i] : 0;
    part[threadIdx.x] = c;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
      const int32_t t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    const int32_t excl = carry + part[threadIdx.x] - c;
    if (i < n) row_ptr[i] = excl, cursor[i] = excl;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) row_ptr[n] = carry;
}

__global__ __launch_bounds__(256) void adj_fill_kernel(const PlanArgs a, int32_t* __restrict__ cursor,
                                                       int32_t* __restrict__ col, float* __restrict__ val) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= a.Ho * a.Wo) return;
  const Corners k = warp_corners(a.m, o % a.Wo, o / a.Wo, a.Ho, a.Wo, a.H, a.W);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (k.idx[i] >= 0) {
      const int pos = atomicAdd(cursor + k.idx[i], 1);
      col[pos] = o;
      val[pos] = k.w[i];
    }
}

// The same plan for the fused upsample + warp (warp_up_kernel): S_up = S * U (Ho*Wo x h*w, U the
// 3x bilinear upsample of persp_trans_detector.py:65), <= 9 entries per output pixel: the
// sample's 3x3 backbone window with weights ay[i] * ax[j] (up_window, the forward's own
// code); zero-weight window cells carry no entry.  Its adjoint takes the gradient straight to
// the backbone-resolution features, without the upsampled gradient in HBM.
struct UpPlanArgs {
  float m[9];
  int H, W, Ho, Wo, h, w;
  float sy, sx;
};
template <bool FILL>
__global__ __launch_bounds__(256) void adj_up_kernel(const UpPlanArgs a, int32_t* __restrict__ counts,
                                                     int32_t* __restrict__ col, float* __restrict__ val) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= a.Ho * a.Wo) return;
  const UpWindow uw = up_window(a.m, o % a.Wo, o / a.Wo, a.Ho, a.Wo, a.H, a.W, a.h, a.w, a.sy, a.sx);
  if (!uw.inside) return;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float wt = uw.ay[i] * uw.ax[j];
      if (wt == 0.f || uw.rb + i > a.h - 1 || uw.cb + j > a.w - 1) continue;
      const int p = (uw.rb + i) * a.w + uw.cb + j;
      if constexpr (FILL) {
        const int pos = atomicAdd(counts + p, 1);  // counts = the scan's cursor here
        col[pos] = o;
        val[pos] = wt;
      } else {
        atomicAdd(counts + p, 1);
      }
    }
}

__global__ __launch_bounds__(256) void adj_sort_kernel(const int32_t* __restrict__ row_ptr, int n,
                                                       int32_t* __restrict__ col, float* __restrict__ val) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int e0 = row_ptr[i], e1 = row_ptr[i + 1];
  for (int e = e0 + 1; e < e1; ++e) {  // insertion sort by output pixel (segments are short)
    const int c = col[e];
    const float w = val[e];
    int f = e - 1;
    while (f >= e0 && col[f] > c) {
      col[f + 1] = col[f];
      val[f + 1] = val[f];
      --f;
    }
    col[f + 1] = c;
    val[f + 1] = w;
  }
}

// grad_src[b][c][p] (+)= sum_e val[e] * grad_out[b][c][col[e]], e in row p of the plan.
// Thread = source pixel, loop over the block's channel chunk; the pixel's first kAdjReg
// entries stay in registers across the channels.  Workgroups of one (view, batch, channel
// chunk) are consecutive in the XCD-remapped order, so an XCD sweeps neighbouring pixels of
// the same grad_out planes (its L2 holds them).
#ifndef MVBEV_ADJ_G8
#define MVBEV_ADJ_G8 1  // split grad_out: a thread per (pixel, 8-channel group), warp_adjoint_split8_kernel
#endif
constexpr int kAdjReg = 6;
constexpr int kAdjCPB = 32;
constexpr int kAdjU = 8;
struct AdjView {
  const float* go;
  int64_t gB, gC;
  int64_t gP;  // pixel stride of a split grad_out in 32-B units (1; the group count when pixel-major)
  float* gs;
  int64_t sB, sC;
  const int32_t* rp;
  const int32_t* col;
  const float* val;
};
struct AdjArgs {
  AdjView v[kWarpMaxViews];
  int nviews, B, C, P, pblocks, chunks, nwg, accumulate;
  int src_cl;  // warp_adjoint_pix_kernel: grad_src channels-last (sC = 1, pixel stride C), else dense planes
  // warp_adjoint_pix_kernel (round 6): 16-B stores of 4 elements along grad_src's contiguous dimension (every
  // view's grad_src 16-B aligned, its batch / channel strides and P (planes) or C (channels-last) multiples of 4)
  int vec4;
};

__global__ __launch_bounds__(256) void warp_adjoint_kernel(const AdjArgs a) {
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int pb = lb % a.pblocks;
  int r = lb / a.pblocks;
  const int chunk = r % a.chunks;
  r /= a.chunks;
  const int view = r % a.nviews;
  const int b = r / a.nviews;
  const int p = pb * 256 + threadIdx.x;
  if (p >= a.P) return;
  const AdjView& vw = a.v[view];
  const int e0 = vw.rp[p], e1 = vw.rp[p + 1];
  const int ne = min(e1 - e0, kAdjReg);
  int cl[kAdjReg];
  float wt[kAdjReg];
#pragma unroll
  for (int j = 0; j < kAdjReg; ++j) {
    cl[j] = j < ne ? vw.col[e0 + j] : 0;
    wt[j] = j < ne ? vw.val[e0 + j] : 0.f;
  }
  const int c0 = chunk * kAdjCPB, c1 = min(a.C, c0 + kAdjCPB);
  const float* go = vw.go + (int64_t)b * vw.gB;
  float* gs = vw.gs + (int64_t)b * vw.sB + p;
  // kAdjU channels per iteration: their gathers are independent, so up to kAdjU * kAdjReg
  // loads are in flight per lane before the first add needs one
  int c = c0;
  for (; c + kAdjU <= c1; c += kAdjU) {
    float s[kAdjU];
#pragma unroll
    for (int q = 0; q < kAdjU; ++q) {
      const float* g = go + (int64_t)(c + q) * vw.gC;
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < kAdjReg; ++j)
        if (j < ne) t += wt[j] * g[cl[j]];
      s[q] = t;
    }
    for (int e = e0 + kAdjReg; e < e1; ++e) {
      const int oc = vw.col[e];
      const float w = vw.val[e];
#pragma unroll
      for (int q = 0; q < kAdjU; ++q) s[q] += w * go[(int64_t)(c + q) * vw.gC + oc];
    }
#pragma unroll
    for (int q = 0; q < kAdjU; ++q) {
      float* d = gs + (int64_t)(c + q) * vw.sC;
      *d = a.accumulate ? s[q] + *d : s[q];
    }
  }
  for (; c < c1; ++c) {
    const float* g = go + (int64_t)c * vw.gC;
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < kAdjReg; ++j)
      if (j < ne) t += wt[j] * g[cl[j]];
    for (int e = e0 + kAdjReg; e < e1; ++e) t += vw.val[e] * g[vw.col[e]];
    float* d = gs + (int64_t)c * vw.sC;
    *d = a.accumulate ? t + *d : t;
  }
}

// Same gather with grad_out in the split-bf16 blocked layout (what the dgrad conv writes with
// a split output: per pixel and 8-channel group 16 B hi + 16 B lo; gB / gC strides in 32-B
// units): one entry costs two 16-B loads for 8 channels instead of eight 4-B gathers.
__global__ __launch_bounds__(256) void warp_adjoint_split_kernel(const AdjArgs a) {
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int pb = lb % a.pblocks;
  int r = lb / a.pblocks;
  const int chunk = r % a.chunks;
  r /= a.chunks;
  const int view = r % a.nviews;
  const int b = r / a.nviews;
  const int p = pb * 256 + threadIdx.x;
  if (p >= a.P) return;
  const AdjView& vw = a.v[view];
  const int e0 = vw.rp[p], e1 = vw.rp[p + 1];
  const int ne = min(e1 - e0, kAdjReg);
  int cl[kAdjReg];
  float wt[kAdjReg];
#pragma unroll
  for (int j = 0; j < kAdjReg; ++j) {
    cl[j] = j < ne ? vw.col[e0 + j] : 0;
    wt[j] = j < ne ? vw.val[e0 + j] : 0.f;
  }
  const int c0 = chunk * kAdjCPB, c1 = min(a.C, c0 + kAdjCPB);  // c0 % 8 == 0
  const u32x4* go = reinterpret_cast<const u32x4*>(vw.go) + 2 * (int64_t)b * vw.gB;
  float* gs = vw.gs + (int64_t)b * vw.sB + p;
  for (int c = c0; c < c1; c += 8) {
    const u32x4* g = go + 2 * (int64_t)(c >> 3) * vw.gC;
    float s[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = 0.f;
    auto add = [&](int oc, float w) __attribute__((always_inline)) {
      const bf16x8 hi = __builtin_bit_cast(bf16x8, g[2 * (int64_t)oc]);
      const bf16x8 lo = __builtin_bit_cast(bf16x8, g[2 * (int64_t)oc + 1]);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += w * ((float)hi[q] + (float)lo[q]);
    };
#pragma unroll
    for (int j = 0; j < kAdjReg; ++j)
      if (j < ne) add(cl[j], wt[j]);
    // further entries (the fused upsample + warp plan has ~2x the warp's) in batches of 8:
    // the batch's (col, val) loads first, then 8 independent gathers, instead of one
    // dependent (col -> gather) round trip per entry
    for (int eb = e0 + kAdjReg; eb < e1; eb += 8) {
      int cb[8];
      float wb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = eb + j < e1;
        cb[j] = ok ? vw.col[eb + j] : 0;
        wb[j] = ok ? vw.val[eb + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (eb + j < e1) add(cb[j], wb[j]);
    }
    const int nq = min(8, c1 - c);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nq) {
        float* d = gs + (int64_t)(c + q) * vw.sC;
        *d = a.accumulate ? s[q] + *d : s[q];
      }
  }
}

// The split gather with a thread per (source pixel, 8-channel group): a workgroup = 32 pixels x
// 8 groups (64 channels), a half-wave = 32 consecutive pixels of one group (coalesced stores).
// Each thread's chain of dependent gathers is one channel group's instead of a 32-channel
// chunk's (4x shorter), and a pixel's entries are shared by its 8 group threads.
// PIX pixels x 8 groups per workgroup: 32 for the warp plan (<= 4 entries per source pixel),
// 16 where source pixels carry many entries (the S.U plan: 0.69 -> 0.58 ms at cfg2; 64: 0.85)
constexpr int kAsGroups = 8;
#ifndef MVBEV_ADJ_PPT
#define MVBEV_ADJ_PPT 2  // source pixels per thread of the plain warp plan's gather (warp_adjoint_split8m_kernel; cfg2: 1 0.945 ms, 2 0.886, 4 1.19)
#endif
template <int PIX>
__global__ __launch_bounds__(PIX * kAsGroups) void warp_adjoint_split8_kernel(const AdjArgs a) {
  constexpr int kAsPix = PIX;
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int pb = lb % a.pblocks;
  int r = lb / a.pblocks;
  const int chunk = r % a.chunks;
  r /= a.chunks;
  const int view = r % a.nviews;
  const int b = r / a.nviews;
  const int p = pb * kAsPix + (threadIdx.x & (kAsPix - 1));
  const int c = (chunk * kAsGroups + threadIdx.x / kAsPix) * 8;
  if (p >= a.P || c >= a.C) return;
  const AdjView& vw = a.v[view];
  const int e0 = vw.rp[p], e1 = vw.rp[p + 1];
  const u32x4* g = reinterpret_cast<const u32x4*>(vw.go) + 2 * (int64_t)b * vw.gB + 2 * (int64_t)(c >> 3) * vw.gC;
  float s[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = 0.f;
  // entries in batches of 8: the batch's (col, val) loads, then 8 independent gathers
  for (int eb = e0; eb < e1; eb += 8) {
    int cb[8];
    float wb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = eb + j < e1;
      cb[j] = ok ? vw.col[eb + j] : 0;
      wb[j] = ok ? vw.val[eb + j] : 0.f;
    }
    u32x4 hv[8], lv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (eb + j < e1) {
        hv[j] = g[2 * (int64_t)cb[j]];
        lv[j] = g[2 * (int64_t)cb[j] + 1];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (eb + j < e1) {
        const bf16x8 hi = __builtin_bit_cast(bf16x8, hv[j]), lo = __builtin_bit_cast(bf16x8, lv[j]);
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += wb[j] * ((float)hi[q] + (float)lo[q]);
      }
  }
  float* gs = vw.gs + (int64_t)b * vw.sB + (int64_t)c * vw.sC + p;
  const int nq = min(8, a.C - c);
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < nq) {
      float* d = gs + (int64_t)q * vw.sC;
      *d = a.accumulate ? s[q] + *d : s[q];
    }
}

// The plain warp plan (<= 4 entries per source pixel, no long lists) with PPT source pixels per
// thread, PIX apart: every pixel's row pointers, then its first 4 (col, val) entries, then their
// gathers are issued together — the chain rp -> entries -> gather -> store is three dependent
// round trips, and one pixel per thread left the launch latency-bound (cfg2: 1.03 ms for 1.86 GB
// of source gradient).  Entries past the first 4 (rare) run the batch-of-8 loop.
template <int PIX, int PPT>
__global__ __launch_bounds__(PIX * kAsGroups) void warp_adjoint_split8m_kernel(const AdjArgs a) {
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int pb = lb % a.pblocks;
  int r = lb / a.pblocks;
  const int chunk = r % a.chunks;
  r /= a.chunks;
  const int view = r % a.nviews;
  const int b = r / a.nviews;
  const int c = (chunk * kAsGroups + threadIdx.x / PIX) * 8;
  if (c >= a.C) return;
  const AdjView& vw = a.v[view];
  const u32x4* g = reinterpret_cast<const u32x4*>(vw.go) + 2 * (int64_t)b * vw.gB + 2 * (int64_t)(c >> 3) * vw.gC;
  int p[PPT], e0[PPT], e1[PPT];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    p[j] = (pb * PPT + j) * PIX + (threadIdx.x & (PIX - 1));
    const bool ok = p[j] < a.P;
    e0[j] = ok ? vw.rp[p[j]] : 0;
    e1[j] = ok ? vw.rp[p[j] + 1] : 0;
  }
  int cb[PPT][4];
  float wb[PPT][4];
#pragma unroll
  for (int j = 0; j < PPT; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = e0[j] + q < e1[j];
      cb[j][q] = ok ? vw.col[e0[j] + q] : 0;
      wb[j][q] = ok ? vw.val[e0[j] + q] : 0.f;
    }
  u32x4 hv[PPT][4], lv[PPT][4];
#pragma unroll
  for (int j = 0; j < PPT; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (e0[j] + q < e1[j]) {
        hv[j][q] = g[2 * (int64_t)cb[j][q]];
        lv[j][q] = g[2 * (int64_t)cb[j][q] + 1];
      }
  float s[PPT][8];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) s[j][k] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (e0[j] + q < e1[j]) {
        const bf16x8 hi = __builtin_bit_cast(bf16x8, hv[j][q]), lo = __builtin_bit_cast(bf16x8, lv[j][q]);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[j][k] += wb[j][q] * ((float)hi[k] + (float)lo[k]);
      }
    for (int eb = e0[j] + 4; eb < e1[j]; ++eb) {  // (rare) further entries, in order
      const u32x4 h = g[2 * (int64_t)vw.col[eb]], l = g[2 * (int64_t)vw.col[eb] + 1];
      const float w = vw.val[eb];
      const bf16x8 hi = __builtin_bit_cast(bf16x8, h), lo = __builtin_bit_cast(bf16x8, l);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[j][k] += w * ((float)hi[k] + (float)lo[k]);
    }
  }
  const int nq = min(8, a.C - c);
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    if (p[j] >= a.P) continue;
    float* gs = vw.gs + (int64_t)b * vw.sB + (int64_t)c * vw.sC + p[j];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < nq) {
        float* d = gs + (int64_t)k * vw.sC;
        *d = a.accumulate ? s[j][k] + *d : s[j][k];
      }
  }
}

// Pixel-major split grad_out (MVBEV_LAYOUT_SPLIT_BF16_PIX: an output pixel's 8-channel groups side by
// side): lanes = (pixel slot, 8-channel group), the group fastest, so one entry's 64 channels (8 lanes,
// 256 B of one output pixel) are a single contiguous gather instead of eight 32-B pieces a plane apart.
// Each (pixel, group) sums its entries in CSR order exactly as warp_adjoint_split8(m)_kernel does; the
// block's [64 channels][NPIX pixels] result goes through LDS (pitch NPIX + 1: conflict-free both ways)
// into coalesced row stores of the source planes.  NPIX = 64 for the plain plan (2 pixels per lane),
// 32 for the upsampled (S.U) plan's longer lists.
#ifndef MVBEV_ADJ_PIX_EMPTY
#define MVBEV_ADJ_PIX_EMPTY 1  // blocks without entries store their zeros directly, no LDS pass (cfg2 plain plan: 0.695 -> 0.682 ms)
#endif
#ifndef MVBEV_ADJ_PIX_NPIX
#define MVBEV_ADJ_PIX_NPIX 64  // source pixels per block of the plain plan's pixel-major gather (32: 0.75 ms, 128: 0.79 vs 0.65-0.68)
#endif
template <int NPIX>
__global__ __launch_bounds__(256) void warp_adjoint_pix_kernel(const AdjArgs a) {
  constexpr int kSlots = 32, kPpt = NPIX / kSlots, kPitch = NPIX + 1;
  static_assert(NPIX % kSlots == 0, "pixels per block");
  __shared__ float tr[64 * kPitch];
  const int lb = xcd_remap(blockIdx.x, a.nwg);
  const int pb = lb % a.pblocks;
  int r = lb / a.pblocks;
  const int chunk = r % a.chunks;
  r /= a.chunks;
  const int view = r % a.nviews;
  const int b = r / a.nviews;
  const AdjView& vw = a.v[view];
  const int gq = threadIdx.x & 7, slot = threadIdx.x >> 3;
  const int c = chunk * 64 + gq * 8;
  const int p0 = pb * NPIX;
  const u32x4* g = reinterpret_cast<const u32x4*>(vw.go) + 2 * ((int64_t)b * vw.gB + (int64_t)(c >> 3) * vw.gC);
  const int np = min(NPIX, a.P - p0), c0 = chunk * 64;
  // the source gradient's (channel, pixel) element: planes (pixels contiguous) or channels-last
  const int64_t ps = a.src_cl ? (int64_t)a.C : 1;
  float* gs0 = vw.gs + (int64_t)b * vw.sB + (int64_t)c0 * vw.sC + (int64_t)p0 * ps;
#if MVBEV_ADJ_PIX_EMPTY
  if (vw.rp[p0] == vw.rp[p0 + np]) {  // no entries in the block (rp is monotone): zeros, no LDS pass
    if (a.accumulate) return;
    if (a.vec4) {  // 16-B stores: a quarter of the store instructions (the TA/TD path binds this kernel)
      for (int i = threadIdx.x; i < 16 * NPIX; i += 256) {
        const int cr = a.src_cl ? 4 * (i % 16) : i / (NPIX / 4), pl = a.src_cl ? i / 16 : 4 * (i % (NPIX / 4));
        if (pl < np && c0 + cr < a.C)
          *reinterpret_cast<floatx4*>(gs0 + (int64_t)cr * vw.sC + (int64_t)pl * ps) = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      return;
    }
    for (int i = threadIdx.x; i < 64 * NPIX; i += 256) {
      // the fastest index along the contiguous dimension: pixels for planes, channels for channels-last
      const int cr = a.src_cl ? i % 64 : i / NPIX, pl = a.src_cl ? i / 64 : i % NPIX;
      if (pl < np && c0 + cr < a.C) gs0[(int64_t)cr * vw.sC + (int64_t)pl * ps] = 0.f;
    }
    return;
  }
#endif
#pragma unroll
  for (int j = 0; j < kPpt; ++j) {
    const int pl = j * kSlots + slot, p = p0 + pl;
    float s[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = 0.f;
    if (p < a.P && c < a.C) {
      const int e0 = vw.rp[p], e1 = vw.rp[p + 1];
      for (int eb = e0; eb < e1; eb += 4) {  // batches of 4: the (col, val) loads, then 4 gathers in flight
        int cb[4];
        float wb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = eb + q < e1;
          cb[q] = ok ? vw.col[eb + q] : 0;
          wb[q] = ok ? vw.val[eb + q] : 0.f;
        }
        u32x4 hv[4], lv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (eb + q < e1) {
            const int64_t o = 2 * (int64_t)cb[q] * vw.gP;
            hv[q] = g[o];
            lv[q] = g[o + 1];
          }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (eb + q < e1) {
            const bf16x8 hi = __builtin_bit_cast(bf16x8, hv[q]), lo = __builtin_bit_cast(bf16x8, lv[q]);
#pragma unroll
            for (int k = 0; k < 8; ++k) s[k] += wb[q] * ((float)hi[k] + (float)lo[k]);
          }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tr[(gq * 8 + k) * kPitch + pl] = s[k];
  }
  __syncthreads();
  if (a.vec4) {  // 4 elements along the contiguous dimension per lane: 4 conflict-free LDS reads, one 16-B store
    for (int i = threadIdx.x; i < 16 * NPIX; i += 256) {
      const int cr = a.src_cl ? 4 * (i % 16) : i / (NPIX / 4), pl = a.src_cl ? i / 16 : 4 * (i % (NPIX / 4));
      if (pl < np && c0 + cr < a.C) {
        floatx4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = a.src_cl ? tr[(cr + e) * kPitch + pl] : tr[cr * kPitch + pl + e];
        floatx4* d = reinterpret_cast<floatx4*>(gs0 + (int64_t)cr * vw.sC + (int64_t)pl * ps);
        *d = a.accumulate ? v + *d : v;
      }
    }
    return;
  }
  for (int i = threadIdx.x; i < 64 * NPIX; i += 256) {
    const int cr = a.src_cl ? i % 64 : i / NPIX, pl = a.src_cl ? i / 64 : i % NPIX;
    if (pl < np && c0 + cr < a.C) {
      float* d = gs0 + (int64_t)cr * vw.sC + (int64_t)pl * ps;
      const float v = tr[cr * kPitch + pl];
      *d = a.accumulate ? v + *d : v;
    }
  }
}

// fp32 rows [n][W] -> MVBEV_LAYOUT_SPLIT_ROWS [n][W / 8][hi 8, lo 8] (W % 8 == 0), the rounding
// of store_split8 / split4 (hi = RNE bf16, lo = RNE bf16 of the remainder)
__global__ void split_rows_kernel(const floatx4* __restrict__ x, int64_t runs, u32x4_t* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= runs) return;
  const floatx4 a = x[2 * i], b = x[2 * i + 1];
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  store_split8(out + 2 * i, v);
}

// ---------------------------------------------------------------------------------------------
// wgrad launch geometry
static int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return n;
}

// Pixel partitions: one workgroup per CU fits (LDS), so P minimises the rounds per unit of
// work, ceil(tiles * P / CUs) / P, with a small per-partition cost (workspace + reduce).
// cost: one partition's workspace write + reduce read in units of a P = 1 round (direct form:
// 0.004; the Winograd form's rounds are ~4x shorter and its workspace 5/3 larger: 0.07).
static int wgrad_partitions(int64_t tiles, int64_t nchunks, double cost = 0.004) {
  const int G = std::max(cu_count(), 1);
  int best = 1;
  double best_t = 1e30;
  for (int P = 1; P <= 64 && P <= nchunks; ++P) {
    const double t = (double)ceil_div(tiles * P, G) / P + cost * P;
    if (t < best_t) best_t = t, best = P;
  }
  return best;
}

struct WGeo {
  int64_t tiles, nchunks;
  int P;
};
static WGeo wgrad_geo(const mvbev_conv_desc* d, int64_t Cout) {
  WGeo g;
  g.tiles = (Cout / MT) * ceil_div(d->K, NT);
  g.nchunks = d->B * d->H * ceil_div(d->W, PX);
  g.P = wgrad_partitions(g.tiles, g.nchunks);
  return g;
}

}  // namespace bwd
}  // namespace mvbev

extern "C" {

size_t mvbev_conv3x3_wgrad_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout) {
  using namespace mvbev::bwd;
  if (!desc || Cout <= 0 || desc->K <= 0 || desc->H <= 0 || desc->W <= 0 || desc->B <= 0) return 0;
  const WGeo g = wgrad_geo(desc, Cout);
  return (size_t)g.P * 9 * (size_t)Cout * (size_t)desc->K * sizeof(float);
}

int mvbev_split_rows_bf16(const float* x, int64_t rows, int64_t W, void* out, void* stream) {
  using namespace mvbev;
  if (!x || !out) return MVBEV_ERR_NULL;
  if (rows <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (W % 8 != 0) return MVBEV_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(x) & 15) != 0 || (reinterpret_cast<uintptr_t>(out) & 15) != 0)
    return MVBEV_ERR_ALIGN;
  const int64_t runs = rows * (W / 8);
  hipLaunchKernelGGL(bwd::split_rows_kernel, dim3((unsigned)ceil_div(runs, 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const bwd::floatx4*>(x), runs, static_cast<u32x4_t*>(out));
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_wgrad_bf16x3_ex2(const void* x, int x_layout, const mvbev_conv_desc* d, const void* dy_,
                                   int dy_layout, int64_t Cout, int dilation, const int32_t* chan_map,
                                   int64_t Cin_w, float* dw, const int32_t* chunk_list, const int32_t* chunk_off,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  using namespace mvbev;
  using namespace mvbev::bwd;
  const float* dy = static_cast<const float*>(dy_);  // SPLIT_ROWS: the same bytes per row
  if (!x || !d || !dy || !dw || !workspace) return MVBEV_ERR_NULL;
  if (dy_layout != MVBEV_LAYOUT_F32 && dy_layout != MVBEV_LAYOUT_SPLIT_ROWS) return MVBEV_ERR_SHAPE;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || Cin_w <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % MT != 0 || Cout > 65535 || d->K % 8 != 0 || d->group % 8 != 0 || d->K % d->group != 0)
    return MVBEV_ERR_SHAPE;
  if (d->in_row0 != 0 || d->in_rows != d->H || d->out_row0 != 0 || d->out_rows != d->H) return MVBEV_ERR_SHAPE;
  if (!chan_map && d->K > Cin_w) return MVBEV_ERR_SHAPE;
  if (d->H * d->W > (int64_t)INT32_MAX / 2 || d->B * d->H * ceil_div(d->W, PX) > INT32_MAX) return MVBEV_ERR_SHAPE;
  if (x_layout != MVBEV_LAYOUT_F32 && x_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;
  const WGeo g = wgrad_geo(d, Cout);
  const size_t need = (size_t)g.P * 9 * (size_t)Cout * (size_t)d->K * sizeof(float);
  if (workspace_bytes < need) return MVBEV_ERR_SHAPE;
  WArgs a;
  a.x = x; a.dy = dy; a.ws = static_cast<float*>(workspace);
  a.group_stride = d->group_stride; a.batch_stride = d->batch_stride;
  a.group = (int)d->group; a.K = (int)d->K; a.Cout = (int)Cout; a.B = (int)d->B;
  a.H = (int)d->H; a.W = (int)d->W;
  a.segs = (int)ceil_div(d->W, PX); a.nchunks = (int)g.nchunks; a.P = g.P;
  a.n_ct = (int)(Cout / MT); a.n_kt = (int)ceil_div(d->K, NT); a.ntiles = (int)g.tiles;
  a.vec_dy = (d->W % 4 == 0) && ((reinterpret_cast<uintptr_t>(dy) & 15) == 0);
  if ((chunk_list == nullptr) != (chunk_off == nullptr)) return MVBEV_ERR_NULL;
  if (chunk_list && d->group % NT != 0) return MVBEV_ERR_SHAPE;  // a channel tile inside one group
  a.clist = chunk_list;
  a.coff = chunk_off;
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)(g.P * g.tiles)), block(NTH);
  const bool split = x_layout == MVBEV_LAYOUT_SPLIT_BF16;
  // the DMA kernel's packed chunk ids (b, y, segment) and 32-bit chunk-invariant offsets
  const int64_t coff_max = ((d->K - 1) / d->group) * d->group_stride + (d->group - 8) * d->H * d->W;
  const bool dma_fits = d->B < 128 && d->H <= 4096 && a.segs <= 4096 && d->batch_stride % 8 == 0 &&
                        d->group_stride % 8 == 0 && Cout * d->H * d->W < INT32_MAX &&
                        coff_max / 4 + 2 * d->H * d->W < INT32_MAX;
  const bool dma = MVBEV_WGRAD_DMA && split && a.vec_dy && dma_fits && (dilation == 1 || dilation == 2) &&
                   g.nchunks / g.P + 1 <= WG_MAXC;
  a.dy_rows = dy_layout == MVBEV_LAYOUT_SPLIT_ROWS;
  if (a.dy_rows && (!dma || d->W % 8 != 0)) return MVBEV_ERR_SHAPE;  // pre-split rows: the DMA kernel only
  if (dma) {
    if (dilation == 1) hipLaunchKernelGGL((wgrad_dma_kernel<1>), grid, dim3(NTH), 0, s, a, WinoT{0});
    else hipLaunchKernelGGL((wgrad_dma_kernel<2>), grid, dim3(NTH), 0, s, a, WinoT{0});
  } else if (dilation == 1) {
    if (split) hipLaunchKernelGGL((wgrad_kernel<SplitIn, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<float, 1>), grid, block, 0, s, a);
  } else if (dilation == 2) {
    if (split) hipLaunchKernelGGL((wgrad_kernel<SplitIn, 2>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<float, 2>), grid, block, 0, s, a);
  } else {
    return MVBEV_ERR_DILATION;
  }
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)ceil_div(d->K, kWrK), (unsigned)Cout), dim3(kWrThreads), 0, s,
                     static_cast<const float*>(workspace), g.P, (int)Cout, (int)d->K, chan_map, (int)Cin_w, dw);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

// 3-row tiles r3 of the forward's row transform: ceil(H / 3) (dilation 1), 4 per 12-row tile (dilation 2)
static int64_t wino_r3(int64_t H, int dil) { return dil == 1 ? mvbev::ceil_div(H, 3) : 4 * mvbev::ceil_div(H, 12); }

size_t mvbev_wino_dy_rows_bytes(int64_t B, int64_t Cout, int64_t H, int64_t W, int dilation) {
  if (B <= 0 || Cout <= 0 || H <= 0 || W <= 0 || (dilation != 1 && dilation != 2)) return 0;
  return (size_t)B * 5 * (size_t)Cout * (size_t)wino_r3(H, dilation) * (size_t)W * 4;
}

int mvbev_wino_dy_rows_f32(const float* dy, int64_t B, int64_t Cout, int64_t H, int64_t W, int dilation,
                           void* out, size_t out_bytes, void* stream) {
  using namespace mvbev;
  if (!dy || !out) return MVBEV_ERR_NULL;
  if (B <= 0 || Cout <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (dilation != 1 && dilation != 2) return MVBEV_ERR_DILATION;
  if (W % 8 != 0 || B * Cout * H * W > (int64_t)INT32_MAX * 8) return MVBEV_ERR_SHAPE;
  if (out_bytes < mvbev_wino_dy_rows_bytes(B, Cout, H, W, dilation)) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(out)) & 15) != 0) return MVBEV_ERR_ALIGN;
  const int64_t R3 = wino_r3(H, dilation), n = B * Cout * R3 * (W / 8);
  hipLaunchKernelGGL(bwd::wino_dy_rows_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const bwd::floatx4*>(dy), (int)B, (int)Cout, (int)H, (int)W, (int)R3, dilation,
                     static_cast<u32x4_t*>(out));
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

// Winograd geometry: P over the 5 x tiles workgroup set, chunks (b, r3 < R3, segment) per xi
static mvbev::bwd::WGeo wgrad_wino_geo(const mvbev_conv_desc* d, int64_t Cout, int dil) {
  using namespace mvbev;
  using namespace mvbev::bwd;
  WGeo g;
  g.tiles = (Cout / MT) * ceil_div(d->K, 2 * NT);  // 128 input channels per workgroup
  g.nchunks = d->B * wino_r3(d->H, dil) * ceil_div(d->W, PX);
  g.P = wgrad_partitions(5 * g.tiles, g.nchunks, 0.07);
  // a partition's chunk ids are staged in LDS (WG_MAXC): more partitions for long chunk lists (large
  // grids, batches) rather than a refusal the training backward could not fall back from (its forward
  // may not have written the slab)
  while (g.nchunks / g.P + 1 > WG_MAXC && g.P < g.nchunks) ++g.P;
  return g;
}

size_t mvbev_conv3x3_wgrad_wino_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout, int dilation) {
  if (!desc || Cout <= 0 || desc->K <= 0 || desc->H <= 0 || desc->W <= 0 || desc->B <= 0) return 0;
  if (dilation != 1 && dilation != 2) return 0;
  const mvbev::bwd::WGeo g = wgrad_wino_geo(desc, Cout, dilation);
  return (size_t)g.P * 15 * (size_t)Cout * (size_t)desc->K * sizeof(float);
}

int mvbev_conv3x3_wgrad_wino_bf16x3(const void* t, size_t t_bytes, const mvbev_conv_desc* d, const void* dy_wino,
                                    size_t dy_wino_bytes, int64_t Cout, int dilation, const int32_t* chan_map,
                                    int64_t Cin_w, float* dw, const int32_t* chunk_list, const int32_t* chunk_off,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  using namespace mvbev;
  using namespace mvbev::bwd;
  if (!t || !d || !dy_wino || !dw || !workspace) return MVBEV_ERR_NULL;
  if (dilation != 1 && dilation != 2) return MVBEV_ERR_DILATION;
  if ((chunk_list == nullptr) != (chunk_off == nullptr)) return MVBEV_ERR_NULL;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || Cin_w <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % MT != 0 || Cout > 65535 || d->K % 8 != 0 || d->group % 8 != 0 || d->K % d->group != 0 ||
      d->W % 8 != 0)
    return MVBEV_ERR_SHAPE;
  if (d->in_row0 != 0 || d->in_rows != d->H || d->out_row0 != 0 || d->out_rows != d->H) return MVBEV_ERR_SHAPE;
  if (!chan_map && d->K > Cin_w) return MVBEV_ERR_SHAPE;
  if (chunk_list && d->group % (2 * NT) != 0) return MVBEV_ERR_SHAPE;  // a channel tile inside one group
  constexpr int kRT = 12;  // conv_wino's workgroup tile rows: T holds 4 row tiles (r3) of each
  const int64_t R3 = wino_r3(d->H, dilation), r5 = 5 * 4 * ceil_div(d->H, kRT), segs = ceil_div(d->W, PX);
  const int64_t t_need = d->B * (d->K / 8) * r5 * d->W * 32;
  if (t_bytes < (size_t)t_need || dy_wino_bytes < mvbev_wino_dy_rows_bytes(d->B, Cout, d->H, d->W, dilation))
    return MVBEV_ERR_SHAPE;
  // 32-bit chunk-invariant offsets and packed chunk ids (b < 128, r3 and segments < 4096)
  if ((d->K / 8) * 2 * r5 * d->W >= INT32_MAX || Cout * R3 * d->W >= INT32_MAX || d->B >= 128 || R3 > 4096 ||
      segs > 4096)
    return MVBEV_ERR_SHAPE;
  const WGeo g = wgrad_wino_geo(d, Cout, dilation);
  if (g.nchunks / g.P + 1 > WG_MAXC) return MVBEV_ERR_SHAPE;
  const size_t need = (size_t)g.P * 15 * (size_t)Cout * (size_t)d->K * sizeof(float);
  if (workspace_bytes < need) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(t) | reinterpret_cast<uintptr_t>(dy_wino)) & 15) != 0) return MVBEV_ERR_ALIGN;
  WArgs a;
  a.x = t; a.dy = static_cast<const float*>(dy_wino); a.ws = static_cast<float*>(workspace);
  a.group_stride = d->group_stride; a.batch_stride = d->batch_stride;
  a.group = (int)d->group; a.K = (int)d->K; a.Cout = (int)Cout; a.B = (int)d->B;
  a.H = (int)R3; a.W = (int)d->W;  // the kernel's rows: the 3-row tiles r3
  a.segs = (int)segs; a.nchunks = (int)g.nchunks; a.P = g.P;
  a.n_ct = (int)(Cout / MT); a.n_kt = (int)ceil_div(d->K, 2 * NT); a.ntiles = (int)g.tiles;
  a.vec_dy = true; a.dy_rows = true;
  a.clist = chunk_list; a.coff = chunk_off;
  hipStream_t s = as_stream(stream);
  if (dilation == 1)
    hipLaunchKernelGGL((wgrad_dma_kernel<1, true>), dim3((unsigned)(g.P * 5 * g.tiles)), dim3(NTH), 0, s, a,
                       WinoT{(int)r5});
  else
    hipLaunchKernelGGL((wgrad_dma_kernel<2, true>), dim3((unsigned)(g.P * 5 * g.tiles)), dim3(NTH), 0, s, a,
                       WinoT{(int)r5});
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(wgrad_wino_reduce_kernel, dim3((unsigned)ceil_div(d->K, kWrK), (unsigned)Cout),
                     dim3(kWinoRedThreads), 0, s, static_cast<const float*>(workspace), g.P, (int)Cout, (int)d->K, chan_map,
                     (int)Cin_w, dw);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_bias_coord_grad_f32(const float* dy, int64_t B, int64_t Cout, int64_t H, int64_t W,
                                      int dilation, float* db, float* dw, int64_t Cin_w, int64_t coord_ch,
                                      void* stream) {
  using namespace mvbev;
  if (!dy || (!db && !dw)) return MVBEV_ERR_NULL;
  if (B <= 0 || Cout <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (H * W > INT32_MAX || Cout > 65535 * 16) return MVBEV_ERR_SHAPE;
  if (dw && (coord_ch < 0 || coord_ch + 2 > Cin_w)) return MVBEV_ERR_SHAPE;
  if (dilation < 1) return MVBEV_ERR_DILATION;
  if (dw && (H > bwd::kCoordTab || W > bwd::kCoordTab)) return MVBEV_ERR_SHAPE;
  hipLaunchKernelGGL(bwd::bias_coord_grad_kernel, dim3((unsigned)Cout), dim3(bwd::kRedThreads), 0, as_stream(stream), dy,
                     (int)B, (int)Cout, (int)H, (int)W, dilation, db, dw, (int)Cin_w, (int)coord_ch);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_relu_backward_f32(float* dy, const float* y, int64_t n, void* stream) {
  using namespace mvbev;
  if (!dy || !y) return MVBEV_ERR_NULL;
  if (n <= 0) return MVBEV_ERR_RANK;
  if (((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(y)) & 15) != 0) return MVBEV_ERR_ALIGN;
  hipLaunchKernelGGL(bwd::relu_backward_kernel, dim3((unsigned)ceil_div(ceil_div(n, 4), 256)), dim3(256), 0,
                     as_stream(stream), dy, y, n);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_relu_backward_split_f32(float* dy, const void* y_split, int64_t B, int64_t C, int64_t H, int64_t W,
                                  void* dy_split, void* stream) {
  using namespace mvbev;
  if (!dy || !y_split) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (C % 8 != 0 || B > 65535 || C / 8 > 65535) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(y_split) | reinterpret_cast<uintptr_t>(dy_split)) & 15) != 0) return MVBEV_ERR_ALIGN;
  const int64_t HW = H * W;
  hipLaunchKernelGGL(bwd::relu_backward_split_kernel, dim3((unsigned)ceil_div(HW, 256), (unsigned)(C / 8), (unsigned)B),
                     dim3(256), 0, as_stream(stream), dy, static_cast<const u32x4_t*>(y_split), (int)C, HW,
                     static_cast<u32x4_t*>(dy_split));
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_cout1_backward_ex(const float* x, const float* w, const float* dmap, int64_t B, int64_t C,
                                    int64_t H, int64_t W, int dilation, int relu_mask, float* dx, void* dx_split,
                                    float* dw, void* stream) {
  using namespace mvbev;
  if (!x || !w || !dmap || (!dx && !dw) || (dx_split && !dx)) return MVBEV_ERR_NULL;
  if (dx_split && (C % 8 != 0 || (reinterpret_cast<uintptr_t>(dx_split) & 15) != 0)) return MVBEV_ERR_SHAPE;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return MVBEV_ERR_RANK;
  if (H * W > INT32_MAX || B > 65535) return MVBEV_ERR_SHAPE;
  if (dilation < 1) return MVBEV_ERR_DILATION;
  hipStream_t s = as_stream(stream);
  if (dx) {
    const dim3 grid((unsigned)ceil_div(H * W, 256), (unsigned)ceil_div(C, bwd::kCout1Cpb), (unsigned)B);
    hipLaunchKernelGGL(bwd::cout1_dgrad_kernel, grid, dim3(256), 0, s, x, w, dmap, (int)C, (int)H, (int)W,
                       dilation, relu_mask, dx, static_cast<u32x4_t*>(dx_split));
    MVBEV_CHECK_LAUNCH();
  }
  if (dw) {
    hipLaunchKernelGGL(bwd::cout1_wgrad_kernel, dim3((unsigned)C), dim3(bwd::kRedThreads), 0, s, x, dmap, (int)B, (int)C,
                       (int)H, (int)W, dilation, dw);
    MVBEV_CHECK_LAUNCH();
  }
  return MVBEV_OK;
}

int mvbev_warp_views_backward_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                                  int64_t W, int64_t Ho, int64_t Wo, void* stream) {
  using namespace mvbev;
  if (!views) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || nviews <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || C > INT32_MAX || H > INT32_MAX / 2 || W > INT32_MAX / 2 ||
      Ho > INT32_MAX / 2 || Wo > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  WarpArgs a = {};
  for (int i = 0; i < nviews; ++i) {
    const mvbev_warp_view& v = views[i];
    if (!v.src || !v.dst) return MVBEV_ERR_NULL;
    if (v.dst_strides[3] != 1) return MVBEV_ERR_STRIDE;
    a.v[i] = WarpView{v.src, v.src_strides[0], v.src_strides[1], v.src_strides[2], v.src_strides[3],
                      v.dst, v.dst_strides[0], v.dst_strides[1], v.dst_strides[2], nullptr, {}};
    for (int j = 0; j < 9; ++j) a.v[i].m[j] = v.m[j];
  }
  a.nviews = nviews;
  a.B = (int)B; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.tiles_x = (int)ceil_div(Wo, mvbev::bwd::kBwTW);
  a.tiles = a.tiles_x * (int)ceil_div(Ho, mvbev::bwd::kBwTH);
  a.chunks = (int)ceil_div(C, mvbev::bwd::kBwCPB);
  const int64_t nwg = (int64_t)a.tiles * a.chunks * B * nviews;
  if (nwg > INT32_MAX) return MVBEV_ERR_SHAPE;
  a.nwg = (int)nwg;
  hipLaunchKernelGGL(bwd::warp_backward_kernel, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}


int mvbev_warp_adjoint_plan(const float* m, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int32_t* row_ptr,
                            int32_t* col, float* val, int32_t* scratch, void* stream) {
  using namespace mvbev;
  if (!m || !row_ptr || !col || !val || !scratch) return MVBEV_ERR_NULL;
  if (H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return MVBEV_ERR_RANK;
  if (H * W >= INT32_MAX || 4 * Ho * Wo >= INT32_MAX) return MVBEV_ERR_SHAPE;
  bwd::PlanArgs a;
  for (int i = 0; i < 9; ++i) a.m[i] = m[i];
  a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo;
  hipStream_t s = as_stream(stream);
  const int n = (int)(H * W);
  if (hipMemsetAsync(scratch, 0, sizeof(int32_t) * n, s) != hipSuccess) return MVBEV_ERR_HIP;
  const unsigned ob = (unsigned)ceil_div(Ho * Wo, 256);
  hipLaunchKernelGGL(bwd::adj_count_kernel, dim3(ob), dim3(256), 0, s, a, scratch);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_scan_kernel, dim3(1), dim3(1024), 0, s, scratch, n, row_ptr, scratch);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_fill_kernel, dim3(ob), dim3(256), 0, s, a, scratch, col, val);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_sort_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, row_ptr, n, col, val);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_warp_upsampled_adjoint_plan(const float* m, int64_t h, int64_t w, int64_t H, int64_t W, int64_t Ho,
                                      int64_t Wo, int32_t* row_ptr, int32_t* col, float* val, int32_t* scratch,
                                      void* stream) {
  using namespace mvbev;
  if (!m || !row_ptr || !col || !val || !scratch) return MVBEV_ERR_NULL;
  if (h <= 0 || w <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return MVBEV_ERR_RANK;
  if (H < h || W < w || H >= INT32_MAX / 2 || W >= INT32_MAX / 2 || 9 * Ho * Wo >= INT32_MAX) return MVBEV_ERR_SHAPE;
  bwd::UpPlanArgs a;
  for (int i = 0; i < 9; ++i) a.m[i] = m[i];
  a.H = (int)H; a.W = (int)W; a.Ho = (int)Ho; a.Wo = (int)Wo; a.h = (int)h; a.w = (int)w;
  a.sy = (float)h / (float)H;  // area_pixel_compute_scale(align_corners=false), as warp_up_kernel
  a.sx = (float)w / (float)W;
  hipStream_t s = as_stream(stream);
  const int n = (int)(h * w);
  if (hipMemsetAsync(scratch, 0, sizeof(int32_t) * n, s) != hipSuccess) return MVBEV_ERR_HIP;
  const unsigned ob = (unsigned)ceil_div(Ho * Wo, 256);
  hipLaunchKernelGGL(bwd::adj_up_kernel<false>, dim3(ob), dim3(256), 0, s, a, scratch, col, val);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_scan_kernel, dim3(1), dim3(1024), 0, s, scratch, n, row_ptr, scratch);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_up_kernel<true>, dim3(ob), dim3(256), 0, s, a, scratch, col, val);
  MVBEV_CHECK_LAUNCH();
  hipLaunchKernelGGL(bwd::adj_sort_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, row_ptr, n, col, val);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_warp_views_adjoint(const mvbev_warp_adjoint_view* views, int nviews, int grad_out_layout, int64_t B,
                             int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int accumulate,
                             void* stream) {
  using namespace mvbev;
  if (!views) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0 || nviews <= 0) return MVBEV_ERR_RANK;
  if (nviews > kWarpMaxViews || H * W >= INT32_MAX || 4 * Ho * Wo >= INT32_MAX) return MVBEV_ERR_SHAPE;
  if (grad_out_layout != MVBEV_LAYOUT_F32 && grad_out_layout != MVBEV_LAYOUT_SPLIT_BF16 &&
      grad_out_layout != MVBEV_LAYOUT_SPLIT_BF16_PIX)
    return MVBEV_ERR_SHAPE;
  const bool pixm = grad_out_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX;
  const bool split = grad_out_layout == MVBEV_LAYOUT_SPLIT_BF16 || pixm;
  if (pixm && C % 8 != 0) return MVBEV_ERR_SHAPE;
  bwd::AdjArgs a = {};
  for (int i = 0; i < nviews; ++i) {
    const mvbev_warp_adjoint_view& v = views[i];
    if (!v.grad_out || !v.grad_src || !v.row_ptr || !v.col || !v.val) return MVBEV_ERR_NULL;
    // planes must be dense (the plan indexes pixels linearly); pixel-major: groups adjacent, pixels dense;
    // a channels-last grad_src (pixel-major grad_out only): channels adjacent, pixels C apart
    const int64_t gp = pixm ? v.grad_out_strides[3] : 1;
    const bool cl = pixm && v.grad_src_strides[1] == 1 && v.grad_src_strides[3] == C && v.grad_src_strides[2] == W * C;
    if (i > 0 && cl != (a.src_cl != 0)) return MVBEV_ERR_STRIDE;  // one grad_src layout per launch
    a.src_cl = cl ? 1 : 0;
    if ((pixm ? (v.grad_out_strides[1] != 1 || gp < C / 8 || v.grad_out_strides[2] != Wo * gp)
              : (v.grad_out_strides[3] != 1 || v.grad_out_strides[2] != Wo)) ||
        (!cl && (v.grad_src_strides[3] != 1 || v.grad_src_strides[2] != W)))
      return MVBEV_ERR_STRIDE;
    if (split && (reinterpret_cast<uintptr_t>(v.grad_out) & 15) != 0) return MVBEV_ERR_ALIGN;
    a.v[i] = bwd::AdjView{v.grad_out, v.grad_out_strides[0], v.grad_out_strides[1], gp, v.grad_src,
                          v.grad_src_strides[0], v.grad_src_strides[1], v.row_ptr, v.col, v.val};
  }
  a.nviews = nviews;
  a.B = (int)B; a.C = (int)C; a.P = (int)(H * W);
#ifndef MVBEV_ADJ_PIX_VEC4
#define MVBEV_ADJ_PIX_VEC4 1
#endif
  a.vec4 = MVBEV_ADJ_PIX_VEC4 && pixm && (a.src_cl ? C % 4 == 0 : (H * W) % 4 == 0);
  for (int i = 0; i < nviews && a.vec4; ++i)
    a.vec4 = (reinterpret_cast<uintptr_t>(a.v[i].gs) & 15) == 0 && a.v[i].sB % 4 == 0 && (a.src_cl || a.v[i].sC % 4 == 0);
  const bool g8 = split && MVBEV_ADJ_G8;
  // many entries per source pixel (a source smaller than the grid: the S.U plan): 16 pixels
  const int pix = H * W < Ho * Wo ? 16 : 32;
  constexpr int kPpt = MVBEV_ADJ_PPT;  // source pixels per thread of the plain plan's gather
  a.pblocks = (int)ceil_div(H * W, g8 ? pix * (pix == 32 ? kPpt : 1) : 256);
  a.chunks = (int)ceil_div(C, g8 ? 8 * bwd::kAsGroups : bwd::kAdjCPB);
  a.accumulate = accumulate ? 1 : 0;
  if (pixm) {  // 64 channels x 64 (plain plan) / 32 (S.U plan) source pixels per block
    a.pblocks = (int)ceil_div(H * W, pix == 32 ? MVBEV_ADJ_PIX_NPIX : 32);
    a.chunks = (int)ceil_div(C, 64);
  }
  const int64_t nwg = (int64_t)a.pblocks * a.chunks * nviews * B;
  if (nwg > INT32_MAX) return MVBEV_ERR_SHAPE;
  a.nwg = (int)nwg;
  if (pixm) {
    if (pix == 32)
      hipLaunchKernelGGL(bwd::warp_adjoint_pix_kernel<MVBEV_ADJ_PIX_NPIX>, dim3((unsigned)nwg), dim3(256), 0,
                         as_stream(stream), a);
    else
      hipLaunchKernelGGL(bwd::warp_adjoint_pix_kernel<32>, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  } else if (g8)
    if (pix == 16)
      hipLaunchKernelGGL(bwd::warp_adjoint_split8_kernel<16>, dim3((unsigned)nwg), dim3(16 * bwd::kAsGroups), 0,
                         as_stream(stream), a);
    else if (kPpt > 1)
      hipLaunchKernelGGL((bwd::warp_adjoint_split8m_kernel<32, kPpt>), dim3((unsigned)nwg), dim3(32 * bwd::kAsGroups),
                         0, as_stream(stream), a);
    else
      hipLaunchKernelGGL(bwd::warp_adjoint_split8_kernel<32>, dim3((unsigned)nwg), dim3(32 * bwd::kAsGroups), 0,
                         as_stream(stream), a);
  else if (split)
    hipLaunchKernelGGL(bwd::warp_adjoint_split_kernel, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(bwd::warp_adjoint_kernel, dim3((unsigned)nwg), dim3(256), 0, as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

}  // extern "C"
