// Dilated 3x3 convolutions of the BEV fusion head (map_classifier) for gfx950.
//
// Replaces nn.Conv2d(Cin->512, 3, p1)+ReLU, nn.Conv2d(512->512, 3, d2, p2)+ReLU and
// nn.Conv2d(512->1, 3, d4, p4, no bias) at multiview_detector/models/persp_trans_detector.py:51-54
// (applied at :81).
//
// mvbev_conv3x3_f32 — implicit GEMM on the fp32-input MFMA (v_mfma_f32_32x32x2_f32: exact
// f32 products, f32 accumulation, 64 FLOP/clk/SIMD = the chip's fp32 peak):
//   D[co][pixel] += sum_{tap, ci} W[co][ci][tap] * X[ci][pixel + d*tap]
//   A operand = weights (M = output channels), B operand = input pixels (N = 32 consecutive
//   columns of one output row), K = (input channel, tap).  With the output channel on the
//   accumulator rows and the pixel on the lane, the epilogue stores 2 x 128 B per register:
//   NCHW output, fully coalesced.
//   Workgroup tile: TH=4 rows x TW=32 cols of pixels x BN=128 output channels, 4 waves
//   (wave = 2 pixel rows x 64 channels = 2x2 MFMA tiles of 32x32).  K is walked in chunks of
//   KC=8 input channels; per chunk the (TH+2d) x (TW+2d) input halo of all 8 channels and the
//   9 x 8 x 128 weight slab are staged in LDS and every staged input element feeds all 9 taps.
//   The next chunk's global loads are issued into registers before the MFMAs of the current
//   chunk (async-STAGE split) and written to LDS after the next barrier; out-of-image halo
//   elements load a safe in-bounds address and are zeroed by a select at LDS-store time,
//   so no wait on those loads sits in front of the MFMAs.
//
//   Input addressing (mvbev_conv_desc): input channel ci of batch item b lives at
//     x + (ci / group) * group_stride + b * batch_stride + (ci % group) * in_rows * W
//   which covers a plain [B][Cin][H][W] tensor (group = Cin) and the view-major fused
//   ground-plane tensor [views][B][C][H][W] (group = C) without a repack.  Row bands: the
//   input buffer holds global rows [in_row0, in_row0 + in_rows) and the kernel computes
//   global output rows [out_row0, out_row0 + out_rows); zero padding applies at the true
//   image border (rows < 0 or >= H) — used by the view-parallel multi-GPU fusion.
//   Epilogue: + bias[co] and/or + init[co][row][col] (the precomputed coord-channel term),
//   optional ReLU (NaN-preserving, like torch.relu).
//
// mvbev_conv3x3_cout1_f32 — Cout = 1 is a 4608-long dot product per pixel: HBM/L2-bound, no
//   MFMA.  Block = 64 pixels of a row x 8 waves; each wave sums an eighth of the channels, four
//   channels per step with independent accumulators (memory-level parallelism), wave-uniform
//   (scalar) weight loads; partial sums reduced through LDS.
#include "common.h"

namespace mvbev {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));  // native vector (HIP's float4 struct blocks SROA)

constexpr int KC = MVBEV_CONV_KC;  // input channels per staged chunk
constexpr int BN = MVBEV_CONV_BN;  // output channels per workgroup
constexpr int TW = 32;             // output cols per workgroup (= MFMA N)

// packed[chunk][cotile][tap][kk][col] = w[cotile*BN+col][map(chunk*KC+kk)][tap]
// map = identity (chan_map == nullptr) or chan_map[k]; unmapped (-1) / k >= K -> 0.
__global__ void pack_conv3x3_kernel(const float* __restrict__ w, float* __restrict__ wp, int Cout,
                                    int Cin_w, const int32_t* __restrict__ chan_map, int K,
                                    int K_pad, const int32_t* gate, int32_t gate_tag) {
  if (gate && *gate != gate_tag) return;  // (ABI 12200) the training guard's per-step pack: gated
  const int64_t total = (int64_t)K_pad * 9 * Cout;
  const int n_cot = Cout / BN;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int col = r % BN; r /= BN;
    const int kk = r % KC; r /= KC;
    const int tap = r % 9; r /= 9;
    const int cot = r % n_cot;
    const int chunk = (int)(r / n_cot);
    const int k = chunk * KC + kk;
    int ci = k < K ? (chan_map ? chan_map[k] : k) : -1;
    if (ci >= Cin_w) ci = -1;
    const int co = cot * BN + col;
    wp[i] = ci >= 0 ? w[((int64_t)co * Cin_w + ci) * 9 + tap] : 0.f;
  }
}

struct ConvArgs {
  const float* x;
  const float* wp;
  const float* bias;
  const float* init;
  float* y;
  int64_t group_stride, batch_stride;
  int group, nchunks, Cout, H, W;
  int in_row0, in_rows, out_row0, out_rows;
  int tiles_x, tiles_y, n_cot, nwg;
  const int32_t* gate;  // run only when *gate == gate_tag (NULL: always; the non-finite guard's path)
  int32_t gate_tag;
  int band_rows;  // > 0: y in row bands [bands][B][Cout][band_rows][W], global row g at band g / band_rows
  int B;
};

#ifndef MVBEV_CONV_MINWAVES
#define MVBEV_CONV_MINWAVES 2  // waves per SIMD the register budget must allow
#endif
#ifndef MVBEV_CONV_WAVES
#define MVBEV_CONV_WAVES 4     // waves per workgroup: 4 (2 WGs/CU, single LDS buffer) or 8 (1 WG/CU)
#endif
#ifndef MVBEV_CONV_DBUF
#define MVBEV_CONV_DBUF 0      // double-buffered LDS, one barrier per K chunk
#endif

// Tile geometry: each wave owns 2 output rows x 64 output channels (2x2 MFMA 32x32 tiles);
// NWAVES/2 row pairs x 2 channel halves per workgroup -> TH = NWAVES rows.
template <int NWAVES> struct TileCfg {
  static constexpr int NT = 64 * NWAVES;
  static constexpr int TH = NWAVES;
};

template <int DIL, bool RELU, int NWAVES, bool DBUF>
__global__ __launch_bounds__(64 * NWAVES, MVBEV_CONV_MINWAVES) void conv3x3_mfma_f32_kernel(
    const ConvArgs a) {
  constexpr int NT = TileCfg<NWAVES>::NT;
  constexpr int TH_ = TileCfg<NWAVES>::TH;
  constexpr int XH = TH_ + 2 * DIL, XW = TW + 2 * DIL;
  constexpr int XS = KC * XH * XW;        // input halo floats per chunk
  constexpr int WS = 9 * KC * BN;         // weight floats per chunk
  constexpr int WS4 = WS / 4;             // float4 elements of the weight slab
  constexpr int WLD = (WS4 + NT - 1) / NT;
  constexpr int XLD = (XS + NT - 1) / NT;
  constexpr int NBUF = DBUF ? 2 : 1;
  constexpr int BUF = WS + ((XS + 3) / 4) * 4;  // floats per LDS buffer (16-B aligned parts)
  __shared__ __attribute__((aligned(16))) float lds[NBUF * BUF];
  if (a.gate && *a.gate != a.gate_tag) return;

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int cot = wg % a.n_cot;
  int rest = wg / a.n_cot;
  const int tx = rest % a.tiles_x;
  rest /= a.tiles_x;
  const int ty = rest % a.tiles_y;
  const int b = rest / a.tiles_y;
  const int x0 = tx * TW;
  const int y0 = a.out_row0 + ty * TH_;  // global output row of the tile's first row
  const int W = a.W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;

  const int64_t plane = (int64_t)a.in_rows * W;
  const float* xb = a.x + (int64_t)b * a.batch_stride;
  const floatx4* wsrc = reinterpret_cast<const floatx4*>(a.wp) + (int64_t)cot * WS4;
  const int64_t wchunk = (int64_t)a.n_cot * WS4;
  const int chunks_per_group = a.group / KC;

  // Per-thread halo element coordinates are chunk-invariant: precompute offsets/validity.
  int xoff[XLD];
  bool xok[XLD];
#pragma unroll
  for (int i = 0; i < XLD; ++i) {
    const int e = tid + NT * i;
    const int kk = e / (XH * XW);
    const int r = (e / XW) % XH;
    const int c = e % XW;
    const int gy = y0 - DIL + r, gx = x0 - DIL + c;  // global input coordinates
    const int by = gy - a.in_row0;                    // row inside the input buffer
    xok[i] = e < XS && gy >= 0 && gy < a.H && by >= 0 && by < a.in_rows && gx >= 0 && gx < W;
    xoff[i] = xok[i] ? (int)(kk * plane + (int64_t)by * W + gx) : 0;
  }

  // Staging registers for the next chunk (native vectors, compile-time indices only).
  floatx4 wreg[WLD];
  float xreg[XLD];
#define MVBEV_LOAD_CHUNK(ch)                                                                  \
  do {                                                                                        \
    const floatx4* ws_ = wsrc + (int64_t)(ch) * wchunk;                                       \
    _Pragma("unroll") for (int i = 0; i < WLD; ++i) {                                         \
      if (WS4 % NT == 0 || tid + NT * i < WS4) wreg[i] = ws_[tid + NT * i];                   \
    }                                                                                         \
    const int g_ = (ch) / chunks_per_group;                                                   \
    const float* xc_ =                                                                        \
        xb + g_ * a.group_stride + (int64_t)((ch) - g_ * chunks_per_group) * KC * plane;      \
    _Pragma("unroll") for (int i = 0; i < XLD; ++i) xreg[i] = xc_[xoff[i]]; /* select at store */ \
  } while (0)
#define MVBEV_STORE_CHUNK(buf)                                                                \
  do {                                                                                        \
    float* Wd_ = lds + (buf) * BUF;                                                           \
    float* Xd_ = Wd_ + WS;                                                                    \
    _Pragma("unroll") for (int i = 0; i < WLD; ++i) {                                         \
      if (WS4 % NT == 0 || tid + NT * i < WS4)                                                \
        reinterpret_cast<floatx4*>(Wd_)[tid + NT * i] = wreg[i];                              \
    }                                                                                         \
    _Pragma("unroll") for (int i = 0; i < XLD; ++i) {                                         \
      const int e = tid + NT * i;                                                             \
      if (XS % NT == 0 || e < XS) Xd_[e] = xok[i] ? xreg[i] : 0.f;                            \
    }                                                                                         \
  } while (0)

  floatx16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  const int prow = 2 * (wave % (NWAVES / 2));  // this wave's two output rows within the tile
  const int cw = 64 * (wave / (NWAVES / 2));   // this wave's 64 output channels within BN

  auto compute = [&](const float* Ws, const float* Xs) __attribute__((always_inline)) {
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int tap = ky * 3 + kx;
#pragma unroll
        for (int kp = 0; kp < KC / 2; ++kp) {
          const int k = 2 * kp + kh;
          const float* wrow = Ws + (tap * KC + k) * BN + cw + l32;
          const float a0 = wrow[0];
          const float a1 = wrow[32];
          const float* xrow = Xs + (k * XH + prow + ky * DIL) * XW + l32 + kx * DIL;
          const float b0 = xrow[0];
          const float b1 = xrow[XW];
          acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
          acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
          acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
        }
      }
    }
  };

  MVBEV_LOAD_CHUNK(0);
  if constexpr (DBUF) {
    // Double buffer: chunk ch+1 is loaded to registers before the MFMAs of chunk ch and
    // stored to the other buffer right after them; one barrier per chunk.
    MVBEV_STORE_CHUNK(0);
    __syncthreads();
    for (int ch = 0; ch < a.nchunks; ++ch) {
      const int cur = ch & 1;
      const bool more = ch + 1 < a.nchunks;
      if (more) MVBEV_LOAD_CHUNK(ch + 1);
      compute(lds + cur * BUF, lds + cur * BUF + WS);
      if (more) MVBEV_STORE_CHUNK(cur ^ 1);
      __syncthreads();
    }
  } else {
    for (int ch = 0; ch < a.nchunks; ++ch) {
      __syncthreads();
      MVBEV_STORE_CHUNK(0);
      __syncthreads();
      if (ch + 1 < a.nchunks) MVBEV_LOAD_CHUNK(ch + 1);
      compute(lds, lds + WS);
    }
  }
#undef MVBEV_LOAD_CHUNK
#undef MVBEV_STORE_CHUNK

  // Epilogue: D[i = co][j = pixel]; lane holds j = l32 and rows i = (r&3) + 8(r>>2) + 4 kh.
  const int col = x0 + l32;
  const int64_t oplane = (int64_t)a.out_rows * W;
  const int64_t iplane = (int64_t)a.H * W;  // init is full-size [Cout][H][W]
  auto emit = [&](const floatx16& acc, int ci_tile, int rj) {
    const int row = y0 + prow + rj;
    if (row >= a.out_row0 + a.out_rows || col >= W) return;
    // the output address chosen once, outside the unrolled store loop (a branch inside it puts the
    // accumulators in scratch): plain [B][Cout][out_rows][W], or row bands (ABI 11900)
    int64_t ybase, cstride;
    if (a.band_rows > 0) {
      const int band = row / a.band_rows;
      cstride = (int64_t)a.band_rows * W;
      ybase = ((int64_t)band * a.B + b) * a.Cout * cstride + (int64_t)(row - band * a.band_rows) * W + col;
    } else {
      cstride = oplane;
      ybase = (int64_t)b * a.Cout * oplane + (int64_t)(row - a.out_row0) * W + col;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cot * BN + cw + 32 * ci_tile + (r & 3) + 8 * (r >> 2) + 4 * kh;
      float v = acc[r];
      if (a.bias) v += a.bias[co];
      if (a.init) v += a.init[co * iplane + (int64_t)row * W + col];
      if (RELU) v = v < 0.f ? 0.f : v;  // torch.relu keeps NaN
      a.y[ybase + co * cstride] = v;
    }
  };
  emit(acc00, 0, 0);
  emit(acc01, 0, 1);
  emit(acc10, 1, 0);
  emit(acc11, 1, 1);
}

constexpr int C1_WAVES = 8;  // waves per conv3 block: each sums C/8 channels of 64 pixels

template <int DIL>
__global__ __launch_bounds__(64 * C1_WAVES) void conv3x3_cout1_kernel(
    const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int C, int H,
    int W, int in_row0, int in_rows, int out_row0, const int32_t* gate, int32_t gate_tag) {
  __shared__ float part[C1_WAVES][64];
  if (gate && *gate != gate_tag) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = blockIdx.x * 64 + lane;
  const int row = out_row0 + blockIdx.y;  // global output row
  const int b = blockIdx.z;
  const int64_t plane = (int64_t)in_rows * W;
  const float* xb = x + (int64_t)b * C * plane;
  bool okx[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int xx = col + (kx - 1) * DIL;
    okx[kx] = xx >= 0 && xx < W;
  }
  bool oky[3];  // block-uniform
  int64_t rowoff[3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = row + (ky - 1) * DIL;
    const int by = yy - in_row0;
    oky[ky] = yy >= 0 && yy < H && by >= 0 && by < in_rows;
    rowoff[ky] = oky[ky] ? (int64_t)by * W : 0;
  }
  // contiguous channel range per wave, 4 channels per step with independent accumulators
  // (36 independent loads in flight per step; scalar weight loads)
  const int cpw = (C + C1_WAVES - 1) / C1_WAVES;
  const int c0 = wave * cpw, c1 = min(C, c0 + cpw);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  auto tapsum = [&](int c, float& a) __attribute__((always_inline)) {
    const float* xc = xb + (int64_t)c * plane;
    const float* wc = w + c * 9;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      if (!oky[ky]) continue;
      const float* xr = xc + rowoff[ky];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float v = okx[kx] ? xr[col + (kx - 1) * DIL] : 0.f;
        a += wc[ky * 3 + kx] * v;
      }
    }
  };
  int c = c0;
  for (; c + 4 <= c1; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) tapsum(c + u, acc[u]);
  }
  for (; c < c1; ++c) tapsum(c, acc[0]);
  part[wave][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (wave == 0 && col < W) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < C1_WAVES; ++i) sum += part[i][lane];
    y[((int64_t)b * gridDim.y + blockIdx.y) * W + col] = sum;
  }
}

// conv3 when DIL % 4 == 0 and W % 4 == 0 (the path's dilation-4 layer): a lane owns 4
// adjacent output pixels, so each tap is ONE 16-B load (the +-DIL taps stay 16-B aligned)
// instead of four 4-B loads (the scalar kernel above issues 4608 load instructions per
// pixel).  A block owns 16 pixel quads (flattened over the output rows) and splits the
// channels 64 ways: lane = (quad, channel subset) with 4 subsets per wave x 16 waves, so a
// 120x360 map runs as 675 blocks; sums reduce by shuffles, then over waves in LDS (fixed order).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int C1Q_WAVES = 16;
constexpr int C1Q_QUADS = 16;                          // quads per block
constexpr int C1Q_SUBS = C1Q_WAVES * (64 / C1Q_QUADS);  // channel subsets per block
template <int DIL>
__global__ __launch_bounds__(64 * C1Q_WAVES) void conv3x3_cout1_q4_kernel(
    const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int C, int H,
    int W, int in_row0, int in_rows, int out_row0, int out_rows, const int32_t* gate, int32_t gate_tag) {
  static_assert(DIL % 4 == 0, "16-B aligned taps");
  __shared__ f32x4_t part[C1Q_WAVES][C1Q_QUADS];
  if (gate && *gate != gate_tag) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qi = lane % C1Q_QUADS, sub = wave * (64 / C1Q_QUADS) + lane / C1Q_QUADS;
  const int qw = W / 4;
  // XCD-contiguous ranges of quads: the blocks of rows r-4 .. r+4 (which share input rows)
  // run on one XCD and hit its L2
  const int q = xcd_remap(blockIdx.x, gridDim.x) * C1Q_QUADS + qi;
  const bool active = q < out_rows * qw;
  const int r = active ? q / qw : 0;
  const int col = active ? 4 * (q - r * qw) : 0;
  const int row = out_row0 + r;
  const int b = blockIdx.y;
  const int64_t plane = (int64_t)in_rows * W;
  const float* xb = x + (int64_t)b * C * plane;
  int64_t off[3][3];
  bool ok[3][3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = row + (ky - 1) * DIL, by = yy - in_row0;
    const bool oky = active && yy >= 0 && yy < H && by >= 0 && by < in_rows;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int xx = col + (kx - 1) * DIL;
      ok[ky][kx] = oky && xx >= 0 && xx < W;  // xx % 4 == 0 and W % 4 == 0: the whole quad is in
      off[ky][kx] = ok[ky][kx] ? (int64_t)by * W + xx : 0;
    }
  }
  const int cps = (C + C1Q_SUBS - 1) / C1Q_SUBS;
  const int c0 = min(C, sub * cps), c1 = min(C, c0 + cps);
  f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  auto tapsum = [&](int c, f32x4_t& a) __attribute__((always_inline)) {
    const float* xc = xb + (int64_t)c * plane;
    const float* wc = w + c * 9;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(xc + off[ky][kx]);
        a += wc[ky * 3 + kx] * (ok[ky][kx] ? v : f32x4_t{0.f, 0.f, 0.f, 0.f});
      }
  };
  int c = c0;
  for (; c + 2 <= c1; c += 2) {
    tapsum(c, acc[0]);
    tapsum(c + 1, acc[1]);
  }
  if (c < c1) tapsum(c, acc[0]);
  f32x4_t s = acc[0] + acc[1];
#pragma unroll
  for (int o = C1Q_QUADS; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += __shfl_xor(s[e], o);
  if (lane < C1Q_QUADS) part[wave][qi] = s;
  __syncthreads();
  if (wave == 0 && lane < C1Q_QUADS && active) {
    f32x4_t sum = part[0][qi];
#pragma unroll
    for (int i = 1; i < C1Q_WAVES; ++i) sum += part[i][qi];
    *reinterpret_cast<f32x4_t*>(y + ((int64_t)b * out_rows + r) * W + col) = sum;
  }
}

// y = relu?(y + init) in place, NaN-preserving, and the non-finite report (ABI 11900): y [B][C][rows][W]
// holds grid rows [row0, row0 + rows) of init [C][H][W] (the coord term + bias).  Any non-finite result
// stores tag into *flag — the partial-sum multi-GPU mode's summed conv1 pre-activation, whose NaN / inf
// pattern is the reference's when every rank's partial is exact (the guard's gated exact conv2 then runs).
template <bool VEC>
__global__ __launch_bounds__(256) void bias_relu_nonfinite_kernel(float* __restrict__ y, const float* __restrict__ init,
                                                                  int C, int rows, int W, int H, int row0, int relu,
                                                                  int64_t n, int32_t* flag, int32_t tag) {
  constexpr int V = VEC ? 4 : 1;
  const int Wv = W / V;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = i % ((int64_t)rows * Wv), bc = i / ((int64_t)rows * Wv);
    const int r = (int)(pix / Wv), q = (int)(pix - (int64_t)r * Wv);
    const int c = (int)(bc % C);
    const int64_t io = ((int64_t)c * H + row0 + r) * W + (int64_t)q * V;
    if constexpr (VEC) {
      floatx4 v = reinterpret_cast<floatx4*>(y)[i];
      const floatx4 t = *reinterpret_cast<const floatx4*>(init + io);
      v += t;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (relu) v[e] = v[e] < 0.f ? 0.f : v[e];
        bad = bad || !isfinite(v[e]);
      }
      reinterpret_cast<floatx4*>(y)[i] = v;
    } else {
      float v = y[i] + init[io];
      if (relu) v = v < 0.f ? 0.f : v;
      bad = bad || !isfinite(v);
      y[i] = v;
    }
  }
  if (flag && bad) *flag = tag;
}

// conv1's coord term (ABI 12300): init[c][r][q] = bias[c] + sum over the 3 x 3 taps of conv1's two coord-channel
// weights times the coord map (persp_trans_detector.py:103-112: grid / (n - 1) * 2 - 1 in float64, then
// .float(); zero outside the grid, conv2d's padding, :51).  Input-independent, recomputed when the weights
// change (every training step).  A VALU kernel: a thread per output pixel evaluates its 3 x 3 coord window once
// (the float64 divisions) and loops over kCtCh output channels — 18 products and one coalesced store each, the
// channel's weights and bias wave-uniform (scalar loads).  The fp32-MFMA conv over an 8-channel padded coord
// input it replaces took 72 us at cfg2, this 39 us (one thread per (channel, pixel) with the divisions redone per
// channel took 108 us; unrolling the channel loop by 8: 42 us).
constexpr int kCtCh = 32;  // output channels per block
__global__ __launch_bounds__(256) void coord_term_kernel(const float* __restrict__ w, int64_t w_cout_stride,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         int Cout, int H, int W) {
  const int r = blockIdx.y, q = blockIdx.x * 256 + threadIdx.x;
  if (q >= W) return;
  float xv[3][3], yv[3][3];  // [ky][kx] the window's coord values, 0 where the tap is padding
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int qq = q + k - 1, rr = r + k - 1;
    const bool cv = qq >= 0 && qq < W, rv = rr >= 0 && rr < H;
    const float x = (float)((double)qq / (double)(W - 1) * 2.0 - 1.0);
    const float y = (float)((double)rr / (double)(H - 1) * 2.0 - 1.0);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      xv[j][k] = (cv && r + j - 1 >= 0 && r + j - 1 < H) ? x : 0.f;  // tap (ky = j, kx = k)
      yv[k][j] = (rv && q + j - 1 >= 0 && q + j - 1 < W) ? y : 0.f;  // tap (ky = k, kx = j)
    }
  }
  const int c0 = blockIdx.z * kCtCh, c1 = min(Cout, c0 + kCtCh);
  float* o = out + (int64_t)r * W + q;
  for (int c = c0; c < c1; ++c) {
    const float* wc = w + (int64_t)c * w_cout_stride;  // [2][3][3]: the x channel, then the y channel
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        acc = fmaf(wc[ky * 3 + kx], xv[ky][kx], acc);
        acc = fmaf(wc[9 + ky * 3 + kx], yv[ky][kx], acc);
      }
    o[(int64_t)c * H * W] = acc + (bias ? bias[c] : 0.f);
  }
}

}  // namespace mvbev

extern "C" {

int mvbev_coord_term_f32(const float* w1, int64_t cin, int64_t coord_c0, const float* bias, int64_t Cout, int64_t H,
                         int64_t W, float* out, void* stream) {
  using namespace mvbev;
  if (!w1 || !out) return MVBEV_ERR_NULL;
  if (cin <= 0 || Cout <= 0 || H <= 1 || W <= 1) return MVBEV_ERR_RANK;
  if (coord_c0 < 0 || coord_c0 + 2 > cin || H > 65535 || H * W > INT32_MAX - 256) return MVBEV_ERR_SHAPE;
  const dim3 grid((unsigned)ceil_div(W, (int64_t)256), (unsigned)H, (unsigned)ceil_div(Cout, (int64_t)kCtCh));
  hipLaunchKernelGGL(coord_term_kernel, grid, dim3(256), 0, as_stream(stream), w1 + coord_c0 * 9, cin * 9, bias, out,
                     (int)Cout, (int)H, (int)W);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_bias_relu_nonfinite_f32(float* y, const float* init, int64_t B, int64_t C, int64_t rows, int64_t W,
                                  int64_t H, int64_t row0, int relu, int32_t* flag, int32_t tag, void* stream) {
  using namespace mvbev;
  if (!y || !init) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || rows <= 0 || W <= 0 || H <= 0) return MVBEV_ERR_RANK;
  if (row0 < 0 || row0 + rows > H || C > INT32_MAX || H > INT32_MAX) return MVBEV_ERR_SHAPE;
  const bool vec = W % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 && (reinterpret_cast<uintptr_t>(init) & 15) == 0;
  const int64_t n = B * C * rows * W / (vec ? 4 : 1);
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(n, 256), 8192));
  if (vec)
    hipLaunchKernelGGL(bias_relu_nonfinite_kernel<true>, grid, dim3(256), 0, as_stream(stream), y, init, (int)C,
                       (int)rows, (int)W, (int)H, (int)row0, relu, n, flag, tag);
  else
    hipLaunchKernelGGL(bias_relu_nonfinite_kernel<false>, grid, dim3(256), 0, as_stream(stream), y, init, (int)C,
                       (int)rows, (int)W, (int)H, (int)row0, relu, n, flag, tag);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

size_t mvbev_conv3x3_packed_floats(int64_t Cout, int64_t K) {
  if (Cout <= 0 || K <= 0) return 0;
  return (size_t)mvbev::round_up(K, mvbev::KC) * 9 * (size_t)Cout;
}

int mvbev_pack_conv3x3_weight_f32_gated(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map,
                                        int64_t K, float* w_packed, const int32_t* gate, int32_t gate_tag,
                                        void* stream);

int mvbev_pack_conv3x3_weight_f32(const float* w, int64_t Cout, int64_t Cin_w,
                                  const int32_t* chan_map, int64_t K, float* w_packed,
                                  void* stream) {
  return mvbev_pack_conv3x3_weight_f32_gated(w, Cout, Cin_w, chan_map, K, w_packed, nullptr, 0, stream);
}

int mvbev_pack_conv3x3_weight_f32_gated(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map,
                                        int64_t K, float* w_packed, const int32_t* gate, int32_t gate_tag,
                                        void* stream) {
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout <= 0 || Cin_w <= 0 || K <= 0) return MVBEV_ERR_RANK;
  if (Cout % mvbev::BN != 0) return MVBEV_ERR_SHAPE;
  if (!chan_map && K != Cin_w) return MVBEV_ERR_SHAPE;
  const int64_t k_pad = mvbev::round_up(K, mvbev::KC);
  const int64_t total = k_pad * 9 * Cout;
  const int blocks = (int)std::min<int64_t>(mvbev::ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(mvbev::pack_conv3x3_kernel, dim3(blocks), dim3(256), 0,
                     mvbev::as_stream(stream), w, w_packed, (int)Cout, (int)Cin_w, chan_map,
                     (int)K, (int)k_pad, gate, gate_tag);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_f32_ex(const float* x, const mvbev_conv_desc* d, const float* w_packed, const float* bias,
                         const float* init, int64_t Cout, int dilation, int relu, float* y, int64_t y_band_rows,
                         const int32_t* gate, int32_t gate_tag, void* stream);

int mvbev_conv3x3_f32(const float* x, const mvbev_conv_desc* d, const float* w_packed,
                      const float* bias, const float* init, int64_t Cout, int dilation, int relu,
                      float* y, const int32_t* gate, int32_t gate_tag, void* stream) {
  return mvbev_conv3x3_f32_ex(x, d, w_packed, bias, init, Cout, dilation, relu, y, 0, gate, gate_tag, stream);
}

int mvbev_conv3x3_f32_ex(const float* x, const mvbev_conv_desc* d, const float* w_packed, const float* bias,
                         const float* init, int64_t Cout, int dilation, int relu, float* y, int64_t y_band_rows,
                         const int32_t* gate, int32_t gate_tag, void* stream) {
  using namespace mvbev;
  if (y_band_rows < 0 || y_band_rows > INT32_MAX) return MVBEV_ERR_SHAPE;
  if (!x || !d || !w_packed || !y) return MVBEV_ERR_NULL;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || d->in_rows <= 0 ||
      d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % BN != 0 || d->K % KC != 0 || d->group % KC != 0 || d->K % d->group != 0)
    return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H) return MVBEV_ERR_SHAPE;
  if (d->in_rows * d->W * KC > (int64_t)INT32_MAX || d->H > INT32_MAX / 2 || d->W > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(w_packed) & 15) != 0) return MVBEV_ERR_ALIGN;
  ConvArgs a{};
  a.x = x; a.wp = w_packed; a.bias = bias; a.init = init; a.y = y;
  a.group_stride = d->group_stride; a.batch_stride = d->batch_stride;
  a.group = (int)d->group; a.nchunks = (int)(d->K / KC); a.Cout = (int)Cout;
  a.H = (int)d->H; a.W = (int)d->W;
  a.in_row0 = (int)d->in_row0; a.in_rows = (int)d->in_rows;
  a.out_row0 = (int)d->out_row0; a.out_rows = (int)d->out_rows;
  a.gate = gate;
  a.gate_tag = gate_tag;
  a.band_rows = (int)y_band_rows;
  a.B = (int)d->B;
  constexpr int kWaves = MVBEV_CONV_WAVES;
  constexpr bool kDbuf = MVBEV_CONV_DBUF != 0;
  a.tiles_x = (int)ceil_div(d->W, TW);
  a.tiles_y = (int)ceil_div(d->out_rows, TileCfg<kWaves>::TH);
  a.n_cot = (int)(Cout / BN);
  const int64_t nwg = (int64_t)a.tiles_x * a.tiles_y * a.n_cot * d->B;
  if (nwg > (int64_t)INT32_MAX) return MVBEV_ERR_SHAPE;
  a.nwg = (int)nwg;
  hipStream_t s = as_stream(stream);
#define MVBEV_CONV_LAUNCH(D, R)                                                           \
  hipLaunchKernelGGL((conv3x3_mfma_f32_kernel<D, R, kWaves, kDbuf>), dim3((unsigned)nwg), \
                     dim3(TileCfg<kWaves>::NT), 0, s, a)
  if (dilation == 1) {
    if (relu) MVBEV_CONV_LAUNCH(1, true); else MVBEV_CONV_LAUNCH(1, false);
  } else if (dilation == 2) {
    if (relu) MVBEV_CONV_LAUNCH(2, true); else MVBEV_CONV_LAUNCH(2, false);
  } else {
    return MVBEV_ERR_DILATION;
  }
#undef MVBEV_CONV_LAUNCH
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_cout1_f32(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                            int64_t in_row0, int64_t in_rows, int64_t out_row0, int64_t out_rows,
                            const float* w, int dilation, float* y, const int32_t* gate, int32_t gate_tag,
                            void* stream) {
  using namespace mvbev;
  if (!x || !w || !y) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || in_rows <= 0 || out_rows <= 0)
    return MVBEV_ERR_RANK;
  if (out_row0 < 0 || out_row0 + out_rows > H || out_rows > 65535 || B > 65535)
    return MVBEV_ERR_SHAPE;
  hipStream_t s = as_stream(stream);
  if (dilation == 4 && W % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(y) & 15) == 0 && out_rows * (W / 4) <= (int64_t)INT32_MAX - 64) {
    dim3 qgrid((unsigned)ceil_div(out_rows * (W / 4), C1Q_QUADS), (unsigned)B);
    hipLaunchKernelGGL(conv3x3_cout1_q4_kernel<4>, qgrid, dim3(64 * C1Q_WAVES), 0, s, x, w, y, (int)C, (int)H,
                       (int)W, (int)in_row0, (int)in_rows, (int)out_row0, (int)out_rows, gate, gate_tag);
    MVBEV_CHECK_LAUNCH();
    return MVBEV_OK;
  }
  dim3 grid((unsigned)ceil_div(W, 64), (unsigned)out_rows, (unsigned)B);
#define MVBEV_C1_LAUNCH(D)                                                                      \
  hipLaunchKernelGGL(conv3x3_cout1_kernel<D>, grid, dim3(64 * C1_WAVES), 0, s, x, w, y, (int)C,  \
                     (int)H, (int)W, (int)in_row0, (int)in_rows, (int)out_row0, gate, gate_tag)
  switch (dilation) {
    case 1: MVBEV_C1_LAUNCH(1); break;
    case 2: MVBEV_C1_LAUNCH(2); break;
    case 4: MVBEV_C1_LAUNCH(4); break;
    default: return MVBEV_ERR_DILATION;
  }
#undef MVBEV_C1_LAUNCH
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

}  // extern "C"
