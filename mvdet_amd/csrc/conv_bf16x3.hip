// 3xbf16 split-precision 3x3 conv (fp32 in, fp32 out) on the bf16 MFMA for gfx950.
//
// Same operation and descriptor as mvbev_conv3x3_f32 (map_classifier[0:4],
// multiview_detector/models/persp_trans_detector.py:51-53), computed as
//     a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi,   a_hi = bf16(a), a_lo = bf16(a - a_hi)
// with fp32 accumulation in v_mfma_f32_32x32x16_bf16.  Each operand keeps 16 mantissa bits
// (the dropped a_lo*b_lo term and the rounding of the lo parts are <= ~2^-16 relative per
// product), i.e. fp32-class accuracy: measured <= ~1e-5 normwise vs fp32 on the fusion
// convs, against a parity gate of 1e-3 (and tighter than the TF32 that cuDNN's default uses
// for these convs on NVIDIA).  The bf16 MFMA issues 16x the fp32 MFMA's FLOP/clk, so the
// three passes still run 5.3x the fp32 rate.  Inputs may be fp32 or fp16 (an fp16 value is
// exactly hi + lo, so the fp16-storage config 4 path is exact in its products).
//
// Mapping: K is walked in chunks of 16 input channels (two 8-channel sub-blocks, each
// located on its own, so any channel group that is a multiple of 8 works); a chunk is 9
// MFMA K-blocks of 16 = (one tap, 16 channels): no padding MFMAs.  Lane l of the 32x32x16
// MFMA holds A[co = l&31][k = 8(l>>5) + j] and B[k][pixel = l&31], so the lane's 8 K-values
// are the 8 channels of sub-block l>>5 at one tap: the weights are pre-packed
// [tap][sub][co][8 ch] and the input halo is staged channel-innermost [sub][row][col][8 ch],
// both read as one ds_read_b128 per fragment (16 consecutive lanes = 256 contiguous bytes:
// conflict-free).  The input halo is split into hi/lo once at LDS-store time (or arrives
// pre-split); weights are split once at pack time.
// Workgroup tile: NW/2 row pairs x 32 cols x 128 output channels; wave = 2 rows x 64
// channels (2x2 accumulators of 32x32, the same epilogue as the fp32 kernel).
#include "common.h"

#include <type_traits>

namespace mvbev {
namespace b3 {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int SB = MVBEV_CONV_KC;  // 8 channels per sub-block (= the split layout's group)
constexpr int KC = 2 * SB;         // 16 input channels per chunk
constexpr int NKB = 9;             // K-blocks per chunk: one per tap
constexpr int BN = MVBEV_CONV_BN;  // 128 output channels per workgroup
constexpr int TW = 32;             // output columns per workgroup (= MFMA N)
constexpr int WPART = NKB * KC * BN;      // bf16 per part (hi or lo) per (chunk, cout tile)
constexpr int WBYTES = 2 * WPART * 2;     // hi + lo bytes per (chunk, cout tile) = 72 KiB
constexpr int W16 = WBYTES / 16;          // 16-B pieces (4608)

// packed[chunk][cot][part][tap][sub][co][j]: input channel = map(chunk*16 + sub*8 + j)
__global__ void pack_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int Cout,
                            int Cin_w, const int32_t* __restrict__ chan_map, int K, int K_pad) {
  const int n_cot = Cout / BN;
  const int64_t total = (int64_t)(K_pad / KC) * n_cot * 2 * WPART;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int j = r % SB; r /= SB;
    const int co = r % BN; r /= BN;
    const int sub = r % 2; r /= 2;
    const int tap = r % NKB; r /= NKB;
    const int part = r % 2; r /= 2;
    const int cot = r % n_cot;
    const int chunk = (int)(r / n_cot);
    const int k = chunk * KC + sub * SB + j;
    int ci = k < K ? (chan_map ? chan_map[k] : k) : -1;
    if (ci >= Cin_w) ci = -1;
    const float v = ci >= 0 ? w[((int64_t)(cot * BN + co) * Cin_w + ci) * 9 + tap] : 0.f;
    const __bf16 hi = (__bf16)v;
    out[i] = part ? (__bf16)(v - (float)hi) : hi;
  }
}

// Data-gradient packing (conv backward): the dgrad of a stride-1 3x3 conv with padding =
// dilation is the same conv over dy with w'[k][co][t] = w[co][k][8 - t].  Packed-conv output
// channel o = forward input channel chan_map[o] (-1 or o >= K_map: zero), packed input channel
// k = forward output channel k; same layout as pack_kernel.
__global__ void pack_dgrad_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int Cout_p,
                                  int Cf_out, int Cf_in, const int32_t* __restrict__ chan_map, int K_map,
                                  int K_pad) {
  const int n_cot = Cout_p / BN;
  const int64_t total = (int64_t)(K_pad / KC) * n_cot * 2 * WPART;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int j = r % SB; r /= SB;
    const int co = r % BN; r /= BN;
    const int sub = r % 2; r /= 2;
    const int tap = r % NKB; r /= NKB;
    const int part = r % 2; r /= 2;
    const int cot = r % n_cot;
    const int chunk = (int)(r / n_cot);
    const int k = chunk * KC + sub * SB + j;
    const int o = cot * BN + co;
    int ci = o < K_map ? (chan_map ? chan_map[o] : o) : -1;
    if (ci >= Cf_in) ci = -1;
    const float v = (ci >= 0 && k < Cf_out) ? w[((int64_t)k * Cf_in + ci) * 9 + (NKB - 1 - tap)] : 0.f;
    const __bf16 hi = (__bf16)v;
    out[i] = part ? (__bf16)(v - (float)hi) : hi;
  }
}

struct Args {
  const void* x;
  const u32x4* wp;
  const float* bias;
  const float* init;
  float* y;
  int64_t group_stride, batch_stride;
  int B, group, K, nchunks, Cout, H, W;
  int in_row0, in_rows, out_row0, out_rows;
  int tiles_x, tiles_y, n_cot, nwg;
  // split-K tail (sk_ws != nullptr): tiles [0, dp_tiles) run whole (full rounds over the
  // CUs); each remaining tile is cut into `split` K-ranges run by separate workgroups,
  // which leave raw partial sums in sk_ws for sk_fixup_kernel
  float* sk_ws;
  int dp_tiles, split;
  // frustum mask (optional): per output tile (tile_y * tiles_x + tile_x) bit g = input
  // channel group g can be non-zero in the tile's halo; clear groups' chunks are skipped
  const uint32_t* gmask;
  int cpg;  // K-chunks per channel group when gmask is set
  // with gmask: pixel tiles (b, ty, tx) in dispatch order (heaviest first, optional) and
  // their count; blocks interleave them over the XCDs, the Cout tiles of one pixel tile
  // stay on one XCD (they share the halo reads)
  const int32_t* tile_order;
  int npix;
  int mgroup;    // row-Winograd conv: consecutive ordered pixel tiles per XCD turn (MVBEV_MASK_GROUP's runtime form)
  bool y_split;  // y in the split-bf16 blocked layout (the next conv's 16-B staging copies)
  bool y_pix;    // with y_split: pixel-major split-bf16 [B][out_rows][W][Cout / 8][hi, lo] (the warp adjoint's gathers)
  // output-side mask (optional, dgrad of the fused conv): per output tile, bit g clear =
  // output channel group g (cot_pg Cout tiles each) is never read, so its tiles are skipped
  const uint32_t* cmask;
  int cot_pg;
  // fused single-output-channel conv after this one (ring kernel only): w3 [Cout][9] fp32;
  // p3 receives, per (Cout tile, 64-channel half) set, tap and output pixel, the partial
  // sum over the set's channels of w3[co][tap] * act(y[co][pixel]) ([B][2 n_cot][9][out_rows][W]);
  // y may then be null (not stored)
  const float* w3;
  float* p3;
  // ring kernel schedule (optional, mvbev_conv_schedule): block i runs items[i] = (tile, first
  // chunk, end chunk of the tile's active-chunk sequence, partial slot or -1); split tiles'
  // raw partial sums (slots of kRingSlotF4 floatx4) are finished by conv_ring_fixup_kernel from
  // fix[f] = (tile, first slot, pieces)
  const int4* items;
  int nitems;
  const int4* fix;
  int nfix;
  // edge strip (ring kernel, optional): pixel tiles [tiles_y * tiles_x, + edge_tiles) of each
  // batch item are edge_rows x (W - edge_x0) tiles of columns [edge_x0, W) (RingGeo EW)
  int edge_tiles, edge_x0, edge_rows, edge_w;
  // fp32 y in row bands (optional, > 0): computed row r (from out_row0) goes to band r / band_rows,
  // y = [bands][B][Cout][band_rows][W] — the reduce-scatter's input of the partial-sum multi-GPU
  // mode, written in place (no band-major copy)
  int band_rows;
};

// Input tag: the split-bf16 blocked layout written by mvbev_warp_views_split_bf16 and by this
// kernel's own split epilogue (per pixel and 8-channel group: 16 B hi, 16 B lo).
struct SplitIn {};

template <typename T> __device__ inline float ld(const T* p);
template <> __device__ inline float ld<float>(const float* p) { return *p; }
template <> __device__ inline float ld<_Float16>(const _Float16* p) { return (float)*p; }

#ifndef MVBEV_B3_MINWAVES
#define MVBEV_B3_MINWAVES 1
#endif
#ifndef MVBEV_MASK_GROUP
#define MVBEV_MASK_GROUP 1  // consecutive ordered pixel tiles per XCD turn (ring kernel, cfg2 conv1: 1 2.17-2.24 ms, 2 2.23-2.28, 4 2.41)
#endif
#ifndef MVBEV_B3_DEPTH
#define MVBEV_B3_DEPTH 2  // staging-register ring depth (1 or 2)
#endif

// One finished 32x32 accumulator block (output channels co0..co0+31 at output pixel
// (row, col) of this lane): bias, coord-term init, ReLU, store fp32 or split-bf16.
// INIT = false: the caller folded the init term into its accumulators already (the row-Winograd convs' prologue)
template <bool RELU, bool INIT = true>
__device__ inline void store_block(const Args& a, int b, int row, int col, int co0, const floatx16& acc) {
  const int kh = (threadIdx.x & 63) >> 5;
  const int W = a.W;
  const int64_t oplane = (int64_t)a.out_rows * W;
  const int64_t iplane = (int64_t)a.H * W;
  const bool valid = row < a.out_row0 + a.out_rows && col < W;
  if (!a.y_split) {
    if (!valid) return;
    // the pixel's address and the channel stride, plain or banded, chosen once (a branch inside the
    // unrolled loop put the accumulators in scratch)
    const int rr = row - a.out_row0;
    const int band = a.band_rows > 0 ? rr / a.band_rows : 0;
    const int64_t cstride = a.band_rows > 0 ? (int64_t)a.band_rows * W : oplane;
    float* yp = a.y + ((int64_t)band * a.B + b) * a.Cout * cstride +
                (int64_t)(a.band_rows > 0 ? rr - band * a.band_rows : rr) * W + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
      float v = acc[r];
      if (a.bias) v += a.bias[co];
      if (INIT && a.init) v += a.init[co * iplane + (int64_t)row * W + col];
      if (RELU) v = v < 0.f ? 0.f : v;
      yp[co * cstride] = v;
    }
    return;
  }
  // split-bf16 output: the lane holds channels 4kh..4kh+3 of four 8-channel groups; its
  // partner lane (lane ^ 32) holds the other half.  kh = 0 writes each group's 16-B hi
  // piece, kh = 1 its lo piece, after swapping the half the partner needs (every lane
  // takes part in the shuffles; only the store is predicated).
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned int hp[2], lp[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int r = 4 * q + 2 * h + e;
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        float v = acc[r];
        if (a.bias) v += a.bias[co];
        if (INIT && a.init && valid) v += a.init[co * iplane + (int64_t)row * W + col];
        if (RELU) v = v < 0.f ? 0.f : v;
        v2[e] = v;
      }
      const __bf16 h0 = (__bf16)v2[0], h1 = (__bf16)v2[1];
      const __bf16 l0 = (__bf16)(v2[0] - (float)h0), l1 = (__bf16)(v2[1] - (float)h1);
      hp[h] = (unsigned)__builtin_bit_cast(unsigned short, h0) |
              ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
      lp[h] = (unsigned)__builtin_bit_cast(unsigned short, l0) |
              ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
    }
    // v_permlane32_swap (the hi dword of the upper half-wave <-> the lo dword of the lower): lanes 0-31 then hold
    // their hi and the upper lanes' hi (the group's 16-B hi piece), lanes 32-63 the lower lanes' lo and their own lo
    // (the lo piece) — in VALU, without the two ds_bpermute round trips of a __shfl_xor(.., 32) per dword
    const auto x0 = __builtin_amdgcn_permlane32_swap(hp[0], lp[0], false, false);
    const auto x1 = __builtin_amdgcn_permlane32_swap(hp[1], lp[1], false, false);
    const u32x4 piece = u32x4{x0[0], x1[0], x0[1], x1[1]};
    if (valid) {
      const int64_t g = co0 / 8 + q;
      u32x4* out = reinterpret_cast<u32x4*>(a.y);
      const int64_t pix = ((int64_t)b * a.out_rows + (row - a.out_row0)) * W + col;
      out[2 * (a.y_pix ? pix * (a.Cout / 8) + g
                       : (((int64_t)b * (a.Cout / 8) + g) * a.out_rows + (row - a.out_row0)) * W + col) + kh] = piece;
    }
  }
}

// Output of one finished tile from the accumulators of the tile's waves; shared by the
// conv kernel and the stream-K fixup.
template <bool RELU, int NW>
__device__ inline void tile_epilogue(const Args& a, int tile, const floatx16 (&acc)[2][2]) {
  constexpr int TH = NW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cot = tile % a.n_cot;
  int rest = tile / a.n_cot;
  const int tx = rest % a.tiles_x;
  rest /= a.tiles_x;
  const int ty = rest % a.tiles_y;
  const int b = rest / a.tiles_y;
  const int y0 = a.out_row0 + ty * TH;
  const int prow = 2 * (wave % (NW / 2));
  const int cw = 64 * (wave / (NW / 2));
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
      store_block<RELU>(a, b, y0 + prow + pt, tx * TW + (lane & 31), cot * BN + cw + 32 * ct, acc[ct][pt]);
}

// stream-K partial slot: [slot][16 float4 of the thread's 64 accumulators][thread] (coalesced)
template <int NW>
__device__ inline void store_partial(float* ws, int slot, const floatx16 (&acc)[2][2]) {
  constexpr int NT = 64 * NW;
  floatx4* p = reinterpret_cast<floatx4*>(ws) + (int64_t)slot * 16 * NT + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        p[(int64_t)((i * 2 + j) * 4 + q) * NT] = v;
      }
}

template <int NW>
__device__ inline void add_partial(const float* ws, int slot, floatx16 (&acc)[2][2]) {
  constexpr int NT = 64 * NW;
  const floatx4* p = reinterpret_cast<const floatx4*>(ws) + (int64_t)slot * 16 * NT + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 v = p[(int64_t)((i * 2 + j) * 4 + q) * NT];
        acc[i][j][4 * q] += v[0];
        acc[i][j][4 * q + 1] += v[1];
        acc[i][j][4 * q + 2] += v[2];
        acc[i][j][4 * q + 3] += v[3];
      }
}

// Finishes the split tail tiles: block t sums the `split` partial slots of tail tile t in
// K order (deterministic) and writes the tile like the conv kernel's epilogue.
template <bool RELU, int NW>
__global__ __launch_bounds__(64 * NW) void sk_fixup_kernel(const Args a) {
  const int t = blockIdx.x;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};
  for (int p = 0; p < a.split; ++p) add_partial<NW>(a.sk_ws, t * a.split + p, acc);
  tile_epilogue<RELU, NW>(a, a.dp_tiles + t, acc);
}

template <typename TIn, int DIL, bool RELU, int NW>
__global__ __launch_bounds__(64 * NW, MVBEV_B3_MINWAVES) void conv_kernel(const Args a) {
  constexpr int NT = 64 * NW;
  constexpr int TH = NW;                 // NW/2 row pairs, 2 channel halves
  constexpr int XH = TH + 2 * DIL, XW = TW + 2 * DIL;
  constexpr int XPIX = XH * XW;          // halo pixels per sub-block
  constexpr int XPT = (XPIX + NT - 1) / NT;
  constexpr int WLD = (W16 + NT - 1) / NT;
  constexpr int XPAD = XPT * NT;         // X image entries incl. a dummy tail for idle threads
  constexpr int BUF = W16 + 4 * XPAD;    // 16-B pieces: W, then X [sub][part][XPAD]
  __shared__ __attribute__((aligned(16))) u32x4 lds[BUF];

  const int W = a.W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, kh = lane >> 5;
  const int64_t plane = (int64_t)a.in_rows * W;
  const int64_t wchunk = (int64_t)a.n_cot * W16;
  const int n = a.nchunks;

  // a whole tile, or (split-K tail) one K-range of a tail tile
  // XCD remap within each phase: the whole tiles (dispatched first, a multiple of the CU
  // count) and the tail pieces each get contiguous ranges per XCD
  const int bid = blockIdx.x;
  const bool tail = a.sk_ws && bid >= a.dp_tiles;
  const int wg = tail ? a.dp_tiles + xcd_remap(bid - a.dp_tiles, a.nwg - a.dp_tiles)
                      : xcd_remap(bid, a.sk_ws ? a.dp_tiles : a.nwg);
  int tile = wg, k0 = 0, k1 = n, piece = -1;  // K-range in (active) chunk order
  if (a.gmask) {  // uneven per-tile work: spread pixel tiles over the XCDs, heaviest first
    // XCD x runs groups of MVBEV_MASK_GROUP consecutive slots of the order (tiles with the
    // same view set, so concurrent workgroups share weight chunks in L2), groups dealt
    // round-robin over the XCDs (balance)
    constexpr int G = MVBEV_MASK_GROUP;
    const int x = bid & 7, j = bid >> 3;
    const int q = j / a.n_cot;
    const int slot = G * (8 * (q / G) + x) + q % G;
    if (slot >= a.npix) return;  // padding block (whole block, before any barrier)
    tile = (a.tile_order ? a.tile_order[slot] : slot) * a.n_cot + j % a.n_cot;
  }
  if (tail) {
    piece = wg - a.dp_tiles;
    tile = a.dp_tiles + piece / a.split;
    const int p = piece % a.split;
    k0 = (int)((int64_t)n * p / a.split);
    k1 = (int)((int64_t)n * (p + 1) / a.split);
  }
  const int cot = tile % a.n_cot;
  int rest = tile / a.n_cot;
  const int tx = rest % a.tiles_x;
  rest /= a.tiles_x;
  const int ty = rest % a.tiles_y;
  const int b = rest / a.tiles_y;
  const int x0 = tx * TW;
  const int y0 = a.out_row0 + ty * TH;
  // output-side mask: a tile of output channels nobody reads (whole block, before any barrier)
  if (a.cmask && !((a.cmask[ty * a.tiles_x + tx] >> (cot / a.cot_pg)) & 1u)) return;
  const u32x4* wsrc = a.wp + (int64_t)cot * W16;
  // frustum mask: iterate only the chunks of groups that can be non-zero in this tile
  const uint32_t gm = a.gmask ? a.gmask[ty * a.tiles_x + tx] : 0u;
  if (a.gmask) k1 = __builtin_popcount(gm) * a.cpg;  // (never combined with the split-K tail)
  auto chunk_of = [&](int i) -> int {
    if (!a.gmask) return i;
    uint32_t m = gm;
    for (int j = i / a.cpg; j > 0; --j) m &= m - 1;  // drop the lower set groups
    return __builtin_ctz(m) * a.cpg + i % a.cpg;
  };

  // halo pixels of this thread (chunk-invariant): plane offset + validity
  int xoff[XPT];
  bool xok[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int p = tid + NT * i;
    const int r = p / XW, c = p % XW;
    const int gy = y0 - DIL + r, gx = x0 - DIL + c;
    const int by = gy - a.in_row0;
    xok[i] = p < XPIX && gy >= 0 && gy < a.H && by >= 0 && by < a.in_rows && gx >= 0 && gx < W;
    xoff[i] = xok[i] ? (int)((int64_t)by * W + gx) : 0;
  }

  constexpr bool SPLIT = std::is_same<TIn, SplitIn>::value;
  using XElem = typename std::conditional<SPLIT, float, TIn>::type;  // element type when not split
  // staging-register ring: DEPTH chunks of global loads in flight ahead of the MFMAs
  constexpr int DEPTH = MVBEV_B3_DEPTH;
  u32x4 wreg[DEPTH][WLD];
  float xreg[DEPTH][2][XPT][SPLIT ? 1 : SB];
  u32x4 xs[DEPTH][2][XPT][SPLIT ? 2 : 1];
  bool sok[DEPTH][2];
  // Sub-block base (elements) of packed channel k0; sub-blocks past K read sub-block 0's
  // pixels (always valid memory) and are zeroed at store time.
#define B3_SUB_BASE(k0)                                                                      \
  ({                                                                                         \
    const int g_ = (k0) / a.group;                                                           \
    (int64_t)b * a.batch_stride + g_ * a.group_stride + (int64_t)((k0) - g_ * a.group) * plane; \
  })
#define B3_LOAD(ci, sl)                                                                      \
  do {                                                                                       \
    const int ch_ = chunk_of(ci);                                                            \
    const u32x4* ws_ = wsrc + (int64_t)ch_ * wchunk;                                         \
    _Pragma("unroll") for (int i = 0; i < WLD; ++i) {                                        \
      if (W16 % NT == 0 || tid + NT * i < W16) wreg[sl][i] = ws_[tid + NT * i];              \
    }                                                                                        \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                       \
      const int k0_ = ch_ * KC + s_ * SB;                                                    \
      sok[sl][s_] = k0_ < a.K;                                                               \
      const int64_t cb_ = B3_SUB_BASE(sok[sl][s_] ? k0_ : ch_ * KC);                         \
      if constexpr (SPLIT) {                                                                 \
        const u32x4* xc_ = static_cast<const u32x4*>(a.x) + cb_ / 4;                         \
        _Pragma("unroll") for (int i = 0; i < XPT; ++i) {                                    \
          xs[sl][s_][i][0] = xc_[2 * xoff[i]];                                               \
          xs[sl][s_][i][1] = xc_[2 * xoff[i] + 1];                                           \
        }                                                                                    \
      } else {                                                                               \
        const XElem* xc_ = static_cast<const XElem*>(a.x) + cb_;                             \
        _Pragma("unroll") for (int i = 0; i < XPT; ++i) {                                    \
          _Pragma("unroll") for (int j = 0; j < SB; ++j)                                     \
            xreg[sl][s_][i][j] = ld<XElem>(xc_ + j * plane + xoff[i]);                       \
        }                                                                                    \
      }                                                                                      \
    }                                                                                        \
  } while (0)
#define B3_STORE(sl)                                                                         \
  do {                                                                                       \
    _Pragma("unroll") for (int i = 0; i < WLD; ++i) {                                        \
      if (W16 % NT == 0 || tid + NT * i < W16) lds[tid + NT * i] = wreg[sl][i];              \
    }                                                                                        \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                       \
      u32x4* Xhi = lds + W16 + s_ * 2 * XPAD;                                                \
      u32x4* Xlo = Xhi + XPAD;                                                               \
      _Pragma("unroll") for (int i = 0; i < XPT; ++i) {                                      \
        /* unconditional: threads past the halo write the dummy tail (no branch, so the    \
           compiler's vmcnt counting stays exact across the prefetch ring) */              \
        const int p = tid + NT * i;                                                          \
        const bool ok_ = xok[i] && sok[sl][s_];                                              \
        if constexpr (SPLIT) {                                                               \
          const u32x4 z_ = {0u, 0u, 0u, 0u};                                                 \
          Xhi[p] = ok_ ? xs[sl][s_][i][0] : z_;                                              \
          Xlo[p] = ok_ ? xs[sl][s_][i][1] : z_;                                              \
        } else {                                                                             \
          bf16x8 hi, lo;                                                                     \
          _Pragma("unroll") for (int j = 0; j < SB; ++j) {                                   \
            const float v = ok_ ? xreg[sl][s_][i][j] : 0.f;                                  \
            const __bf16 h_ = (__bf16)v;                                                     \
            hi[j] = h_;                                                                      \
            lo[j] = (__bf16)(v - (float)h_);                                                 \
          }                                                                                  \
          Xhi[p] = __builtin_bit_cast(u32x4, hi);                                            \
          Xlo[p] = __builtin_bit_cast(u32x4, lo);                                            \
        }                                                                                    \
      }                                                                                      \
    }                                                                                        \
  } while (0)

  const int prow = 2 * (wave % (NW / 2));
  const int cw = 64 * (wave / (NW / 2));
  // per tap B offsets in the halo image (lane half kh reads sub-block kh)
  int boff[NKB];
#pragma unroll
  for (int t = 0; t < NKB; ++t) boff[t] = kh * 2 * XPAD + (prow + (t / 3) * DIL) * XW + l32 + (t % 3) * DIL;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};

#ifndef MVBEV_B3_PIPE
#define MVBEV_B3_PIPE 1  // read tap t+1's fragments from LDS under tap t's MFMAs
#endif
  auto compute = [&]() __attribute__((always_inline)) {
    const u32x4* Wl = lds;
    const u32x4* X = lds + W16;
    // fragment registers: [set][ahi0, ahi1, alo0, alo1] and [set][bhi0, bhi1, blo0, blo1]
    constexpr int NSET = MVBEV_B3_PIPE ? 2 : 1;
    bf16x8 fa[NSET][4], fb[NSET][4];
    auto fetch = [&](int t, int st) __attribute__((always_inline)) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int wi = (t * 2 + kh) * BN + cw + 32 * ct + l32;
        fa[st][ct] = __builtin_bit_cast(bf16x8, Wl[wi]);
        fa[st][2 + ct] = __builtin_bit_cast(bf16x8, Wl[NKB * 2 * BN + wi]);
      }
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        fb[st][pt] = __builtin_bit_cast(bf16x8, X[boff[t] + pt * XW]);
        fb[st][2 + pt] = __builtin_bit_cast(bf16x8, X[boff[t] + XPAD + pt * XW]);
      }
    };
    auto mfmas = [&](int st) __attribute__((always_inline)) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[st][2 + ct], fb[st][pt], acc[ct][pt], 0, 0, 0);
          acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[st][ct], fb[st][2 + pt], acc[ct][pt], 0, 0, 0);
          acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[st][ct], fb[st][pt], acc[ct][pt], 0, 0, 0);
        }
    };
    if constexpr (NSET == 2) {
      fetch(0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // tap 0's reads first
#pragma unroll
      for (int t = 0; t < NKB; ++t) {
        if (t + 1 < NKB) fetch(t + 1, (t + 1) & 1);
        mfmas(t & 1);
        if (t + 1 < NKB) {
          // interleave: the next tap's 8 fragment reads between this tap's first 8 MFMAs
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < NKB; ++t) {
        fetch(t, 0);
        mfmas(0);
      }
    }
  };

  if (k1 <= k0) {
    // no view reaches this tile: the output is the epilogue terms alone
  } else if constexpr (DEPTH == 2) {
    // Two chunks of loads in flight: slot 0 holds even chunks, slot 1 odd ones. Loads are
    // unconditional (index clamped; the last chunk is re-read at most twice) so the
    // loop body is straight-line and the compiler's vmcnt counting stays exact.
    const int last = k1 - 1;
    B3_LOAD(k0, 0);
    B3_LOAD(min(k0 + 1, last), 1);
    int ch = k0;
    for (; ch + 1 < k1; ch += 2) {
      __syncthreads();
      B3_STORE(0);
      __syncthreads();
      B3_LOAD(min(ch + 2, last), 0);
      compute();
      __syncthreads();
      B3_STORE(1);
      __syncthreads();
      B3_LOAD(min(ch + 3, last), 1);
      compute();
    }
    if (ch < k1) {
      __syncthreads();
      B3_STORE(0);
      __syncthreads();
      compute();
    }
  } else {
    B3_LOAD(k0, 0);
    for (int ch = k0; ch < k1; ++ch) {
      __syncthreads();
      B3_STORE(0);
      __syncthreads();
      if (ch + 1 < k1) B3_LOAD(ch + 1, 0);
      compute();
    }
  }
#undef B3_LOAD
#undef B3_STORE
#undef B3_SUB_BASE

  if (piece < 0) {
    tile_epilogue<RELU, NW>(a, tile, acc);
  } else {  // one K-range of a tail tile: raw partial sums, finished by sk_fixup_kernel
    store_partial<NW>(a.sk_ws, piece, acc);
  }
}

// ---------------------------------------------------------------------------------------
// Ring kernel: the default for split-bf16 input (conv1 over the warped slab, conv2 over y1).
//
// conv_kernel above stages each 16-channel chunk (72 KiB of weights + the halo) through
// registers into one LDS image between two barriers, so every chunk's ds_write pass runs
// while the MFMAs idle, and the 2-deep register ring holds the VGPR file at 256.  Here the
// staging is LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write) into a ring, and the
// freed registers buy a taller wave tile:
//   * unit = (chunk, kernel column kw): 3 taps x 16 channels x 128 Cout = 24 KiB of weights;
//     W ring of 3 unit slots, halo images (whole chunk) double-buffered: 136 KiB (d1) /
//     152 KiB (d2) of LDS, one workgroup per CU;
//   * workgroup tile 12 rows x 32 cols x 128 Cout, 8 waves = 4 row groups x 2 Cout halves,
//     wave = 3 output rows x 64 Cout (2x3 accumulators).  Rows of a wave are DIL apart, so a
//     kernel column's 3 taps read only 5 distinct input rows: the B fragments of a unit are
//     loaded once (10 ds_read_b128) and reused by its 3 taps;
//   * one barrier per unit, placed before the unit's last tap: the wait before it retires
//     W(u+1) (and the next chunk's halo), the DMA after it refills the slot of unit u (whose
//     last fragments were read before the barrier) with W(u+3), so two units of DMA latency
//     are hidden, and the last tap's MFMAs cover the next unit's fragment reads.
// Counted waits only (vmcnt per unit position, raw s_barrier): __syncthreads() would drain
// the DMAs in flight (cdna_hip_programming.md §5, "Pipelining across barriers").
// Accumulation order per output: chunk, then kw, then kh (the register kernel: chunk, tap);
// the same fp32-accumulated 3xbf16 products, so the same accuracy.
constexpr int RT = 12;                          // output rows per workgroup tile
constexpr int RNW = 8;                          // waves
constexpr int RNT = 64 * RNW;
constexpr int RUNIT = 2 * 3 * 2 * BN;           // 16-B pieces of one W unit (hi + lo): 1536
constexpr int RHALF = RUNIT / 2;                // one part (hi or lo) of a unit
#ifndef MVBEV_RING_DMAW
#define MVBEV_RING_DMAW 4  // waves that issue the LDS-DMAs: 4 = one wave per SIMD issues them while its partner
                           // only computes (conv1 -3 %, conv2 -2 % vs all 8 waves issuing)
#endif
constexpr int RNIW = MVBEV_RING_DMAW;           // issuing waves
constexpr int RNIT = 64 * RNIW;                 // issuing lanes
constexpr int RNWI = RUNIT / RNIT;              // LDS-DMA instructions per issuing wave per W unit (3)
static_assert(RNIW == 4 || RNIW == 8, "issuing waves");
static_assert(RUNIT % RNIT == 0, "W unit must split evenly over the waves");
// EW: tile width.  32 = the regular 12 x 32 tile (an MFMA's 32 pixels are one row segment);
// 8 / 16 = an edge-strip tile of 12 * 32 / EW rows x EW columns for the last W % 32 columns
// (an MFMA's 32 pixels are 32 / EW row segments 12 rows apart, so the 3 taps of a kernel
// column still share a wave's 5 fragment rows).  Same pixel count, halo of the same size class.
template <int DIL, int EW = TW> struct RingGeo {
  static_assert(EW == 8 || EW == 16 || EW == 32, "tile width");
  static constexpr int XH = RT * (TW / EW) + 2 * DIL, XW = EW + 2 * DIL, XPIX = XH * XW;
  static constexpr int NX = (4 * XPIX + RNIT - 1) / RNIT;  // LDS-DMA instructions per issuing wave per halo
  static constexpr int XBUF = NX * RNIT;                   // entries per halo buffer (incl. tail)
  static constexpr int LDS = 3 * RUNIT + 2 * XBUF;       // 16-B entries
  static_assert(LDS * 16 <= 160 * 1024, "LDS");
};
__device__ u32x4 g_ring_zero[1];  // zero-initialised source of padding halo entries

// first output row (tile-relative) of row group rg; its rows are base + pt * DIL, pt < 3
template <int DIL>
__device__ inline int ring_base_row(int rg) {
  static_assert(DIL == 1 || DIL == 2, "dilation");
  return DIL == 1 ? 3 * rg : (rg >> 1) * 6 + (rg & 1);
}

template <int AUX = 0>
__device__ inline void glds16(const u32x4* src, u32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, AUX);
}
// (Variants measured and removed, DESIGN.md §4: non-temporal halo DMAs, s_setprio around the MFMA
// stream, DMAs placed one per MFMA, staggered barriers for waves 4-7; the timing ablations live in
// the round-2/3 records, not in this source.)

// Epilogue of a conv followed by a single-output-channel conv (conv2 -> conv3, map_classifier[2:5],
// persp_trans_detector.py:53-54): instead of storing the activation, each lane forms, for its
// pixel and the 9 taps of the next conv, the dot product of its channels' activations with
// w3[co][tap]; the two lane halves are added, and lanes 0-31 store one partial per (set,
// tap, pixel), set = (Cout tile, 64-channel half of the wave).  cout1_reduce_kernel then sums
// the sets' shifted taps in a fixed order.  w3 is staged in LDS ([tap][128 co] of this Cout
// tile) after the K loop: 4 consecutive channels = one ds_read_b128 per (tap, 8-channel quad).
template <bool RELU, int NPT = 3>
__device__ __attribute__((always_inline)) inline void cout1_partials(const Args& a, int b, int row_base, int dil,
                                                                    int col, int cot, int cw,
                                      const floatx16 (&acc)[2][NPT], u32x4* lds) {
  const int tid = threadIdx.x, kh = (tid & 63) >> 5;
  // LDS (the ring buffers, free after the K loop): w3s [9][128] then the bias [128]
  float* w3s = reinterpret_cast<float*>(lds);
  float* bs = w3s + 9 * BN;
  __syncthreads();  // every wave is past its last fragment read of the ring buffers
  for (int i = tid; i < 10 * BN; i += blockDim.x) {
    const int t = i / BN, co = i - t * BN;
    w3s[i] = t < 9 ? a.w3[(int64_t)(cot * BN + co) * 9 + t] : (a.bias ? a.bias[cot * BN + co] : 0.f);
  }
  __syncthreads();
  const int W = a.W;
  const int nsets = 2 * a.n_cot, set = 2 * cot + cw / 64;
  // per row: per (Cout block, 4-channel quad) the 4 activations, then the 9 taps' weights one
  // floatx4 at a time (9 sums + 4 activations + 4 weights live; the weights re-read per row)
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) {
    float s[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) s[t] = 0.f;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cl = cw + 32 * ct + 8 * q + 4 * kh;  // 4 consecutive channels of this lane
        const floatx4 bq = *reinterpret_cast<const floatx4*>(bs + cl);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = acc[ct][pt][4 * q + e] + bq[e];
          v[e] = RELU ? (t < 0.f ? 0.f : t) : t;
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const floatx4 w = *reinterpret_cast<const floatx4*>(w3s + t * BN + cl);
#pragma unroll
          for (int e = 0; e < 4; ++e) s[t] += w[e] * v[e];
        }
        __builtin_amdgcn_sched_barrier(0);  // one quad's weights in registers at a time
      }
#pragma unroll
    for (int t = 0; t < 9; ++t) s[t] += __shfl_xor(s[t], 32);
    const int row = row_base + pt * dil;
    if (kh == 0 && row < a.out_row0 + a.out_rows && col < W) {
      float* p = a.p3 + ((((int64_t)b * nsets + set) * 9) * a.out_rows + (row - a.out_row0)) * W + col;
#pragma unroll
      for (int t = 0; t < 9; ++t) p[(int64_t)t * a.out_rows * W] = s[t];
    }
  }
}

// map[b][0][q][c] = sum over sets s, taps t of p3[b][s][t][q + d(t/3 - 1)][c + d(t%3 - 1)]
// (zero outside the image): the single-output conv from the partials above, fixed order.
// Block = 64 map columns x 4 waves: wave g sums the sets g, g + 4, ... (each set's 9 shifted taps in
// tap order), then wave 0 adds the 4 waves' sums in wave order — a fixed order, 4x the waves of one
// thread per output (the reduce was latency-bound at under one wave per SIMD: 27 -> ~10 us at cfg2).
constexpr int kC1rGroups = 4;
__global__ __launch_bounds__(64 * kC1rGroups) void cout1_reduce_kernel(const float* __restrict__ p3, int nsets, int H,
                                                                      int W, int rows_p, int row0_p, int dil,
                                                                      float* __restrict__ map, int map_row0,
                                                                      int map_rows) {
  __shared__ float part[kC1rGroups][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, qr = blockIdx.y, b = blockIdx.z;
  const int q = map_row0 + qr;
  const float* pb = p3 + (int64_t)b * nsets * 9 * rows_p * W;
  float acc = 0.f;
  if (c < W) {
    for (int s = g; s < nsets; s += kC1rGroups)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r = q + dil * (t / 3 - 1), cc = c + dil * (t % 3 - 1);
        if (r >= 0 && r < H && cc >= 0 && cc < W)
          acc += pb[(((int64_t)s * 9 + t) * rows_p + (r - row0_p)) * W + cc];
      }
  }
  part[g][lane] = acc;
  __syncthreads();
  if (g == 0 && c < W) {
    float sum = part[0][lane];
#pragma unroll
    for (int k = 1; k < kC1rGroups; ++k) sum += part[k][lane];
    map[((int64_t)b * map_rows + qr) * W + c] = sum;
  }
}

// The ring kernel's output of a finished tile: rows row_base + pt * DIL (pt < 3) of this wave,
// the lane's column, output channels cot * BN + cw + 32 ct (+ the fused Cout-1 partials).
template <int DIL, bool RELU, bool P3, bool INIT = true>
__device__ __attribute__((always_inline)) inline void ring_epilogue(const Args& a, int b, int row_base, int col,
                                                                   int cot, int cw, const floatx16 (&acc)[2][3],
                                                                   u32x4* lds) {
  if constexpr (P3) {
    cout1_partials<RELU>(a, b, row_base, DIL, col, cot, cw, acc, lds);
  } else {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
        store_block<RELU, INIT>(a, b, row_base + pt * DIL, col, cot * BN + cw + 32 * ct, acc[ct][pt]);
  }
}

// The init term (conv1's coord term) of this lane's outputs: rows row_base + pt * DIL (pt < NPT), column col, output
// channels co0 + 32 ct + (r & 3) + 8 (r >> 2) + 4 kh (store_block's lane layout); 0 outside the image.  Read at a
// row-Winograd conv's start, beside its first DMAs, and folded into its accumulators: the epilogue's 6-8 rounds of
// 16 dependent init loads per lane cost 3-4.5 % of conv1 (cfg2 1.37 vs 1.31 ms without them,
// profiles/r06av_init_epilogue_cost.jsonl)
template <int NPT, int NA>
__device__ __attribute__((always_inline)) inline void load_init(const Args& a, int row_base, int dil, int col, int co0,
                                                                floatx16 (&v)[2][NA]) {
  static_assert(NPT <= NA, "rows");
  // 32-bit element offsets from the uniform base (co * H * W < 2^31: the host's shape checks), one channel at a
  // time over the rows (the 96-128 offsets of all of them at once cost registers the K loop needs)
  const int kh = (threadIdx.x & 63) >> 5;
  const uint32_t iplane = (uint32_t)a.H * (uint32_t)a.W;
  bool ok[NPT];
  uint32_t roff[NPT];
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) {
    const int row = row_base + pt * dil;
    ok[pt] = row < a.H && col < a.W;
    roff[pt] = ok[pt] ? (uint32_t)row * (uint32_t)a.W + (uint32_t)col : 0u;
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t co = (uint32_t)(co0 + 32 * ct + (r & 3) + 8 * (r >> 2) + 4 * kh);
      const float* p = a.init + co * iplane;
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) v[ct][pt][r] = ok[pt] ? p[roff[pt]] : 0.f;
    }
}

// split tiles' raw partial sums: slot s = [24 floatx4 of a thread's 96 accumulators][RNT threads]
constexpr int kRingSlotF4 = 24 * RNT;
__device__ inline void ring_store_partial(float* ws, int slot, const floatx16 (&acc)[2][3]) {
  floatx4* p = reinterpret_cast<floatx4*>(ws) + (int64_t)slot * kRingSlotF4 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        p[((i * 3 + j) * 4 + q) * RNT] = floatx4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                                                  acc[i][j][4 * q + 3]};
}

// Finishes split tiles: block f sums fix[f]'s pieces in K order (deterministic) and writes the
// tile with the ring kernel's own epilogue.
template <int DIL, bool RELU, bool P3>
__global__ __launch_bounds__(RNT) void conv_ring_fixup_kernel(const Args a) {
  __shared__ __attribute__((aligned(16))) u32x4 lds[P3 ? 10 * BN / 4 : 1];  // cout1_partials' w3 + bias
  const int4 f = a.fix[blockIdx.x];
  floatx16 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = floatx16{0};
  for (int piece = 0; piece < f.z; ++piece) {
    const floatx4* p = reinterpret_cast<const floatx4*>(a.sk_ws) + (int64_t)(f.y + piece) * kRingSlotF4 + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const floatx4 v = p[((i * 3 + j) * 4 + q) * RNT];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] += v[e];
        }
  }
  // the ring kernel's tile decode and lane -> pixel map (edge-strip tiles: EW = a.edge_w)
  const int tile = f.x, cot = tile % a.n_cot, rest = tile / a.n_cot;
  const int t_main = a.tiles_y * a.tiles_x, t_all = t_main + a.edge_tiles;
  const int pp = rest % t_all, b = rest / t_all;
  const bool edge = pp >= t_main;
  const int ty = pp / a.tiles_x;
  const int x0 = edge ? a.edge_x0 : (pp - ty * a.tiles_x) * TW;
  const int y0 = a.out_row0 + (edge ? (pp - t_main) * a.edge_rows : ty * RT);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l32 = threadIdx.x & 31;
  const int ew = edge ? a.edge_w : TW;
  ring_epilogue<DIL, RELU, P3>(a, b, y0 + ring_base_row<DIL>(wave & 3) + 12 * (l32 / ew), x0 + l32 % ew, cot,
                               64 * (wave >> 2), acc, lds);
}

template <int DIL, bool RELU, bool P3 = false, int EWE = 0>
__global__ __launch_bounds__(RNT, 1) void conv_ring_kernel(const Args a) {
  constexpr int LDSN = EWE ? (RingGeo<DIL>::LDS > RingGeo<DIL, EWE ? EWE : TW>::LDS ? RingGeo<DIL>::LDS
                                                                                   : RingGeo<DIL, EWE ? EWE : TW>::LDS)
                           : RingGeo<DIL>::LDS;
  __shared__ __attribute__((aligned(16))) u32x4 lds[LDSN];
  u32x4* const Xlds = lds + 3 * RUNIT;

  const int W = a.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, kl = lane >> 5;  // lane half = 8-channel sub-block of a K-block
  const int64_t plane = (int64_t)a.in_rows * W;
  const int64_t wchunk = (int64_t)a.n_cot * W16;

  // One work item: chunks [ci0, ci1) of `tile`'s active-chunk sequence (all of it unscheduled);
  // pslot >= 0: a piece of a split tile, whose raw partial sums conv_ring_fixup_kernel finishes.
  auto run_item = [&](const int tile, const int ci0, int ci1, const int pslot) __attribute__((always_inline)) {
  // tile = (b, pixel tile pp, cot); pixel tiles: the tiles_y x tiles_x grid, then the edge strip
  const int cot = tile % a.n_cot;
  const int rest = tile / a.n_cot;
  const int t_main = a.tiles_y * a.tiles_x, t_all = t_main + a.edge_tiles;
  const int pp = rest % t_all;
  const int b = rest / t_all;
  const bool edge = EWE != 0 && pp >= t_main;
  const int ty = pp / a.tiles_x;
  const int x0 = edge ? a.edge_x0 : (pp - ty * a.tiles_x) * TW;
  const int y0 = a.out_row0 + (edge ? (pp - t_main) * a.edge_rows : ty * RT);
  // output-side mask: a tile of output channels nobody reads (whole item, before any barrier)
  if (a.cmask && !((a.cmask[pp] >> (cot / a.cot_pg)) & 1u)) return;
  const u32x4* wsrc = a.wp + (int64_t)cot * W16;
  const uint32_t gm = a.gmask ? a.gmask[pp] : 0u;
  // this block's chunks: [ci0, ci1) of the tile's active-chunk sequence (all of it unscheduled)
  const int nch_tile = a.gmask ? __builtin_popcount(gm) * a.cpg : a.nchunks;
  ci1 = min(ci1, nch_tile);
  const int nch = max(ci1 - ci0, 0);
  auto chunk_of = [&](int i) -> int {  // physical chunk of the block's i-th chunk
    i += ci0;
    if (!a.gmask) return i;
    uint32_t m = gm;
    for (int j = i / a.cpg; j > 0; --j) m &= m - 1;
    return __builtin_ctz(m) * a.cpg + i % a.cpg;
  };

  auto body = [&](auto ew_tag) __attribute__((always_inline)) {
  constexpr int EW = decltype(ew_tag)::value;
  using G = RingGeo<DIL, EW>;
  constexpr int XW = G::XW, XPIX = G::XPIX, NX = G::NX, XBUF = G::XBUF;
  static_assert(G::LDS <= LDSN, "LDS");
  // the lane's pixel in its MFMA block: row offset (a multiple of the 12-row period) and column
  const int lr = 12 * (l32 / EW), lc = l32 % EW;
  // LDS-DMA sources, chunk-invariant parts.  Halo entry e = (sub, part, pixel) of the image
  // [sub][part][XH][XW]; lane j-th instruction covers entries (j * RNIW + wave) * 64 + lane.
  int xo[NX];  // piece offset in the sub-block's plane (2 * pixel + part); -1 = zero entry
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    const int e = (j * RNIW + wave) * 64 + lane;
    const int part = (e / XPIX) & 1, pix = e % XPIX;
    const int r = pix / XW, c = pix % XW;
    const int gy = y0 - DIL + r, gx = x0 - DIL + c, by = gy - a.in_row0;
    const bool ok = e < 4 * XPIX && gy >= 0 && gy < a.H && by >= 0 && by < a.in_rows && gx >= 0 && gx < W;
    xo[j] = ok ? 2 * (by * W + gx) + part : -1;
  }
  // W unit image [part][kh][sub][co]; packed source [part][tap = 3 kh + kw][sub][co].  The
  // DMA source offsets (and the halo entries' sub-block) are recomputed per issue: a few VALU
  // ops instead of registers held across the MFMA loop.
  auto wo = [&](int j) __attribute__((always_inline)) -> int {
    const int e = (j * RNIW + wave) * 64 + lane;
    const int part = e / RHALF, r = e % RHALF;
    return part * (NKB * 2 * BN) + (r / (2 * BN)) * 3 * (2 * BN) + r % (2 * BN);
  };
  const int U = 3 * nch;
  // W unit (physical chunk ch, kernel column kw) -> slot
  auto issue_w_ch = [&](int ch, int kw, int slot) __attribute__((always_inline)) {
    const u32x4* src = wsrc + (int64_t)ch * wchunk + kw * 2 * BN;
    u32x4* dst = lds + slot * RUNIT + wave * 64;
    if (RNIW == RNW || wave < RNIW)
#pragma unroll
      for (int j = 0; j < RNWI; ++j) glds16(src + wo(j), dst + j * RNIT);
  };
  auto issue_w = [&](int u) __attribute__((always_inline)) {  // W unit u -> slot u % 3
    const int uu = min(u, U - 1);
    const int ci = uu / 3;
    issue_w_ch(chunk_of(ci), uu - 3 * ci, u % 3);
  };
  // halo of physical chunk ch -> buffer xb
  auto issue_x_ch = [&](int ch, int xb) __attribute__((always_inline)) {
    // sub-block sources computed unconditionally (clamped channel) and selected per lane, so
    // the issue is straight-line code the scheduler can spread between MFMAs
    const u32x4* xs[2];
    bool kv[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k0 = ch * KC + s * SB;
      kv[s] = k0 < a.K;
      const int kc = kv[s] ? k0 : 0;
      const int g = kc / a.group;
      const int64_t cb = (int64_t)b * a.batch_stride + g * a.group_stride + (int64_t)(kc - g * a.group) * plane;
      xs[s] = static_cast<const u32x4*>(a.x) + cb / 4;
    }
    u32x4* dst = Xlds + xb * XBUF + wave * 64;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const bool s1 = (j * RNIW + wave) * 64 + lane >= 2 * XPIX;
      const bool z = xo[j] < 0 || !(s1 ? kv[1] : kv[0]);
      if (RNIW == RNW || wave < RNIW) glds16(z ? g_ring_zero : (s1 ? xs[1] : xs[0]) + xo[j], dst + j * RNIT);
    }
  };
  auto issue_x = [&](int i) __attribute__((always_inline)) {  // halo of chunk i -> buffer i & 1
    issue_x_ch(chunk_of(min(i, nch - 1)), i & 1);
  };
  // Physical id of the chunk after the current one: every DMA issued while chunk ci is
  // computed fetches chunk ci + 1 (W(u + 3) and the next halo).  Advanced branch-free (scalar
  // selects) once per chunk, so the unit body stays one basic block for the scheduler; past
  // the last chunk it stays at the last one (dummy loads that keep the vmcnt counts exact).
  int nx_i = 1, nx_sub = a.gmask ? (ci0 + 1) % a.cpg : 0;
  int nx_ph = chunk_of(min(1, nch - 1));
  uint32_t nx_m = gm;  // lowest set bit = the group of sequence chunk ci0 + 1
  if (a.gmask)
    for (int j = (ci0 + 1) / a.cpg; j > 0; --j) nx_m &= nx_m - 1;
  auto advance = [&]() __attribute__((always_inline)) {
    const bool more = nx_i + 1 < nch;
    const bool wrap = a.gmask && nx_sub + 1 == a.cpg;
    const uint32_t m2 = wrap ? (nx_m & (nx_m - 1)) : nx_m;
    const int ph2 = wrap ? (int)__builtin_ctz(m2 | 0x80000000u) * a.cpg : nx_ph + 1;
    nx_m = more ? m2 : nx_m;
    nx_ph = more ? ph2 : nx_ph;
    nx_sub = more ? (wrap ? 0 : nx_sub + 1) : nx_sub;
    nx_i += 1;
  };

  const int rg = wave & 3;
  const int base = ring_base_row<DIL>(rg);
  const int cw = 64 * (wave >> 2);
  floatx16 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = floatx16{0};
  bf16x8 fb[2][5][2];  // [set][input row m (rows base + m * DIL)][hi, lo]
  bf16x8 fa[2][2][2];  // [set][ct][hi, lo]
  auto fetch_b = [&](int st, int xb, int kw) __attribute__((always_inline)) {
    const u32x4* X = Xlds + xb * XBUF + kl * 2 * XPIX + (base + lr) * XW + lc + kw * DIL;
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int p = 0; p < 2; ++p) fb[st][m][p] = __builtin_bit_cast(bf16x8, X[p * XPIX + m * DIL * XW]);
  };
  auto fetch_a = [&](int st, int slot, int kh) __attribute__((always_inline)) {
    const u32x4* Wl = lds + slot * RUNIT + kh * 2 * BN + kl * BN + cw + l32;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int p = 0; p < 2; ++p) fa[st][ct][p] = __builtin_bit_cast(bf16x8, Wl[p * RHALF + 32 * ct]);
  };
  auto mfmas = [&](int as, int bs, int kh) __attribute__((always_inline)) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int pt = 0; pt < 3; ++pt) {
        const int m = pt + kh;
        acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[as][ct][1], fb[bs][m][0], acc[ct][pt], 0, 0, 0);
        acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[as][ct][0], fb[bs][m][1], acc[ct][pt], 0, 0, 0);
        acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[as][ct][0], fb[bs][m][0], acc[ct][pt], 0, 0, 0);
      }
  };
  // interleave n fragment reads with the first n of a tap's 18 MFMAs
  auto interleave = [&](auto nreads) __attribute__((always_inline)) {
    constexpr int n = decltype(nreads)::value;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 18 - n, 0);
  };

  if (nch > 0) {
    // prologue: W(0), halo(0), W(1), W(2) in flight; wait for the first two
    issue_w(0);
    issue_x(0);
    issue_w(1);
    issue_w(2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * RNWI) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    fetch_b(0, 0, 0);
    fetch_a(0, 0, 0);
    // unit u = u0 + R, R < 6 compile-time: kw = R % 3, W slot R % 3, halo buffer (R / 3) & 1,
    // fragment set R & 1 (u0 is a multiple of 6)
#define RING_UNIT(R)                                                                           \
  do {                                                                                         \
    constexpr int KW = (R) % 3, P = (R) & 1, SLOT = (R) % 3;                                    \
    constexpr int NSLOT = ((R) + 1) % 3, NXB = (((R) + 1) / 3) & 1, NKW = ((R) + 1) % 3;        \
    const int u_ = u0 + (R);                                                                   \
    if (u_ >= U) break;                                                                        \
    fetch_a(P ^ 1, SLOT, 1);                                                                   \
    mfmas(P, P, 0);                                                                            \
    interleave(std::integral_constant<int, 4>{});                                              \
    fetch_a(P, SLOT, 2);                                                                       \
    mfmas(P ^ 1, P, 1);                                                                        \
    interleave(std::integral_constant<int, 4>{});                                              \
    /* retire W(u+1) (+ the next chunk's halo at kw 2); LDS reads of this unit's slot done */ \
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(KW == 1 ? RNWI + NX : RNWI) : "memory"); \
    __builtin_amdgcn_s_barrier();                                                              \
    asm volatile("" ::: "memory");                                                             \
    issue_w_ch(nx_ph, KW, SLOT);                                                               \
    if (KW == 0) issue_x_ch(nx_ph, ((R) / 3 + 1) & 1);                                         \
    if (KW == 2) advance();                                                                    \
    fetch_b(P ^ 1, NXB, NKW);                                                                  \
    fetch_a(P ^ 1, NSLOT, 0);                                                                  \
    mfmas(P, P, 2);                                                                            \
    interleave(std::integral_constant<int, 14>{});                                             \
  } while (0)
    for (int u0 = 0; u0 < U; u0 += 6) {
      RING_UNIT(0);
      RING_UNIT(1);
      RING_UNIT(2);
      RING_UNIT(3);
      RING_UNIT(4);
      RING_UNIT(5);
    }
#undef RING_UNIT
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the block exits
  }

  if (pslot >= 0) {
    ring_store_partial(a.sk_ws, pslot, acc);  // a piece of a split tile: conv_ring_fixup_kernel finishes it
  } else {
    ring_epilogue<DIL, RELU, P3>(a, b, y0 + base + lr, x0 + lc, cot, cw, acc, lds);
  }
  };  // body
  if constexpr (EWE != 0) {
    if (edge) body(std::integral_constant<int, EWE>{});
    else body(std::integral_constant<int, TW>{});
  } else {
    body(std::integral_constant<int, TW>{});
  }
  };  // run_item

  int tile = xcd_remap(blockIdx.x, a.nwg);
  int ci0 = 0, ci1 = INT_MAX, pslot = -1;  // chunk range of this block, partial slot
  if (a.items) {  // host schedule: the item of this block (tile < 0: padding)
    if ((int)blockIdx.x >= a.nitems) return;
    const int4 it = a.items[blockIdx.x];
    if (it.x < 0) return;
    tile = it.x, ci0 = it.y, ci1 = it.z, pslot = it.w;
  } else if (a.gmask) {  // frustum mask: ordered pixel tiles dealt to the XCDs (see conv_kernel)
    constexpr int Gq = MVBEV_MASK_GROUP;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int q = j / a.n_cot;
    const int slot = Gq * (8 * (q / Gq) + x) + q % Gq;
    if (slot >= a.npix) return;  // padding block (whole block, before any barrier)
    tile = (a.tile_order ? a.tile_order[slot] : slot) * a.n_cot + j % a.n_cot;
  }
  run_item(tile, ci0, ci1, pslot);
}

#ifndef MVBEV_B3_RING
#define MVBEV_B3_RING 1  // split-bf16 input: the LDS-DMA ring kernel (0: conv_kernel)
#endif

#ifndef MVBEV_B3_WAVES
#define MVBEV_B3_WAVES 8
#endif

// Split-K tail geometry.  One workgroup per CU fits (LDS), so tiles run in rounds of G = CU
// count; when the last round is partial its tiles are cut into `split` K-ranges so the tail
// fills the CUs: split minimises ceil(tail * s / G) * (n / s + c) chunk-times, c = the
// measured per-piece overhead (pipeline fill from cold caches, partial store, fixup pass):
// at cfg1 (n = 48, tail 128) splitting in 2 saves 8.5 % of conv1, at cfg2 (n = 224, tail
// 208) every split measured slower, which c = 12 reproduces.  Partial slots: 64 x 512 floats.
constexpr double kSkPieceOverhead = 12.0;
static int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return n;
}
constexpr size_t kSkSlotBytes = (size_t)64 * 64 * MVBEV_B3_WAVES * sizeof(float);
#ifndef MVBEV_B3_SK
#define MVBEV_B3_SK 1  // split-K tail when the workspace allows it
#endif
struct SkPlan {
  int64_t dp_tiles = 0, tail = 0;
  int split = 1;
};
static SkPlan sk_plan(int64_t tiles, int64_t nchunks) {
  SkPlan p;
  const int G = MVBEV_B3_SK ? cu_count() : 0;
  if (G <= 0 || tiles % G == 0 || nchunks < 4) return p;
  p.tail = tiles % G;
  p.dp_tiles = tiles - p.tail;
  double best = (double)nchunks;  // s = 1: one (partial) round of whole tiles
  for (int s = 2; s <= 16 && nchunks / s >= 2; ++s) {
    const double t = (double)ceil_div(p.tail * s, G) * ((double)nchunks / s + kSkPieceOverhead);
    if (t < 0.97 * best) {
      best = t;
      p.split = s;
    }
  }
  if (p.split == 1) p.tail = 0, p.dp_tiles = tiles;
  return p;
}
static int64_t conv_tiles(const mvbev_conv_desc* d, int64_t Cout) {
  return ceil_div(d->W, TW) * ceil_div(d->out_rows, MVBEV_B3_WAVES) * (Cout / BN) * d->B;
}

// Pixel-tile space of the ring kernel (split-bf16 input).  MVBEV_TILES_EDGE_STRIP, for
// 0 < W % 32 <= 16: the regular 12 x 32 tiles cover columns [0, 32 * floor(W / 32)) and the last
// W % 32 columns are cut into edge-strip tiles of (12 * 32 / EW) rows x EW columns (EW = 8 or 16,
// the same 384 pixels per tile), so no MFMA column is spent past W.  g = {tiles_x, tiles_y,
// edge_tiles, edge width (the EW the kernel uses), edge rows}.
static int ring_tile_space(const mvbev_conv_desc* d, int tile_space, int64_t g[5]) {
  if (!d || d->W <= 0 || d->out_rows <= 0) return MVBEV_ERR_RANK;
  g[1] = ceil_div(d->out_rows, RT);
  if (tile_space == MVBEV_TILES_GRID) {
    g[0] = ceil_div(d->W, TW), g[2] = 0, g[3] = 0, g[4] = 0;
    return MVBEV_OK;
  }
  if (tile_space != MVBEV_TILES_EDGE_STRIP) return MVBEV_ERR_SHAPE;
  const int64_t r = d->W % TW;
  if (r == 0 || r > 16) return MVBEV_ERR_SHAPE;  // nothing to trim / a regular tile is as good
  g[0] = d->W / TW;
  g[3] = r <= 8 ? 8 : 16;
  g[4] = RT * (TW / g[3]);
  g[2] = ceil_div(d->out_rows, g[4]);
  return MVBEV_OK;
}

template <typename TIn>
static int launch(const void* x, const mvbev_conv_desc* d, const void* w_packed,
                  const float* bias, const float* init, int64_t Cout, int dilation, int relu,
                  float* y, int y_layout, const uint32_t* group_mask, const int32_t* tile_order,
                  void* workspace, size_t ws_bytes, void* stream, const uint32_t* out_mask = nullptr,
                  int cot_pg = 1, const float* w3 = nullptr, float* p3 = nullptr,
                  const mvbev_conv_schedule* sched = nullptr, int tile_space = MVBEV_TILES_GRID) {
  if (!x || !d || !w_packed || (!y && !p3) || (!w3 != !p3)) return MVBEV_ERR_NULL;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || d->in_rows <= 0 ||
      d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % BN != 0 || d->K % SB != 0 || d->group % SB != 0 || d->K % d->group != 0)
    return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H) return MVBEV_ERR_SHAPE;
  if (d->in_rows * d->W > (int64_t)INT32_MAX || d->H > INT32_MAX / 2 || d->W > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(w_packed) & 15) != 0) return MVBEV_ERR_ALIGN;
  constexpr int NW = MVBEV_B3_WAVES;
  Args a{};
  a.x = x; a.wp = static_cast<const u32x4*>(w_packed); a.bias = bias; a.init = init; a.y = y;
  a.group_stride = d->group_stride; a.batch_stride = d->batch_stride;
  a.B = (int)d->B; a.group = (int)d->group; a.K = (int)d->K; a.nchunks = (int)ceil_div(d->K, KC);
  a.Cout = (int)Cout;
  a.H = (int)d->H; a.W = (int)d->W;
  a.in_row0 = (int)d->in_row0; a.in_rows = (int)d->in_rows;
  a.out_row0 = (int)d->out_row0; a.out_rows = (int)d->out_rows;
  // split-bf16 input runs the LDS-DMA ring kernel (12-row tiles, no split-K tail)
  const bool ring = std::is_same<TIn, SplitIn>::value && MVBEV_B3_RING && (dilation == 1 || dilation == 2);
  if (p3 && (!ring || init)) return MVBEV_ERR_SHAPE;  // the fused cout1 epilogue: ring kernel, no init term
  a.w3 = w3;
  a.p3 = p3;
  a.tiles_x = (int)ceil_div(d->W, TW); a.tiles_y = (int)ceil_div(d->out_rows, ring ? RT : NW);
  a.n_cot = (int)(Cout / BN);
  a.edge_tiles = 0, a.edge_x0 = 0, a.edge_rows = 0, a.edge_w = 0;
  int edge_w = 0;
  if (tile_space == MVBEV_TILES_EDGE_STRIP) {  // ring kernel, no schedule / output-side mask
    int64_t g[5];
    if (!ring || out_mask || ring_tile_space(d, tile_space, g) != MVBEV_OK) return MVBEV_ERR_SHAPE;
    a.tiles_x = (int)g[0];
    a.edge_tiles = (int)g[2], edge_w = (int)g[3], a.edge_rows = (int)g[4];
    a.edge_w = edge_w;
    a.edge_x0 = (int)(g[0] * TW);
  } else if (tile_space != MVBEV_TILES_GRID) {
    return MVBEV_ERR_SHAPE;
  }
  const int64_t tiles = ((int64_t)a.tiles_x * a.tiles_y + a.edge_tiles) * a.n_cot * d->B;
  if (tiles * a.nchunks > (int64_t)INT32_MAX * 8) return MVBEV_ERR_SHAPE;
  a.gmask = nullptr;
  a.cpg = 0;
  if (group_mask) {  // frustum mask: needs whole chunks per group and <= 32 groups
    if (d->group % KC != 0 || d->K / d->group > 32) return MVBEV_ERR_SHAPE;
    a.gmask = group_mask;
    a.cpg = (int)(d->group / KC);
  }
  a.tile_order = group_mask ? tile_order : nullptr;
  a.cmask = out_mask;
  a.cot_pg = cot_pg;
  if (out_mask && (cot_pg <= 0 || a.n_cot > 32 * cot_pg || group_mask)) return MVBEV_ERR_SHAPE;
  if (out_mask) workspace = nullptr;  // skipped tiles never write split-K partial sums
  if (y_layout != MVBEV_LAYOUT_F32 && y_layout != MVBEV_LAYOUT_SPLIT_BF16 &&
      !(y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX && ring && !p3))
    return MVBEV_ERR_SHAPE;
  a.y_split = y_layout == MVBEV_LAYOUT_SPLIT_BF16 || y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX;
  a.y_pix = y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX;
  a.npix = (int)(tiles / a.n_cot);
  const SkPlan plan = (group_mask || ring) ? SkPlan() : sk_plan(tiles, a.nchunks);
  const bool sk = workspace && plan.split > 1 &&
                  ws_bytes >= (size_t)(plan.tail * plan.split) * kSkSlotBytes;
  a.sk_ws = sk ? static_cast<float*>(workspace) : nullptr;
  a.dp_tiles = (int)(sk ? plan.dp_tiles : tiles);
  a.split = sk ? plan.split : 1;
  int64_t nwg = group_mask ? (int64_t)a.n_cot * round_up(a.npix, 8 * MVBEV_MASK_GROUP)
                           : (sk ? plan.dp_tiles + plan.tail * plan.split : tiles);
  a.items = nullptr, a.nitems = 0, a.fix = nullptr, a.nfix = 0;
  if (sched) {  // host schedule (ring kernel): items replace the tile order, pieces their fixup
    if (!ring || sched->nitems < 0 || sched->nfix < 0 || sched->nslots < 0 || (!sched->items && sched->nitems) ||
        (sched->nfix && (!sched->fixups || !sched->partials)))
      return MVBEV_ERR_SHAPE;
    if (sched->partial_bytes < (size_t)sched->nslots * sizeof(floatx4) * kRingSlotF4) return MVBEV_ERR_SHAPE;
    if ((reinterpret_cast<uintptr_t>(sched->items) & 15) || (reinterpret_cast<uintptr_t>(sched->fixups) & 15) ||
        (reinterpret_cast<uintptr_t>(sched->partials) & 15))
      return MVBEV_ERR_ALIGN;
    a.items = reinterpret_cast<const int4*>(sched->items);
    a.nitems = sched->nitems;
    a.fix = reinterpret_cast<const int4*>(sched->fixups);
    a.nfix = sched->nfix;
    a.sk_ws = static_cast<float*>(sched->partials);
    nwg = sched->nitems;
    if (nwg == 0) return MVBEV_OK;
  }
  if (nwg > (int64_t)INT32_MAX) return MVBEV_ERR_SHAPE;
  a.nwg = (int)nwg;
  hipStream_t s = as_stream(stream);
#define B3_LAUNCH(D, R)                                                                   \
  do {                                                                                    \
    hipLaunchKernelGGL((conv_kernel<TIn, D, R, NW>), dim3((unsigned)nwg), dim3(64 * NW),   \
                       0, s, a);                                                          \
    if (sk)                                                                               \
      hipLaunchKernelGGL((sk_fixup_kernel<R, NW>), dim3((unsigned)plan.tail),              \
                         dim3(64 * NW), 0, s, a);                                         \
  } while (0)
#define RING_LAUNCH(D, R)                                                                         \
  do {                                                                                            \
    if (p3)                                                                                       \
      hipLaunchKernelGGL((conv_ring_kernel<D, R, true>), dim3((unsigned)nwg), dim3(RNT), 0, s, a); \
    else if (edge_w == 8 && D == 1 && R)                                                          \
      hipLaunchKernelGGL((conv_ring_kernel<1, true, false, 8>), dim3((unsigned)nwg), dim3(RNT), 0, s, a); \
    else if (edge_w == 16 && D == 1 && R)                                                         \
      hipLaunchKernelGGL((conv_ring_kernel<1, true, false, 16>), dim3((unsigned)nwg), dim3(RNT), 0, s, a); \
    else if (edge_w != 0)                                                                         \
      return MVBEV_ERR_SHAPE;                                                                     \
    else                                                                                          \
      hipLaunchKernelGGL((conv_ring_kernel<D, R>), dim3((unsigned)nwg), dim3(RNT), 0, s, a);       \
    if (a.nfix > 0) {                                                                             \
      if (p3)                                                                                     \
        hipLaunchKernelGGL((conv_ring_fixup_kernel<D, R, true>), dim3((unsigned)a.nfix), dim3(RNT), 0, s, a); \
      else                                                                                        \
        hipLaunchKernelGGL((conv_ring_fixup_kernel<D, R, false>), dim3((unsigned)a.nfix), dim3(RNT), 0, s, a); \
    }                                                                                             \
  } while (0)
  if (ring) {
    if (dilation == 1) {
      if (relu) RING_LAUNCH(1, true); else RING_LAUNCH(1, false);
    } else {
      if (relu) RING_LAUNCH(2, true); else RING_LAUNCH(2, false);
    }
  } else if (dilation == 1) {
    if (relu) B3_LAUNCH(1, true); else B3_LAUNCH(1, false);
  } else if (dilation == 2) {
    if (relu) B3_LAUNCH(2, true); else B3_LAUNCH(2, false);
  } else {
    return MVBEV_ERR_DILATION;
  }
#undef B3_LAUNCH
#undef RING_LAUNCH
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

// ---------------------------------------------------------------------------------------
// Row-Winograd conv1 (forward, dilation 1, split-bf16 input): F(3,3) along the rows.
//
// The ring kernel's wave computes 3 output rows from 5 input rows per kernel column kw,
//     y_i = sum_kh w[kh] d[i + kh]    (i, kh < 3: 9 products per channel and pixel).
// With the interpolation points {0, 1, -1, 2, inf} that is  y = A^T [(G w) . (B^T d)]:
// 5 products.  B^T d is computed once per frame by wino_rows_kernel into the T layout (the
// split-bf16 blocked layout over 5 transformed rows per 3-row output tile), G w once per
// weight version (pack_wino_kernel).  The conv is the ring kernel with the unit (chunk, kw)
// replaced by (chunk, xi): per unit a wave runs its 3 kernel columns against one transformed
// row (18 MFMAs into acc[ct][xi]) and the epilogue applies A^T to the 5 accumulators (exact
// small-integer weights, fp32).  Per (chunk, kw): 5 instead of 9 MFMA K-blocks (x0.556).
//   A^T = [1 1 1 1 0; 0 1 -1 2 0; 0 1 1 4 1]
//   G   = [1/2 0 0; -1/2 -1/2 -1/2; -1/6 1/6 -1/6; 1/6 1/3 2/3; 0 0 1]
//   B^T = [2 -1 -2 1 0; 0 -2 -1 1 0; 0 2 -3 1 0; 0 -1 0 1 0; 0 2 -1 -2 1]
// T and G w are split hi/lo like the slab and the direct weights (the products keep the
// 3xbf16 accuracy); the transforms' roundings add about as much error again as the direct
// conv's (numpy emulation at K = 2048: 1.1e-5 vs 5.6e-6 normwise), far inside the 1e-3 gate.
namespace wino {
constexpr int NXI = 5;                            // transformed rows per 3-row output tile
constexpr int XH = 4 * NXI;                       // T rows of a 12-row workgroup tile
#ifndef MVBEV_WINO_NIW
#define MVBEV_WINO_NIW 4  // DMA-issuing waves, one per SIMD (cfg2 winoconv, buffer-load DMAs: 4 1.40 ms, 8 1.51-1.52; with the per-unit address arithmetic of round 2: 8 1.59-1.67, 4 1.73-1.79)
#endif
constexpr int NIW = MVBEV_WINO_NIW;               // DMA-issuing waves
constexpr int NIT = 64 * NIW;
constexpr int NWI = RUNIT / NIT;                  // weight DMAs per issuing wave per unit (6)
// a unit (chunk, xi) stages its weights (3 kernel columns) and its T row of the 4 row tiles,
// [sub][part][row tile][XW], together in one ring slot; a kernel column's taps are DIL columns
// apart, so the row carries DIL halo columns on each side
template <int DIL> struct Geo {
  static constexpr int XW = TW + 2 * DIL;              // T columns of a unit's row
  static constexpr int TROW = 2 * 2 * 4 * XW;          // T entries of a unit (544 / 576)
  static constexpr int NXT = (TROW + NIT - 1) / NIT;   // T DMAs per issuing wave per unit (2)
};
constexpr int NXTMAX = (2 * 2 * 4 * (TW + 4) + NIT - 1) / NIT;  // T pieces of the widest (dilation 2) unit
static_assert(Geo<1>::NXT <= NXTMAX && Geo<2>::NXT <= NXTMAX, "T pieces");
constexpr int SLOT = RUNIT + NXTMAX * NIT;        // 16-B entries per ring slot
constexpr int NSLOT = 4;                          // 3 units of DMA in flight
constexpr int LDS = NSLOT * SLOT;                 // 160 KiB
static_assert(LDS * 16 <= 160 * 1024, "LDS");
constexpr int NTAP = 3 * NXI;                     // packed taps (xi, kw)
constexpr int WPART = NTAP * KC * BN;             // bf16 per part per (chunk, cout tile)
constexpr int W16 = 2 * WPART * 2 / 16;           // 16-B pieces per (chunk, cout tile)
}  // namespace wino

// packed[chunk][cot][part][3 xi + kw][sub][co][j] = split(sum_kh G[xi][kh] w[co][map(k)][kh][kw]).
// A thread per (chunk, cot, kw, sub, co, j) loads the kernel column g[kh] once and writes its 5 xi x
// 2 parts (per step a training forward + backward re-packs 2 x 3584 x 512 weights: one thread per
// output, 10 x the column loads, took ~0.2 ms per big weight).
// swap (a data gradient's weights): the packed [Cout][K] weight is w^T with its taps reversed,
// packed[o][i][kh][kw] = w[i][o][2 - kh][2 - kw], read from the forward weight w [K][Cin_w][3][3]
// (o < Cout <= Cin_w) without a transposed copy.
__global__ void pack_wino_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int Cout, int Cin_w,
                                 const int32_t* __restrict__ chan_map, int K, int K_pad, bool swap) {
  const int n_cot = Cout / BN;
  const int64_t total = (int64_t)(K_pad / KC) * n_cot * 3 * 2 * BN * SB;  // columns
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int j = r % SB; r /= SB;
    const int co = r % BN; r /= BN;
    const int sub = r % 2; r /= 2;
    const int kw = r % 3; r /= 3;
    const int cot = r % n_cot;
    const int chunk = (int)(r / n_cot);
    const int k = chunk * KC + sub * SB + j;
    int ci = k < K ? (chan_map ? chan_map[k] : k) : -1;
    if (!swap && ci >= Cin_w) ci = -1;  // (swap: ci is the forward weight's output row, < K)
    double g0 = 0.0, g1 = 0.0, g2 = 0.0;
    if (ci >= 0 && !swap) {
      const float* g = w + ((int64_t)(cot * BN + co) * Cin_w + ci) * 9 + kw;  // g[3 kh]
      g0 = g[0], g1 = g[3], g2 = g[6];
    } else if (ci >= 0) {
      const float* g = w + ((int64_t)ci * Cin_w + cot * BN + co) * 9 + (2 - kw);  // reversed taps
      g0 = g[6], g1 = g[3], g2 = g[0];
    }
    const double u[wino::NXI] = {0.5 * g0, -0.5 * (g0 + g1 + g2), (g1 - g0 - g2) / 6.0,
                                 (g0 + 2.0 * g1 + 4.0 * g2) / 6.0, g2};
    // element (part, tap = 3 xi + kw, sub, co, j) of the (chunk, cot) block
    __bf16* o = out + ((int64_t)chunk * n_cot + cot) * 2 * wino::WPART + ((int64_t)sub * BN + co) * SB + j;
#pragma unroll
    for (int xi = 0; xi < wino::NXI; ++xi) {
      const float v = (float)u[xi];
      const __bf16 hi = (__bf16)v;
      const int tap = 3 * xi + kw;
      o[(int64_t)tap * KC * BN] = hi;
      o[(int64_t)(wino::NTAP + tap) * KC * BN] = (__bf16)(v - (float)hi);
    }
  }
}

struct WinoRowsArgs {
  const u32x4* x;
  u32x4* t;
  int64_t group_stride, batch_stride;  // elements, as mvbev_conv_desc
  int K, group, H, W, in_row0, in_rows, out_row0, tiles_x, tiles_y, dil;
  const uint32_t* gmask;
  const int32_t* gate;  // (ABI 12200) NULL, or run only when *gate == gate_tag (the training guard's exact T)
  int32_t gate_tag;
};

__device__ inline void bf16x8_to_f32(const u32x4 v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

// T[b][k / 8][5 r3 + xi][hi, lo][col][8] = split((B^T d)[xi]) (a row's hi plane, then its lo plane:
// a unit's T DMAs read whole contiguous 16-B runs),
//   d[m] = x[b][k][out_row0 + base(r3) + dil (m - 1)][col] (zero outside the image and the input rows),
// r3 < 4 tiles_y: the 3-row tiles of the conv's 12 x 32 workgroup tiles, rows base(r3) + dil pt
// (pt < 3): base = 3 r3 for dilation 1; for dilation 2 the 12 rows hold two interleaved pairs of
// row tiles, base = 12 (r3 / 4) + ring_base_row<2>(r3 % 4) (the ring kernel's wave rows).  Workgroup = (pixel tile, channel group, b);
// with a frustum mask the groups it clears for the tile are skipped: the conv never reads them
// there, and the T columns a neighbouring tile's halo reads from a skipped tile are zero both
// in T (zero-filled, never written) and in the true transform (the mask covers the halo).
__global__ __launch_bounds__(256) void wino_rows_kernel(const WinoRowsArgs a) {
  constexpr int KB = 8;  // 8-channel blocks per workgroup: 4 x 32 x 8 items, 4 per thread
  if (a.gate && *a.gate != a.gate_tag) return;
  const int pp = blockIdx.x, b = blockIdx.z;
  const int nbg = (a.group / SB + KB - 1) / KB;
  const int g = blockIdx.y / nbg, kb0 = (blockIdx.y - g * nbg) * KB;
  if (a.gmask && !((a.gmask[pp] >> g) & 1u)) return;
  const int W = a.W;
  const int ty = pp / a.tiles_x;
  const int x0 = (pp - ty * a.tiles_x) * TW;
  const int nb = a.group / SB, K8 = a.K / SB, R5 = 5 * 4 * a.tiles_y;
  const int64_t plane = (int64_t)a.in_rows * W;
  const int c = threadIdx.x % TW, q = (threadIdx.x / TW) % 4, kq = threadIdx.x / (4 * TW);  // kq < 2
  const int col = x0 + c, r3 = 4 * ty + q;
  if (col >= W) return;
  const int base = 12 * ty + (a.dil == 1 ? 3 * q : ring_base_row<2>(q));
  // the 5 input rows of the row tile (all 4 items of the thread share them)
  int64_t roff[5];
  bool rok[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    const int row = a.out_row0 + base + a.dil * (m - 1), by = row - a.in_row0;
    rok[m] = row >= 0 && row < a.H && by >= 0 && by < a.in_rows;
    roff[m] = 2 * ((int64_t)by * W + col);
  }
  u32x4 raw[4][5][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // all loads first: 40 in flight per thread
    const int kb = kb0 + kq + 2 * i;
    const bool kok = kb < nb && g * a.group + kb * SB < a.K;
    const u32x4* src = a.x + ((int64_t)b * a.batch_stride + (int64_t)g * a.group_stride +
                              (int64_t)(kok ? kb : 0) * SB * plane) / 4;
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int p = 0; p < 2; ++p) raw[i][m][p] = (kok && rok[m]) ? src[roff[m] + p] : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kb = kb0 + kq + 2 * i, k0 = g * a.group + kb * SB;
    if (kb >= nb || k0 >= a.K) continue;
    float d[5][8];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      float h[8], l[8];
      bf16x8_to_f32(raw[i][m][0], h);
      bf16x8_to_f32(raw[i][m][1], l);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[m][j] = h[j] + l[j];
    }
    // T row = its hi plane [W][8] then its lo plane (16-B units)
    u32x4* dst = a.t + 2 * (((int64_t)b * K8 + k0 / SB) * R5 * W + (int64_t)5 * r3 * W) + col;
#pragma unroll
    for (int xi = 0; xi < 5; ++xi) {
      unsigned hp[4], lp[4];
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        unsigned short hs[2], ls[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * e4 + e;
          const float d0 = d[0][j], d1 = d[1][j], d2 = d[2][j], d3 = d[3][j], d4 = d[4][j];
          const float v = xi == 0 ? 2.f * d0 - d1 - 2.f * d2 + d3
                        : xi == 1 ? -2.f * d1 - d2 + d3
                        : xi == 2 ? 2.f * d1 - 3.f * d2 + d3
                        : xi == 3 ? d3 - d1
                                  : 2.f * d1 - d2 - 2.f * d3 + d4;
          const __bf16 hv = (__bf16)v, lv = (__bf16)(v - (float)hv);
          hs[e] = __builtin_bit_cast(unsigned short, hv);
          ls[e] = __builtin_bit_cast(unsigned short, lv);
        }
        hp[e4] = (unsigned)hs[0] | ((unsigned)hs[1] << 16);
        lp[e4] = (unsigned)ls[0] | ((unsigned)ls[1] << 16);
      }
      dst[2 * (int64_t)xi * W] = u32x4{hp[0], hp[1], hp[2], hp[3]};
      dst[2 * (int64_t)xi * W + W] = u32x4{lp[0], lp[1], lp[2], lp[3]};
    }
  }
}

// One unit barrier per two units (2 units of DMA lookahead instead of 3) for conv2 only (cfg2: conv2
// 0.349 -> 0.342 ms, conv1 1.43 -> 1.45); T pieces that hold no T entry are not issued (per-wave wait
// counts); the T DMAs keep the default cache policy (nt measured +0.5 % on conv1, +1 % on conv2).
// DIL 2 (conv2): the wave's row tile is the ring kernel's interleaved rows base + 2 pt; P3: the
// epilogue forms conv3's partial sums (cout1_partials) instead of storing y
#ifndef MVBEV_WINO_STAMPS
#define MVBEV_WINO_STAMPS 0  // diagnostic builds only: per-workgroup start / end clocks and CU of the last launch
#endif
#if MVBEV_WINO_STAMPS
__device__ long long g_wino_stamps[4 * 65536];
#endif
// acc[.][0..2] = the init term (i0, i1, i2) of a wave's 3 rows -> M = (i0 - i2, (i1 + i2) / 2, (i2 - i1) / 2), element
// by element in place (A^T M = (i0, i1, i2))
__device__ __attribute__((always_inline)) inline void init_to_m(floatx16 (&acc)[2][wino::NXI]) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float i0 = acc[ct][0][r], i1 = acc[ct][1][r], i2 = acc[ct][2][r];
      acc[ct][0][r] = i0 - i2;
      acc[ct][1][r] = 0.5f * (i1 + i2);
      acc[ct][2][r] = 0.5f * (i2 - i1);
    }
}

template <bool RELU, int DIL, bool P3>
__global__ __launch_bounds__(RNT, 1) void conv_wino_kernel(const Args a) {
  using namespace wino;
  using G = Geo<DIL>;
#if MVBEV_WINO_STAMPS
  const long long stamp0 = wall_clock64();
#endif
  constexpr int XW = G::XW, TROW = G::TROW, NXT = G::NXT;
  __shared__ __attribute__((aligned(16))) u32x4 lds[LDS];
  const int W = a.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, kl = lane >> 5;

  int tile = xcd_remap(blockIdx.x, a.nwg);
  if (a.gmask) {  // ordered pixel tiles dealt to the XCDs, as the ring kernel (groups of a.mgroup)
    const int Gq = a.mgroup;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int q = j / a.n_cot;
    const int slot = Gq * (8 * (q / Gq) + x) + q % Gq;
    if (slot >= a.npix) return;  // padding block (whole block, before any barrier)
    tile = (a.tile_order ? a.tile_order[slot] : slot) * a.n_cot + j % a.n_cot;
  }
  const int cot = tile % a.n_cot, rest = tile / a.n_cot;
  const int t_main = a.tiles_y * a.tiles_x;
  const int pp = rest % t_main, b = rest / t_main;
  const int ty = pp / a.tiles_x;
  const int x0 = (pp - ty * a.tiles_x) * TW;
  const int y0 = a.out_row0 + ty * RT;
  // (a data gradient's output-side frustum mask: output channel group cot / cot_pg of this pixel
  // tile is never read — the whole block leaves before any barrier)
  if (a.cmask && !((a.cmask[pp] >> (cot / a.cot_pg)) & 1u)) return;
  const uint32_t gm = a.gmask ? a.gmask[pp] : 0u;
  const int nch = a.gmask ? __builtin_popcount(gm) * a.cpg : a.nchunks;
  const int K8 = a.K / SB;
  const int64_t tplane2 = 2LL * (XH * a.tiles_y) * W;  // 16-B pieces per 8-channel block of T
  const uint32_t tplane_b = (uint32_t)(tplane2 * 16);  // < 2^30 (host check)
  // The DMAs are buffer loads: a wave-uniform descriptor per unit (built by scalar code from the
  // chunk's base) and per-lane byte offsets computed ONCE here — the per-unit address arithmetic
  // of 64-bit per-lane pointers (and a select of a zero source) was ~90 instructions right after
  // each unit's barrier, with both waves of a SIMD stalled on it.  Padding entries (outside the
  // grid, past the T row) carry an out-of-range offset: the range check makes them zero.
  // Weights: entry e of a unit = [part][kw][sub][co] from the packed [part][3 xi + kw][sub][co].
  // T: entry e = (sub, part, row tile, col) -> T row XH ty + NXI rt + xi, column x0 - DIL + col.
  constexpr uint32_t kOOB = 0x80000000u;
  uint32_t wvo[NWI], tvo[NXTMAX];  // fixed size: a template-dependent array captured by the lambdas below silently drops the kernel's host stub (hipcc, ROCm 7.2)
#pragma unroll
  for (int j = 0; j < NWI; ++j) {
    const int e = (j * NIW + wave) * 64 + lane;
    wvo[j] = (uint32_t)(((e / RHALF) * (NTAP * 2 * BN) + e % RHALF) * 16);
    asm volatile("" : "+v"(wvo[j]));  // keep it in a register, not rematerialised per unit
  }
#pragma unroll
  for (int j = 0; j < NXT; ++j) {
    const int e = (j * NIW + wave) * 64 + lane;
    const int sub = e / (TROW / 2), part = (e / (TROW / 4)) & 1, rt = (e % (TROW / 4)) / XW, c = e % XW;
    const int gx = x0 - DIL + c;
    const bool z = e >= TROW || gx < 0 || gx >= W;
    tvo[j] = z ? kOOB : (uint32_t)sub * tplane_b + (uint32_t)((2 * (XH * ty + NXI * rt) * W + part * W + gx) * 16);
    asm volatile("" : "+v"(tvo[j]));
  }
  // the tile's physical chunks, walked incrementally: group = lowest set bit of the mask left,
  // chunk = group * cpg + index in the group (past the last chunk the walk stays there: dummy
  // loads that keep the vmcnt counts exact)
  const int cpg = a.gmask ? a.cpg : max(nch, 1);
  uint32_t rem = a.gmask ? gm : 1u;
  int gbase = a.gmask ? __builtin_ctz(gm | 0x80000000u) * cpg : 0, ci = 0, wi = 0;
  auto step = [&]() __attribute__((always_inline)) {
    if (wi + 1 < nch) {
      ++wi;
      if (++ci == cpg) {
        ci = 0;
        rem &= rem - 1;
        gbase = __builtin_ctz(rem | 0x80000000u) * cpg;
      }
    }
    return gbase + ci;
  };
  const char* wcot = reinterpret_cast<const char*>(a.wp + (int64_t)cot * wino::W16);
  const char* tb0 = reinterpret_cast<const char*>(static_cast<const u32x4*>(a.x) + (int64_t)b * K8 * tplane2);
  struct ChunkBase {
    const char* w;
    const char* t;
    bool kv1;  // the chunk's second 8-channel block exists (K % 16 == 8: not in the last chunk)
  };
  auto base_of = [&](int ph) __attribute__((always_inline)) {
    return ChunkBase{wcot + (int64_t)ph * a.n_cot * wino::W16 * 16, tb0 + (int64_t)(2 * ph) * tplane2 * 16,
                     2 * ph + 1 < K8};
  };
  auto issue_unit = [&](const ChunkBase& cb, int xi, int slot) __attribute__((always_inline)) {
    if (wave >= NIW) return;
    u32x4* dst = lds + slot * SLOT + wave * 64;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(cb.w + xi * 3 * 2 * BN * 16), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < NWI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(dst + j * NIT), 16,
                                               wvo[j], 0, 0, 0);
    const int32_t rows_b = xi * W * 32;
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(cb.t + rows_b), (short)0, cb.kv1 ? 0x7fffffff : (int)(tplane_b - rows_b), 0x00020000);
#pragma unroll
    for (int j = 0; j < NXT; ++j)
      if ((j * NIW + wave) * 64 < TROW)  // pieces wholly past the T row: not issued
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(dst + RUNIT + j * NIT),
                                                 16, tvo[j], 0, 0, 0);
  };
  // the current chunk and the next
  ChunkBase cur = base_of(gbase + ci);
  ChunkBase nx = base_of(step());
  auto advance = [&]() __attribute__((always_inline)) {
    cur = nx;
    nx = base_of(step());
  };

  const int rg = wave & 3;
  const int cw = 64 * (wave >> 2);
  floatx16 acc[2][NXI];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NXI; ++j) acc[i][j] = floatx16{0};
  // the init term i of the wave's 3 rows, loaded into acc[.][0..2] here (beside the first DMAs: the loads are older
  // than them, so the prologue's counted wait covers them) and turned after the first barrier into
  // M = (i0 - i2, (i1 + i2) / 2, (i2 - i1) / 2, 0, 0), whose A^T is exactly (i0, i1, i2): the epilogue adds nothing
  // (ring_epilogue<..., INIT = false>)
  if constexpr (!P3) {  // (conv2 -> conv3 partials: no init term)
    if (a.init) load_init<3>(a, y0 + ring_base_row<DIL>(rg), DIL, x0 + l32, cot * BN + cw, acc);
  }
  // one B set, refilled per kernel column right after its MFMAs (kw 0, 1 of the next unit after
  // the unit's barrier, kw 2 at the unit's start); two A sets alternating per kernel column
  bf16x8 fb[3][2];     // [kw][hi, lo]
  bf16x8 fa[2][2][2];  // [set][ct][hi, lo]
  auto fetch_b = [&](int kw, int slot) __attribute__((always_inline)) {
    const u32x4* X = lds + slot * SLOT + RUNIT + kl * (TROW / 2) + rg * XW + l32 + DIL * kw;
#pragma unroll
    for (int p = 0; p < 2; ++p) fb[kw][p] = __builtin_bit_cast(bf16x8, X[p * (TROW / 4)]);
  };
  auto fetch_a = [&](int st, int slot, int kw) __attribute__((always_inline)) {
    const u32x4* Wl = lds + slot * SLOT + kw * 2 * BN + kl * BN + cw + l32;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int p = 0; p < 2; ++p) fa[st][ct][p] = __builtin_bit_cast(bf16x8, Wl[p * RHALF + 32 * ct]);
  };
  auto sched6 = [&](auto nreads) __attribute__((always_inline)) {
    constexpr int n = decltype(nreads)::value;  // fragment reads spread over a kernel column's 6 MFMAs
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i < n) __builtin_amdgcn_sched_group_barrier(0x100, (n + 5) / 6, 0);
    }
  };

  // LDS-DMA pieces per wave per unit: waves < WHI issue NPU_HI, the others NPU_LO (the last T
  // piece only where it holds T entries)
  constexpr int NXT_LO = TROW / NIT;
  constexpr int WHI = (TROW % NIT + 63) / 64;
  static_assert(NXT_LO + (WHI > 0) == NXT, "T pieces");
  constexpr int NPU_HI = NWI + NXT;
  constexpr int NPU_LO = NWI + NXT_LO;
  const bool whi = wave < WHI;
#ifndef MVBEV_WINO_PB2
#define MVBEV_WINO_PB2 1  // conv2 (dilation 2): one barrier per two units (0: one per unit, as conv1)
#endif
  constexpr bool PB = DIL == 2 && MVBEV_WINO_PB2;  // one barrier per two units for conv2
  if (nch > 0) {
    const int U = NXI * nch;
    // prologue: units 0-3 (chunk 0, rows 0-3) in flight, wait for unit 0
    issue_unit(cur, 0, 0);
    issue_unit(cur, 1, 1);
    issue_unit(cur, 2, 2);
    issue_unit(cur, 3, 3);
    if (PB) {  // units 0 and 1 landed (the first barrier, after unit 1, retires 2 and 3)
      if (whi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPU_HI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPU_LO) : "memory");
    } else {
      if (whi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPU_HI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPU_LO) : "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (!P3) init_to_m(acc);  // (zeros without an init term: no branch)
    fetch_b(0, 0);
    fetch_b(1, 0);
    fetch_a(0, 0, 0);
    // unit u = u0 + R, R < 10 compile-time (u0 a multiple of 10): xi = R % 5, fragment set
    // R & 1; ring slot u % 4 (runtime)
#define WINO_MFMAS(AS, KW, XI)                                                                       \
  _Pragma("unroll") for (int ct = 0; ct < 2; ++ct) {                                                 \
    acc[ct][XI] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][1], fb[KW][0], acc[ct][XI], 0, 0, 0); \
    acc[ct][XI] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][0], fb[KW][1], acc[ct][XI], 0, 0, 0); \
    acc[ct][XI] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][0], fb[KW][0], acc[ct][XI], 0, 0, 0); \
  }
#define WINO_UNIT(R)                                                                                 \
  do {                                                                                               \
    constexpr int XI = (R) % 5, P = (R) & 1;                                                          \
    if (u0 + (R) >= U) break;                                                                        \
    constexpr int slot = (R) & 3, nslot = ((R) + 1) & 3; /* u0 % 20 == 0 */                        \
    fetch_a(P ^ 1, slot, 1);                                                                         \
    fetch_b(2, slot);                                                                                \
    WINO_MFMAS(P, 0, XI);                                                                            \
    sched6(std::integral_constant<int, 6>{});                                                        \
    fetch_a(P, slot, 2);                                                                             \
    WINO_MFMAS(P ^ 1, 1, XI);                                                                        \
    sched6(std::integral_constant<int, 4>{});                                                        \
    if (!PB) {                                                                         \
      /* retire unit u+1; every LDS read of this unit's slot is done */                               \
      if (whi) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NPU_HI) : "memory");     \
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NPU_LO) : "memory");          \
      __builtin_amdgcn_s_barrier();                                                                  \
      asm volatile("" ::: "memory");                                                                 \
      /* unit u+4 into this slot: (chunk, xi 4) at xi 0, else (next chunk, xi - 1) */                \
      issue_unit(XI == 0 ? cur : nx, (XI + 4) % 5, slot);                                            \
    } else if (P == 1) {                                                                             \
      /* PAIRB: one barrier per two units, after the odd one: retire units u+1, u+2 (all in      \
         flight), then units u+3, u+4 into the slots of u-1 and u */                                  \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                   \
      __builtin_amdgcn_s_barrier();                                                                  \
      asm volatile("" ::: "memory");                                                                 \
      issue_unit(XI <= 1 ? cur : nx, (XI + 3) % 5, (u0 + (R) + 3) & 3);                              \
      issue_unit(XI == 0 ? cur : nx, (XI + 4) % 5, slot);                                            \
    }                                                                                                \
    if (XI == 4) advance();                                                                          \
    fetch_b(0, nslot);                                                                               \
    fetch_b(1, nslot);                                                                               \
    fetch_a(P ^ 1, nslot, 0);                                                                        \
    WINO_MFMAS(P, 2, XI);                                                                            \
    sched6(std::integral_constant<int, 8>{});                                                        \
  } while (0)
    // 20 units per trip (the lcm of the 5 xi of a chunk and the 4 ring slots): the slot of every unit
    // is a compile-time constant, so no per-unit LDS address arithmetic (1-2 % on conv1 at cfg2 vs 10
    // units per trip, profiles/r04n_u20.jsonl)
    for (int u0 = 0; u0 < U; u0 += 20) {
      WINO_UNIT(0); WINO_UNIT(1); WINO_UNIT(2); WINO_UNIT(3); WINO_UNIT(4);
      WINO_UNIT(5); WINO_UNIT(6); WINO_UNIT(7); WINO_UNIT(8); WINO_UNIT(9);
      WINO_UNIT(10); WINO_UNIT(11); WINO_UNIT(12); WINO_UNIT(13); WINO_UNIT(14);
      WINO_UNIT(15); WINO_UNIT(16); WINO_UNIT(17); WINO_UNIT(18); WINO_UNIT(19);
    }
#undef WINO_UNIT
#undef WINO_MFMAS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the block exits
  } else if constexpr (!P3) {  // no chunk in this tile (frustum): M = the init term's transform alone, as above
    init_to_m(acc);
  }
  // y = A^T M per (Cout block, lane element): the 3 output rows of the wave's row tile
  floatx16 y[2][3];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const floatx16 m0 = acc[ct][0], m1 = acc[ct][1], m2 = acc[ct][2], m3 = acc[ct][3], m4 = acc[ct][4];
    y[ct][0] = m0 + m1 + m2 + m3;
    y[ct][1] = m1 - m2 + 2.f * m3;
    y[ct][2] = m1 + m2 + 4.f * m3 + m4;
  }
  ring_epilogue<DIL, RELU, P3, false>(a, b, y0 + ring_base_row<DIL>(rg), x0 + l32, cot, cw, y, lds);
#if MVBEV_WINO_STAMPS
  __syncthreads();
  if (threadIdx.x < 4 && blockIdx.x < 65536) {  // lanes 0-3 store one field each (vector stores)
    const long long v = threadIdx.x == 0 ? stamp0 : threadIdx.x == 1 ? wall_clock64()
                      : threadIdx.x == 2 ? (long long)__smid() : (long long)tile;
    g_wino_stamps[4 * blockIdx.x + threadIdx.x] = v;
  }
#endif
}

// (Round 4, VERDICT r03 item 5: a one-wave-per-SIMD form — 4 waves of 2 row tiles x 64 Cout, xi-major
// accumulation with the A^T fold after each xi's K sum, 12 + 12 fragment reads per 36 MFMAs — was
// parity-green but ran 1.75-1.85 ms vs 1.40-1.45 for conv1 and 0.41-0.47 vs 0.34-0.37 for conv2 +
// conv3 partials (profiles/r04b_kbench.jsonl): with one wave per SIMD every unit barrier drains the
// MFMA pipe, which the second wave of this kernel keeps fed.  Removed)

static int wino_rows_launch(const void* x, const mvbev_conv_desc* d, int dil, const uint32_t* group_mask, void* t,
                            size_t t_bytes, void* stream, const int32_t* gate = nullptr, int32_t gate_tag = 0) {
  if (!x || !d || !t) return MVBEV_ERR_NULL;
  if (dil != 1 && dil != 2) return MVBEV_ERR_DILATION;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || d->in_rows <= 0 || d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (d->K % SB != 0 || d->group % SB != 0 || d->K % d->group != 0) return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H || d->K / d->group > 65535 || d->B > 65535)
    return MVBEV_ERR_SHAPE;
  const int64_t tiles_y = ceil_div(d->out_rows, RT), tiles_x = ceil_div(d->W, TW);
  const int64_t need = d->B * (d->K / SB) * 5 * 4 * tiles_y * d->W * 32;
  if ((size_t)need > t_bytes || 2 * need / 32 > (int64_t)INT32_MAX * 8) return MVBEV_ERR_SHAPE;
  if (group_mask && d->K / d->group > 32) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(t)) & 15) != 0) return MVBEV_ERR_ALIGN;
  WinoRowsArgs a;
  a.x = static_cast<const u32x4*>(x);
  a.t = static_cast<u32x4*>(t);
  a.group_stride = d->group_stride, a.batch_stride = d->batch_stride;
  a.K = (int)d->K, a.group = (int)d->group, a.H = (int)d->H, a.W = (int)d->W;
  a.in_row0 = (int)d->in_row0, a.in_rows = (int)d->in_rows, a.out_row0 = (int)d->out_row0;
  a.tiles_x = (int)tiles_x, a.tiles_y = (int)tiles_y;
  a.dil = dil;
  a.gmask = group_mask;
  a.gate = gate, a.gate_tag = gate_tag;
  const int64_t nbg = ceil_div(d->group / SB, 8);  // wino_rows_kernel's KB
  if ((d->K / d->group) * nbg > 65535) return MVBEV_ERR_SHAPE;
  hipLaunchKernelGGL(wino_rows_kernel, dim3((unsigned)(tiles_x * tiles_y), (unsigned)((d->K / d->group) * nbg), (unsigned)d->B),
                     dim3(256), 0, as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

static int wino_launch(const void* t, const mvbev_conv_desc* d, const void* w_packed, const float* bias,
                       const float* init, int64_t Cout, int relu, float* y, int y_layout,
                       const uint32_t* group_mask, const int32_t* tile_order, void* stream, int dil = 1,
                       const float* w3 = nullptr, float* p3 = nullptr, int64_t band_rows = 0,
                       const uint32_t* out_mask = nullptr, int64_t cot_pg = 1) {
  if (!t || !d || !w_packed || (!y && !p3)) return MVBEV_ERR_NULL;
  if (dil != 1 && dil != 2) return MVBEV_ERR_DILATION;
  if (p3 && (!w3 || group_mask || init)) return MVBEV_ERR_SHAPE;  // the conv2 -> conv3 form: dense, bias only
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % BN != 0 || d->K % SB != 0 || d->group % SB != 0 || d->K % d->group != 0) return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H || d->H > INT32_MAX / 2 || d->W > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  if (y_layout != MVBEV_LAYOUT_F32 && y_layout != MVBEV_LAYOUT_SPLIT_BF16 &&
      !(y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX && !p3))
    return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(w_packed) | reinterpret_cast<uintptr_t>(t)) & 15) != 0) return MVBEV_ERR_ALIGN;
  Args a{};
  a.x = t; a.wp = static_cast<const u32x4*>(w_packed); a.bias = bias; a.init = init; a.y = y;
  a.w3 = w3; a.p3 = p3;
  a.B = (int)d->B; a.group = (int)d->group; a.K = (int)d->K; a.nchunks = (int)ceil_div(d->K, KC);
  a.Cout = (int)Cout; a.H = (int)d->H; a.W = (int)d->W;
  a.in_row0 = 0; a.in_rows = (int)d->H;
  a.out_row0 = (int)d->out_row0; a.out_rows = (int)d->out_rows;
  a.tiles_x = (int)ceil_div(d->W, TW); a.tiles_y = (int)ceil_div(d->out_rows, RT);
  a.n_cot = (int)(Cout / BN);
  const int64_t tiles = (int64_t)a.tiles_x * a.tiles_y * a.n_cot * d->B;
  if (tiles > INT32_MAX / 2 || 2LL * 5 * 4 * a.tiles_y * a.W * (d->K / SB) * d->B > (int64_t)INT32_MAX * 64)
    return MVBEV_ERR_SHAPE;
  // the kernel's 32-bit DMA offsets span two 8-channel planes of T: 2 * 32 B * XH * tiles_y * W < 2^31
  if (2LL * 32 * wino::XH * a.tiles_y * a.W >= (1LL << 31)) return MVBEV_ERR_SHAPE;
  if (group_mask) {
    if (d->group % KC != 0 || d->K / d->group > 32) return MVBEV_ERR_SHAPE;
    a.gmask = group_mask;
    a.cpg = (int)(d->group / KC);
  }
  a.tile_order = group_mask ? tile_order : nullptr;
  if (out_mask) {  // output-side mask (dense K): no input mask, no conv3 partials, <= 32 channel groups
    if (group_mask || p3 || band_rows || cot_pg <= 0 || a.n_cot > 32 * cot_pg) return MVBEV_ERR_SHAPE;
    a.cmask = out_mask;
    a.cot_pg = (int)cot_pg;
  }
  a.y_split = y_layout == MVBEV_LAYOUT_SPLIT_BF16 || y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX;
  a.y_pix = y_layout == MVBEV_LAYOUT_SPLIT_BF16_PIX;
  if (band_rows < 0 || (band_rows > 0 && (a.y_split || p3 || band_rows > d->out_rows))) return MVBEV_ERR_SHAPE;
  a.band_rows = (int)band_rows;
  a.npix = (int)(tiles / a.n_cot);
  // XCD turns of 8 consecutive ordered pixel tiles (equal view sets: the same weight-chunk stream, shared in
  // the XCD's L2) once the launch is >= 8 rounds deep; shallower launches deal them one at a time, where
  // the balance of the first rounds decides (cfg2, 1.9 rounds: groups of 4 +7 %; cfg5, 42 rounds: 8 -5 %,
  // cfg3 -2 %: profiles/r05o_mask_group_ab.jsonl, r05v_mask_group_large_ab.jsonl)
  a.mgroup = (group_mask && tiles >= 8 * (int64_t)std::max(cu_count(), 1)) ? 8 : 1;
  const int64_t nwg = group_mask ? (int64_t)a.n_cot * round_up(a.npix, 8 * a.mgroup) : tiles;
  a.nwg = (int)nwg;
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nwg), blk(RNT);
  if (p3) {
    if (dil != 2 || !relu) return MVBEV_ERR_SHAPE;  // conv2 -> conv3 of map_classifier (the only use)
    hipLaunchKernelGGL((conv_wino_kernel<true, 2, true>), grid, blk, 0, s, a);
  } else if (dil == 2) {
    if (relu) hipLaunchKernelGGL((conv_wino_kernel<true, 2, false>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((conv_wino_kernel<false, 2, false>), grid, blk, 0, s, a);
  } else if (relu) {
    hipLaunchKernelGGL((conv_wino_kernel<true, 1, false>), grid, blk, 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_wino_kernel<false, 1, false>), grid, blk, 0, s, a);
  }
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}


// ---------------------------------------------------------------------------------------------
// Row-Winograd F(4,3), xi-major (round 6).
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// (points 0, +-1, +-2, inf).  A wave's 4 output rows come from 6 transformed rows: 6 x 3 MFMA K-blocks
// per 16-channel chunk and 4 rows instead of F(3,3)'s 5 per 3 (-10 % of the MFMAs, T at 6/4 instead of
// 5/3 of the slab).  Accumulating per transformed row as the F(3,3) kernel does would need acc[2][6]
// (192 registers) beside the fragments — past the 256 a wave has at two waves per SIMD.  This kernel walks
// K xi-major instead: every (chunk, xi) unit is the F(3,3) kernel's unit (the same weight and T DMAs, the
// same 18 MFMAs per wave), but the units of one xi run back to back over all chunks into ONE accumulator
// pair, which is folded into the 4 output rows (y[r] += A^T[r][xi] M_xi, fp32) when the xi's K sum is
// complete: y[2][4] + acc[2] = 160 accumulator registers, as F(3,3)'s acc[2][5].  Workgroup tile 16 rows
// (4 row tiles of 4) x 32 columns x 128 Cout; dilation 2: row tile q holds rows base + 2 pt,
// base = 8 (q / 2) + q % 2.  T43[b][k / 8][6 r4 + xi][hi, lo][W][8], r4 < 4 ceil(out_rows / 16).
namespace w43 {
constexpr int NXI = 6;              // transformed rows per 4-row output tile
constexpr int RT4 = 16;             // output rows per workgroup tile
constexpr int XH = 4 * NXI;         // T rows of a workgroup tile
constexpr int NTAP = 3 * NXI;       // packed taps (xi, kw)
constexpr int WPART = NTAP * KC * BN;
constexpr int W16 = 2 * WPART * 2 / 16;  // 16-B pieces per (chunk, cout tile)
template <int DIL>
__device__ inline int base_row(int rg) {
  return DIL == 1 ? 4 * rg : (rg >> 1) * 8 + (rg & 1);
}
}  // namespace w43

// packed[chunk][cot][part][3 xi + kw][sub][co][j] = split(sum_kh G43[xi][kh] w[co][map(k)][kh][kw])
__global__ void pack_wino43_kernel(const float* __restrict__ w, __bf16* __restrict__ out, int Cout, int Cin_w,
                                   const int32_t* __restrict__ chan_map, int K, int K_pad) {
  const int n_cot = Cout / BN;
  const int64_t total = (int64_t)(K_pad / KC) * n_cot * 3 * 2 * BN * SB;  // kernel columns
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int j = r % SB; r /= SB;
    const int co = r % BN; r /= BN;
    const int sub = r % 2; r /= 2;
    const int kw = r % 3; r /= 3;
    const int cot = r % n_cot;
    const int chunk = (int)(r / n_cot);
    const int k = chunk * KC + sub * SB + j;
    int ci = k < K ? (chan_map ? chan_map[k] : k) : -1;
    if (ci >= Cin_w) ci = -1;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0;
    if (ci >= 0) {
      const float* g = w + ((int64_t)(cot * BN + co) * Cin_w + ci) * 9 + kw;  // g[3 kh]
      g0 = g[0], g1 = g[3], g2 = g[6];
    }
    const double u[w43::NXI] = {0.25 * g0, -(g0 + g1 + g2) / 6.0, (g1 - g0 - g2) / 6.0,
                                g0 / 24.0 + g1 / 12.0 + g2 / 6.0, g0 / 24.0 - g1 / 12.0 + g2 / 6.0, g2};
    __bf16* o = out + ((int64_t)chunk * n_cot + cot) * 2 * w43::WPART + ((int64_t)sub * BN + co) * SB + j;
#pragma unroll
    for (int xi = 0; xi < w43::NXI; ++xi) {
      const float v = (float)u[xi];
      const __bf16 hi = (__bf16)v;
      const int tap = 3 * xi + kw;
      o[(int64_t)tap * KC * BN] = hi;
      o[(int64_t)(w43::NTAP + tap) * KC * BN] = (__bf16)(v - (float)hi);
    }
  }
}

// T43 of a split-bf16 input (the slab, or y1 for conv2): a thread per (column, row tile q of the 16-row
// tile, 8-channel block pair kq) and 2 blocks; d[m] = x[base + dil (m - 1)], m < 6 (zero outside the image
// and the input rows).  With a frustum mask the groups it clears for the tile are skipped (as wino_rows).
__global__ __launch_bounds__(256) void wino43_rows_kernel(const WinoRowsArgs a) {
  constexpr int KB = 4;  // 8-channel blocks per workgroup: 4 x 32 x 2 threads, 2 blocks each
  const int pp = blockIdx.x, b = blockIdx.z;
  const int nbg = (a.group / SB + KB - 1) / KB;
  const int g = blockIdx.y / nbg, kb0 = (blockIdx.y - g * nbg) * KB;
  if (a.gmask && !((a.gmask[pp] >> g) & 1u)) return;
  const int W = a.W;
  const int ty = pp / a.tiles_x;
  const int x0 = (pp - ty * a.tiles_x) * TW;
  const int nb = a.group / SB, K8 = a.K / SB, R6 = w43::NXI * 4 * a.tiles_y;
  const int64_t plane = (int64_t)a.in_rows * W;
  const int c = threadIdx.x % TW, q = (threadIdx.x / TW) % 4, kq = threadIdx.x / (4 * TW);  // kq < 2
  const int col = x0 + c, r4 = 4 * ty + q;
  if (col >= W) return;
  const int base = w43::RT4 * ty + (a.dil == 1 ? 4 * q : (q >> 1) * 8 + (q & 1));
  int64_t roff[6];
  bool rok[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const int row = a.out_row0 + base + a.dil * (m - 1), by = row - a.in_row0;
    rok[m] = row >= 0 && row < a.H && by >= 0 && by < a.in_rows;
    roff[m] = 2 * ((int64_t)by * W + col);
  }
  u32x4 raw[2][6][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kb = kb0 + kq + 2 * i;
    const bool kok = kb < nb && g * a.group + kb * SB < a.K;
    const u32x4* src = a.x + ((int64_t)b * a.batch_stride + (int64_t)g * a.group_stride +
                              (int64_t)(kok ? kb : 0) * SB * plane) / 4;
#pragma unroll
    for (int m = 0; m < 6; ++m)
#pragma unroll
      for (int p = 0; p < 2; ++p) raw[i][m][p] = (kok && rok[m]) ? src[roff[m] + p] : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kb = kb0 + kq + 2 * i, k0 = g * a.group + kb * SB;
    if (kb >= nb || k0 >= a.K) continue;
    float d[6][8];
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      float h[8], l[8];
      bf16x8_to_f32(raw[i][m][0], h);
      bf16x8_to_f32(raw[i][m][1], l);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[m][j] = h[j] + l[j];
    }
    u32x4* dst = a.t + 2 * (((int64_t)b * K8 + k0 / SB) * R6 * W + (int64_t)w43::NXI * r4 * W) + col;
#pragma unroll
    for (int xi = 0; xi < w43::NXI; ++xi) {
      unsigned hp[4], lp[4];
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        unsigned short hs[2], ls[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * e4 + e;
          const float d0 = d[0][j], d1 = d[1][j], d2 = d[2][j], d3 = d[3][j], d4 = d[4][j], d5 = d[5][j];
          const float v = xi == 0 ? 4.f * d0 - 5.f * d2 + d4
                        : xi == 1 ? -4.f * d1 - 4.f * d2 + d3 + d4
                        : xi == 2 ? 4.f * d1 - 4.f * d2 - d3 + d4
                        : xi == 3 ? -2.f * d1 - d2 + 2.f * d3 + d4
                        : xi == 4 ? 2.f * d1 - d2 - 2.f * d3 + d4
                                  : 4.f * d1 - 5.f * d3 + d5;
          const __bf16 hv = (__bf16)v, lv = (__bf16)(v - (float)hv);
          hs[e] = __builtin_bit_cast(unsigned short, hv);
          ls[e] = __builtin_bit_cast(unsigned short, lv);
        }
        hp[e4] = (unsigned)hs[0] | ((unsigned)hs[1] << 16);
        lp[e4] = (unsigned)ls[0] | ((unsigned)ls[1] << 16);
      }
      dst[2 * (int64_t)xi * W] = u32x4{hp[0], hp[1], hp[2], hp[3]};
      dst[2 * (int64_t)xi * W + W] = u32x4{lp[0], lp[1], lp[2], lp[3]};
    }
  }
}

// The F(4,3) conv: conv_wino_kernel's ring, DMAs, fragment schedule and epilogues, with units walked
// xi-major (above).  Two walkers of the tile's chunk sequence: the DMA side issues unit u + 4 while the
// compute side runs unit u; at the end of each xi's K sum the accumulators are folded into y.
template <bool RELU, int DIL, bool P3>
__global__ __launch_bounds__(RNT, 1) void conv_wino43_kernel(const Args a) {
  using namespace wino;  // the ring geometry (NIW, NIT, NWI, Geo, SLOT, NSLOT, LDS) is F(3,3)'s
  using G = Geo<DIL>;
  constexpr int XW = G::XW, TROW = G::TROW, NXT = G::NXT;
  constexpr int NX6 = w43::NXI;
  __shared__ __attribute__((aligned(16))) u32x4 lds[LDS];
  const int W = a.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, kl = lane >> 5;

  int tile = xcd_remap(blockIdx.x, a.nwg);
  if (a.gmask) {
    const int Gq = a.mgroup;
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int q = j / a.n_cot;
    const int slot = Gq * (8 * (q / Gq) + x) + q % Gq;
    if (slot >= a.npix) return;
    tile = (a.tile_order ? a.tile_order[slot] : slot) * a.n_cot + j % a.n_cot;
  }
  const int cot = tile % a.n_cot, rest = tile / a.n_cot;
  const int t_main = a.tiles_y * a.tiles_x;
  const int pp = rest % t_main, b = rest / t_main;
  const int ty = pp / a.tiles_x;
  const int x0 = (pp - ty * a.tiles_x) * TW;
  const int y0 = a.out_row0 + ty * w43::RT4;
  const uint32_t gm = a.gmask ? a.gmask[pp] : 0u;
  const int nch = a.gmask ? __builtin_popcount(gm) * a.cpg : a.nchunks;
  const int K8 = a.K / SB;
  const int64_t tplane2 = 2LL * (w43::XH * a.tiles_y) * W;
  const uint32_t tplane_b = (uint32_t)(tplane2 * 16);
  constexpr uint32_t kOOB = 0x80000000u;
  uint32_t wvo[NWI], tvo[NXTMAX];
#pragma unroll
  for (int j = 0; j < NWI; ++j) {
    const int e = (j * NIW + wave) * 64 + lane;
    wvo[j] = (uint32_t)(((e / RHALF) * (w43::NTAP * 2 * BN) + e % RHALF) * 16);
    asm volatile("" : "+v"(wvo[j]));
  }
#pragma unroll
  for (int j = 0; j < NXT; ++j) {
    const int e = (j * NIW + wave) * 64 + lane;
    const int sub = e / (TROW / 2), part = (e / (TROW / 4)) & 1, rt = (e % (TROW / 4)) / XW, c = e % XW;
    const int gx = x0 - DIL + c;
    const bool z = e >= TROW || gx < 0 || gx >= W;
    tvo[j] = z ? kOOB : (uint32_t)sub * tplane_b + (uint32_t)((2 * (w43::XH * ty + NX6 * rt) * W + part * W + gx) * 16);
    asm volatile("" : "+v"(tvo[j]));
  }
  // the DMA side's walker (issuing waves only; a scalar branch): unit (ixi, iwi-th chunk of the tile's
  // sequence = chunk ph, index ici of its group), its weight / T bases stepped per chunk (the per-unit
  // address arithmetic of a walker that multiplies out every base cost 90-130 scalar instructions per
  // unit on every wave, ~4x the F(3,3) kernel's); past the last unit it stays on it (dummy loads that
  // keep the vmcnt counts exact)
  const int cpg = a.gmask ? a.cpg : max(nch, 1);
  const uint32_t rem0 = a.gmask ? gm : 1u;
  const int gbase0 = a.gmask ? __builtin_ctz(gm | 0x80000000u) * cpg : 0;
  const int64_t wstep = (int64_t)a.n_cot * w43::W16 * 16, tstep = 2 * tplane2 * 16;
  const char* w_first = reinterpret_cast<const char*>(a.wp + (int64_t)cot * w43::W16) + gbase0 * wstep;
  const char* t_first = reinterpret_cast<const char*>(static_cast<const u32x4*>(a.x) + (int64_t)b * K8 * tplane2) +
                        gbase0 * tstep;
  const char* iwp = w_first;
  const char* itp = t_first;
  uint32_t irem = rem0;
  int ph = gbase0, ici = 0, iwi = 0, ixi = 0, irows_b = 0;
  auto issue_next = [&](int slot) __attribute__((always_inline)) {
    if (wave >= NIW) return;
    u32x4* dst = lds + slot * SLOT + wave * 64;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(iwp), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < NWI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(dst + j * NIT), 16,
                                               wvo[j], 0, 0, 0);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(itp), (short)0, 2 * ph + 1 < K8 ? 0x7fffffff : (int)(tplane_b - irows_b), 0x00020000);
#pragma unroll
    for (int j = 0; j < NXT; ++j)
      if ((j * NIW + wave) * 64 < TROW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(dst + RUNIT + j * NIT),
                                                 16, tvo[j], 0, 0, 0);
    if (iwi + 1 < nch) {
      ++iwi;
      if (++ici == cpg) {  // the next set group of the mask
        ici = 0;
        irem &= irem - 1;
        const int nph = __builtin_ctz(irem | 0x80000000u) * cpg;
        iwp += (nph - ph) * wstep;
        itp += (nph - ph) * tstep;
        ph = nph;
      } else {
        ++ph;
        iwp += wstep;
        itp += tstep;
      }
    } else if (ixi + 1 < NX6) {  // the next xi: the chunk sequence from its start
      ++ixi;
      iwi = 0, ici = 0, irem = rem0, ph = gbase0;
      irows_b = ixi * W * 32;
      iwp = w_first + ixi * 3 * 2 * BN * 16;
      itp = t_first + irows_b;
    }
  };

  const int rg = wave & 3;
  const int cw = 64 * (wave >> 2);
  floatx16 acc[2], y[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc[i] = floatx16{0};
#pragma unroll
    for (int r = 0; r < 4; ++r) y[i][r] = floatx16{0};
  }
  if (a.init)  // the output rows start at the init term (the epilogue adds nothing: store_block<..., false>)
    load_init<4>(a, y0 + w43::base_row<DIL>(rg), DIL, x0 + l32, cot * BN + cw, y);  // (y: [2][4])
  bf16x8 fb[3][2];
  bf16x8 fa[2][2][2];
  auto fetch_b = [&](int kw, int slot) __attribute__((always_inline)) {
    const u32x4* X = lds + slot * SLOT + RUNIT + kl * (TROW / 2) + rg * XW + l32 + DIL * kw;
#pragma unroll
    for (int p = 0; p < 2; ++p) fb[kw][p] = __builtin_bit_cast(bf16x8, X[p * (TROW / 4)]);
  };
  auto fetch_a = [&](int st, int slot, int kw) __attribute__((always_inline)) {
    const u32x4* Wl = lds + slot * SLOT + kw * 2 * BN + kl * BN + cw + l32;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int p = 0; p < 2; ++p) fa[st][ct][p] = __builtin_bit_cast(bf16x8, Wl[p * RHALF + 32 * ct]);
  };
  auto sched6 = [&](auto nreads) __attribute__((always_inline)) {
    constexpr int n = decltype(nreads)::value;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i < n) __builtin_amdgcn_sched_group_barrier(0x100, (n + 5) / 6, 0);
    }
  };
  // y[r] += A^T[r][xi] M_xi: A^T column xi = (1, s p, p^2, s p^3), p = (xi + 1) / 2, s = +-1 (xi 1-4);
  // (1, 0, 0, 0) for xi 0, (0, 0, 0, 1) for xi 5
  auto fold = [&](int xi) __attribute__((always_inline)) {
    const float p = (float)((xi + 1) >> 1), sp = (xi & 1) ? p : -p;
    const bool mid = xi > 0 && xi < 5;
    const float c0 = xi < 5 ? 1.f : 0.f, c1 = mid ? sp : 0.f, c2 = mid ? p * p : 0.f,
                c3 = mid ? sp * p * p : (xi == 5 ? 1.f : 0.f);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      y[ct][0] += c0 * acc[ct];
      y[ct][1] += c1 * acc[ct];
      y[ct][2] += c2 * acc[ct];
      y[ct][3] += c3 * acc[ct];
      acc[ct] = floatx16{0};
    }
  };

  constexpr int NXT_LO = TROW / NIT;
  constexpr int WHI = (TROW % NIT + 63) / 64;
  static_assert(NXT_LO + (WHI > 0) == NXT, "T pieces");
  constexpr int NPU_HI = NWI + NXT;
  constexpr int NPU_LO = NWI + NXT_LO;
  const bool whi = wave < WHI;
  if (nch > 0) {
    const int U = NX6 * nch;
    int cleft = nch, cxi = 0;  // the compute side: units left in xi cxi
    issue_next(0);
    issue_next(1);
    issue_next(2);
    issue_next(3);
    if (whi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPU_HI) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPU_LO) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    fetch_b(0, 0);
    fetch_b(1, 0);
    fetch_a(0, 0, 0);
#define W43_MFMAS(AS, KW)                                                                              \
  _Pragma("unroll") for (int ct = 0; ct < 2; ++ct) {                                                   \
    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][1], fb[KW][0], acc[ct], 0, 0, 0);     \
    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][0], fb[KW][1], acc[ct], 0, 0, 0);     \
    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[AS][ct][0], fb[KW][0], acc[ct], 0, 0, 0);     \
  }
#define W43_UNIT(R)                                                                                    \
  do {                                                                                                 \
    constexpr int P = (R) & 1, slot = (R) & 3, nslot = ((R) + 1) & 3; /* u0 % 4 == 0 */               \
    if (u0 + (R) >= U) break;                                                                          \
    fetch_a(P ^ 1, slot, 1);                                                                           \
    fetch_b(2, slot);                                                                                  \
    W43_MFMAS(P, 0);                                                                                   \
    sched6(std::integral_constant<int, 6>{});                                                          \
    fetch_a(P, slot, 2);                                                                               \
    W43_MFMAS(P ^ 1, 1);                                                                               \
    sched6(std::integral_constant<int, 4>{});                                                          \
    if (whi) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NPU_HI) : "memory");             \
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NPU_LO) : "memory");                  \
    __builtin_amdgcn_s_barrier();                                                                      \
    asm volatile("" ::: "memory");                                                                     \
    issue_next(slot); /* unit u + 4 into this slot */                                                  \
    fetch_b(0, nslot);                                                                                 \
    fetch_b(1, nslot);                                                                                 \
    fetch_a(P ^ 1, nslot, 0);                                                                          \
    W43_MFMAS(P, 2);                                                                                   \
    sched6(std::integral_constant<int, 8>{});                                                          \
    if (--cleft == 0) {                                                                                \
      fold(cxi);                                                                                       \
      ++cxi;                                                                                           \
      cleft = nch;                                                                                     \
    }                                                                                                  \
  } while (0)
    for (int u0 = 0; u0 < U; u0 += 4) {
      W43_UNIT(0); W43_UNIT(1); W43_UNIT(2); W43_UNIT(3);
    }
#undef W43_UNIT
#undef W43_MFMAS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the block exits
  }
  const int row_base = y0 + w43::base_row<DIL>(rg), col = x0 + l32;
  if constexpr (P3) {
    cout1_partials<RELU, 4>(a, b, row_base, DIL, col, cot, cw, y, lds);
  } else {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int pt = 0; pt < 4; ++pt)
        store_block<RELU, false>(a, b, row_base + pt * DIL, col, cot * BN + cw + 32 * ct, y[ct][pt]);
  }
}

static int wino43_rows_launch(const void* x, const mvbev_conv_desc* d, int dil, const uint32_t* group_mask, void* t,
                              size_t t_bytes, void* stream) {
  if (!x || !d || !t) return MVBEV_ERR_NULL;
  if (dil != 1 && dil != 2) return MVBEV_ERR_DILATION;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || d->in_rows <= 0 || d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (d->K % SB != 0 || d->group % SB != 0 || d->K % d->group != 0) return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H || d->K / d->group > 65535 || d->B > 65535)
    return MVBEV_ERR_SHAPE;
  const int64_t tiles_y = ceil_div(d->out_rows, w43::RT4), tiles_x = ceil_div(d->W, TW);
  const int64_t need = d->B * (d->K / SB) * w43::NXI * 4 * tiles_y * d->W * 32;
  if ((size_t)need > t_bytes || 2 * need / 32 > (int64_t)INT32_MAX * 8) return MVBEV_ERR_SHAPE;
  if (group_mask && d->K / d->group > 32) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(t)) & 15) != 0) return MVBEV_ERR_ALIGN;
  WinoRowsArgs a{};
  a.x = static_cast<const u32x4*>(x);
  a.t = static_cast<u32x4*>(t);
  a.group_stride = d->group_stride, a.batch_stride = d->batch_stride;
  a.K = (int)d->K, a.group = (int)d->group, a.H = (int)d->H, a.W = (int)d->W;
  a.in_row0 = (int)d->in_row0, a.in_rows = (int)d->in_rows, a.out_row0 = (int)d->out_row0;
  a.tiles_x = (int)tiles_x, a.tiles_y = (int)tiles_y;
  a.dil = dil;
  a.gmask = group_mask;
  const int64_t nbg = ceil_div(d->group / SB, 4);  // wino43_rows_kernel's KB
  if ((d->K / d->group) * nbg > 65535) return MVBEV_ERR_SHAPE;
  hipLaunchKernelGGL(wino43_rows_kernel, dim3((unsigned)(tiles_x * tiles_y), (unsigned)((d->K / d->group) * nbg),
                                              (unsigned)d->B),
                     dim3(256), 0, as_stream(stream), a);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

static int wino43_launch(const void* t, const mvbev_conv_desc* d, const void* w_packed, const float* bias,
                         const float* init, int64_t Cout, int dil, int relu, float* y, int y_layout,
                         const uint32_t* group_mask, const int32_t* tile_order, const float* w3, float* p3,
                         void* stream) {
  if (!t || !d || !w_packed || (!y && !p3)) return MVBEV_ERR_NULL;
  if (dil != 1 && dil != 2) return MVBEV_ERR_DILATION;
  if (p3 && (!w3 || group_mask || init || dil != 2 || !relu)) return MVBEV_ERR_SHAPE;
  if (d->B <= 0 || d->K <= 0 || d->H <= 0 || d->W <= 0 || Cout <= 0 || d->out_rows <= 0 || d->group <= 0)
    return MVBEV_ERR_RANK;
  if (Cout % BN != 0 || d->K % SB != 0 || d->group % SB != 0 || d->K % d->group != 0) return MVBEV_ERR_SHAPE;
  if (d->out_row0 < 0 || d->out_row0 + d->out_rows > d->H || d->H > INT32_MAX / 2 || d->W > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  if (y_layout != MVBEV_LAYOUT_F32 && y_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;
  if (((reinterpret_cast<uintptr_t>(w_packed) | reinterpret_cast<uintptr_t>(t)) & 15) != 0) return MVBEV_ERR_ALIGN;
  Args a{};
  a.x = t; a.wp = static_cast<const u32x4*>(w_packed); a.bias = bias; a.init = init; a.y = y;
  a.w3 = w3; a.p3 = p3;
  a.B = (int)d->B; a.group = (int)d->group; a.K = (int)d->K; a.nchunks = (int)ceil_div(d->K, KC);
  a.Cout = (int)Cout; a.H = (int)d->H; a.W = (int)d->W;
  a.in_row0 = 0; a.in_rows = (int)d->H;
  a.out_row0 = (int)d->out_row0; a.out_rows = (int)d->out_rows;
  a.tiles_x = (int)ceil_div(d->W, TW); a.tiles_y = (int)ceil_div(d->out_rows, w43::RT4);
  a.n_cot = (int)(Cout / BN);
  const int64_t tiles = (int64_t)a.tiles_x * a.tiles_y * a.n_cot * d->B;
  if (tiles > INT32_MAX / 2 || 2LL * w43::NXI * 4 * a.tiles_y * a.W * (d->K / SB) * d->B > (int64_t)INT32_MAX * 64)
    return MVBEV_ERR_SHAPE;
  if (2LL * 32 * w43::XH * a.tiles_y * a.W >= (1LL << 31)) return MVBEV_ERR_SHAPE;
  if (group_mask) {
    if (d->group % KC != 0 || d->K / d->group > 32) return MVBEV_ERR_SHAPE;
    a.gmask = group_mask;
    a.cpg = (int)(d->group / KC);
  }
  a.tile_order = group_mask ? tile_order : nullptr;
  a.y_split = y_layout == MVBEV_LAYOUT_SPLIT_BF16;
  a.npix = (int)(tiles / a.n_cot);
  a.mgroup = (group_mask && tiles >= 8 * (int64_t)std::max(cu_count(), 1)) ? 8 : 1;
  const int64_t nwg = group_mask ? (int64_t)a.n_cot * round_up(a.npix, 8 * a.mgroup) : tiles;
  a.nwg = (int)nwg;
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nwg), blk(RNT);
  if (p3) hipLaunchKernelGGL((conv_wino43_kernel<true, 2, true>), grid, blk, 0, s, a);
  else if (dil == 2) {
    if (relu) hipLaunchKernelGGL((conv_wino43_kernel<true, 2, false>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((conv_wino43_kernel<false, 2, false>), grid, blk, 0, s, a);
  } else if (relu) {
    hipLaunchKernelGGL((conv_wino43_kernel<true, 1, false>), grid, blk, 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_wino43_kernel<false, 1, false>), grid, blk, 0, s, a);
  }
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

}  // namespace b3
}  // namespace mvbev

extern "C" {

size_t mvbev_conv3x3_packed_bytes_bf16x3(int64_t Cout, int64_t K) {
  if (Cout <= 0 || K <= 0) return 0;
  return (size_t)(mvbev::round_up(K, mvbev::b3::KC) / mvbev::b3::KC) *
         (size_t)(Cout / mvbev::b3::BN) * mvbev::b3::WBYTES;
}

int mvbev_pack_conv3x3_weight_bf16x3(const float* w, int64_t Cout, int64_t Cin_w,
                                     const int32_t* chan_map, int64_t K, void* w_packed,
                                     void* stream) {
  using namespace mvbev;
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout <= 0 || Cin_w <= 0 || K <= 0) return MVBEV_ERR_RANK;
  if (Cout % b3::BN != 0) return MVBEV_ERR_SHAPE;
  if (!chan_map && K != Cin_w) return MVBEV_ERR_SHAPE;
  const int64_t k_pad = round_up(K, b3::KC);
  const int64_t total = (int64_t)mvbev_conv3x3_packed_bytes_bf16x3(Cout, K) / 2;
  const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(b3::pack_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), w,
                     static_cast<__bf16*>(w_packed), (int)Cout, (int)Cin_w, chan_map, (int)K,
                     (int)k_pad);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_pack_conv3x3_dgrad_bf16x3(const float* w, int64_t Cout_w, int64_t Cin_w, const int32_t* chan_map,
                                    int64_t K_out, void* w_packed, void* stream) {
  using namespace mvbev;
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout_w <= 0 || Cin_w <= 0 || K_out <= 0) return MVBEV_ERR_RANK;
  if (!chan_map && K_out > Cin_w) return MVBEV_ERR_SHAPE;
  const int64_t cout_p = round_up(K_out, b3::BN);
  const int64_t k_pad = round_up(Cout_w, b3::KC);
  const int64_t total = (int64_t)mvbev_conv3x3_packed_bytes_bf16x3(cout_p, Cout_w) / 2;
  const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(b3::pack_dgrad_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), w,
                     static_cast<__bf16*>(w_packed), (int)cout_p, (int)Cout_w, (int)Cin_w, chan_map,
                     (int)K_out, (int)k_pad);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_conv3x3_bf16x3_tile_rows(int x_layout, int dilation) {
  const bool ring = x_layout == MVBEV_LAYOUT_SPLIT_BF16 && MVBEV_B3_RING && (dilation == 1 || dilation == 2);
  return ring ? mvbev::b3::RT : MVBEV_B3_WAVES;
}

size_t mvbev_conv3x3_bf16x3_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout) {
  using namespace mvbev::b3;
  if (!desc || Cout <= 0 || desc->W <= 0 || desc->out_rows <= 0 || desc->B <= 0 || desc->K <= 0)
    return 0;
  const SkPlan p = sk_plan(conv_tiles(desc, Cout), mvbev::ceil_div(desc->K, KC));
  return p.split > 1 ? (size_t)(p.tail * p.split) * kSkSlotBytes : 0;
}

int mvbev_conv3x3_bf16x3_ex(const void* x, int x_layout, const mvbev_conv_desc* desc,
                            const void* w_packed, const float* bias, const float* init,
                            int64_t Cout, int dilation, int relu, void* y, int y_layout,
                            const uint32_t* group_mask, const int32_t* tile_order, void* workspace,
                            size_t workspace_bytes, void* stream) {
  using namespace mvbev::b3;
  if (x_layout == MVBEV_LAYOUT_SPLIT_BF16)
    return launch<SplitIn>(x, desc, w_packed, bias, init, Cout, dilation, relu,
                           static_cast<float*>(y), y_layout, group_mask, tile_order, workspace,
                           workspace_bytes, stream);
  if (x_layout == MVBEV_LAYOUT_F16)
    return launch<_Float16>(x, desc, w_packed, bias, init, Cout, dilation, relu,
                            static_cast<float*>(y), y_layout, group_mask, tile_order, workspace,
                            workspace_bytes, stream);
  return launch<float>(x, desc, w_packed, bias, init, Cout, dilation, relu,
                       static_cast<float*>(y), y_layout, group_mask, tile_order, workspace,
                       workspace_bytes, stream);
}

int mvbev_conv_ring_tile_space(const mvbev_conv_desc* desc, int tile_space, int64_t g[5]) {
  if (!desc || !g) return MVBEV_ERR_NULL;
  return mvbev::b3::ring_tile_space(desc, tile_space, g);
}

int mvbev_conv3x3_bf16x3_ex3(const void* x, int x_layout, const mvbev_conv_desc* desc,
                             const void* w_packed, const float* bias, const float* init,
                             int64_t Cout, int dilation, int relu, void* y, int y_layout,
                             const uint32_t* group_mask, const int32_t* tile_order, int tile_space,
                             void* stream) {
  using namespace mvbev::b3;
  if (x_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;  // the ring kernel's input
  return launch<SplitIn>(x, desc, w_packed, bias, init, Cout, dilation, relu, static_cast<float*>(y), y_layout,
                         group_mask, tile_order, nullptr, 0, stream, nullptr, 1, nullptr, nullptr, nullptr,
                         tile_space);
}

size_t mvbev_conv3x3_bf16x3_cout1_partials_bytes(const mvbev_conv_desc* desc, int64_t Cout) {
  if (!desc || Cout <= 0 || Cout % mvbev::b3::BN != 0 || desc->B <= 0 || desc->W <= 0 || desc->out_rows <= 0) return 0;
  return (size_t)desc->B * (size_t)(2 * (Cout / mvbev::b3::BN)) * 9 * (size_t)desc->out_rows * (size_t)desc->W *
         sizeof(float);
}

int mvbev_conv3x3_bf16x3_cout1_partials(const void* x, const mvbev_conv_desc* desc, const void* w_packed,
                                        const float* bias, int64_t Cout, int dilation, int relu, const float* w3,
                                        void* partials, size_t partials_bytes, void* stream) {
  using namespace mvbev::b3;
  if (!desc || !w3 || !partials) return MVBEV_ERR_NULL;
  const size_t need = mvbev_conv3x3_bf16x3_cout1_partials_bytes(desc, Cout);
  if (need == 0 || partials_bytes < need) return MVBEV_ERR_SHAPE;
  return launch<SplitIn>(x, desc, w_packed, bias, nullptr, Cout, dilation, relu, nullptr, MVBEV_LAYOUT_F32, nullptr,
                         nullptr, nullptr, 0, stream, nullptr, 1, w3, static_cast<float*>(partials));
}

int mvbev_cout1_reduce_partials(const void* partials, const mvbev_conv_desc* desc, int64_t Cout, int dilation3,
                                float* map, int64_t map_row0, int64_t map_rows, void* stream) {
  using namespace mvbev::b3;
  if (!partials || !desc || !map) return MVBEV_ERR_NULL;
  if (dilation3 < 1) return MVBEV_ERR_DILATION;
  if (map_rows <= 0 || Cout <= 0 || desc->B <= 0 || desc->W <= 0 || desc->out_rows <= 0) return MVBEV_ERR_RANK;
  if (Cout % BN != 0) return MVBEV_ERR_SHAPE;
  // every row the map band reads (band +- dilation3, inside the image) must be a computed row
  const int64_t r_lo = std::max<int64_t>(0, map_row0 - dilation3);
  const int64_t r_hi = std::min<int64_t>(desc->H, map_row0 + map_rows + dilation3);
  if (map_row0 < 0 || map_row0 + map_rows > desc->H || r_lo < desc->out_row0 || r_hi > desc->out_row0 + desc->out_rows ||
      map_rows > 65535 || desc->B > 65535 || desc->out_rows * desc->W > INT32_MAX)
    return MVBEV_ERR_SHAPE;
  const dim3 grid((unsigned)mvbev::ceil_div(desc->W, 64), (unsigned)map_rows, (unsigned)desc->B);
  hipLaunchKernelGGL(cout1_reduce_kernel, grid, dim3(64 * kC1rGroups), 0, mvbev::as_stream(stream),
                     static_cast<const float*>(partials), (int)(2 * (Cout / BN)), (int)desc->H, (int)desc->W,
                     (int)desc->out_rows, (int)desc->out_row0, dilation3, map, (int)map_row0, (int)map_rows);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

size_t mvbev_conv_schedule_slot_bytes(void) { return sizeof(mvbev::b3::floatx4) * mvbev::b3::kRingSlotF4; }

int mvbev_conv3x3_dgrad_bf16x3_sched(const void* dy, int dy_layout, const mvbev_conv_desc* desc,
                                     const void* w_packed, int64_t Cout_p, int dilation, void* dx, int dx_layout,
                                     const uint32_t* out_mask, int64_t cot_per_group,
                                     const mvbev_conv_schedule* sched, void* stream) {
  using namespace mvbev::b3;
  if (!sched) return MVBEV_ERR_NULL;
  if (out_mask && (cot_per_group <= 0 || cot_per_group > 65536)) return MVBEV_ERR_SHAPE;
  if (dy_layout != MVBEV_LAYOUT_SPLIT_BF16) return MVBEV_ERR_SHAPE;
  return launch<SplitIn>(dy, desc, w_packed, nullptr, nullptr, Cout_p, dilation, 0, static_cast<float*>(dx),
                         dx_layout, nullptr, nullptr, nullptr, 0, stream, out_mask, (int)cot_per_group, nullptr,
                         nullptr, sched);
}

int mvbev_conv3x3_dgrad_bf16x3_ex(const void* dy, int dy_layout, const mvbev_conv_desc* desc, const void* w_packed,
                                  int64_t Cout_p, int dilation, void* dx, int dx_layout, const uint32_t* out_mask,
                                  int64_t cot_per_group, void* stream) {
  using namespace mvbev::b3;
  if (out_mask && (cot_per_group <= 0 || cot_per_group > 65536)) return MVBEV_ERR_SHAPE;
  if (dy_layout == MVBEV_LAYOUT_SPLIT_BF16)  // the LDS-DMA ring kernel (12-row output tiles)
    return launch<SplitIn>(dy, desc, w_packed, nullptr, nullptr, Cout_p, dilation, 0, static_cast<float*>(dx),
                           dx_layout, nullptr, nullptr, nullptr, 0, stream, out_mask, (int)cot_per_group);
  if (dy_layout != MVBEV_LAYOUT_F32) return MVBEV_ERR_SHAPE;
  return launch<float>(dy, desc, w_packed, nullptr, nullptr, Cout_p, dilation, 0, static_cast<float*>(dx),
                       dx_layout, nullptr, nullptr, nullptr, 0, stream, out_mask, (int)cot_per_group);
}

size_t mvbev_conv3x3_packed_bytes_wino(int64_t Cout, int64_t K) {
  if (Cout <= 0 || K <= 0) return 0;
  return (size_t)(mvbev::round_up(K, mvbev::b3::KC) / mvbev::b3::KC) * (size_t)(Cout / mvbev::b3::BN) *
         mvbev::b3::wino::W16 * 16;
}

int mvbev_pack_conv3x3_weight_wino(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map, int64_t K,
                                   void* w_packed, void* stream) {
  using namespace mvbev;
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout <= 0 || Cin_w <= 0 || K <= 0) return MVBEV_ERR_RANK;
  if (Cout % b3::BN != 0) return MVBEV_ERR_SHAPE;
  if (!chan_map && K != Cin_w) return MVBEV_ERR_SHAPE;
  const int64_t total = (int64_t)mvbev_conv3x3_packed_bytes_wino(Cout, K) / 2 / (2 * b3::wino::NXI);  // threads
  const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(b3::pack_wino_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), w,
                     static_cast<__bf16*>(w_packed), (int)Cout, (int)Cin_w, chan_map, (int)K,
                     (int)round_up(K, b3::KC), false);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_pack_conv3x3_weight_wino_dgrad(const float* w, int64_t Cout_f, int64_t Cin_f, int64_t Cout, void* w_packed,
                                         void* stream) {
  using namespace mvbev;
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout_f <= 0 || Cin_f <= 0 || Cout <= 0) return MVBEV_ERR_RANK;
  if (Cout % b3::BN != 0 || Cout > Cin_f || Cout_f > INT32_MAX / 2 || Cin_f > INT32_MAX / 2) return MVBEV_ERR_SHAPE;
  const int64_t total = (int64_t)mvbev_conv3x3_packed_bytes_wino(Cout, Cout_f) / 2 / (2 * b3::wino::NXI);
  const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(b3::pack_wino_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), w,
                     static_cast<__bf16*>(w_packed), (int)Cout, (int)Cin_f, nullptr, (int)Cout_f,
                     (int)round_up(Cout_f, b3::KC), true);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

#if MVBEV_WINO_STAMPS
int mvbev_debug_wino_stamps(void* host, size_t bytes) {
  const size_t n = std::min(bytes, sizeof(mvbev::b3::g_wino_stamps));
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mvbev::b3::g_wino_stamps), n, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? MVBEV_OK : MVBEV_ERR_HIP;
}
#endif

size_t mvbev_wino_rows_bytes(const mvbev_conv_desc* d) {
  using namespace mvbev;
  if (!d || d->B <= 0 || d->K <= 0 || d->W <= 0 || d->out_rows <= 0) return 0;
  return (size_t)d->B * (size_t)(ceil_div(d->K, b3::SB)) * 5 * 4 * (size_t)ceil_div(d->out_rows, b3::RT) *
         (size_t)d->W * 32;
}

int mvbev_wino_rows_split_bf16(const void* x, const mvbev_conv_desc* desc, const uint32_t* group_mask, void* t,
                               size_t t_bytes, void* stream) {
  return mvbev::b3::wino_rows_launch(x, desc, 1, group_mask, t, t_bytes, stream);
}

int mvbev_wino_rows_split_bf16_dil(const void* x, const mvbev_conv_desc* desc, int dilation,
                                   const uint32_t* group_mask, void* t, size_t t_bytes, void* stream) {
  return mvbev::b3::wino_rows_launch(x, desc, dilation, group_mask, t, t_bytes, stream);
}

int mvbev_wino_rows_split_bf16_gated(const void* x, const mvbev_conv_desc* desc, int dilation,
                                     const uint32_t* group_mask, void* t, size_t t_bytes, const int32_t* gate,
                                     int32_t gate_tag, void* stream) {
  if (!gate) return MVBEV_ERR_NULL;
  return mvbev::b3::wino_rows_launch(x, desc, dilation, group_mask, t, t_bytes, stream, gate, gate_tag);
}

int mvbev_conv3x3_wino_bf16x3(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                              const float* init, int64_t Cout, int relu, void* y, int y_layout, int64_t y_band_rows,
                              const uint32_t* group_mask, const int32_t* tile_order, void* stream) {
  return mvbev::b3::wino_launch(t, desc, w_packed, bias, init, Cout, relu, static_cast<float*>(y), y_layout,
                                group_mask, tile_order, stream, 1, nullptr, nullptr, y_band_rows);
}

int mvbev_conv3x3_wino_bf16x3_dil(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                                  int64_t Cout, int dilation, int relu, void* y, int y_layout, void* stream) {
  return mvbev::b3::wino_launch(t, desc, w_packed, bias, nullptr, Cout, relu, static_cast<float*>(y), y_layout,
                                nullptr, nullptr, stream, dilation);
}

int mvbev_conv3x3_wino_bf16x3_dgrad(const void* t, const mvbev_conv_desc* desc, const void* w_packed, int64_t Cout,
                                    void* dx, int dx_layout, const uint32_t* out_mask, int64_t cot_per_group,
                                    void* stream) {
  if (out_mask && (cot_per_group <= 0 || cot_per_group > 65536)) return MVBEV_ERR_SHAPE;
  return mvbev::b3::wino_launch(t, desc, w_packed, nullptr, nullptr, Cout, 0, static_cast<float*>(dx), dx_layout,
                                nullptr, nullptr, stream, 1, nullptr, nullptr, 0, out_mask, cot_per_group);
}

int mvbev_conv3x3_wino_bf16x3_cout1_partials(const void* t, const mvbev_conv_desc* desc, const void* w_packed,
                                             const float* bias, int64_t Cout, int dilation, int relu, const float* w3,
                                             void* partials, size_t partials_bytes, void* stream) {
  if (!desc || !w3 || !partials) return MVBEV_ERR_NULL;
  const size_t need = mvbev_conv3x3_bf16x3_cout1_partials_bytes(desc, Cout);
  if (need == 0 || partials_bytes < need) return MVBEV_ERR_SHAPE;
  return mvbev::b3::wino_launch(t, desc, w_packed, bias, nullptr, Cout, relu, nullptr, MVBEV_LAYOUT_F32, nullptr,
                                nullptr, stream, dilation, w3, static_cast<float*>(partials));
}

}  // extern "C"

/* row-Winograd F(4,3) (xi-major; ABI 12400) */
extern "C" {

size_t mvbev_conv3x3_packed_bytes_wino43(int64_t Cout, int64_t K) {
  if (Cout <= 0 || K <= 0) return 0;
  return (size_t)(mvbev::round_up(K, mvbev::b3::KC) / mvbev::b3::KC) * (size_t)(Cout / mvbev::b3::BN) *
         mvbev::b3::w43::W16 * 16;
}

int mvbev_pack_conv3x3_weight_wino43(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map, int64_t K,
                                     void* w_packed, void* stream) {
  using namespace mvbev;
  if (!w || !w_packed) return MVBEV_ERR_NULL;
  if (Cout <= 0 || Cin_w <= 0 || K <= 0) return MVBEV_ERR_RANK;
  if (Cout % b3::BN != 0) return MVBEV_ERR_SHAPE;
  if (!chan_map && K != Cin_w) return MVBEV_ERR_SHAPE;
  const int64_t total = (int64_t)mvbev_conv3x3_packed_bytes_wino43(Cout, K) / 2 / (2 * b3::w43::NXI);  // threads
  const int blocks = (int)std::min<int64_t>(ceil_div(total, 256), 8192);
  hipLaunchKernelGGL(b3::pack_wino43_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), w,
                     static_cast<__bf16*>(w_packed), (int)Cout, (int)Cin_w, chan_map, (int)K,
                     (int)round_up(K, b3::KC));
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

size_t mvbev_wino43_rows_bytes(const mvbev_conv_desc* d) {
  using namespace mvbev;
  if (!d || d->B <= 0 || d->K <= 0 || d->W <= 0 || d->out_rows <= 0) return 0;
  return (size_t)d->B * (size_t)(ceil_div(d->K, b3::SB)) * b3::w43::NXI * 4 *
         (size_t)ceil_div(d->out_rows, b3::w43::RT4) * (size_t)d->W * 32;
}

int mvbev_wino43_rows_split_bf16(const void* x, const mvbev_conv_desc* desc, int dilation, const uint32_t* group_mask,
                                 void* t, size_t t_bytes, void* stream) {
  return mvbev::b3::wino43_rows_launch(x, desc, dilation, group_mask, t, t_bytes, stream);
}

int mvbev_conv3x3_wino43_bf16x3(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                                const float* init, int64_t Cout, int dilation, int relu, void* y, int y_layout,
                                const uint32_t* group_mask, const int32_t* tile_order, void* stream) {
  return mvbev::b3::wino43_launch(t, desc, w_packed, bias, init, Cout, dilation, relu, static_cast<float*>(y),
                                  y_layout, group_mask, tile_order, nullptr, nullptr, stream);
}

int mvbev_conv3x3_wino43_bf16x3_cout1_partials(const void* t, const mvbev_conv_desc* desc, const void* w_packed,
                                               const float* bias, int64_t Cout, int dilation, int relu,
                                               const float* w3, void* partials, size_t partials_bytes, void* stream) {
  if (!desc || !w3 || !partials) return MVBEV_ERR_NULL;
  const size_t need = mvbev_conv3x3_bf16x3_cout1_partials_bytes(desc, Cout);
  if (need == 0 || partials_bytes < need) return MVBEV_ERR_SHAPE;
  return mvbev::b3::wino43_launch(t, desc, w_packed, bias, nullptr, Cout, dilation, relu, nullptr, MVBEV_LAYOUT_F32,
                                  nullptr, nullptr, w3, static_cast<float*>(partials), stream);
}

}  // extern "C"
