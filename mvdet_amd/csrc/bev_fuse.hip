// One-call project + fuse (SURVEY §8(b) "mvbev_bev_fuse"): the whole inference hot path of
// PerspTransDetector.forward (persp_trans_detector.py:62-82, after the backbone) behind a plan,
// for callers that are not the Python engine (mvdet_amd/pipeline.py makes the same calls).
//
//   plan_init (host only)  ->  prepare (once per geometry and weight version: weight packs, coord
//   term, frustum mask, heavy-first tile order, the non-finite-geometry check; one stream sync)
//   ->  fuse (per frame, enqueued, no sync): warp (+ the fused 3x upsample) writing conv1's
//   row-Winograd transform straight into T, the Winograd conv1 (+ coord term, bias, ReLU), conv2
//   (row-Winograd too: y1's dilation-2 transform, then the conv) with conv3's per-tap partials in its
//   epilogue, their reduce -> map [B][1][Ho][Wo].
//
// Geometry that can produce a non-finite warp sample runs the direct conv1 on the split slab
// instead (the reference's NaN pattern; see mvbev_warp_nonfinite_views).  Non-finite FEATURES
// (plan.guard, the row-Winograd path): the fused warp reports a NaN / inf it samples into a device
// flag, and the guard's exact path — the reference-order warp (+ upsample) into an fp32 slab, the
// fp32-MFMA conv1 / conv2 and the single-output conv3, each a no-op unless the flag is set — then
// rewrites the map, so a NaN / inf reaches exactly the outputs it reaches in the reference (no host
// sync: the decision is taken on the device).  Everything here is a sequence of the library's own C
// entry points over one caller-owned workspace.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "common.h"

namespace {

constexpr int64_t kMid = 512;  // map_classifier's hidden width (persp_trans_detector.py:51-53)
constexpr int64_t kKC = MVBEV_CONV_KC;
constexpr int64_t kTileW = MVBEV_CONV_TILE_W;
constexpr size_t kAlign = 256;

enum Region { R_MAP1, R_PACK1, R_PACK2, R_INIT, R_MASK, R_ORDER, R_NF, R_BIG, R_Y1, R_T2,
              R_GFLAG, R_GPACK1, R_GPACK2, R_GSLAB, R_P3, R_COUNT };
static_assert(R_COUNT <= 24, "mvbev_bev_plan.off");

size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

template <typename T> T* at(void* ws, const mvbev_bev_plan* p, int r) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + p->off[r]);
}

mvbev_conv_desc conv1_desc(const mvbev_bev_plan* p) {
  const mvbev_bev_geometry& g = p->g;
  mvbev_conv_desc d;
  d.B = g.B; d.K = g.num_views * p->Cs; d.H = g.Ho; d.W = g.Wo;
  d.group = p->Cs; d.group_stride = g.B * p->Cs * g.Ho * g.Wo; d.batch_stride = p->Cs * g.Ho * g.Wo;
  d.in_row0 = 0; d.in_rows = g.Ho; d.out_row0 = 0; d.out_rows = g.Ho;
  return d;
}

mvbev_conv_desc conv2_desc(const mvbev_bev_plan* p) {
  const mvbev_bev_geometry& g = p->g;
  mvbev_conv_desc d;
  d.B = g.B; d.K = kMid; d.H = g.Ho; d.W = g.Wo;
  d.group = kMid; d.group_stride = 0; d.batch_stride = kMid * g.Ho * g.Wo;
  d.in_row0 = 0; d.in_rows = g.Ho; d.out_row0 = 0; d.out_rows = g.Ho;
  return d;
}

int kind_of(const mvbev_bev_geometry& g) { return g.src_kind & ~(MVBEV_BEV_SRC_CHANNELS_LAST | MVBEV_BEV_NO_GUARD); }

// the guard's exact path runs in output-row chunks whose fp32 slab window (rows + 14) holds at most this
// many bytes (ABI 11900; a whole-grid fp32 slab would double the plan's largest region for a rare path)
// (MVBEV_BEV_GUARD_BYTES in the environment overrides it at plan_init: tests exercise several chunks)
constexpr size_t kGuardBytes = size_t(1) << 30;
int64_t guard_chunk_rows(const mvbev_bev_geometry& g, int64_t Cs, size_t budget) {
  const size_t per_row = (size_t)g.num_views * g.B * Cs * g.Wo * 4;
  const int64_t n = (int64_t)(budget / per_row) - 14;
  return std::min<int64_t>(g.Ho, std::max<int64_t>(12, n));
}

// a view's source strides: NCHW, or channels-last (MVBEV_BEV_SRC_CHANNELS_LAST) of the same [B][C][sh][sw]
void src_strides(const mvbev_bev_geometry& g, int64_t sh, int64_t sw, int64_t (&st)[4]) {
  if (g.src_kind & MVBEV_BEV_SRC_CHANNELS_LAST) {
    st[0] = g.C * sh * sw; st[1] = 1; st[2] = sw * g.C; st[3] = g.C;
  } else {
    st[0] = g.C * sh * sw; st[1] = sh * sw; st[2] = sw; st[3] = 1;
  }
}

// the views of one frame as mvbev_warp_view entries writing slot s of the split slab (32-B units)
void slab_views(const mvbev_bev_plan* p, const void* const* views, void* slab, mvbev_warp_view* out) {
  const mvbev_bev_geometry& g = p->g;
  const bool backbone = kind_of(g) == MVBEV_BEV_SRC_BACKBONE_F32;
  const int64_t sh = backbone ? g.h : g.H, sw = backbone ? g.w : g.W;
  const int64_t G = p->Cs / kKC;
  for (int s = 0; s < g.num_views; ++s) {
    mvbev_warp_view& v = out[s];
    v.src = views[s];
    src_strides(g, sh, sw, v.src_strides);
    v.dst = static_cast<char*>(slab) + (size_t)s * g.B * G * g.Ho * g.Wo * 32;
    v.dst_strides[0] = G * g.Ho * g.Wo; v.dst_strides[1] = g.Ho * g.Wo; v.dst_strides[2] = g.Wo;
    v.dst_strides[3] = 1;
    std::memcpy(v.m, g.m[s], sizeof(v.m));
  }
}

// row tiles of the whole grid's row-Winograd transform: 4 ceil(Ho / 12) three-row tiles (F(3,3)), or
// 4 ceil(Ho / 16) four-row tiles (F(4,3), plan wino 2)
int64_t t_tile_rows(const mvbev_bev_plan* p) {
  return p->wino == 2 ? 4 * ((p->g.Ho + 15) / 16) : 4 * ((p->g.Ho + 11) / 12);
}

// The F(4,3) policy of ProjectFuse.wino43_pays (pipeline.py): 16-row tiles wasting at most 3 % of the grid's
// rows (conv1, frustum-masked: workgroups of uneven cost dealt heaviest first) and, for conv2 -> conv3
// (workgroups of equal cost), a launch at least 8 rounds of workgroups deep
bool w43_rows_ok(int64_t Ho) { return (double)(((Ho + 15) / 16) * 16 - Ho) <= 0.03 * (double)Ho; }
bool w43_deep(const mvbev_bev_geometry& g) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return ((g.Ho + 15) / 16) * ((g.Wo + kTileW - 1) / kTileW) * g.B * (kMid / 128) >= 8 * (int64_t)cus;
}

// the same writing slot s's channels of T (the Winograd transform of the whole grid; T43 with plan wino 2)
void t_views(const mvbev_bev_plan* p, const void* const* views, void* t, mvbev_warp_view* out) {
  const mvbev_bev_geometry& g = p->g;
  const bool backbone = kind_of(g) == MVBEV_BEV_SRC_BACKBONE_F32;
  const int64_t sh = backbone ? g.h : g.H, sw = backbone ? g.w : g.W;
  const int64_t nx = p->wino == 2 ? 6 : 5, r3 = t_tile_rows(p), K8 = g.num_views * p->Cs / kKC;
  for (int s = 0; s < g.num_views; ++s) {
    mvbev_warp_view& v = out[s];
    v.src = views[s];
    src_strides(g, sh, sw, v.src_strides);
    v.dst = static_cast<char*>(t) + (size_t)32 * (s * (p->Cs / kKC)) * nx * r3 * g.Wo;
    v.dst_strides[0] = K8 * nx * r3 * g.Wo; v.dst_strides[1] = nx * r3 * g.Wo; v.dst_strides[2] = g.Wo;
    v.dst_strides[3] = 1;
    std::memcpy(v.m, g.m[s], sizeof(v.m));
  }
}

#define BEV_TRY(x)                 \
  do {                             \
    const int st_ = (x);           \
    if (st_ != MVBEV_OK) return st_; \
  } while (0)
// the same while host buffers are still the source / target of enqueued copies: drain the stream
// before returning, so no copy outlives the host memory it reads or writes
#define BEV_TRY_SYNC(x, s)                    \
  do {                                        \
    const int st_ = (x);                      \
    if (st_ != MVBEV_OK) {                    \
      (void)hipStreamSynchronize(s);          \
      return st_;                             \
    }                                         \
  } while (0)

}  // namespace

extern "C" {

int mvbev_bev_plan_init(const mvbev_bev_geometry* g, mvbev_bev_plan* p) {
  if (!g || !p) return MVBEV_ERR_NULL;
  if (g->num_views <= 0 || g->B <= 0 || g->C <= 0 || g->H <= 0 || g->W <= 0 || g->Ho <= 0 || g->Wo <= 0)
    return MVBEV_ERR_RANK;
  if (g->num_views > MVBEV_BEV_MAX_VIEWS) return MVBEV_ERR_SHAPE;
  const int kind = kind_of(*g);
  if (kind != MVBEV_BEV_SRC_F32 && kind != MVBEV_BEV_SRC_F16 && kind != MVBEV_BEV_SRC_BACKBONE_F32)
    return MVBEV_ERR_SHAPE;
  if ((g->src_kind & MVBEV_BEV_SRC_CHANNELS_LAST) && (kind == MVBEV_BEV_SRC_F16 || g->C % 32 != 0))
    return MVBEV_ERR_SHAPE;  // channels-last: fp32 sources in whole 32-channel groups
  if (kind == MVBEV_BEV_SRC_BACKBONE_F32 && (g->h <= 0 || g->w <= 0 || g->h > g->H || g->w > g->W))
    return MVBEV_ERR_SHAPE;
  std::memset(p, 0, sizeof(*p));
  p->g = *g;
  p->Cs = (g->C + kKC - 1) / kKC * kKC;
  const int64_t K = g->num_views * p->Cs;
  p->frustum = p->Cs % 16 == 0 ? 1 : 0;  // the conv's group mask needs 16-channel chunks
  // the row-Winograd conv1 reads T, which the warp writes directly from fp32 sources (the fused
  // warp + transform kernels); fp16 sources take the direct conv1 on the split slab, as the
  // engine's fp16-storage path does; prepare also falls back for non-finite geometry
  p->wino = (kind != MVBEV_BEV_SRC_F16 && g->W >= 2 && (kind != MVBEV_BEV_SRC_BACKBONE_F32 || g->w >= 4)) ? 1 : 0;
  // (ABI 12400) F(4,3) where it pays: conv1 (wino 2) and conv2 -> conv3 (wino2 2, decided in prepare)
  if (p->wino && w43_rows_ok(g->Ho)) p->wino = 2;
  const int64_t tiles_y = p->wino == 2 ? (g->Ho + 15) / 16 : (g->Ho + 11) / 12, tiles_x = (g->Wo + kTileW - 1) / kTileW;
  p->tiles = tiles_y * tiles_x;
  mvbev_conv_desc d1 = conv1_desc(p), d2 = conv2_desc(p);
  const size_t t_bytes = std::max(mvbev_wino_rows_bytes(&d1), mvbev_wino43_rows_bytes(&d1));
  const size_t slab_bytes = (size_t)g->num_views * g->B * p->Cs * g->Ho * g->Wo * 4;
  size_t sz[R_COUNT] = {};
  sz[R_MAP1] = (size_t)K * 4;
  sz[R_PACK1] = std::max({mvbev_conv3x3_packed_bytes_wino(kMid, K), mvbev_conv3x3_packed_bytes_wino43(kMid, K),
                          mvbev_conv3x3_packed_bytes_bf16x3(kMid, K)});
  sz[R_PACK2] = std::max({mvbev_conv3x3_packed_bytes_wino(kMid, kMid), mvbev_conv3x3_packed_bytes_wino43(kMid, kMid),
                          mvbev_conv3x3_packed_bytes_bf16x3(kMid, kMid)});
  sz[R_INIT] = (size_t)kMid * g->Ho * g->Wo * 4;
  // (sized for the 12 x 32 tiles: prepare falls back to them from F(4,3)'s 16 x 32 for non-finite geometry)
  const int64_t tiles12 = ((g->Ho + 11) / 12) * tiles_x;
  sz[R_MASK] = (size_t)tiles12 * 4;
  sz[R_ORDER] = (size_t)g->B * tiles12 * 4;
  sz[R_NF] = 4;
  sz[R_BIG] = std::max(t_bytes, slab_bytes);  // T (Winograd) or the split slab (direct conv1)
  sz[R_Y1] = (size_t)g->B * kMid * g->Ho * g->Wo * 4;
  sz[R_T2] = std::max({mvbev_wino_rows_bytes(&d2), mvbev_wino43_rows_bytes(&d2),  // conv2's row transform of y1
                       (size_t)g->B * kMid * g->Ho * g->Wo * 4});                     // (the guard: its y2)
  // the non-finite guard (row-Winograd plans): flag, fp32 packs of conv1 / conv2, the fp32 slab; its y1
  // reuses R_Y1 and its y2 R_T2 (both free once the fast path's conv2 has run)
  p->guard = p->wino && !(g->src_kind & MVBEV_BEV_NO_GUARD);
  sz[R_GFLAG] = 4;
  sz[R_GPACK1] = p->guard ? 4 * mvbev_conv3x3_packed_floats(kMid, K) : 0;
  sz[R_GPACK2] = p->guard ? 4 * mvbev_conv3x3_packed_floats(kMid, kMid) : 0;
  // one row chunk's fp32 slab window (bounded: kGuardBytes); its y1 / y2 fit R_Y1 / R_T2
  size_t budget = kGuardBytes;
  if (const char* e = std::getenv("MVBEV_BEV_GUARD_BYTES")) budget = (size_t)std::strtoull(e, nullptr, 10);
  const int64_t gr = guard_chunk_rows(*g, p->Cs, budget);
  sz[R_GSLAB] = p->guard ? std::min(slab_bytes, (size_t)g->num_views * g->B * p->Cs * std::min<int64_t>(g->Ho, gr + 14) *
                                                    g->Wo * 4) : 0;
  sz[R_P3] = mvbev_conv3x3_bf16x3_cout1_partials_bytes(&d2, kMid);
  size_t o = 0;
  for (int r = 0; r < R_COUNT; ++r) {
    p->off[r] = o;
    o = align_up(o + sz[r]);
  }
  p->workspace_bytes = o;
  return MVBEV_OK;
}

size_t mvbev_bev_fuse_workspace_bytes(const mvbev_bev_geometry* g) {
  mvbev_bev_plan p;
  return mvbev_bev_plan_init(g, &p) == MVBEV_OK ? p.workspace_bytes : 0;
}

int mvbev_bev_fuse_prepare(mvbev_bev_plan* p, const float* w1, const float* b1, const float* w2, const float* b2,
                           const float* w3, void* ws, size_t ws_bytes, void* stream) {
  if (!p || !w1 || !w2 || !w3 || !ws) return MVBEV_ERR_NULL;
  if (p->workspace_bytes == 0 || ws_bytes < p->workspace_bytes) return MVBEV_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(ws) % kAlign) return MVBEV_ERR_ALIGN;
  const mvbev_bev_geometry& g = p->g;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t K = g.num_views * p->Cs, nc = g.num_views * g.C, cin = nc + 2;
  // conv1's channel map: slot s channel c -> module channel s*C + c (view-major concat, :77)
  std::vector<int32_t> map1((size_t)K);
  for (int64_t k = 0; k < K; ++k) {
    const int64_t sl = k / p->Cs, c = k % p->Cs;
    map1[(size_t)k] = c < g.C ? (int32_t)(sl * g.C + c) : -1;
  }
  if (hipMemcpyAsync(at<int32_t>(ws, p, R_MAP1), map1.data(), map1.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess) {
    (void)hipStreamSynchronize(s);
    return MVBEV_ERR_HIP;
  }
  // geometry: non-finite samples (-> direct conv1), the frustum mask of the 12 x 32 conv tiles
  std::vector<mvbev_warp_view> mv((size_t)g.num_views);
  std::memset(mv.data(), 0, mv.size() * sizeof(mvbev_warp_view));
  for (int v = 0; v < g.num_views; ++v) std::memcpy(mv[(size_t)v].m, g.m[v], sizeof(mv[0].m));
  BEV_TRY_SYNC(mvbev_warp_nonfinite_views(mv.data(), g.num_views, g.H, g.W, g.Ho, g.Wo, at<uint32_t>(ws, p, R_NF),
                                          stream), s);
  if (p->frustum)  // (over F(4,3)'s 16 x 32 tiles with plan wino 2: the transform's and the conv's)
    BEV_TRY_SYNC(mvbev_warp_tile_mask(mv.data(), g.num_views, g.H, g.W, g.Ho, g.Wo, 0, g.Ho, p->wino == 2 ? 16 : 12,
                                      kTileW, 1, at<uint32_t>(ws, p, R_MASK), stream), s);
  uint32_t nf = 0;
  std::vector<uint32_t> mask((size_t)p->tiles, 0);
  if (hipMemcpyAsync(&nf, at<uint32_t>(ws, p, R_NF), 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      (p->frustum && hipMemcpyAsync(mask.data(), at<uint32_t>(ws, p, R_MASK), mask.size() * 4, hipMemcpyDeviceToHost,
                                    s) != hipSuccess)) {
    (void)hipStreamSynchronize(s);
    return MVBEV_ERR_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess) return MVBEV_ERR_HIP;
  if (nf != 0 && p->wino == 2) {  // non-finite geometry: the direct conv1 on 12-row tiles (the mask is rebuilt)
    p->tiles = ((g.Ho + 11) / 12) * ((g.Wo + kTileW - 1) / kTileW);
    mask.assign((size_t)p->tiles, 0);
    if (p->frustum) {
      BEV_TRY_SYNC(mvbev_warp_tile_mask(mv.data(), g.num_views, g.H, g.W, g.Ho, g.Wo, 0, g.Ho, 12, kTileW, 1,
                                        at<uint32_t>(ws, p, R_MASK), stream), s);
      if (hipMemcpyAsync(mask.data(), at<uint32_t>(ws, p, R_MASK), mask.size() * 4, hipMemcpyDeviceToHost, s) !=
              hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return MVBEV_ERR_HIP;
    }
  }
  p->wino = nf == 0 ? p->wino : 0;
  // conv2's Winograd form (y1 finite), as the engine's wino_conv2_active; F(4,3) as its conv2_form
  p->wino2 = nf == 0 ? (w43_rows_ok(g.Ho) && w43_deep(g) ? 2 : 1) : 0;
  if (p->frustum) {
    // heavy-first run order: most active views first, equal view sets adjacent (ops.heavy_first_order)
    const int64_t T = p->tiles, n = g.B * T;
    std::vector<int32_t> order((size_t)n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      const uint32_t ma = mask[(size_t)(a % T)], mb = mask[(size_t)(b % T)];
      const int pa = __builtin_popcount(ma), pb = __builtin_popcount(mb);
      if (pa != pb) return pa > pb;
      if (ma != mb) return ma < mb;
      return a < b;
    });
    const bool ok = hipMemcpyAsync(at<int32_t>(ws, p, R_ORDER), order.data(), order.size() * 4, hipMemcpyHostToDevice,
                                   s) == hipSuccess;
    if (hipStreamSynchronize(s) != hipSuccess || !ok) return MVBEV_ERR_HIP;  // the host order buffer's lifetime
  }
  // weights: conv1 (G w for the Winograd form, or the direct pack), conv2, and the coord term
  if (p->wino == 2)
    BEV_TRY(mvbev_pack_conv3x3_weight_wino43(w1, kMid, cin, at<int32_t>(ws, p, R_MAP1), K, at<void>(ws, p, R_PACK1),
                                             stream));
  else if (p->wino)
    BEV_TRY(mvbev_pack_conv3x3_weight_wino(w1, kMid, cin, at<int32_t>(ws, p, R_MAP1), K, at<void>(ws, p, R_PACK1),
                                           stream));
  else
    BEV_TRY(mvbev_pack_conv3x3_weight_bf16x3(w1, kMid, cin, at<int32_t>(ws, p, R_MAP1), K, at<void>(ws, p, R_PACK1),
                                             stream));
  if (p->wino2 == 2)
    BEV_TRY(mvbev_pack_conv3x3_weight_wino43(w2, kMid, kMid, nullptr, kMid, at<void>(ws, p, R_PACK2), stream));
  else if (p->wino2)
    BEV_TRY(mvbev_pack_conv3x3_weight_wino(w2, kMid, kMid, nullptr, kMid, at<void>(ws, p, R_PACK2), stream));
  else
    BEV_TRY(mvbev_pack_conv3x3_weight_bf16x3(w2, kMid, kMid, nullptr, kMid, at<void>(ws, p, R_PACK2), stream));
  p->guard = p->guard && p->wino;  // non-finite geometry already runs the direct convs
  if (p->guard) {  // the exact path's fp32 packs; its slab's padding channels stay zero
    BEV_TRY(mvbev_pack_conv3x3_weight_f32(w1, kMid, cin, at<int32_t>(ws, p, R_MAP1), K, at<float>(ws, p, R_GPACK1),
                                          stream));
    BEV_TRY(mvbev_pack_conv3x3_weight_f32(w2, kMid, kMid, nullptr, kMid, at<float>(ws, p, R_GPACK2), stream));
    if (hipMemsetAsync(at<void>(ws, p, R_GSLAB), 0, p->off[R_GSLAB + 1] - p->off[R_GSLAB], s) != hipSuccess)
      return MVBEV_ERR_HIP;
  }
  // coord term = conv1 bias + conv1 over the two coord channels (:21, :77): input-independent (ABI 12300)
  BEV_TRY(mvbev_coord_term_f32(w1, cin, nc, b1, kMid, g.Ho, g.Wo, at<float>(ws, p, R_INIT), stream));
  // T / the slab: zero once; later warps skip the pixels whose samples fall outside the source
  if (hipMemsetAsync(at<void>(ws, p, R_BIG), 0, p->off[R_BIG + 1] - p->off[R_BIG], s) != hipSuccess)
    return MVBEV_ERR_HIP;
  p->b2 = b2;
  p->w3 = w3;
  p->prepared = 1;
  return MVBEV_OK;
}

int mvbev_bev_fuse(const mvbev_bev_plan* p, const void* const* views, float* map, void* ws, size_t ws_bytes,
                   void* stream) {
  if (!p || !views || !map || !ws) return MVBEV_ERR_NULL;
  if (!p->prepared || ws_bytes < p->workspace_bytes) return MVBEV_ERR_SHAPE;
  const mvbev_bev_geometry& g = p->g;
  for (int v = 0; v < g.num_views; ++v)
    if (!views[v]) return MVBEV_ERR_NULL;
  mvbev_warp_view wv[MVBEV_BEV_MAX_VIEWS];
  std::memset(wv, 0, sizeof(wv));
  const mvbev_conv_desc d1 = conv1_desc(p), d2 = conv2_desc(p);
  void* big = at<void>(ws, p, R_BIG);
  const uint32_t* mask = p->frustum ? at<uint32_t>(ws, p, R_MASK) : nullptr;
  const int32_t* order = p->frustum ? at<int32_t>(ws, p, R_ORDER) : nullptr;
  const bool backbone = kind_of(g) == MVBEV_BEV_SRC_BACKBONE_F32;
  void* y1 = at<void>(ws, p, R_Y1);
  int32_t* gflag = p->guard ? at<int32_t>(ws, p, R_GFLAG) : nullptr;
  if (gflag && hipMemsetAsync(gflag, 0, 4, static_cast<hipStream_t>(stream)) != hipSuccess) return MVBEV_ERR_HIP;
  // a4 + a5 + a6 (+ conv1's B^T): the warp of every view in one launch
  if (p->wino) {
    t_views(p, views, big, wv);
    const int64_t r3 = t_tile_rows(p);
    const int wf = MVBEV_WARP_DST_ZEROED | (p->wino == 2 ? MVBEV_WARP_WINO43 : 0);
    if (backbone)
      BEV_TRY(mvbev_warp_views_upsampled_wino_rows(wv, g.num_views, g.B, g.C, g.h, g.w, g.H, g.W, g.Ho, g.Wo, r3, wf,
                                                   gflag, 1, stream));
    else
      BEV_TRY(mvbev_warp_views_wino_rows(wv, g.num_views, g.B, g.C, g.H, g.W, g.Ho, g.Wo, r3, wf, gflag, 1, stream));
  } else {
    slab_views(p, views, big, wv);
    if (backbone)
      BEV_TRY(mvbev_warp_views_upsampled_ex(wv, g.num_views, 0, g.B, g.C, g.h, g.w, g.H, g.W, g.Ho, g.Wo,
                                            MVBEV_LAYOUT_SPLIT_BF16, MVBEV_WARP_DST_ZEROED, stream));
    else
      BEV_TRY(mvbev_warp_views_split_bf16_ex(wv, g.num_views, kind_of(g) == MVBEV_BEV_SRC_F16 ? 1 : 0, g.B, g.C, g.H,
                                             g.W, g.Ho, g.Wo, MVBEV_WARP_DST_ZEROED, stream));
  }
  // a7: conv1 + coord term + bias + ReLU -> y1 (split-bf16, conv2's input)
  if (p->wino == 2)
    BEV_TRY(mvbev_conv3x3_wino43_bf16x3(big, &d1, at<void>(ws, p, R_PACK1), nullptr, at<float>(ws, p, R_INIT), kMid, 1,
                                        1, y1, MVBEV_LAYOUT_SPLIT_BF16, mask, order, stream));
  else if (p->wino)
    BEV_TRY(mvbev_conv3x3_wino_bf16x3(big, &d1, at<void>(ws, p, R_PACK1), nullptr, at<float>(ws, p, R_INIT), kMid, 1,
                                      y1, MVBEV_LAYOUT_SPLIT_BF16, 0, mask, order, stream));
  else
    BEV_TRY(mvbev_conv3x3_bf16x3_ex(big, MVBEV_LAYOUT_SPLIT_BF16, &d1, at<void>(ws, p, R_PACK1), nullptr,
                                    at<float>(ws, p, R_INIT), kMid, 1, 1, y1, MVBEV_LAYOUT_SPLIT_BF16, mask, order,
                                    nullptr, 0, stream));
  // a8 + a9: conv2 + ReLU with conv3's per-tap partials in its epilogue, then their reduce
  void* p3 = at<void>(ws, p, R_P3);
  static_assert(R_P3 == R_COUNT - 1, "the partials are the workspace's last region");
  if (p->wino2 == 2) {  // F(4,3) (ABI 12400)
    void* t2 = at<void>(ws, p, R_T2);
    BEV_TRY(mvbev_wino43_rows_split_bf16(y1, &d2, 2, nullptr, t2, p->off[R_T2 + 1] - p->off[R_T2], stream));
    BEV_TRY(mvbev_conv3x3_wino43_bf16x3_cout1_partials(t2, &d2, at<void>(ws, p, R_PACK2), p->b2, kMid, 2, 1, p->w3, p3,
                                                       p->workspace_bytes - p->off[R_P3], stream));
  } else if (p->wino2) {  // the dilation-2 row transform of y1, then the Winograd conv with the partials epilogue
    void* t2 = at<void>(ws, p, R_T2);
    BEV_TRY(mvbev_wino_rows_split_bf16_dil(y1, &d2, 2, nullptr, t2, p->off[R_T2 + 1] - p->off[R_T2], stream));
    BEV_TRY(mvbev_conv3x3_wino_bf16x3_cout1_partials(t2, &d2, at<void>(ws, p, R_PACK2), p->b2, kMid, 2, 1, p->w3, p3,
                                                     p->workspace_bytes - p->off[R_P3], stream));
  } else {
    BEV_TRY(mvbev_conv3x3_bf16x3_cout1_partials(y1, &d2, at<void>(ws, p, R_PACK2), p->b2, kMid, 2, 1, p->w3, p3,
                                                p->workspace_bytes - p->off[R_P3], stream));
  }
  BEV_TRY(mvbev_cout1_reduce_partials(p3, &d2, kMid, 4, map, 0, g.Ho, stream));
  if (gflag) {  // the non-finite guard: each launch exits at once unless the warp set the flag
    // in output-row chunks: chunk [a, b) needs y2 rows [a - 4, b + 4), y1 rows [a - 6, b + 6) and the slab's
    // rows [a - 7, b + 7) (the dilation-1/2/4 chain, clipped to the grid)
    float* gslab = at<float>(ws, p, R_GSLAB);
    float* gy1 = at<float>(ws, p, R_Y1);
    float* gy2 = at<float>(ws, p, R_T2);
    // the chunk rows the plan sized R_GSLAB for (R rows per window: gr + 14, or the whole grid)
    const int64_t Rw = (int64_t)((p->off[R_GSLAB + 1] - p->off[R_GSLAB]) / ((size_t)g.num_views * g.B * p->Cs * g.Wo * 4));
    const int64_t gr = Rw >= g.Ho ? g.Ho : Rw - 14, sh = backbone ? g.h : g.H, sw = backbone ? g.w : g.W;
    for (int64_t a = 0; a < g.Ho; a += gr) {
      const int64_t b = std::min(g.Ho, a + gr);
      const int64_t a2 = std::max<int64_t>(0, a - 4), b2 = std::min(g.Ho, b + 4);
      const int64_t a1 = std::max<int64_t>(0, a2 - 2), b1 = std::min(g.Ho, b2 + 2);
      // every chunk's window has the same R rows (shifted inside the grid at the bottom), so the slab's
      // padding channels (Cs > C: zero weights) stay the zeros prepare wrote — a stale value there could be
      // an inf from another chunk's real channels, and 0 * inf is NaN
      const int64_t R = std::min(g.Ho, Rw);
      const int64_t s0 = std::min(std::max<int64_t>(0, a1 - 1), g.Ho - R);
      const int64_t plane = R * g.Wo;
      int32_t row0s[MVBEV_BEV_MAX_VIEWS];
      for (int s = 0; s < g.num_views; ++s) {
        mvbev_warp_view& v = wv[s];
        v.src = views[s];
        src_strides(g, sh, sw, v.src_strides);
        v.dst = gslab + (size_t)s * g.B * p->Cs * plane;
        v.dst_strides[0] = p->Cs * plane; v.dst_strides[1] = plane; v.dst_strides[2] = g.Wo; v.dst_strides[3] = 1;
        std::memcpy(v.m, g.m[s], sizeof(v.m));
        row0s[s] = (int32_t)s0;
      }
      BEV_TRY(mvbev_warp_views_exact_rows(wv, row0s, g.num_views, 0, g.B, g.C, sh, sw, g.H, g.W, g.Ho, g.Wo, R, gflag,
                                          1, stream));
      mvbev_conv_desc e1 = d1, e2 = d2;
      e1.group_stride = g.B * p->Cs * plane; e1.batch_stride = p->Cs * plane;
      e1.in_row0 = s0; e1.in_rows = R; e1.out_row0 = a1; e1.out_rows = b1 - a1;
      e2.batch_stride = kMid * (b1 - a1) * g.Wo; e2.in_row0 = a1; e2.in_rows = b1 - a1; e2.out_row0 = a2;
      e2.out_rows = b2 - a2;
      BEV_TRY(mvbev_conv3x3_f32(gslab, &e1, at<float>(ws, p, R_GPACK1), nullptr, at<float>(ws, p, R_INIT), kMid, 1, 1,
                                gy1, gflag, 1, stream));
      BEV_TRY(mvbev_conv3x3_f32(gy1, &e2, at<float>(ws, p, R_GPACK2), p->b2, nullptr, kMid, 2, 1, gy2, gflag, 1,
                                stream));
      for (int64_t bi = 0; bi < g.B; ++bi)  // (a row chunk of a B > 1 map is not one contiguous block)
        BEV_TRY(mvbev_conv3x3_cout1_f32(gy2 + bi * kMid * (b2 - a2) * g.Wo, 1, kMid, g.Ho, g.Wo, a2, b2 - a2, a, b - a,
                                        p->w3, 4, map + (bi * g.Ho + a) * g.Wo, gflag, 1, stream));
    }
  }
  return MVBEV_OK;
}

}  // extern "C"
