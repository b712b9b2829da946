/*
 * mvbev.h — C ABI of the MI355X-native MVDet project+fuse hot path.
 *
 * libmvbev.so (built from the HIP sources in mvdet_amd/csrc for gfx950) exports exactly the
 * functions below.  Plain pointers and sizes only: every tensor argument is a
 * caller-owned DEVICE pointer (PyTorch caching allocator, hipMalloc, ...), every
 * call is enqueued on the caller's HIP stream (passed as `void*`, NULL = the
 * null stream), no call allocates, copies to the host or synchronises, and all
 * calls are reentrant (no global mutable state).
 *
 * Return value: 0 (MVBEV_OK) on success, a negative MVBEV_ERR_* code for a bad
 * argument (nothing is launched), or MVBEV_ERR_HIP when the launch itself
 * failed.  mvbev_status_string() turns a code into text.
 *
 * Reference interfaces replaced (ErikBrorsson/MVDet @ 2024-08-07):
 *   mvbev_warp_perspective_f32 / _f16
 *       kornia.geometry.transform.warp_perspective(img_feature, proj_mat,
 *       reducedgrid_shape)   multiview_detector/models/persp_trans_detector.py:69
 *       (kornia 0.6.11: normalize -> inverse -> meshgrid -> transform_points ->
 *       F.grid_sample(bilinear, zeros, align_corners=True)).  The caller passes
 *       the kornia src_norm<-dst_norm 3x3 (host-computed, same recipe) so the
 *       device does transform + divide + bilinear gather.  dst strides let every
 *       view write straight into its channel slice of the fused ground-plane
 *       tensor: the torch.cat at persp_trans_detector.py:77 becomes zero-copy.
 *   mvbev_fill_coord_map_f32
 *       self.coord_map.repeat([B,1,1,1]) concatenated as the last two channels
 *       (persp_trans_detector.py:21,77,103-112).
 *   mvbev_pack_conv3x3_weight_f32, mvbev_conv3x3_f32
 *       nn.Conv2d(Cin->Cout, 3, padding=d, dilation=d) (+ nn.ReLU) of
 *       map_classifier[0:4]   persp_trans_detector.py:51-53, :81; the conv1 contribution of
 *       the two constant coord channels plus its bias is input-independent and enters as
 *       the `init` term (once per weight version: mvbev_coord_term_f32, ABI 12300).
 *   mvbev_pack_conv3x3_weight_bf16x3, mvbev_conv3x3_bf16x3
 *       the same convs in 3xbf16 split precision on the bf16 MFMA (5.3x the fp32 rate)
 *   mvbev_conv3x3_cout1_f32
 *       nn.Conv2d(512->1, 3, padding=4, dilation=4, bias=False) of
 *       map_classifier[4]      persp_trans_detector.py:54, :81
 *   (the same-size F.interpolate at persp_trans_detector.py:82 is an exact
 *    identity and has no entry point.)
 */
#ifndef MVBEV_H_
#define MVBEV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVBEV_OK 0
#define MVBEV_ERR_RANK (-1)      /* a size is <= 0 / a rank assumption is violated */
#define MVBEV_ERR_SHAPE (-2)     /* inconsistent sizes (e.g. Cout not a multiple of 128) */
#define MVBEV_ERR_STRIDE (-3)    /* unsupported stride (innermost stride must be 1 where stated) */
#define MVBEV_ERR_ALIGN (-4)     /* pointer misaligned for the vector width used */
#define MVBEV_ERR_NULL (-5)      /* a required pointer is NULL */
#define MVBEV_ERR_DILATION (-6)  /* dilation not supported by this entry point */
#define MVBEV_ERR_HIP (-100)     /* the HIP launch failed (hipGetLastError) */

/* Input-channel granule of the conv kernels: packed K and every channel group must be
 * a multiple of this. */
#define MVBEV_CONV_KC 8
/* Output-channel granule of mvbev_conv3x3_f32. */
#define MVBEV_CONV_BN 128

const char* mvbev_status_string(int status);
/* Library / ABI version, e.g. 10000 for 1.0.0. */
int mvbev_version(void);  /* 12400: row-Winograd F(4,3) (mvbev_pack_conv3x3_weight_wino43, mvbev_wino43_rows_split_bf16, mvbev_conv3x3_wino43_bf16x3, mvbev_conv3x3_wino43_bf16x3_cout1_partials); 12300: mvbev_coord_term_f32 (conv1's coord term as one VALU pass); 12200: the training forward's non-finite guard (mvbev_store_gated_f32, mvbev_pack_conv3x3_weight_f32_gated, mvbev_wino_rows_split_bf16_gated), per-geometry staging boxes of the fused warps (mvbev_warp_wino_boxes, mvbev_warp_views_wino_rows_ex, mvbev_warp_upsampled_wino_boxes, mvbev_warp_views_upsampled_wino_rows_ex); 12100: MVBEV_LAYOUT_SPLIT_BF16_PIX (conv data gradients' output, the warp adjoint's input); 12000: conv1's and conv2's weight gradients from the forward's row-Winograd transforms (mvbev_wino_dy_rows_f32, mvbev_conv3x3_wgrad_wino_bf16x3); 11900: row windows (mvbev_warp_views_split_bf16_rows with the non-finite report, mvbev_warp_views_exact_rows with fp16 sources), mvbev_conv3x3_f32_ex (row-band output), mvbev_bias_relu_nonfinite_f32, mvbev_zero_gated — the non-finite guard of the multi-GPU modes and the banded exact path; 11800: mvbev_conv3x3_wino_bf16x3_dgrad (row-Winograd data gradient, output-side mask); 11700: channels-last sources for the fused warps (mvbev_warp_views_wino_rows, mvbev_warp_views_upsampled_wino_rows), mvbev_nchw_to_nhwc_f32; 11600: the non-finite-feature guard (mvbev_warp_views_exact_f32; the fused warps' nonfinite report; gate arguments of mvbev_conv3x3_f32 / mvbev_conv3x3_cout1_f32; mvbev_bev_plan.guard); 11500: row-Winograd conv2 -> conv3 partials (mvbev_wino_rows_split_bf16_dil, mvbev_conv3x3_wino_bf16x3_dil, mvbev_conv3x3_wino_bf16x3_cout1_partials); 11400: mvbev_warp_nonfinite_views (non-finite geometry routes to the direct conv1); the NMS candidate order replays torch's CPU sort (ties included), mvbev_point_nms (no workspace) retired; mvbev_conv3x3_bf16x3_sched / _sched3 retired (forward schedules measured slower); 11300: row-Winograd conv1 (mvbev_pack_conv3x3_weight_wino, mvbev_wino_rows_split_bf16, mvbev_conv3x3_wino_bf16x3); 11200: mvbev_conv3x3_bf16x3_sched3 (schedules over the edge-strip tiles); 11100: edge-strip conv tiles (mvbev_conv_ring_tile_space, mvbev_conv3x3_bf16x3_ex3); 11000: ring-kernel schedules (mvbev_conv_schedule, mvbev_conv3x3_bf16x3_sched, mvbev_conv3x3_dgrad_bf16x3_sched); 10900: mvbev_conv3x3_wgrad_bf16x3_ex2 (pre-split dy rows), mvbev_split_rows_bf16; 10800: mvbev_warp_upsampled_adjoint_plan (training from backbone features), mvbev_conv3x3_cout1_backward_ex; 10700: training on split-bf16 y1 (mvbev_relu_backward_split_f32, mvbev_conv3x3_dgrad_bf16x3_ex); 10600: conv2 -> conv3 fused (mvbev_conv3x3_bf16x3_cout1_partials, mvbev_cout1_reduce_partials); 10500: mvbev_point_nms_ws (any K); 10400: MVBEV_WARP_DST_ZEROED warps; 10300: LDS-DMA ring conv (12-row tiles for split-bf16 input); 10200: native backward (10100: frustum masks, split-K tail, fused upsample+warp) */

/* Bilinear homography warp, zero padding, align_corners=True (kornia 0.6.11).
 *   src    : [B][C][H][W] fp32, element strides src_strides[4] (any, >= 0)
 *   m      : device fp32 [B][3][3] row-major src_norm <- dst_norm (kornia's
 *            _torch_inverse_cast(normalize_homography(M, (H,W), (Ho,Wo))))
 *   dst    : [B][C][Ho][Wo] fp32 at element strides dst_strides[4]
 *            (dst_strides[3] must be 1); may point into a larger tensor. */
int mvbev_warp_perspective_f32(const float* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m,
                               float* dst, int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream);

/* Same with fp16 storage for src and dst (fp32 coordinate and blend math). */
int mvbev_warp_perspective_f16(const void* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m,
                               void* dst, int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream);

/* One view of a batched warp: all views share B, C, H, W, Ho, Wo. */
typedef struct mvbev_warp_view {
  const void* src;           /* [B][C][H][W] device, element strides src_strides */
  int64_t src_strides[4];
  void* dst;                 /* [B][C][Ho][Wo] device view, element strides dst_strides ([3] == 1) */
  int64_t dst_strides[4];
  float m[9];                /* src_norm <- dst_norm (row-major), same for every batch item */
} mvbev_warp_view;

/* Warp every view of a frame in ONE launch (the detector's per-camera loop at
 * persp_trans_detector.py:62-75, warp + concat).  views: host array of nviews (<= 16). */
int mvbev_warp_views_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                         int64_t H, int64_t W, int64_t Ho, int64_t Wo, void* stream);
/* Same, writing the split-bf16 blocked layout (MVBEV_LAYOUT_SPLIT_BF16) the 3xbf16 conv
 * reads without any conversion: for (batch, group of 8 channels, row, col) 32 bytes = bf16
 * hi[8] then bf16 lo[8], value = hi + lo.  dst_strides are in 32-byte units
 * {batch, channel group, row, col (must be 1)}; channels beyond C in the last group are 0.
 * src is fp32 (src_is_f16 = 0) or fp16.  (ABI 11600: the flag-less form is retired.)
 * flags of the _ex warps.  MVBEV_WARP_DST_ZEROED: the caller guarantees every dst already
 * holds zeros wherever the view's sample falls outside the source (e.g. a persistent slab
 * zero-filled at allocation and only ever written by this warp with the same matrices), so
 * those pixels — exactly 0 in the result — are skipped instead of rewritten.  Pixels with
 * non-finite coordinates (NaN output) are always written. */
#define MVBEV_WARP_DST_ZEROED 1
/* flag of mvbev_warp_views_wino_rows (ABI 11900): the sources are fp16 (fp32 math; T split-bf16 as for
 * fp32 sources) — config 4's fp16 features on the fused warp + B^T and the row-Winograd conv1. */
#define MVBEV_WARP_SRC_F16 2
/* MVBEV_WARP_WINO43 (ABI 12400; mvbev_warp_views_wino_rows_ex / _upsampled_wino_rows_ex): the fused warp
 * writes the F(4,3) transform T43 (mvbev_wino43_rows_bytes' layout) instead of T; r3_rows then counts
 * four-row tiles (4 * ceil(out_rows / 16)), 3 per 14 x 16 block; the block's staging-box table is
 * mvbev_warp_wino_boxes' with r3_rows = 4 * ceil(r4_rows / 3) (the same 12-row blocks). */
#define MVBEV_WARP_WINO43 4
int mvbev_warp_views_split_bf16_ex(const mvbev_warp_view* views, int nviews, int src_is_f16,
                                   int64_t B, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                   int flags, void* stream);
/* Row windows (ABI 11900): view i's dst holds out_rows rows of the Ho-row grid starting at grid row
 * row0s[i] (host int32 array; 0 <= row0s[i], row0s[i] + out_rows <= Ho), so one launch can warp the row
 * windows the multi-GPU band exchange sends (several entries may share a source).  nonfinite (may be
 * NULL): nf_tag is stored into the device int32 *nonfinite when a sample the warp produces is non-finite
 * (a NaN / inf feature it reads, or non-finite coordinates) — the non-finite guard's report, as the
 * fused row-Winograd warps give it. */
int mvbev_warp_views_split_bf16_rows(const mvbev_warp_view* views, const int32_t* row0s, int nviews, int src_is_f16,
                                     int64_t B, int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                     int64_t out_rows, int flags, int32_t* nonfinite, int32_t nf_tag, void* stream);
/* Gated zero fill: bytes (a multiple of 16, 16-B aligned dst) of zeros when *gate == gate_tag, else no
 * write (ABI 11900: re-zeroes the band exchange's send chunks after a frame whose exact path wrote them). */
int mvbev_zero_gated(void* dst, int64_t bytes, const int32_t* gate, int32_t gate_tag, void* stream);
/* Gated store (ABI 12200): fp32 src [B][C][H][W] (element strides, src_strides[3] == 1) into dst when
 * *gate == gate_tag, else no write.  dst_layout MVBEV_LAYOUT_F32: fp32 at element strides (dst_strides[3]
 * == 1); MVBEV_LAYOUT_SPLIT_BF16: the split-bf16 blocked layout, dst_strides in 32-byte units {batch,
 * channel group, row, col (1)}, a non-finite value stored as hi = value, lo = 0 (hi + lo keeps it; the
 * fast path's split gives lo = NaN).  The training forward's non-finite guard stores its exact-path
 * activations (conv1's input, y1, y2) where the native backward reads them
 * (persp_trans_detector.py:65-81 under trainer.py:38-47). */
int mvbev_store_gated_f32(const float* src, const int64_t src_strides[4], void* dst, const int64_t dst_strides[4],
                          int64_t B, int64_t C, int64_t H, int64_t W, int dst_layout, const int32_t* gate,
                          int32_t gate_tag, void* stream);
/* Fused bilinear upsample + warp.  views[i].src is the
 * backbone-resolution map [B][C][h][w] that persp_trans_detector.py:65 upsamples with
 * F.interpolate(size=(H, W), mode='bilinear', align_corners=False) before the warp at :69;
 * every bilinear corner of the warp is that upsample evaluated on the fly (one 3x3 source
 * window per output pixel), so the [B][C][H][W] intermediate is never written.  m is the
 * kornia matrix for the UPSAMPLED size (H, W) — the same one mvbev_warp_views_* take.
 * Upsampling only (H >= h, W >= w).  out_layout: MVBEV_LAYOUT_F32 (fp32 src) or
 * MVBEV_LAYOUT_SPLIT_BF16 (fp32 or fp16 src); dst strides as in the entry points above.
 * NaN/inf in the source map are outside the contract (a zero-weight tap of the window may
 * propagate them). */
int mvbev_warp_views_upsampled(const mvbev_warp_view* views, int nviews, int src_is_f16,
                               int64_t B, int64_t C, int64_t h, int64_t w, int64_t H, int64_t W,
                               int64_t Ho, int64_t Wo, int out_layout, void* stream);
int mvbev_warp_views_upsampled_ex(const mvbev_warp_view* views, int nviews, int src_is_f16,
                                  int64_t B, int64_t C, int64_t h, int64_t w, int64_t H, int64_t W,
                                  int64_t Ho, int64_t Wo, int out_layout, int flags, void* stream);
/* Frustum mask for the conv (see mvbev_conv3x3_bf16x3_ex): for output tiles of tile_h x
 * tile_w pixels over grid rows [row0, row0 + rows) of the Ho x Wo warp output, bit s of
 * mask[tile] is set when view s's warp (views[s].m, src size H x W) can be non-zero
 * anywhere in the tile grown by `halo` pixels — some pixel samples inside the source, or
 * its coordinates are non-finite (NaN output).  Uses the warp kernels' own fp32 coordinate
 * code, so a clear bit is exact.  Only views[].m is read; nviews <= 16. */
int mvbev_warp_tile_mask(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W,
                         int64_t Ho, int64_t Wo, int64_t row0, int64_t rows, int64_t tile_h,
                         int64_t tile_w, int64_t halo, uint32_t* mask, void* stream);
/* *bits (device uint32, overwritten) = the views (bit s = views[s], nviews <= 16) whose warp has
 * an output pixel of the Ho x Wo grid with non-finite sample coordinates, i.e. a NaN in the warped
 * features of persp_trans_detector.py:69 (a degenerate homography; kornia's 0/0 meshgrid when Ho
 * or Wo is 1).  The warp kernels' own fp32 coordinate code.  Only views[].m is read.  The
 * row-Winograd conv1 mixes a 3-row tile's rows before its products, so a caller routes such
 * geometry to the direct conv, which keeps NaN to the taps that read it as the reference's
 * nn.Conv2d (:51) does. */
int mvbev_warp_nonfinite_views(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W, int64_t Ho,
                               int64_t Wo, uint32_t* bits, void* stream);
/* fp16 storage for src and dst, fp32 math. */
int mvbev_warp_views_f16(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                         int64_t H, int64_t W, int64_t Ho, int64_t Wo, void* stream);

/* Coord-map channels: dst[b][0][v][u] = u/(Wo-1)*2-1, dst[b][1][v][u] = v/(Ho-1)*2-1
 * (computed in float64, rounded to fp32 as numpy->torch does at :106-107). */
int mvbev_fill_coord_map_f32(float* dst, int64_t B, int64_t Ho, int64_t Wo,
                             const int64_t dst_strides[4], void* stream);

/* Number of floats of the packed weight buffer for Cout output channels and K packed
 * input channels (K rounded up to MVBEV_CONV_KC). */
size_t mvbev_conv3x3_packed_floats(int64_t Cout, int64_t K);

/* Re-lay an nn.Conv2d weight w[Cout][Cin_w][3][3] (contiguous fp32, device) into the MFMA
 * staging layout for K packed input channels: packed channel k takes weight channel
 * chan_map[k] (device int32[K]; -1 = zero weights), or k itself when chan_map is NULL
 * (then K must equal Cin_w).  Lets the fused tensor's channel order differ from the
 * module's (view-major slots, coord channels handled separately). */
int mvbev_pack_conv3x3_weight_f32(const float* w, int64_t Cout, int64_t Cin_w,
                                  const int32_t* chan_map, int64_t K, float* w_packed,
                                  void* stream);
/* The same pack, run only when *gate == gate_tag (ABI 12200): the training forward's non-finite guard
 * re-packs the exact path's fp32 weights every step (the optimizer changes them) at the cost of a launch
 * that exits at once when the features are finite. */
int mvbev_pack_conv3x3_weight_f32_gated(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map,
                                        int64_t K, float* w_packed, const int32_t* gate, int32_t gate_tag,
                                        void* stream);

/* Geometry of one conv launch (all sizes in elements). */
typedef struct mvbev_conv_desc {
  int64_t B;             /* batch items */
  int64_t K;             /* packed input channels (multiple of MVBEV_CONV_KC) */
  int64_t H, W;          /* full image (ground grid) height / width */
  int64_t group;         /* channels per contiguous channel group (multiple of KC, divides K) */
  int64_t group_stride;  /* elements between consecutive channel groups */
  int64_t batch_stride;  /* elements between consecutive batch items */
  int64_t in_row0;       /* global row held by input-buffer row 0 */
  int64_t in_rows;       /* rows in the input buffer (channel plane = in_rows * W) */
  int64_t out_row0;      /* first global output row computed */
  int64_t out_rows;      /* output rows computed (y holds exactly these rows) */
} mvbev_conv_desc;

/* y = act(conv3x3(x, w, dilation=d, padding=d) [+ bias] [+ init]), fp32 MFMA, fp32 accumulate.
 *   x      : input channel ci of item b at x + (ci/group)*group_stride + b*batch_stride
 *            + (ci%group)*in_rows*W  ([B][K][H][W]: group=K; view-major [S][B][C][H][W]: group=C)
 *   w_packed : from mvbev_pack_conv3x3_weight_f32 with the same Cout and K
 *   bias   : [Cout] or NULL;  init : [Cout][H][W] (full-size, broadcast over B) or NULL
 *   relu   : 0/1 (NaN-preserving);  dilation : 1 or 2
 *   y      : [B][Cout][out_rows][W] contiguous fp32, Cout % MVBEV_CONV_BN == 0
 *   Zero padding at the image border; input rows outside the buffer are read as zero, so
 *   a band caller must supply every row the output band needs. */
int mvbev_conv3x3_f32(const float* x, const mvbev_conv_desc* desc, const float* w_packed,
                      const float* bias, const float* init, int64_t Cout, int dilation,
                      int relu, float* y, const int32_t* gate, int32_t gate_tag, void* stream);
/* The same with a row-banded output (ABI 11900): y_band_rows > 0 puts global output row g at row
 * g % y_band_rows of band g / y_band_rows of y = [bands][B][Cout][y_band_rows][W] — the partial-sum
 * multi-GPU mode's reduce-scatter input (as mvbev_conv3x3_wino_bf16x3's band_rows); 0 = the plain y. */
int mvbev_conv3x3_f32_ex(const float* x, const mvbev_conv_desc* desc, const float* w_packed, const float* bias,
                         const float* init, int64_t Cout, int dilation, int relu, float* y, int64_t y_band_rows,
                         const int32_t* gate, int32_t gate_tag, void* stream);
/* y = relu?(y + init) in place (NaN-preserving ReLU) for y [B][C][rows][W] holding grid rows
 * [row0, row0 + rows) of init [C][H][W]; stores tag into the device int32 *flag (NULL: no report) when a
 * result is non-finite (ABI 11900: the coord term + bias + ReLU of the partial-sum mode's summed conv1
 * pre-activation — persp_trans_detector.py:51 — and its non-finite guard). */
int mvbev_bias_relu_nonfinite_f32(float* y, const float* init, int64_t B, int64_t C, int64_t rows, int64_t W,
                                  int64_t H, int64_t row0, int relu, int32_t* flag, int32_t tag, void* stream);
/* conv1's coord term (ABI 12300; persp_trans_detector.py:103-112 coord map, :77 its concat, :51 conv1):
 * out [Cout][H][W] fp32 = bias (NULL: 0) + conv2d over the two coord channels [x = col / (W-1) * 2 - 1,
 * y = row / (H-1) * 2 - 1] (float64 then float, zero padding 1) with conv1's weights w1 [Cout][cin][3][3]
 * at input channels coord_c0 (x) and coord_c0 + 1 (y).  The input-independent part of conv1, added as its
 * accumulators' initial value. */
int mvbev_coord_term_f32(const float* w1, int64_t cin, int64_t coord_c0, const float* bias, int64_t Cout, int64_t H,
                         int64_t W, float* out, void* stream);
/* gate (this entry point, mvbev_conv3x3_cout1_f32, mvbev_warp_views_exact_f32; ABI 11600): a device
 * int32; when non-NULL the launch does its work only if *gate == gate_tag at the time it runs (every
 * workgroup exits at once otherwise) — a decision taken on the device in stream order, so a caller
 * can enqueue a conditional path without a host sync (the non-finite guard of mvbev_bev_fuse and
 * the Python engine).  NULL: always run. */

/* Input layouts of mvbev_conv3x3_bf16x3 (descriptor strides are always in 4-byte
 * "channel-element" units, i.e. as for an fp32 tensor of the same logical shape). */
#define MVBEV_LAYOUT_F32 0        /* plain fp32 channel planes */
#define MVBEV_LAYOUT_F16 1        /* plain fp16 channel planes (strides in elements) */
#define MVBEV_LAYOUT_SPLIT_BF16 2 /* per (8-channel group, pixel): bf16 hi[8], bf16 lo[8] */
#define MVBEV_LAYOUT_SPLIT_ROWS 3 /* per (channel, row, 8-pixel run): bf16 hi[8], bf16 lo[8]
                                     (W % 8 == 0; the same bytes per row as fp32) */
#define MVBEV_LAYOUT_SPLIT_BF16_PIX 4 /* pixel-major split-bf16: per (pixel, 8-channel group) bf16 hi[8], lo[8],
                                         [B][rows][W][C/8] (ABI 12100): the conv data gradients' output for the
                                         warp adjoint, whose gather then reads a pixel's channels in one piece */

/* 3xbf16 split-precision variant of mvbev_conv3x3_f32 (mvbev_conv3x3_bf16x3_ex below; same
 * descriptor and semantics): a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi on the bf16 MFMA, fp32
 * accumulation; ~2^-16 relative per product (fp32-class; see conv_bf16x3.hip).  x_layout:
 * MVBEV_LAYOUT_* (fp32, the config-4 fp16 slab, or the pre-split slab).
 * Weights packed by mvbev_pack_conv3x3_weight_bf16x3 (bytes: mvbev_conv3x3_packed_bytes_bf16x3). */
size_t mvbev_conv3x3_packed_bytes_bf16x3(int64_t Cout, int64_t K);
int mvbev_pack_conv3x3_weight_bf16x3(const float* w, int64_t Cout, int64_t Cin_w,
                                     const int32_t* chan_map, int64_t K, void* w_packed,
                                     void* stream);
/* Output tile of mvbev_conv3x3_bf16x3_ex (rows x columns), the granule of group_mask below:
 * MVBEV_CONV_TILE_H rows for fp32/fp16 input; split-bf16 input (the LDS-DMA ring kernel)
 * uses the row count mvbev_conv3x3_bf16x3_tile_rows returns (12). */
#define MVBEV_CONV_TILE_H 8
#define MVBEV_CONV_TILE_W 32
int mvbev_conv3x3_bf16x3_tile_rows(int x_layout, int dilation);

/* The 3xbf16 conv (ABI 11600: the form without mask / order / workspace is retired).
 *   y, y_layout: MVBEV_LAYOUT_F32 ([B][Cout][out_rows][W] fp32, as above) or
 *     MVBEV_LAYOUT_SPLIT_BF16 ([B][Cout/8][out_rows][W] pieces of bf16 hi[8], lo[8]: the
 *     next conv's input without a conversion pass).
 *   group_mask (optional, device): one uint32 per output tile, tiles row-major over
 *     ceil(out_rows / tile_rows(x_layout, dilation)) x ceil(W / MVBEV_CONV_TILE_W) (rows from out_row0);
 *     bit g clear = input channel group g (desc->group channels, group % 16 == 0, at most 32
 *     groups) is exactly zero over the tile and its 3x3 dilated halo, so its K-chunks are
 *     skipped for that tile (identical result).  mvbev_warp_tile_mask builds it from the
 *     views' homographies: a camera's warped features are exactly 0 outside its frustum.
 *   tile_order (optional, device, with group_mask): the B x tiles pixel tiles (index
 *     (b * tiles_y + tile_y) * tiles_x + tile_x) in the order to run them — heaviest
 *     first evens out the per-tile work the mask makes uneven.
 *   workspace (optional, device): scratch for the split-K tail — when the output tiles do
 *     not fill a whole number of rounds over the CUs (one workgroup per CU), the tiles of
 *     the last, partial round are cut into K-ranges run by separate workgroups and a second
 *     launch sums each tile's pieces in K order (deterministic).  workspace_bytes() returns
 *     what this shape needs (0 = not used); a NULL / smaller workspace keeps whole tiles.
 *     Not combined with group_mask. */
size_t mvbev_conv3x3_bf16x3_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout);
int mvbev_conv3x3_bf16x3_ex(const void* x, int x_layout, const mvbev_conv_desc* desc,
                            const void* w_packed, const float* bias, const float* init,
                            int64_t Cout, int dilation, int relu, void* y, int y_layout,
                            const uint32_t* group_mask, const int32_t* tile_order, void* workspace,
                            size_t workspace_bytes, void* stream);
/* Pixel-tile spaces of the split-bf16-input (ring) conv.  MVBEV_TILES_GRID: the 12 x 32 tile
 * grid of mvbev_conv3x3_bf16x3_ex (tiles_y x ceil(W / 32) per batch item, row-major; the last
 * tile column computes up to 31 columns past W).  MVBEV_TILES_EDGE_STRIP (0 < W % 32 <= 16):
 * the 12 x 32 grid over columns [0, 32 * floor(W / 32)), then edge_tiles tiles of edge_rows x EW
 * pixels (EW = 8 or 16, edge_rows = 384 / EW) over the last W % 32 columns, top to bottom — the
 * same 384 pixels per tile and no MFMA column past W (Wildtrack's W = 360: 11 regular tile
 * columns + 3 strips of 48 x 8).  mvbev_conv_ring_tile_space fills
 * g = {tiles_x, tiles_y, edge_tiles, EW, edge_rows} for desc's output rows and W (0 edges for
 * the grid), or returns MVBEV_ERR_SHAPE when the space does not apply. */
#define MVBEV_TILES_GRID 0
#define MVBEV_TILES_EDGE_STRIP 1
int mvbev_conv_ring_tile_space(const mvbev_conv_desc* desc, int tile_space, int64_t g[5]);
/* mvbev_conv3x3_bf16x3_ex with the tiles of tile_space (split-bf16 x only, no workspace):
 * group_mask[pp] / tile_order (b * tiles + pp) index pixel tiles pp of that space (edge-strip
 * masks: mvbev_warp_tile_mask with tile_h = edge_rows, tile_w = EW, last tile column).
 * MVBEV_TILES_EDGE_STRIP: dilation 1 with ReLU (conv1, map_classifier[0:2]).  Same y, bitwise,
 * as the grid tiles. */
int mvbev_conv3x3_bf16x3_ex3(const void* x, int x_layout, const mvbev_conv_desc* desc,
                             const void* w_packed, const float* bias, const float* init,
                             int64_t Cout, int dilation, int relu, void* y, int y_layout,
                             const uint32_t* group_mask, const int32_t* tile_order, int tile_space,
                             void* stream);

/* Row-Winograd form of the forward conv1 (map_classifier[0:2], persp_trans_detector.py:51-52,
 * dilation 1): F(3,3) along the rows, y = A^T [(G w) . (B^T d)] per kernel column, 5 instead of 9
 * MFMA K-blocks per (16-channel chunk, kernel column); same 3xbf16 split products, fp32 accumulate.
 * Replaces the same call as mvbev_conv3x3_bf16x3_ex with dilation 1 (the reference's
 * nn.Conv2d(512*N+2, 512, 3, padding=1) forward, :51), in two steps:
 *   1. mvbev_wino_rows_split_bf16: the split-bf16 input x (desc as mvbev_conv3x3_bf16x3_ex) ->
 *      T = B^T over each 3-row output tile's 5 input rows, split-bf16 blocked
 *      [B][K/8][5 * 4 * ceil(out_rows / 12)][hi, lo][W][8] (mvbev_wino_rows_bytes; ABI 11500: a row's hi plane, then
 *      its lo plane — was [W][hi, lo][8]).  With
 *      group_mask (12 x 32 tiles, as the conv) the cleared (tile, group) pairs are not written:
 *      T must then be zero-filled once and only ever written by this call with the same mask.
 *   2. mvbev_conv3x3_wino_bf16x3: y from T (desc: B, K, H, W, group, out_row0, out_rows as in
 *      step 1), weights from mvbev_pack_conv3x3_weight_wino (same arguments as
 *      mvbev_pack_conv3x3_weight_bf16x3), bias / init / relu / y / y_layout / group_mask /
 *      tile_order as mvbev_conv3x3_bf16x3_ex (grid tiles, 12 x 32). */
/* Warp + the row transform of step 1 in one pass, from fp32 sources (mvbev_warp_views_split_bf16's
 * views and matrices): the T rows of r3_rows 3-row output tiles (3 * r3_rows >= Ho; the conv's
 * T has 4 * ceil(out_rows / 12) of them) are written for each view's channels at its dst, whose
 * dst_strides are in 32-byte units: [0] per batch item, [1] per 8-channel group, [2] per T row
 * (= Wo: the row's hi plane, then its lo plane), [3] = 1 — the view's slice of T.  The warped slab itself is never written.  flags:
 * MVBEV_WARP_DST_ZEROED = T is zero-filled and only written by this geometry, so a (tile,
 * column) whose 5 samples all fall outside the source is skipped.  Replaces :69 + :77 + the
 * first step of conv1 (:51) for inference. */
int mvbev_warp_views_wino_rows(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                               int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                               int32_t nf_tag, void* stream);
/* (ABI 12200) The per-(view, block) source boxes of the NCHW form of mvbev_warp_views_wino_rows, once per
 * geometry (views[i].m only; src / dst unused): boxes = device int32 [nviews][mvbev_warp_wino_boxes_count(Wo,
 * r3_rows)][4], 16-B aligned.  Passed to mvbev_warp_views_wino_rows_ex (same views, sizes and r3_rows), every
 * block of a (view, tile) takes its staging box from the table instead of reducing it, and a block none of
 * whose samples falls inside the source (with MVBEV_WARP_DST_ZEROED) returns at once; boxes = NULL is
 * mvbev_warp_views_wino_rows.  Channels-last sources (the line-per-pixel kernel, same block tiles) use it for the
 * early return only. */
int64_t mvbev_warp_wino_boxes_count(int64_t Wo, int64_t r3_rows);
int mvbev_warp_wino_boxes(const mvbev_warp_view* views, int nviews, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                          int64_t r3_rows, int32_t* boxes, void* stream);
int mvbev_warp_views_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H,
                                  int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int flags, int32_t* nonfinite,
                                  int32_t nf_tag, const int32_t* boxes, void* stream);
/* The same from backbone-resolution maps [B][C][h][w] (fp32, unit column stride, w >= 4): the
 * fused 3x upsample + warp of mvbev_warp_views_upsampled (m for the upsampled size H x W) and the
 * row transform in one pass (the detector's inference path, :65 + :69 + :77 + conv1's first step).
 * ABI 11700, both fused warps: channels-last sources (src_strides[1] == 1, [3] >= C, the other strides
 * multiples of 4 floats, 16-B aligned, C % 32 == 0; the same logical [B][C][h][w] tensor in torch's
 * channels_last memory format) run a line-per-pixel form (one 128-B line holds a pixel's 32 channels
 * of a block); same T up to fp32 rounding of the bilinear sums. */
int mvbev_warp_views_upsampled_wino_rows(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t h,
                                         int64_t w, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows,
                                         int flags, int32_t* nonfinite, int32_t nf_tag, void* stream);
/* (ABI 12200) As mvbev_warp_wino_boxes for the channels-last upsample warp: the per-(view, block) boxes of the
 * blocks' 3x3 backbone windows (h x w maps, m for the upsampled H x W), once per geometry; passed to
 * mvbev_warp_views_upsampled_wino_rows_ex (same views, sizes and r3_rows) every block of a (view, tile) takes its
 * staging box from the table and a block none of whose samples falls inside the source (with
 * MVBEV_WARP_DST_ZEROED) returns at once.  The table has mvbev_warp_wino_boxes_count(Wo, r3_rows) entries per
 * view; NCHW maps ignore it. */
int mvbev_warp_upsampled_wino_boxes(const mvbev_warp_view* views, int nviews, int64_t h, int64_t w, int64_t H,
                                    int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows, int32_t* boxes, void* stream);
int mvbev_warp_views_upsampled_wino_rows_ex(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t h,
                                            int64_t w, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t r3_rows,
                                            int flags, int32_t* nonfinite, int32_t nf_tag, const int32_t* boxes,
                                            void* stream);
/* nonfinite (both fused warps, ABI 11600; NULL = no report): nf_tag is stored into the device int32
 * *nonfinite when a sample reads a NaN / inf feature (conservatively also when finite values overflow).
 * The fused form folds B^T (and the upsample's taps into one 3x3 window), so it cannot keep the
 * reference's NaN / inf pattern for such features; the caller's exact path, gated on the report, can:
 *   mvbev_warp_views_exact_f32 — the warp (h = H, w = W) or the 3x upsample + warp (h x w backbone
 *   maps, persp_trans_detector.py:65 + :69) in the reference's own evaluation order: per in-bounds
 *   corner the PyTorch upsample value (both taps of each axis multiplied, zero weights included; no
 *   fma contraction in the source index), times its grid_sample weight; out-of-bounds corners selected
 *   to 0.  fp32 src [B][C][h][w], fp32 dst [B][C][Ho][Wo] at element strides ([3] == 1); gate as
 *   mvbev_conv3x3_f32's. */
int mvbev_warp_views_exact_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t h, int64_t w,
                               int64_t H, int64_t W, int64_t Ho, int64_t Wo, const int32_t* gate, int32_t gate_tag,
                               void* stream);
/* The same on row windows and fp16 sources (ABI 11900): view i's dst holds out_rows rows of the Ho-row
 * grid starting at grid row row0s[i] (host int32 array) — the exact path in row bands of bounded memory,
 * and the band exchange's windows; src_is_f16: fp16 sources (fp32 math). */
int mvbev_warp_views_exact_rows(const mvbev_warp_view* views, const int32_t* row0s, int nviews, int src_is_f16,
                                int64_t B, int64_t C, int64_t h, int64_t w, int64_t H, int64_t W, int64_t Ho,
                                int64_t Wo, int64_t out_rows, const int32_t* gate, int32_t gate_tag, void* stream);
/* NCHW -> channels-last copy (ABI 11700): view i's fp32 [B][C][H][W] map at views[i].src /
 * src_strides into a contiguous [B][H][W][C] buffer at views[i].dst (dst_strides, m ignored), every
 * view in one launch — the input of the channels-last fused upsample warp for NCHW producers. */
int mvbev_nchw_to_nhwc_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C, int64_t H, int64_t W,
                           void* stream);
size_t mvbev_conv3x3_packed_bytes_wino(int64_t Cout, int64_t K);
int mvbev_pack_conv3x3_weight_wino(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map,
                                   int64_t K, void* w_packed, void* stream);
size_t mvbev_wino_rows_bytes(const mvbev_conv_desc* desc);
int mvbev_wino_rows_split_bf16(const void* x, const mvbev_conv_desc* desc, const uint32_t* group_mask, void* t,
                               size_t t_bytes, void* stream);
int mvbev_conv3x3_wino_bf16x3(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                              const float* init, int64_t Cout, int relu, void* y, int y_layout, int64_t y_band_rows,
                              const uint32_t* group_mask, const int32_t* tile_order, void* stream);
/* y_band_rows (ABI 11600; MVBEV_LAYOUT_F32 only, 0 = plain [B][Cout][out_rows][W]): y in row bands,
 * computed row r (from out_row0) at band r / y_band_rows, y = [bands][B][Cout][y_band_rows][W] (rows
 * past out_rows in the last band untouched) — the reduce-scatter input of the partial-sum multi-GPU
 * mode, written in place. */
/* The same two steps for dilation 2 (conv2, map_classifier[2:4], persp_trans_detector.py:53:
 * nn.Conv2d(512, 512, 3, padding=2, dilation=2)): the 12-row workgroup tile holds two interleaved
 * pairs of 3-row tiles (rows r, r + 2, r + 4), whose T = B^T over the 5 input rows r - 2 ... r + 6
 * (step 2); a kernel column's taps are 2 columns apart.  mvbev_wino_rows_split_bf16_dil(dilation 1)
 * is mvbev_wino_rows_split_bf16; T has the same size (mvbev_wino_rows_bytes).  The conv: no init,
 * no mask (dense), y fp32 or split-bf16 (_dil), or, replacing
 * mvbev_conv3x3_bf16x3_cout1_partials (same desc, bias, w3, partials layout and size; relu,
 * dilation 2), conv3's partial sums from the epilogue (_cout1_partials, ABI 11500). */
int mvbev_wino_rows_split_bf16_dil(const void* x, const mvbev_conv_desc* desc, int dilation,
                                   const uint32_t* group_mask, void* t, size_t t_bytes, void* stream);
/* The same transform, run only when *gate == gate_tag (gate not NULL; ABI 12200): the training guard's
 * T / T2 of its exact-path conv1 input / y1 for the native weight gradients. */
int mvbev_wino_rows_split_bf16_gated(const void* x, const mvbev_conv_desc* desc, int dilation,
                                     const uint32_t* group_mask, void* t, size_t t_bytes, const int32_t* gate,
                                     int32_t gate_tag, void* stream);
int mvbev_conv3x3_wino_bf16x3_dil(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                                  int64_t Cout, int dilation, int relu, void* y, int y_layout, void* stream);
int mvbev_conv3x3_wino_bf16x3_cout1_partials(const void* t, const mvbev_conv_desc* desc, const void* w_packed,
                                             const float* bias, int64_t Cout, int dilation, int relu, const float* w3,
                                             void* partials, size_t partials_bytes, void* stream);
/* Row-Winograd F(4,3) (ABI 12400; persp_trans_detector.py:51 conv1 and :53-54 conv2 -> conv3): the same
 * convs as mvbev_conv3x3_wino_bf16x3 / _cout1_partials from 6 transformed rows per 4 output rows (points
 * 0, +-1, +-2, inf) instead of 5 per 3 — 10 % fewer MFMAs, the K sum walked xi-major.  T43 =
 * [B][K/8][6 * 4 * ceil(out_rows / 16)][hi, lo][W][8] (mvbev_wino43_rows_bytes; dilation 2: row tile q of
 * a 16-row tile holds rows 8 (q / 2) + q % 2 + 2 pt), written by mvbev_wino43_rows_split_bf16 from the
 * split-bf16 input; weights from mvbev_pack_conv3x3_weight_wino43 (arguments as
 * mvbev_pack_conv3x3_weight_wino); group_mask / tile_order over 16 x 32 output tiles
 * (mvbev_warp_tile_mask with 16-row tiles); y fp32 or split-bf16. */
size_t mvbev_conv3x3_packed_bytes_wino43(int64_t Cout, int64_t K);
int mvbev_pack_conv3x3_weight_wino43(const float* w, int64_t Cout, int64_t Cin_w, const int32_t* chan_map, int64_t K,
                                     void* w_packed, void* stream);
size_t mvbev_wino43_rows_bytes(const mvbev_conv_desc* desc);
int mvbev_wino43_rows_split_bf16(const void* x, const mvbev_conv_desc* desc, int dilation, const uint32_t* group_mask,
                                 void* t, size_t t_bytes, void* stream);
int mvbev_conv3x3_wino43_bf16x3(const void* t, const mvbev_conv_desc* desc, const void* w_packed, const float* bias,
                                const float* init, int64_t Cout, int dilation, int relu, void* y, int y_layout,
                                const uint32_t* group_mask, const int32_t* tile_order, void* stream);
int mvbev_conv3x3_wino43_bf16x3_cout1_partials(const void* t, const mvbev_conv_desc* desc, const void* w_packed,
                                               const float* bias, int64_t Cout, int dilation, int relu,
                                               const float* w3, void* partials, size_t partials_bytes, void* stream);
/* A data gradient as the dilation-1 row-Winograd conv (ABI 11800; the training backward's conv1
 * dgrad, persp_trans_detector.py:51 differentiated): t = the row transform of the split-bf16 dy
 * (mvbev_wino_rows_split_bf16), w_packed = mvbev_pack_conv3x3_weight_wino of the weight with its
 * in / out channels swapped and its taps reversed ([Cout = forward Cin][forward Cout][3][3]), no
 * bias / init / ReLU; dx fp32 or split-bf16 [B][Cout][out_rows][W].  out_mask (optional, int32 per
 * 12 x 32 output tile as mvbev_warp_tile_mask): tiles of output channel group g (cot_per_group
 * 128-channel tiles) whose bit g is clear are not written (a consumer that never reads them). */
/* The data-gradient weights of mvbev_conv3x3_wino_bf16x3_dgrad straight from the forward weight
 * w [Cout_f][Cin_f][3][3] fp32 (ABI 11800): packed as mvbev_pack_conv3x3_weight_wino would pack
 * w'[o][i][kh][kw] = w[i][o][2 - kh][2 - kw] for o < Cout (Cout % 128 == 0, Cout <= Cin_f: the
 * first Cout forward input channels) and i < Cout_f (the packed K). */
int mvbev_pack_conv3x3_weight_wino_dgrad(const float* w, int64_t Cout_f, int64_t Cin_f, int64_t Cout, void* w_packed,
                                         void* stream);
int mvbev_conv3x3_wino_bf16x3_dgrad(const void* t, const mvbev_conv_desc* desc, const void* w_packed, int64_t Cout,
                                    void* dx, int dx_layout, const uint32_t* out_mask, int64_t cot_per_group,
                                    void* stream);

/* conv2 -> conv3 without conv2's activation in HBM (map_classifier[2:5],
 * persp_trans_detector.py:53-54, inference): the split-bf16-input conv of
 * mvbev_conv3x3_bf16x3_ex (desc, w_packed, bias, Cout, dilation, relu as there; no init, no
 * mask) whose epilogue, instead of storing y, writes per (Cout tile, 64-channel half) set s,
 * tap t of the following single-output conv and computed pixel the partial
 *   partials[b][s][t][row - desc->out_row0][col] = sum over the set's channels co of
 *                                                  w3[co][t] * act(y[b][co][row][col])
 * (w3 : [Cout][3][3] fp32, the next conv's weight; 2 * Cout / MVBEV_CONV_BN sets;
 * partials_bytes >= mvbev_conv3x3_bf16x3_cout1_partials_bytes).  mvbev_cout1_reduce_partials
 * then forms map[b][0][r][:] = conv3x3(y, w3, dilation3, padding dilation3)[map_row0 + r]
 * summing the sets' shifted taps in a fixed order; the rows map_row0 +- dilation3 that lie
 * inside the image must be among desc's computed rows.  Same value as storing y and running
 * mvbev_conv3x3_cout1_f32 on it, to fp32 summation order. */
size_t mvbev_conv3x3_bf16x3_cout1_partials_bytes(const mvbev_conv_desc* desc, int64_t Cout);
int mvbev_conv3x3_bf16x3_cout1_partials(const void* x, const mvbev_conv_desc* desc, const void* w_packed,
                                        const float* bias, int64_t Cout, int dilation, int relu, const float* w3,
                                        void* partials, size_t partials_bytes, void* stream);
int mvbev_cout1_reduce_partials(const void* partials, const mvbev_conv_desc* desc, int64_t Cout, int dilation3,
                                float* map, int64_t map_row0, int64_t map_rows, void* stream);

/* y[b][0][r][:] = conv3x3(x[b], w, dilation=d, padding=d)[out_row0 + r], one output channel,
 * no bias.  x : [B][C][in_rows][W] holding global rows [in_row0, in_row0+in_rows) of an
 * H x W image;  w : [C][3][3] contiguous fp32;  y : [B][1][out_rows][W]. */
int mvbev_conv3x3_cout1_f32(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                            int64_t in_row0, int64_t in_rows, int64_t out_row0, int64_t out_rows,
                            const float* w, int dilation, float* y, const int32_t* gate, int32_t gate_tag,
                            void* stream);

/* ---- one-call project + fuse ----------------------------------------------
 * The inference hot path of PerspTransDetector.forward after the backbone
 * (persp_trans_detector.py:62-82: the per-view warp at :69 (+ the 3x upsample of :65 for
 * backbone-resolution sources), the concat at :77, map_classifier at :81, the identity
 * interpolate at :82) for a caller that does not want to orchestrate the entry points above
 * itself.  Three calls over one caller-owned device workspace:
 *   mvbev_bev_plan_init      host only: validates the geometry, lays out the workspace
 *   mvbev_bev_fuse_prepare   once per geometry and weight version: conv1's packing (G w for the
 *                            row-Winograd form), conv2's, the coord term (conv1 bias + conv1 over
 *                            the 2 coord channels, :21), the frustum mask, the heavy-first tile
 *                            order and the non-finite-geometry check; ONE stream sync (the mask
 *                            and the check are read back to plan the launches)
 *   mvbev_bev_fuse           per frame, enqueued, no sync: map = [B][1][Ho][Wo] fp32
 * Weights are the nn.Conv2d parameters of map_classifier (:51-54), fp32 contiguous device
 * tensors: w1 [512][N*C+2][3][3], b1 [512], w2 [512][512][3][3], b2 [512], w3 [1][512][3][3];
 * b2 and w3 are read again by every mvbev_bev_fuse (keep them alive and unchanged; after an
 * update of any weight call prepare again).  The module's channel order is view-major (view v's
 * channels are v*C .. v*C + C-1, then the 2 coord channels) as torch.cat builds it at :77. */
#define MVBEV_BEV_MAX_VIEWS 16
#define MVBEV_BEV_SRC_F32 0          /* views[v]: [B][C][H][W] fp32 contiguous (kornia's input, :69) */
#define MVBEV_BEV_SRC_F16 1          /* views[v]: [B][C][H][W] fp16 contiguous (fp32 math) */
#define MVBEV_BEV_SRC_BACKBONE_F32 2 /* views[v]: [B][C][h][w] fp32 backbone maps; :65's upsample fused */
#define MVBEV_BEV_SRC_CHANNELS_LAST 16 /* flag OR'ed into an fp32 kind (ABI 11700): views[v] hold the same
                                          tensor channels-last, [B][H][W][C] ([B][h][w][C]) contiguous, C % 32
                                          == 0 — the fused warps' line-per-pixel kernels */
#define MVBEV_BEV_NO_GUARD 32        /* flag (ABI 11900): no non-finite guard — no guard regions in the
                                        workspace (the guard's fp32 slab is one row chunk of at most 1 GiB) */
typedef struct mvbev_bev_geometry {
  int32_t num_views;                /* N, 1 .. 16 (persp_trans_detector.py:58-59) */
  int32_t src_kind;                 /* MVBEV_BEV_SRC_* */
  int64_t B, C;                     /* batch items; channels per view */
  int64_t h, w;                     /* backbone map size (MVBEV_BEV_SRC_BACKBONE_F32 only) */
  int64_t H, W;                     /* the warp's source size (upsample_shape, :23) */
  int64_t Ho, Wo;                   /* the ground grid (reducedgrid_shape) */
  float m[MVBEV_BEV_MAX_VIEWS][9];  /* per view: kornia's src_norm <- dst_norm of proj_mats[v] (:68-69) */
} mvbev_bev_geometry;
typedef struct mvbev_bev_plan {     /* host memory, caller-owned; filled by the calls below */
  mvbev_bev_geometry g;
  int32_t wino;                     /* after prepare: 1 = row-Winograd conv1, 0 = direct (non-finite geometry);
                                       ABI 12400: 2 = row-Winograd F(4,3) (grids whose rows fill 16-row tiles) */
  int32_t frustum;                  /* conv1 skips the views a tile's camera frustum excludes (C % 16 == 0 after padding) */
  int32_t prepared;
  int32_t wino2;                    /* after prepare: 1 = row-Winograd conv2 -> conv3 partials (ABI 11500; finite geometry);
                                       ABI 12400: 2 = F(4,3) (16-row tiles and a launch >= 8 rounds deep) */
  int32_t guard;                    /* 1 = the non-finite-feature guard runs behind the row-Winograd path (ABI 11600) */
  int64_t Cs, tiles;                /* channels per view slot (C rounded to 8); conv1's 12 x 32 tiles (16 x 32 with wino 2) */
  size_t off[24];                   /* workspace regions */
  size_t workspace_bytes;           /* >= what mvbev_bev_fuse_workspace_bytes returns, 256-B aligned base */
  const float* b2;
  const float* w3;
} mvbev_bev_plan;
int mvbev_bev_plan_init(const mvbev_bev_geometry* g, mvbev_bev_plan* plan);
size_t mvbev_bev_fuse_workspace_bytes(const mvbev_bev_geometry* g);
int mvbev_bev_fuse_prepare(mvbev_bev_plan* plan, const float* w1, const float* b1, const float* w2, const float* b2,
                           const float* w3, void* workspace, size_t ws_bytes, void* stream);
/* views: host array of N device pointers (layout per src_kind); map: [B][1][Ho][Wo] fp32.  fp32
 * sources: the warp writes conv1's row-Winograd transform directly; fp16 sources (and geometry
 * with non-finite samples) run the direct conv1 on the split slab.  guard (fp32 sources, ABI
 * 11600): the warp reports a NaN / inf feature it samples into a device flag, and the exact path
 * (mvbev_warp_views_exact_rows into an fp32 slab window, mvbev_conv3x3_f32 twice, mvbev_conv3x3_cout1_f32,
 * each gated on that flag) rewrites the map with the reference's NaN / inf pattern — decided on the
 * device, no host sync; launches that exit at once when the features are finite.  ABI 11900: in
 * output-row chunks whose fp32 slab window holds at most 1 GiB (one chunk at configs 1, 2 and 4);
 * MVBEV_BEV_NO_GUARD in src_kind turns the guard and its workspace regions off. */
int mvbev_bev_fuse(const mvbev_bev_plan* plan, const void* const* views, float* map, void* workspace,
                   size_t ws_bytes, void* stream);

/* ---- native backward: training through the hot path ----------------
 * Replaces the autograd of the stock ops the reference trains through (trainer.py:38-49,
 * loss.backward() at :47): grid_sample's backward under kornia.warp_perspective
 * (persp_trans_detector.py:69) and nn.Conv2d / nn.ReLU backward of map_classifier (:51-54). */

/* Adjoint of mvbev_warp_views_* (bilinear, zeros padding, align_corners=True): for every output
 * pixel whose sample point is finite and inside, each in-bounds corner of the source gradient
 * gets w_corner * grad_out (fp32 atomic adds; no gradient from zero-padded or NaN samples).
 *   views[i].src : grad_out, [B][C][Ho][Wo] fp32 at element strides src_strides
 *   views[i].dst : grad_src, [B][C][H][W] fp32 at element strides dst_strides ([3] must be 1);
 *                  ACCUMULATED into (zero it first for a plain gradient)
 *   views[i].m   : the forward's src_norm <- dst_norm matrix. */
int mvbev_warp_views_backward_f32(const mvbev_warp_view* views, int nviews, int64_t B, int64_t C,
                                  int64_t H, int64_t W, int64_t Ho, int64_t Wo, void* stream);

/* The same adjoint as a deterministic gather (no atomics in the per-channel loop).
 * mvbev_warp_adjoint_plan builds, once per view geometry (m = src_norm <- dst_norm, host
 * array), the CSR transpose of the warp's sparse sampling matrix: for source pixel p, entries
 * row_ptr[p] .. row_ptr[p+1]-1 hold (col = output pixel v*Wo+u, val = bilinear corner weight)
 * in increasing col order.  Device buffers: row_ptr int32[H*W + 1], col int32[4*Ho*Wo], val
 * fp32[4*Ho*Wo] (capacity; row_ptr[H*W] = entries used), scratch int32[H*W]. */
int mvbev_warp_adjoint_plan(const float* m, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int32_t* row_ptr,
                            int32_t* col, float* val, int32_t* scratch, void* stream);
/* The same plan for the fused 3x-upsample + warp of mvbev_warp_views_upsampled (the backbone
 * map h x w upsampled to H x W, persp_trans_detector.py:65, then warped, :69): source pixels are
 * the h x w backbone pixels, <= 9 entries per output pixel (the sample's 3x3 backbone window,
 * weight = upsample weight x warp weight, zero-weight cells omitted).  Buffers: row_ptr
 * int32[h*w + 1], col int32[9*Ho*Wo], val fp32[9*Ho*Wo], scratch int32[h*w].  With it,
 * mvbev_warp_views_adjoint (H, W = h, w) takes the gradient straight to the backbone features. */
int mvbev_warp_upsampled_adjoint_plan(const float* m, int64_t h, int64_t w, int64_t H, int64_t W, int64_t Ho,
                                      int64_t Wo, int32_t* row_ptr, int32_t* col, float* val, int32_t* scratch,
                                      void* stream);

typedef struct mvbev_warp_adjoint_view {
  const float* grad_out;       /* [B][C][Ho][Wo] fp32, element strides (row / column dense) */
  int64_t grad_out_strides[4];
  float* grad_src;             /* [B][C][H][W] fp32, element strides (row / column dense) */
  int64_t grad_src_strides[4];
  const int32_t* row_ptr;      /* the view's plan */
  const int32_t* col;
  const float* val;
} mvbev_warp_adjoint_view;

/* grad_src (accumulate ? += : =) S^T grad_out for every view, one launch (nviews <= 16).
 * grad_out_layout MVBEV_LAYOUT_F32 (element strides) or MVBEV_LAYOUT_SPLIT_BF16 (grad_out =
 * the view's first 8-channel group of a split-bf16 blocked tensor, 16-B aligned, strides in
 * 32-byte units {batch, channel group, row = Wo, col = 1}; value = hi + lo), or (ABI 12100)
 * MVBEV_LAYOUT_SPLIT_BF16_PIX (the same pieces pixel-major: strides {batch, 1, Wo * G, G} with
 * G >= C / 8 groups per pixel; C % 8 == 0) — same grad_src values as the split layout. */
int mvbev_warp_views_adjoint(const mvbev_warp_adjoint_view* views, int nviews, int grad_out_layout, int64_t B,
                             int64_t C, int64_t H, int64_t W, int64_t Ho, int64_t Wo, int accumulate,
                             void* stream);

/* A host-built schedule for the LDS-DMA ring kernel (split-bf16 input, dilation 1 or 2): block i
 * runs items[i] = {tile, c0, c1, slot} — tile = ((b * tiles_y + ty) * tiles_x + tx) * n_cot + cot
 * (12-row tiles, mvbev_conv3x3_bf16x3_tile_rows), chunks [c0, c1) of the tile's active 16-channel
 * chunk sequence (all of K, or the groups a group_mask enables, in order), slot = -1 for a
 * whole tile or the partial-sum slot of a piece of a split tile; tile < 0 = an idle block.
 * fixups[f] = {tile, first slot, pieces, 0}: after the conv, one block per split tile adds its
 * pieces' partial sums in slot order (deterministic) and writes the tile as the kernel would.
 * The order of items is the dispatch order (block i goes to XCD i % 8); the host plans it to
 * balance the CUs (mvdet_amd/schedule.py: e.g. splitting the last, partial round's tiles). */
typedef struct mvbev_conv_schedule {
  const int32_t* items;    /* device [nitems][4], 16-B aligned */
  int32_t nitems;
  const int32_t* fixups;   /* device [nfix][4], 16-B aligned */
  int32_t nfix;
  int32_t nslots;          /* partial slots the items use: 0 .. nslots - 1 */
  void* partials;          /* device, >= nslots * mvbev_conv_schedule_slot_bytes() */
  size_t partial_bytes;
} mvbev_conv_schedule;
size_t mvbev_conv_schedule_slot_bytes(void);
/* mvbev_conv3x3_dgrad_bf16x3_ex (split-bf16 dy only) run as scheduled (the training backward's
 * conv1 data gradient; out_mask as there). */
int mvbev_conv3x3_dgrad_bf16x3_sched(const void* dy, int dy_layout, const mvbev_conv_desc* desc,
                                     const void* w_packed, int64_t Cout_p, int dilation, void* dx, int dx_layout,
                                     const uint32_t* out_mask, int64_t cot_per_group,
                                     const mvbev_conv_schedule* sched, void* stream);

/* Weights for the data gradient of a 3x3 stride-1 conv with padding = dilation: that gradient is
 * the same conv over dy with w'[k][co][t] = w[co][k][8 - t], so mvbev_conv3x3_bf16x3_ex computes
 * it with these weights (Cout' = round_up(K_out, MVBEV_CONV_BN) output channels, K' = Cout_w).
 * Output channel o of the dgrad conv is forward input channel chan_map[o] (device int32[K_out],
 * -1 = zero; NULL = identity).  w: forward weight [Cout_w][Cin_w][3][3] fp32.  Size:
 * mvbev_conv3x3_packed_bytes_bf16x3(round_up(K_out, 128), Cout_w). */
int mvbev_pack_conv3x3_dgrad_bf16x3(const float* w, int64_t Cout_w, int64_t Cin_w,
                                    const int32_t* chan_map, int64_t K_out, void* w_packed,
                                    void* stream);

/* The data-gradient conv itself: mvbev_conv3x3_bf16x3_ex over dy (fp32, desc as for a forward
 * conv over [B][Cout_w][H][W]) with the dgrad packing, no bias / ReLU, dx in dx_layout
 * (MVBEV_LAYOUT_F32 or MVBEV_LAYOUT_SPLIT_BF16), plus an output-side mask: with out_mask
 * (device, one uint32 per output tile as group_mask of the _ex form), the tiles of output
 * channel group g (cot_per_group consecutive 128-channel Cout tiles, e.g. one camera's
 * channels) are skipped where bit g is clear — those dx entries are left unwritten, for a
 * consumer that never reads them (the warp adjoint reads a view's gradient only where the
 * view samples inside its source, which the frustum mask of mvbev_warp_tile_mask bounds). */
/* dy in dy_layout: MVBEV_LAYOUT_F32 or MVBEV_LAYOUT_SPLIT_BF16 (the LDS-DMA ring kernel, dilation 1
 * or 2; its output tiles, and so out_mask's tiles, are mvbev_conv3x3_bf16x3_tile_rows(
 * MVBEV_LAYOUT_SPLIT_BF16, dilation) rows high). */
int mvbev_conv3x3_dgrad_bf16x3_ex(const void* dy, int dy_layout, const mvbev_conv_desc* desc, const void* w_packed,
                                  int64_t Cout_p, int dilation, void* dx, int dx_layout, const uint32_t* out_mask,
                                  int64_t cot_per_group, void* stream);

/* Weight gradient of mvbev_conv3x3_bf16x3_ex (3xbf16 MFMA, fp32 accumulation):
 *   dw[co][chan_map[k]][t] = sum_b,y,x dy[b][co][y][x] * x[b][k][y + (t/3-1)d][x + (t%3-1)d]
 * x as in the forward (desc: whole image, in_row0 = out_row0 = 0, in_rows = out_rows = H;
 * x_layout MVBEV_LAYOUT_F32 or MVBEV_LAYOUT_SPLIT_BF16); dy [B][Cout][H][W] fp32 contiguous,
 * Cout % 128 == 0; dw [Cout][Cin_w][3][3] fp32 — only the channels chan_map names are written
 * (chan_map NULL = identity, K <= Cin_w).  dilation 1 or 2.  workspace: device scratch of
 * mvbev_conv3x3_wgrad_workspace_bytes() (per-partition partial sums; the reduction over
 * partitions runs in a fixed order, so the result is deterministic). */
size_t mvbev_conv3x3_wgrad_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout);
/* Optional chunk lists (both NULL = every chunk): skip the pixel chunks where an input-channel
 * group (desc->group channels, a multiple of 64: one camera's slot of the fused slab) is exactly
 * zero over the 3x3 window: chunk_list[chunk_off[g] .. chunk_off[g+1]) lists, ascending, the chunks
 * (row segments of 32 pixels, index (b * H + y) * ceil(W / 32) + x / 32) where group g can be
 * non-zero (from the frustum mask of mvbev_warp_tile_mask with halo >= dilation).  Device int32.
 * dy in dy_layout: MVBEV_LAYOUT_F32 or MVBEV_LAYOUT_SPLIT_ROWS (dy pre-split by
 * mvbev_split_rows_bf16; the LDS-DMA wgrad path only: split-bf16 x, dilation 1 or 2, W % 8 == 0,
 * else MVBEV_ERR_SHAPE) — bitwise the same dw as from the fp32 dy (the kernel splits an fp32 dy
 * with the same rounding), without the per-segment split pass.  (ABI 11600: the forms without
 * chunk lists / dy layout are retired.) */
int mvbev_conv3x3_wgrad_bf16x3_ex2(const void* x, int x_layout, const mvbev_conv_desc* desc,
                                   const void* dy, int dy_layout, int64_t Cout, int dilation,
                                   const int32_t* chan_map, int64_t Cin_w, float* dw,
                                   const int32_t* chunk_list, const int32_t* chunk_off, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* Row-Winograd weight gradient of a 3x3 conv of dilation 1 or 2 (ABI 12000; conv1 / conv2 of
 * map_classifier, persp_trans_detector.py:51, 53, whose forward ran mvbev_conv3x3_wino_bf16x3[_dil]).  With
 * the forward's y = A^T[(G w) . (B^T d)] per 3-row tile r3 (conv_bf16x3.hip), dW[co][ci][kh][kw] =
 * sum_xi G[xi][kh] M_xi[kw] where
 *   M_xi[kw][co][ci] = sum_{b, r3, x} D_xi[co][r3][x] T_xi[ci][r3][x + dil (kw - 1)],
 *   D_xi = sum_j AT[j][xi] dy[base(r3) + dil j]  (base: the forward's row tiles — 3 r3, or conv2's interleaved ones):
 * t is the forward's transform (mvbev_wino_rows_split_bf16[_dil] / the fused warp's T, t_bytes of it),
 * dy_wino is D (mvbev_wino_dy_rows_f32 of the same dilation), and the products run 3xbf16 as in
 * mvbev_conv3x3_wgrad_bf16x3_ex2, whose arguments the others mean (chunk lists: chunk (b * R3 + r3) *
 * ceil(W / 32) + x / 32 where T_xi of group g can be non-zero — the forward's 12-row frustum mask, tile
 * r3 / 4; R3 = ceil(H / 3) for dilation 1, 4 ceil(H / 12) for dilation 2).  x0.556 of the direct form's
 * MFMAs; W % 8 == 0, desc over all rows, 128-channel groups with chunk lists.  workspace:
 * mvbev_conv3x3_wgrad_wino_workspace_bytes. */
size_t mvbev_wino_dy_rows_bytes(int64_t B, int64_t Cout, int64_t H, int64_t W, int dilation);
/* D[b][xi][co][r3] (r3 < R3, rows past H zero) of fp32 dy [B][Cout][H][W] in MVBEV_LAYOUT_SPLIT_ROWS;
 * AT = [1 1 1 1 0; 0 1 -1 2 0; 0 1 1 4 1]; W % 8 == 0, 16-B aligned. */
int mvbev_wino_dy_rows_f32(const float* dy, int64_t B, int64_t Cout, int64_t H, int64_t W, int dilation,
                           void* out, size_t out_bytes, void* stream);
size_t mvbev_conv3x3_wgrad_wino_workspace_bytes(const mvbev_conv_desc* desc, int64_t Cout, int dilation);
int mvbev_conv3x3_wgrad_wino_bf16x3(const void* t, size_t t_bytes, const mvbev_conv_desc* desc, const void* dy_wino,
                                    size_t dy_wino_bytes, int64_t Cout, int dilation, const int32_t* chan_map,
                                    int64_t Cin_w, float* dw, const int32_t* chunk_list, const int32_t* chunk_off,
                                    void* workspace, size_t workspace_bytes, void* stream);

/* fp32 rows x [rows][W] (16-B aligned, W % 8 == 0) -> out [rows][W / 8] pieces of bf16 hi[8],
 * lo[8] (MVBEV_LAYOUT_SPLIT_ROWS; hi = bf16(x) round-to-nearest-even, lo = bf16(x - hi)). */
int mvbev_split_rows_bf16(const float* x, int64_t rows, int64_t W, void* out, void* stream);

/* db[co] = sum_b,p dy[b][co][p] (db may be NULL) and, when dw != NULL, the weight gradient of the
 * two coord channels (create_coord_map, persp_trans_detector.py:103-112) that are input channels
 * coord_ch, coord_ch + 1 of a conv of the given dilation: dw[co][coord_ch + j][t] (dw is
 * [Cout][Cin_w][3][3]).  dy [B][Cout][H][W] fp32. */
int mvbev_conv3x3_bias_coord_grad_f32(const float* dy, int64_t B, int64_t Cout, int64_t H, int64_t W,
                                      int dilation, float* db, float* dw, int64_t Cin_w,
                                      int64_t coord_ch, void* stream);

/* In place: dy[i] = y[i] > 0 ? dy[i] : 0 (y = the ReLU's output; torch threshold_backward). */
int mvbev_relu_backward_f32(float* dy, const float* y, int64_t n, void* stream);
/* Same with y in the split-bf16 layout (y = hi + lo; [B][C/8][H][W] pieces, C % 8 == 0) and
 * dy fp32 [B][C][H][W]; dy_split (optional, 16-B aligned) also receives the masked dy in the
 * split layout (the next data-gradient conv's input). */
int mvbev_relu_backward_split_f32(float* dy, const void* y_split, int64_t B, int64_t C, int64_t H, int64_t W,
                                  void* dy_split, void* stream);

/* Backward of mvbev_conv3x3_cout1_f32 over a whole image (x [B][C][H][W], w [C][3][3], dmap
 * [B][1][H][W] fp32):  dx[b][c][p] = sum_t w[c][t] dmap[b][p - s_t], zeroed where x <= 0 when
 * relu_mask (x is the previous ReLU's output: its backward fused); dw[c][t] = sum_b,p
 * dmap[b][p] x[b][c][p + s_t].  Any output may be NULL; dx_split (C % 8 == 0, 16-B aligned): dx
 * also in the split-bf16 layout ([B][C/8][H][W] pieces of bf16 hi[8], lo[8]), the input of the
 * next data-gradient conv. */
int mvbev_conv3x3_cout1_backward_ex(const float* x, const float* w, const float* dmap, int64_t B, int64_t C,
                                    int64_t H, int64_t W, int dilation, int relu_mask, float* dx, void* dx_split,
                                    float* dw, void* stream);

/* ---- evaluation post-processing (trainer.py:97-106, 148-157) ---- */

/* map > thres over an H x W map, in row-major (torch.nonzero) order: *count = number of hits
 * (device int32), ij[2k], ij[2k+1] = row, column and scores[k] = value of the first
 * min(count, capacity) hits.  One workgroup; enqueued, no host sync. */
int mvbev_threshold_points(const float* map, int64_t H, int64_t W, float thres, int32_t* count,
                           int32_t* ij, float* scores, int64_t capacity, void* stream);

/* Greedy point NMS of multiview_detector/utils/nms.py:7-43 for any K (trainer.py:154 passes every
 * map cell over cls_thres, up to Ho*Wo): the candidates in the order torch's CPU scores.sort(0)
 * produces (nms.py:22; libstdc++ std::sort of (score, index) pairs, NaN largest — replayed
 * exactly, so equal scores come out as on the reference's CPU, not in index order), read from
 * the end, the top_k largest considered; keep the best, drop every later candidate whose
 * distance sqrt(dx^2+dy^2) (fp32, correctly rounded) is not > dist_thres, repeat (nms.py:29-42).
 * points [K][2] fp32, scores [K] fp32 (device); keep [K] int64 = kept indices then zeros;
 * *count (device int32) = number kept.  workspace: device, >= mvbev_point_nms_workspace_bytes,
 * 4-B aligned.  One workgroup; enqueued, no host sync. */
size_t mvbev_point_nms_workspace_bytes(int64_t K, int64_t top_k);
int mvbev_point_nms_ws(const float* points, const float* scores, int64_t K, float dist_thres,
                       int64_t top_k, int64_t* keep, int32_t* count, void* workspace, size_t ws_bytes,
                       void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MVBEV_H_ */
