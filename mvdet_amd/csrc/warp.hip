// Homography warp (kornia 0.6.11 warp_perspective semantics) for gfx950.
//
// Replaces kornia.geometry.transform.warp_perspective at
// multiview_detector/models/persp_trans_detector.py:69 and, through the dst
// strides, the torch.cat at :77 (each view writes straight into its channel slice
// of the fused ground-plane tensor).
//
// Per output pixel (u = col, v = row) of batch b:
//   g   = kornia create_meshgrid (normalised):  gx = (u/(Wo-1) - 0.5)*2, gy likewise
//   p   = M_b @ [gx, gy, 1]            (M_b = src_norm <- dst_norm, fp32, from the host)
//   s   = |p.z| > 1e-8 ? 1/(p.z + 1e-8) : 1;  (x, y) = s * (p.x, p.y)   (no z>0 mask)
//   ix  = ((x+1)/2)*(W-1), iy = ((y+1)/2)*(H-1)          (GridSampler.h:31, align_corners)
//   out = sum over the 4 in-bounds corners of src * bilinear weight    (zeros padding)
//
// Kernel shape: one thread per output pixel; the pixel's coordinates, corner offsets and
// weights are computed once and reused across the block's channel slice (the dominant
// traffic is the C-deep gather + the C-deep store, both per channel plane).  Stores are
// fully coalesced along u; loads follow the projected source line of the 64 lanes.
#include "common.h"

namespace mvbev {

template <typename T, int UNROLL>
__global__ __launch_bounds__(256) void warp_perspective_kernel(
    const T* __restrict__ src, int64_t sB, int64_t sC, int64_t sH, int64_t sW, int C, int H, int W,
    const float* __restrict__ m, T* __restrict__ dst, int64_t dB, int64_t dC, int64_t dH, int Ho,
    int Wo, int c_per_block) {
  const int b = blockIdx.z;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= Ho * Wo) return;
  const int v = p / Wo;
  const int u = p - v * Wo;
  const int c_begin = blockIdx.y * c_per_block;
  const int c_end = min(C, c_begin + c_per_block);

  // kornia create_meshgrid(normalized_coordinates=True); same fp32 op order.
  const float gx = ((float)u / (float)(Wo - 1) - 0.5f) * 2.0f;
  const float gy = ((float)v / (float)(Ho - 1) - 0.5f) * 2.0f;
  const float* mb = m + 9 * b;
  // transform_points: [gx gy 1] @ M^T, then convert_points_from_homogeneous(eps=1e-8)
  float x = gx * mb[0] + gy * mb[1] + mb[2];
  float y = gx * mb[3] + gy * mb[4] + mb[5];
  const float z = gx * mb[6] + gy * mb[7] + mb[8];
  const float scale = fabsf(z) > 1e-8f ? 1.0f / (z + 1e-8f) : 1.0f;
  x = scale * x;
  y = scale * y;
  // grid_sampler_unnormalize(align_corners=True)
  const float ix = ((x + 1.f) / 2.f) * (float)(W - 1);
  const float iy = ((y + 1.f) / 2.f) * (float)(H - 1);

  T* out = dst + (int64_t)b * dB + (int64_t)v * dH + u;
  // Non-finite sample position (kornia's 0/0 meshgrid when Ho or Wo is 1, or an inf
  // after the divide): torch's bilinear weights become NaN, so every channel is NaN.
  // Otherwise, no corner in bounds -> zeros padding.
  const bool finite = isfinite(ix) && isfinite(iy);
  if (!finite || !(ix > -1.f && ix < (float)W && iy > -1.f && iy < (float)H)) {
    const float fill = finite ? 0.f : __builtin_nanf("");
    for (int c = c_begin; c < c_end; ++c) out[(int64_t)c * dC] = from_f32<T>(fill);
    return;
  }
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  // torch GridSampler bilinear weights (nw, ne, sw, se)
  const float w_nw = (fx1 - ix) * (fy1 - iy);
  const float w_ne = (ix - fx0) * (fy1 - iy);
  const float w_sw = (fx1 - ix) * (iy - fy0);
  const float w_se = (ix - fx0) * (iy - fy0);
  const bool vx0 = x0 >= 0, vx1 = x0 + 1 <= W - 1, vy0 = y0 >= 0, vy1 = y0 + 1 <= H - 1;
  const bool ok_nw = vx0 && vy0, ok_ne = vx1 && vy0, ok_sw = vx0 && vy1, ok_se = vx1 && vy1;
  // Offsets of the 4 corners; invalid corners point at a safe in-bounds pixel and
  // their value is replaced by 0 (select, not multiply: keeps inf/NaN semantics).
  const int cx0 = max(x0, 0), cy0 = max(y0, 0);
  const int cx1 = min(x0 + 1, W - 1), cy1 = min(y0 + 1, H - 1);
  const int64_t o_nw = cy0 * sH + cx0 * sW, o_ne = cy0 * sH + cx1 * sW;
  const int64_t o_sw = cy1 * sH + cx0 * sW, o_se = cy1 * sH + cx1 * sW;

  const T* base = src + (int64_t)b * sB;
  int c = c_begin;
  for (; c + UNROLL <= c_end; c += UNROLL) {
    float vnw[UNROLL], vne[UNROLL], vsw[UNROLL], vse[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const T* pc = base + (int64_t)(c + k) * sC;
      vnw[k] = to_f32<T>(pc[o_nw]);
      vne[k] = to_f32<T>(pc[o_ne]);
      vsw[k] = to_f32<T>(pc[o_sw]);
      vse[k] = to_f32<T>(pc[o_se]);
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      float acc = 0.f;
      acc += (ok_nw ? vnw[k] : 0.f) * w_nw;
      acc += (ok_ne ? vne[k] : 0.f) * w_ne;
      acc += (ok_sw ? vsw[k] : 0.f) * w_sw;
      acc += (ok_se ? vse[k] : 0.f) * w_se;
      out[(int64_t)(c + k) * dC] = from_f32<T>(acc);
    }
  }
  for (; c < c_end; ++c) {
    const T* pc = base + (int64_t)c * sC;
    float acc = 0.f;
    acc += (ok_nw ? to_f32<T>(pc[o_nw]) : 0.f) * w_nw;
    acc += (ok_ne ? to_f32<T>(pc[o_ne]) : 0.f) * w_ne;
    acc += (ok_sw ? to_f32<T>(pc[o_sw]) : 0.f) * w_sw;
    acc += (ok_se ? to_f32<T>(pc[o_se]) : 0.f) * w_se;
    out[(int64_t)c * dC] = from_f32<T>(acc);
  }
}

template <typename T>
static int launch_warp(const T* src, int64_t B, int64_t C, int64_t H, int64_t W,
                       const int64_t* ss, const float* m, T* dst, int64_t Ho, int64_t Wo,
                       const int64_t* ds, void* stream) {
  if (!src || !m || !dst || !ss || !ds) return MVBEV_ERR_NULL;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return MVBEV_ERR_RANK;
  if (ds[3] != 1) return MVBEV_ERR_STRIDE;
  if (Ho * Wo > (int64_t)INT32_MAX || B > 65535 || H > INT32_MAX / 2 || W > INT32_MAX / 2)
    return MVBEV_ERR_SHAPE;
  const int cpb = 64;
  dim3 grid((unsigned)ceil_div(Ho * Wo, 256), (unsigned)ceil_div(C, cpb), (unsigned)B);
  hipLaunchKernelGGL((warp_perspective_kernel<T, 4>), grid, dim3(256), 0, as_stream(stream), src,
                     ss[0], ss[1], ss[2], ss[3], (int)C, (int)H, (int)W, m, dst, ds[0], ds[1],
                     ds[2], (int)Ho, (int)Wo, cpb);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
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

}  // namespace mvbev

extern "C" {

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

int mvbev_version(void) { return 10000; }

int mvbev_warp_perspective_f32(const float* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m, float* dst,
                               int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream) {
  return mvbev::launch_warp<float>(src, B, C, H, W, src_strides, m, dst, Ho, Wo, dst_strides,
                                   stream);
}

int mvbev_warp_perspective_f16(const void* src, int64_t B, int64_t C, int64_t H, int64_t W,
                               const int64_t src_strides[4], const float* m, void* dst,
                               int64_t Ho, int64_t Wo, const int64_t dst_strides[4],
                               void* stream) {
  return mvbev::launch_warp<__half>(static_cast<const __half*>(src), B, C, H, W, src_strides, m,
                                    static_cast<__half*>(dst), Ho, Wo, dst_strides, stream);
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
