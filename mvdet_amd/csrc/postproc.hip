// Evaluation post-processing on the GPU for gfx950.
//
// Replaces the CPU loop of trainer.py:97-106,148-157:
//   map_res > cls_thres, nonzero, (frame, x, y, score) rows           -> mvbev_threshold_points
//   nms(positions, scores, dist_thres, top_k)  (utils/nms.py:7-43)     -> mvbev_point_nms
// Both are single-workgroup kernels: the data are a few thousand points per frame, so the
// cost is launch latency, not bandwidth; what matters is exact agreement with the reference
// (row-major nonzero order, the greedy NMS order, distance compared as sqrt(dx^2+dy^2) > thres
// with a correctly rounded fp32 sqrt like torch.norm).
#include "common.h"

namespace mvbev {

constexpr int kPPThreads = 1024;
constexpr int kNmsMax = 8192;

// Ordered stream compaction of map > thres (row-major, torch.nonzero order).
__global__ __launch_bounds__(kPPThreads) void threshold_kernel(const float* __restrict__ map, int n, int W,
                                                               float thres, int* __restrict__ count,
                                                               int32_t* __restrict__ ij, float* __restrict__ val,
                                                               int cap) {
  __shared__ int wave_sums[kPPThreads / 64];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int start = 0; start < n; start += kPPThreads) {
    const int i = start + tid;
    const float v = i < n ? map[i] : 0.f;
    const bool hit = i < n && v > thres;  // NaN compares false, as in torch
    const unsigned long long ball = __ballot(hit);
    const int before = __popcll(ball & ((1ull << lane) - 1ull));
    if (lane == 0) wave_sums[wave] = __popcll(ball);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wave_sums[w];
    if (hit) {
      const int o = off + before;
      if (o < cap) {
        ij[2 * o] = i / W;
        ij[2 * o + 1] = i - (i / W) * W;
        val[o] = v;
      }
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < kPPThreads / 64; ++w) t += wave_sums[w];
      base += t;
    }
    __syncthreads();
  }
  if (tid == 0) *count = base;
}

// Greedy point NMS with the reference's order: candidates by descending score, ties by
// descending index (torch's ascending sort read from the end; for exactly equal scores torch's
// CPU sort order is unspecified, this kernel's is stable), the top_k largest considered; the
// current best is kept and every later candidate within dist_thres (not strictly farther) is
// dropped.  keep[0..count) = kept indices, keep[count..K) = 0 (torch.zeros_like + writes).
__global__ __launch_bounds__(kPPThreads) void nms_kernel(const float* __restrict__ pts, const float* __restrict__ sc,
                                                         int K, int N, float thres, int top_k,
                                                         int64_t* __restrict__ keep, int* __restrict__ count) {
  __shared__ float key[kNmsMax];
  __shared__ int idx[kNmsMax];
  __shared__ unsigned char removed[kNmsMax];
  __shared__ int next_pos;
  const int tid = threadIdx.x;
  for (int i = tid; i < N; i += kPPThreads) {
    key[i] = i < K ? sc[i] : -__builtin_inff();
    idx[i] = i < K ? i : -1;
    removed[i] = 0;
  }
  __syncthreads();
  // bitonic sort, descending by (score, index)
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < N; i += kPPThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const bool a_first = key[i] > key[j] || (key[i] == key[j] && idx[i] > idx[j]);
          if (a_first != desc) {
            const float tk = key[i]; key[i] = key[j]; key[j] = tk;
            const int ti = idx[i]; idx[i] = idx[j]; idx[j] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  const int M = min(K, top_k);
  for (int i = tid; i < K; i += kPPThreads) keep[i] = 0;
  __syncthreads();
  int kept = 0, p = 0;
  while (p < M) {
    const int cur = idx[p];
    if (tid == 0) keep[kept] = cur;
    ++kept;
    const float cx = pts[2 * cur], cy = pts[2 * cur + 1];
    for (int q = p + 1 + tid; q < M; q += kPPThreads) {
      const int o = idx[q];
      const float dx = cx - pts[2 * o], dy = cy - pts[2 * o + 1];
      if (!(__fsqrt_rn(dx * dx + dy * dy) > thres)) removed[q] = 1;
    }
    if (tid == 0) next_pos = M;
    __syncthreads();
    // next surviving candidate after p
    for (int q = p + 1 + tid; q < M; q += kPPThreads)
      if (!removed[q]) atomicMin(&next_pos, q);
    __syncthreads();
    p = next_pos;
    __syncthreads();
  }
  if (tid == 0) *count = kept;
}

}  // namespace mvbev

extern "C" {

int mvbev_threshold_points(const float* map, int64_t H, int64_t W, float thres, int32_t* count,
                           int32_t* ij, float* scores, int64_t capacity, void* stream) {
  using namespace mvbev;
  if (!map || !count || (capacity > 0 && (!ij || !scores))) return MVBEV_ERR_NULL;
  if (H <= 0 || W <= 0 || capacity < 0) return MVBEV_ERR_RANK;
  if (H * W > INT32_MAX || capacity > INT32_MAX) return MVBEV_ERR_SHAPE;
  hipLaunchKernelGGL(threshold_kernel, dim3(1), dim3(kPPThreads), 0, as_stream(stream), map, (int)(H * W),
                     (int)W, thres, count, ij, scores, (int)capacity);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

int mvbev_point_nms(const float* points, const float* scores, int64_t K, float dist_thres, int64_t top_k,
                    int64_t* keep, int32_t* count, void* stream) {
  using namespace mvbev;
  if (!points || !scores || !keep || !count) return MVBEV_ERR_NULL;
  if (K <= 0 || top_k <= 0) return MVBEV_ERR_RANK;
  if (K > kNmsMax) return MVBEV_ERR_SHAPE;
  int N = 1;
  while (N < K) N <<= 1;
  hipLaunchKernelGGL(nms_kernel, dim3(1), dim3(kPPThreads), 0, as_stream(stream), points, scores, (int)K, N,
                     dist_thres, (int)std::min<int64_t>(top_k, K), keep, count);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

}  // extern "C"
