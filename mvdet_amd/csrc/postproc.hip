// Evaluation post-processing on the GPU for gfx950.
//
// Replaces the CPU loop of trainer.py:97-106,148-157:
//   map_res > cls_thres, nonzero, (frame, x, y, score) rows           -> mvbev_threshold_points
//   nms(positions, scores, dist_thres, top_k)  (utils/nms.py:7-43)     -> mvbev_point_nms
// Both are single-workgroup kernels: the data are a few thousand points per frame, so the
// cost is launch latency, not bandwidth; what matters is exact agreement with the reference
// (row-major nonzero order, the greedy NMS order, distance compared as sqrt(dx^2+dy^2) > thres
// with a correctly rounded fp32 sqrt like torch.norm).  Up to kNmsMax candidates the NMS sorts
// in LDS; above it (an untrained model can put every one of a cfg2 map's 43,200 cells over
// cls_thres, trainer.py:154) the same order and greedy loop run over a caller workspace:
// a bitonic sort in 8192-element LDS chunks plus global merge passes, then the reference's
// own shrinking candidate list (nms.py:40, indices[dists > dist_thres]) as an ordered
// compaction per kept point.
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

// Candidate o survives the current best (cx, cy): torch.norm(...) > dist_thres (nms.py:39-40).
// Not inlined, so both NMS paths evaluate it with the same instructions (contraction included).
__device__ __attribute__((noinline)) bool nms_far(float cx, float cy, const float* __restrict__ pts, int o,
                                                  float thres) {
  const float dx = cx - pts[2 * o], dy = cy - pts[2 * o + 1];
  return __fsqrt_rn(dx * dx + dy * dy) > thres;
}

// (score desc, index desc): the candidate order of both NMS paths
__device__ inline bool nms_before(float ka, int ia, float kb, int ib) {
  return ka > kb || (ka == kb && ia > ib);
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
          const bool a_first = nms_before(key[i], idx[i], key[j], idx[j]);
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
      if (!nms_far(cx, cy, pts, o, thres)) removed[q] = 1;
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

// ---- large-K path: workspace [N] key, [N] idx, [M] alternate candidate list ----
constexpr int kSortChunk = 8192;  // elements per LDS chunk (64 KiB of key + idx)

__global__ __launch_bounds__(kPPThreads) void nms_sort_init_kernel(const float* __restrict__ sc, int K, int N,
                                                                   float* __restrict__ key, int* __restrict__ idx) {
  for (int i = blockIdx.x * kPPThreads + threadIdx.x; i < N; i += gridDim.x * kPPThreads) {
    key[i] = i < K ? sc[i] : -__builtin_inff();
    idx[i] = i < K ? i : -1;
  }
}

// Bitonic stage (size, stride) with stride >= kSortChunk: one compare-exchange per pair.
__global__ __launch_bounds__(kPPThreads) void nms_sort_global_kernel(float* __restrict__ key, int* __restrict__ idx,
                                                                     int N, int size, int stride) {
  for (int i = blockIdx.x * kPPThreads + threadIdx.x; i < N; i += gridDim.x * kPPThreads) {
    const int j = i ^ stride;
    if (j <= i) continue;
    const bool desc = (i & size) == 0;
    if (nms_before(key[i], idx[i], key[j], idx[j]) != desc) {
      const float tk = key[i]; key[i] = key[j]; key[j] = tk;
      const int ti = idx[i]; idx[i] = idx[j]; idx[j] = ti;
    }
  }
}

// Bitonic stages with stride < kSortChunk inside each chunk (block c = elements
// [c * kSortChunk, (c + 1) * kSortChunk)) in LDS: sizes size_lo .. size_hi, the first size
// starting at stride first_stride, later ones at size / 2.  Direction from the global index.
__global__ __launch_bounds__(kPPThreads) void nms_sort_chunk_kernel(float* __restrict__ key, int* __restrict__ idx,
                                                                    int size_lo, int size_hi, int first_stride) {
  __shared__ float k[kSortChunk];
  __shared__ int ix[kSortChunk];
  const int tid = threadIdx.x, base = blockIdx.x * kSortChunk;
  for (int i = tid; i < kSortChunk; i += kPPThreads) {
    k[i] = key[base + i];
    ix[i] = idx[base + i];
  }
  __syncthreads();
  for (int size = size_lo; size <= size_hi; size <<= 1) {
    for (int stride = size == size_lo ? first_stride : size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < kSortChunk; i += kPPThreads) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = ((base + i) & size) == 0;
          if (nms_before(k[i], ix[i], k[j], ix[j]) != desc) {
            const float tk = k[i]; k[i] = k[j]; k[j] = tk;
            const int ti = ix[i]; ix[i] = ix[j]; ix[j] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < kSortChunk; i += kPPThreads) {
    key[base + i] = k[i];
    idx[base + i] = ix[i];
  }
}

// Greedy loop over the sorted candidates cand[0..M): keep the first, compact the others that
// are strictly farther than thres (in order) into the other list, repeat.  One workgroup.
__global__ __launch_bounds__(kPPThreads) void nms_greedy_kernel(const float* __restrict__ pts, int K, int M,
                                                                float thres, int* __restrict__ cand,
                                                                int* __restrict__ alt, int64_t* __restrict__ keep,
                                                                int* __restrict__ count) {
  __shared__ int wave_sums[kPPThreads / 64];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < K; i += kPPThreads) keep[i] = 0;
  int* cur_list = cand;
  int* next_list = alt;
  int n = M, kept = 0;
  while (n > 0) {
    __syncthreads();  // keep[] zeroed / every thread has read the previous round's base
    const int cur = cur_list[0];
    if (tid == 0) {
      keep[kept] = cur;
      base = 0;
    }
    ++kept;
    const float cx = pts[2 * cur], cy = pts[2 * cur + 1];
    __syncthreads();
    for (int start = 1; start < n; start += kPPThreads) {
      const int q = start + tid;
      const int o = q < n ? cur_list[q] : 0;
      const bool hit = q < n && nms_far(cx, cy, pts, o, thres);
      const unsigned long long ball = __ballot(hit);
      const int before = __popcll(ball & ((1ull << lane) - 1ull));
      if (lane == 0) wave_sums[wave] = __popcll(ball);
      __syncthreads();
      int off = base;
      for (int w = 0; w < wave; ++w) off += wave_sums[w];
      if (hit) next_list[off + before] = o;
      __syncthreads();
      if (tid == 0) {
        int t = 0;
        for (int w = 0; w < kPPThreads / 64; ++w) t += wave_sums[w];
        base += t;
      }
      __syncthreads();
    }
    n = base;
    int* t = cur_list;
    cur_list = next_list;
    next_list = t;
  }
  if (tid == 0) *count = kept;
}

static int64_t nms_pow2(int64_t K) {
  int64_t N = kSortChunk;
  while (N < K) N <<= 1;
  return N;
}

}  // namespace mvbev

extern "C" {

size_t mvbev_point_nms_workspace_bytes(int64_t K, int64_t top_k) {
  using namespace mvbev;
  if (K <= kNmsMax || top_k <= 0) return 0;
  const int64_t N = nms_pow2(K), M = std::min(K, top_k);
  return (size_t)(N * (int64_t)(sizeof(float) + sizeof(int)) + M * (int64_t)sizeof(int));
}

int mvbev_point_nms_ws(const float* points, const float* scores, int64_t K, float dist_thres, int64_t top_k,
                       int64_t* keep, int32_t* count, void* workspace, size_t ws_bytes, void* stream) {
  using namespace mvbev;
  if (K <= kNmsMax) return mvbev_point_nms(points, scores, K, dist_thres, top_k, keep, count, stream);
  if (!points || !scores || !keep || !count || !workspace) return MVBEV_ERR_NULL;
  if (top_k <= 0) return MVBEV_ERR_RANK;
  if (K > ((int64_t)1 << 28)) return MVBEV_ERR_SHAPE;
  if (ws_bytes < mvbev_point_nms_workspace_bytes(K, top_k)) return MVBEV_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(workspace) % 4) return MVBEV_ERR_ALIGN;
  const int N = (int)nms_pow2(K), M = (int)std::min<int64_t>(K, top_k);
  float* key = static_cast<float*>(workspace);
  int* idx = reinterpret_cast<int*>(key + N);
  int* alt = idx + N;
  hipStream_t st = as_stream(stream);
  const int grid = std::min(N / kPPThreads, 1024);
  hipLaunchKernelGGL(nms_sort_init_kernel, dim3(grid), dim3(kPPThreads), 0, st, scores, (int)K, N, key, idx);
  hipLaunchKernelGGL(nms_sort_chunk_kernel, dim3(N / kSortChunk), dim3(kPPThreads), 0, st, key, idx, 2,
                     kSortChunk, 1);
  for (int size = 2 * kSortChunk; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride >= kSortChunk; stride >>= 1)
      hipLaunchKernelGGL(nms_sort_global_kernel, dim3(grid), dim3(kPPThreads), 0, st, key, idx, N, size, stride);
    hipLaunchKernelGGL(nms_sort_chunk_kernel, dim3(N / kSortChunk), dim3(kPPThreads), 0, st, key, idx, size, size,
                       kSortChunk / 2);
  }
  // candidate list = the first M sorted indices (the top_k largest, nms.py:30-31)
  hipLaunchKernelGGL(nms_greedy_kernel, dim3(1), dim3(kPPThreads), 0, st, points, (int)K, M, dist_thres, idx, alt,
                     keep, count);
  MVBEV_CHECK_LAUNCH();
  return MVBEV_OK;
}

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
