// Evaluation post-processing on the GPU for gfx950.
//
// Replaces the CPU loop of trainer.py:97-106,148-157:
//   map_res > cls_thres, nonzero, (frame, x, y, score) rows           -> mvbev_threshold_points
//   nms(positions, scores, dist_thres, top_k)  (utils/nms.py:7-43)     -> mvbev_point_nms
// Both are single-workgroup kernels: the data are a few thousand points per frame (an untrained
// model can put all 43,200 cells of a cfg2 map over cls_thres, trainer.py:154), so the cost is
// latency, not bandwidth; what matters is exact agreement with the reference: row-major nonzero
// order; the NMS candidate order of torch's CPU scores.sort(0) including equal scores
// (torch_cpu_sort below replays libstdc++'s introsort); the reference's own shrinking candidate
// list (nms.py:40, indices[dists > dist_thres]) as an ordered compaction per kept point; the
// distance compared as sqrt(dx^2+dy^2) > thres with a correctly rounded fp32 sqrt like torch.norm.
#include "common.h"

namespace mvbev {

constexpr int kPPThreads = 1024;

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
__device__ __attribute__((noinline)) bool nms_far(float cx, float cy, const float* __restrict__ pts, int o,
                                                  float thres) {
  const float dx = cx - pts[2 * o], dy = cy - pts[2 * o + 1];
  return __fsqrt_rn(dx * dx + dy * dy) > thres;
}

// ---- the candidate order: torch's CPU sort, restated ----------------------------------------
// nms.py:22 orders the candidates with scores.sort(0) (ascending) and walks it from the end.  On
// the CPU, torch sorts (value, index) pairs with std::sort under KeyValueCompAsc (NaN largest),
// i.e. libstdc++'s introsort: median-of-three pivot moved to the front, Hoare's unguarded
// partition, recursion while a range holds more than 16 elements with a depth limit of
// 2 floor(log2 n) (past it: heap sort), then one insertion sort.  Equal scores come out in the
// order that process leaves them, not in index order, so the kept set of an NMS over tied scores
// depends on it.  This kernel replays the same introsort exactly, level by level: every range
// of one recursion depth is partitioned at once by the whole workgroup.  A Hoare partition of
// [f + 1, l) around p swaps the k-th element >= p from the left with the k-th element <= p from
// the right for k = 1 .. m, m = max_x min(#left stops before x, #right stops from x), and returns
// cut = L_1 (m = 0), else min(L_{m+1}, R_m) — prefix counts, a scatter and a max per range, so
// the result is the sequential algorithm's (oracle/postproc.py restates both forms; tests pin
// them against torch.sort).  The final insertion sort is a stable sort, and the ranges come out
// ordered, so it runs per range.
__device__ inline bool sort_lt(float a, float b) { return (!isnan(a) && isnan(b)) || a < b; }

struct SortWs {
  float* key;
  int *idx, *segof, *len, *depth, *act, *m, *totL, *totR, *cut, *posL, *posR, *incL, *incR;
};

__device__ inline void pair_swap(const SortWs& w, int i, int j) {
  const float tk = w.key[i]; w.key[i] = w.key[j]; w.key[j] = tk;
  const int ti = w.idx[i]; w.idx[i] = w.idx[j]; w.idx[j] = ti;
}

// libstdc++ __adjust_heap / __push_heap over [f, f + len) (one thread)
__device__ void heap_adjust(const SortWs& w, int f, int hole, int len, float vk, int vi) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (sort_lt(w.key[f + second], w.key[f + second - 1])) --second;
    w.key[f + hole] = w.key[f + second];
    w.idx[f + hole] = w.idx[f + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    w.key[f + hole] = w.key[f + second - 1];
    w.idx[f + hole] = w.idx[f + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && sort_lt(w.key[f + parent], vk)) {
    w.key[f + hole] = w.key[f + parent];
    w.idx[f + hole] = w.idx[f + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  w.key[f + hole] = vk;
  w.idx[f + hole] = vi;
}

// __partial_sort(first, last, last) = __make_heap + __sort_heap (the depth-limit fallback)
__device__ void heap_sort_range(const SortWs& w, int f, int l) {
  const int len = l - f;
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      heap_adjust(w, f, parent, len, w.key[f + parent], w.idx[f + parent]);
      if (parent == 0) break;
    }
  }
  for (int last = l; last - f > 1;) {
    --last;
    const float vk = w.key[last];
    const int vi = w.idx[last];
    w.key[last] = w.key[f];
    w.idx[last] = w.idx[f];
    heap_adjust(w, f, 0, last - f, vk, vi);
  }
}

// segmented inclusive scan of (flag, value) pairs over the workgroup's 1024 chunk summaries
__device__ inline void seg_scan_pair(int& flag, int& a, int& b, int* sf, int* sa, int* sb) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int f2 = __shfl_up(flag, off), a2 = __shfl_up(a, off), b2 = __shfl_up(b, off);
    if (lane >= off && !flag) {
      a += a2;
      b += b2;
      flag = f2;
    }
  }
  if (lane == 63) {
    sf[wave] = flag;
    sa[wave] = a;
    sb[wave] = b;
  }
  __syncthreads();
  if (wave == 0) {  // scan of the 16 wave totals
    int f = lane < kPPThreads / 64 ? sf[lane] : 1, x = lane < kPPThreads / 64 ? sa[lane] : 0,
        y = lane < kPPThreads / 64 ? sb[lane] : 0;
#pragma unroll
    for (int off = 1; off < kPPThreads / 64; off <<= 1) {
      const int f2 = __shfl_up(f, off), x2 = __shfl_up(x, off), y2 = __shfl_up(y, off);
      if (lane >= off && !f) {
        x += x2;
        y += y2;
        f = f2;
      }
    }
    if (lane < kPPThreads / 64) {
      sf[lane] = f;
      sa[lane] = x;
      sb[lane] = y;
    }
  }
  __syncthreads();
  if (wave > 0 && !flag) {  // add the preceding waves' carry
    a += sa[wave - 1];
    b += sb[wave - 1];
    flag = sf[wave - 1];
  }
}

// Introsort replica over w.key / w.idx [0, K) (one workgroup of kPPThreads threads).
__device__ void torch_cpu_sort(const SortWs& w, int K) {
  __shared__ int sf[kPPThreads / 64], sa[kPPThreads / 64], sb[kPPThreads / 64];
  __shared__ int any_active;
  __shared__ int carry_l[kPPThreads], carry_r[kPPThreads];
  const int tid = threadIdx.x;
  const int chunk = (K + kPPThreads - 1) / kPPThreads;
  const int c0 = min(K, tid * chunk), c1 = min(K, c0 + chunk);
  int lg = 0;
  while ((2 << lg) <= K) ++lg;  // floor(log2 K)
  for (int i = c0; i < c1; ++i) {
    w.segof[i] = 0;
    w.len[i] = 0;
    w.act[i] = 0;
  }
  if (tid == 0) {
    w.len[0] = K;
    w.depth[0] = 2 * lg;
  }
  __syncthreads();
  // every active range's children have depth d - 1 and depth-0 ranges are heap-sorted, so the
  // loop ends within 2 floor(log2 K) + 1 levels
  for (int level = 0; level <= 2 * lg + 1; ++level) {
    // A: per range (its head's thread): final / heap fallback / median of three to the front
    if (tid == 0) any_active = 0;
    __syncthreads();
    bool mine_active = false;
    for (int f = c0; f < c1; ++f) {
      if (w.segof[f] != f || w.depth[f] < 0) continue;
      const int l = f + w.len[f];
      w.act[f] = 0;
      if (l - f <= 16) {
        w.depth[f] = -1;  // insertion sort at the end
      } else if (w.depth[f] == 0) {
        heap_sort_range(w, f, l);
        w.depth[f] = -2;  // sorted
      } else {
        const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
        const float ka = w.key[a], kb = w.key[b], kc = w.key[c];
        int pick;
        if (sort_lt(ka, kb)) pick = sort_lt(kb, kc) ? b : (sort_lt(ka, kc) ? c : a);
        else pick = sort_lt(ka, kc) ? a : (sort_lt(kb, kc) ? c : b);
        pair_swap(w, f, pick);
        w.act[f] = 1;
        w.m[f] = 0;
        mine_active = true;
      }
    }
    if (mine_active) any_active = 1;  // benign same-value race
    __syncthreads();
    if (!any_active) break;
    // B1: per chunk, left / right stop counts since the chunk's last range head
    int hf = 0, cl = 0, cr = 0;
    for (int i = c0; i < c1; ++i) {
      const int s = w.segof[i];
      if (s == i) {
        hf = 1;
        cl = cr = 0;
        continue;
      }
      if (!w.act[s]) continue;
      const float p = w.key[s], v = w.key[i];
      cl += !sort_lt(v, p);
      cr += !sort_lt(p, v);
    }
    seg_scan_pair(hf, cl, cr, sf, sa, sb);
    // exclusive carry into this chunk: the inclusive value of chunk tid - 1
    carry_l[tid] = cl;
    carry_r[tid] = cr;
    __syncthreads();
    int rl = tid > 0 ? carry_l[tid - 1] : 0, rr = tid > 0 ? carry_r[tid - 1] : 0;
    // B2: inclusive counts per element; range totals at each range's last element
    for (int i = c0; i < c1; ++i) {
      const int s = w.segof[i];
      if (s == i) {
        rl = rr = 0;
        continue;
      }
      if (!w.act[s]) continue;
      const float p = w.key[s], v = w.key[i];
      rl += !sort_lt(v, p);
      rr += !sort_lt(p, v);
      w.incL[i] = rl;
      w.incR[i] = rr;
      if (i == s + w.len[s] - 1) {
        w.totL[s] = rl;
        w.totR[s] = rr;
      }
    }
    __syncthreads();
    // B3: k-th left stop -> posL[s + k], k-th right stop from the right -> posR[s + k]; m
    for (int i = c0; i < c1; ++i) {
      const int s = w.segof[i];
      if (s == i || !w.act[s]) continue;
      const float p = w.key[s], v = w.key[i];
      const int il = w.incL[i], ir = w.incR[i], tr = w.totR[s];
      if (!sort_lt(v, p)) w.posL[s + il] = i;
      if (!sort_lt(p, v)) w.posR[s + (tr - ir + 1)] = i;
      const int c = min(il, tr - ir);
      if (c > 0) atomicMax(&w.m[s], c);
    }
    __syncthreads();
    // C: the partition's swaps, pair k = (posL[s + k], posR[s + k]) for k = 1 .. m
    for (int j = c0; j < c1; ++j) {
      const int s = w.segof[j];
      if (!w.act[s]) continue;
      const int k = j - s;
      if (k >= 1 && k <= w.m[s]) pair_swap(w, w.posL[j], w.posR[j]);
    }
    __syncthreads();
    // D: the cut, and the two child ranges
    for (int f = c0; f < c1; ++f) {
      if (w.segof[f] != f || !w.act[f]) continue;
      const int m = w.m[f], l = f + w.len[f];
      int cut;
      if (m == 0) {
        cut = w.posL[f + 1];
      } else {
        cut = w.posR[f + m];
        if (m < w.totL[f] && w.posL[f + m + 1] < cut) cut = w.posL[f + m + 1];
      }
      const int d = w.depth[f] - 1;
      w.cut[f] = cut;
      w.len[f] = cut - f;
      w.len[cut] = l - cut;
      w.depth[f] = d;
      w.depth[cut] = d;
    }
    __syncthreads();
    // E: elements right of the cut join the new range
    for (int i = c0; i < c1; ++i) {
      const int s = w.segof[i];
      if (w.act[s] && i >= w.cut[s]) w.segof[i] = w.cut[s];
    }
    __syncthreads();
  }
  // final insertion sort per range (stable, strict <), skipping heap-sorted ranges
  for (int f = c0; f < c1; ++f) {
    if (w.segof[f] != f || w.depth[f] != -1) continue;
    const int l = f + w.len[f];
    for (int i = f + 1; i < l; ++i) {
      const float vk = w.key[i];
      const int vi = w.idx[i];
      int j = i;
      while (j > f && sort_lt(vk, w.key[j - 1])) {
        w.key[j] = w.key[j - 1];
        w.idx[j] = w.idx[j - 1];
        --j;
      }
      w.key[j] = vk;
      w.idx[j] = vi;
    }
  }
  __syncthreads();
}

// Greedy loop over the sorted candidates cand[0..M): keep the first, compact the others that
// are strictly farther than thres (in order) into the other list, repeat.  One workgroup.
__device__ void nms_greedy(const float* __restrict__ pts, int K, int M, float thres, int* cand, int* alt,
                           int64_t* __restrict__ keep, int* __restrict__ count) {
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

// nms.py:7-43 in one workgroup: the candidate order of scores.sort(0) (torch_cpu_sort), its
// top_k largest from the end, then the greedy loop.
__global__ __launch_bounds__(kPPThreads) void point_nms_kernel(const float* __restrict__ pts,
                                                               const float* __restrict__ sc, int K, int M,
                                                               float thres, SortWs w, int* cand, int* alt,
                                                               int64_t* __restrict__ keep, int* __restrict__ count) {
  for (int i = threadIdx.x; i < K; i += kPPThreads) {
    w.key[i] = sc[i];
    w.idx[i] = i;
  }
  __syncthreads();
  torch_cpu_sort(w, K);
  for (int j = threadIdx.x; j < M; j += kPPThreads) cand[j] = w.idx[K - 1 - j];  // indices[-top_k:], last first
  __syncthreads();
  nms_greedy(pts, K, M, thres, cand, alt, keep, count);
}

constexpr int kSortArrays = 14;  // 4-byte arrays of K entries in the workspace: key + SortWs's 13 int arrays

}  // namespace mvbev

extern "C" {

size_t mvbev_point_nms_workspace_bytes(int64_t K, int64_t top_k) {
  using namespace mvbev;
  if (K <= 0 || top_k <= 0) return 0;
  const int64_t M = std::min(K, top_k);
  return (size_t)((kSortArrays * K + 2 * M) * (int64_t)sizeof(int));
}

int mvbev_point_nms_ws(const float* points, const float* scores, int64_t K, float dist_thres, int64_t top_k,
                       int64_t* keep, int32_t* count, void* workspace, size_t ws_bytes, void* stream) {
  using namespace mvbev;
  if (!points || !scores || !keep || !count || !workspace) return MVBEV_ERR_NULL;
  if (K <= 0 || top_k <= 0) return MVBEV_ERR_RANK;
  if (K > ((int64_t)1 << 26)) return MVBEV_ERR_SHAPE;
  if (ws_bytes < mvbev_point_nms_workspace_bytes(K, top_k)) return MVBEV_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(workspace) % 4) return MVBEV_ERR_ALIGN;
  const int M = (int)std::min<int64_t>(K, top_k);
  int* p = static_cast<int*>(workspace);
  SortWs w;
  w.key = reinterpret_cast<float*>(p);
  int** arrays[] = {&w.idx, &w.segof, &w.len, &w.depth, &w.act, &w.m, &w.totL, &w.totR, &w.cut, &w.posL, &w.posR,
                    &w.incL, &w.incR};
  static_assert(sizeof(arrays) / sizeof(arrays[0]) == kSortArrays - 1, "workspace arrays");
  for (int a = 0; a < kSortArrays - 1; ++a) *arrays[a] = p + (int64_t)(a + 1) * K;
  int* cand = p + (int64_t)kSortArrays * K;
  int* alt = cand + M;
  hipLaunchKernelGGL(point_nms_kernel, dim3(1), dim3(kPPThreads), 0, as_stream(stream), points, scores, (int)K, M,
                     dist_thres, w, cand, alt, keep, count);
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

}  // extern "C"
