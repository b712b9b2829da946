// Sustained bf16 MFMA throughput by shape on random operands (MI355X_MICROARCH.md, DVFS
// give-back item 7): 32x32x16, 16x16x32 and the legacy 16x16x16, same output tile per wave
// (64x64 floats), operands in registers, 2 waves per SIMD, every CU busy, >= 2 s per shape
// so the chip settles at the clock it holds under that load.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_shape_bench tools/mfma_shape_bench.hip
//   ./tools/mfma_shape_bench
// or as the library bench.py loads (built by __graft_entry__.build()):
//   hipcc -O3 --offload-arch=gfx950 -fPIC -shared -DMFMA_PROBE_LIB -o mvdet_amd/lib/libmfmaprobe.so tools/mfma_shape_bench.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// each iteration: 64x64 output tile x K=32 per wave = 2*64*64*32 FLOP
__global__ __launch_bounds__(512, 1) void k32x32x16(const bf16x8* src, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a[2][2], b[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) a[i][j] = src[(t * 8 + i * 2 + j) & 65535], b[i][j] = src[(t * 8 + 4 + i * 2 + j) & 65535];
  floatx16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx16{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][k], b[j][k], acc[i][j], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[t] = s;
}

__global__ __launch_bounds__(512, 1) void k16x16x32(const bf16x8* src, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i) a[i] = src[(t * 8 + i) & 65535], b[i] = src[(t * 8 + 4 + i) & 65535];
  floatx4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 4; ++e) s += acc[i][j][e];
  out[t] = s;
}

__global__ __launch_bounds__(512, 1) void k16x16x16(const bf16x8* src, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x4 a[4][2], b[4][2];
  for (int i = 0; i < 4; ++i) {
    bf16x8 x = src[(t * 8 + i) & 65535], y = src[(t * 8 + 4 + i) & 65535];
    a[i][0] = __builtin_shufflevector(x, x, 0, 1, 2, 3);
    a[i][1] = __builtin_shufflevector(x, x, 4, 5, 6, 7);
    b[i][0] = __builtin_shufflevector(y, y, 0, 1, 2, 3);
    b[i][1] = __builtin_shufflevector(y, y, 4, 5, 6, 7);
  }
  floatx4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[i][k], b[j][k], acc[i][j], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 4; ++e) s += acc[i][j][e];
  out[t] = s;
}

// Sustained rate of one shape (0: 32x32x16, 1: 16x16x32, 2: 16x16x16) after `settle_s` seconds
// of back-to-back launches, in TFLOP/s; bench.py loads this as libmfmaprobe.so to report the
// ceiling the device holds at the time of its run beside the spec peak.
static bf16x8* g_src = nullptr;
static float* g_out = nullptr;
extern "C" double mfma_probe_tflops(int shape, double settle_s) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1.0;
  const int blocks = cus * 4, threads = 512, iters = 256;
  if (!g_src) {
    std::vector<uint16_t> h(65536 * 8);
    srand(1);
    for (auto& v : h) {
      const uint16_t mant = rand() & 0x7f, e = 126 + (rand() & 1), sgn = rand() & 1;
      v = (uint16_t)((sgn << 15) | (e << 7) | mant);
    }
    if (hipMalloc(&g_src, h.size() * 2) != hipSuccess ||
        hipMemcpy(g_src, h.data(), h.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&g_out, (size_t)blocks * threads * 4) != hipSuccess)
      return -1.0;
  }
  auto launch = [&]() {
    if (shape == 0) hipLaunchKernelGGL(k32x32x16, dim3(blocks), dim3(threads), 0, 0, g_src, g_out, iters);
    if (shape == 1) hipLaunchKernelGGL(k16x16x32, dim3(blocks), dim3(threads), 0, 0, g_src, g_out, iters);
    if (shape == 2) hipLaunchKernelGGL(k16x16x16, dim3(blocks), dim3(threads), 0, 0, g_src, g_out, iters);
  };
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < settle_s) {
    for (int i = 0; i < 10; ++i) launch();
    if (hipDeviceSynchronize() != hipSuccess) return -1.0;
  }
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1.0;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < 20; ++i) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  const double flop = 2.0 * 64 * 64 * 32 * iters * (double)blocks * (threads / 64);
  return flop / (ms / 20 * 1e-3) / 1e12;
}

#ifndef MFMA_PROBE_LIB
int main() {
  int dev = 0, cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint16_t> h(65536 * 8);
  srand(1);
  for (auto& v : h) {  // random bf16 in +-[0.5, 2): full mantissa, both signs
    const uint16_t mant = rand() & 0x7f, e = 126 + (rand() & 1), sgn = rand() & 1;
    v = (uint16_t)((sgn << 15) | (e << 7) | mant);
  }
  bf16x8* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  const int blocks = cus * 4, threads = 512;  // 8 waves per CU = 2 per SIMD, 4 blocks per CU in sequence
  CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
  const int iters = 256;
  const double flop = 2.0 * 64 * 64 * 32 * iters * (double)blocks * (threads / 64);
  const char* names[3] = {"32x32x16_bf16", "16x16x32_bf16", "16x16x16bf16_1k"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int round = 0; round < 2; ++round)
    for (int s = 0; s < 3; ++s) {
      auto launch = [&]() {
        if (s == 0) hipLaunchKernelGGL(k32x32x16, dim3(blocks), dim3(threads), 0, 0, src, out, iters);
        if (s == 1) hipLaunchKernelGGL(k16x16x32, dim3(blocks), dim3(threads), 0, 0, src, out, iters);
        if (s == 2) hipLaunchKernelGGL(k16x16x16, dim3(blocks), dim3(threads), 0, 0, src, out, iters);
      };
      // settle: ~2 s of back-to-back launches, then time 20 launches
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
        for (int i = 0; i < 10; ++i) launch();
        CHECK(hipDeviceSynchronize());
      }
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("round %d %-16s %8.3f ms/launch  %7.1f TFLOP/s\n", round, names[s], ms / 20, flop / (ms / 20 * 1e-3) / 1e12);
      fflush(stdout);
    }
  return 0;
}
#endif
