// Microbenchmark: cost of the primitives the commit path uses, on random addresses.
// Build: hipcc --offload-arch=gfx950 -O3 atomics.hip -o atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33; return k;
}

// mode 0: plain load; 1: atomicOr returning; 2: atomicOr no-return; 3: 64-bit CAS returning;
// 4: atomicAdd returning (small table); 5: plain load 64-bit (big table)
__global__ void k_prim(int mode, uint32_t* a32, unsigned long long* a64, uint64_t n32, uint64_t n64, uint32_t n,
                       uint32_t seed, uint32_t* sink) {
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = mix64(((uint64_t)seed << 32) | i);
    if (mode == 0) acc += a32[h % n32];
    else if (mode == 1) acc += atomicOr(a32 + h % n32, 1u << (h >> 59));
    else if (mode == 2) atomicOr(a32 + h % n32, 1u << (h >> 59));
    else if (mode == 3) acc += (uint32_t)atomicCAS(a64 + h % n64, ~0ull, h);
    else if (mode == 4) acc += atomicAdd(a32 + h % 45000, 1u);
    else if (mode == 5) acc += (uint32_t)a64[h % n64];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t n32 = 679ull << 20 >> 2, n64 = 8ull << 20;
  uint32_t *a32, *sink;
  unsigned long long* a64;
  CK(hipMalloc(&a32, n32 * 4));
  CK(hipMalloc(&a64, n64 * 8));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a32, 0, n32 * 4));
  CK(hipMemset(a64, 0xff, n64 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"load32 (679MB)", "atomicOr ret", "atomicOr noret", "CAS64 ret (64MB)", "atomicAdd ret (180KB)",
                         "load64 (64MB)"};
  for (uint32_t n : {100000u, 200000u, 1000000u}) {
    for (int grid : {256, 1024}) {
      for (int mode = 0; mode < 6; ++mode) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
          if (mode == 3) CK(hipMemset(a64, 0xff, n64 * 8));
          CK(hipEventRecord(e0));
          hipLaunchKernelGGL(k_prim, dim3(grid), dim3(256), 0, 0, mode, a32, a64, n32, n64, n, 1234u + rep, sink);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
        }
        printf("n=%7u grid=%4d %-24s %8.1f us  %6.2f G/s\n", n, grid, names[mode], best * 1e3, n / (best * 1e-3) / 1e9);
      }
    }
  }
  // empty launch
  float best = 1e9f;
  for (int rep = 0; rep < 10; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_prim, dim3(1024), dim3(256), 0, 0, 0, a32, a64, n32, n64, 0u, 1u, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("empty launch 1024 blocks: %.1f us\n", best * 1e3);
  return 0;
}
