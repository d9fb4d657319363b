// Microbenchmark: launch cost vs grid size and kernarg size, back-to-back in one stream.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Big { uint64_t w[80]; };  // 640 B of kernel arguments

__global__ void k_empty(uint32_t* sink, uint32_t v) { if (v == 0x1234567u) sink[0] = v; }
__global__ void k_big(Big b, uint32_t* sink) { if (b.w[threadIdx.x & 63] == 0x1234567u) sink[0] = 1; }
__global__ void k_lds(uint32_t* sink, uint32_t v) {
  __shared__ uint32_t s[5000];
  s[threadIdx.x] = v;
  __syncthreads();
  if (s[(threadIdx.x + 1) & 255] == 0x1234567u) sink[0] = v;
}

int main() {
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Big b{};
  for (int kind = 0; kind < 3; ++kind) {
    for (int grid : {1, 64, 256, 1024, 2048, 4096}) {
      const int reps = 200;
      float best = 1e9f;
      for (int trial = 0; trial < 3; ++trial) {
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) {
          if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, sink, 1u);
          else if (kind == 1) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, st, b, sink);
          else hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, st, sink, 1u);
        }
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("%-10s grid=%5d  %.2f us per launch (back-to-back)\n", kind == 0 ? "empty" : kind == 1 ? "kernarg640" : "lds20k",
             grid, best * 1e3 / reps);
    }
  }
  // host round trip: launch + stream sync
  float tot = 0;
  for (int r = 0; r < 100; ++r) {
    auto t0 = hipEventRecord(e0, st);
    (void)t0;
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, sink, 1u);
    CK(hipStreamSynchronize(st));
  }
  printf("done\n");
  return 0;
}
