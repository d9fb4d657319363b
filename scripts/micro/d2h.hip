// D2H copy-back microbenchmark: pinned-host hipMemcpyAsync rate, and how much a concurrent
// memory-bound kernel slows down beside it (blit-kernel copies share the CUs; SDMA does not).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r)); exit(1); } } while (0)

__global__ void stream_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i];
    v.x += 1;
    b[i] = v;
  }
}

int main() {
  const size_t bytes = 512ull << 20, sb = 1ull << 30;
  void *d, *h, *sa, *sbuf;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 1, bytes));
  CK(hipHostMalloc(&h, bytes, hipHostMallocPortable));
  CK(hipMalloc(&sa, sb));
  CK(hipMalloc(&sbuf, sb));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, k0, k1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&k0)); CK(hipEventCreate(&k1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, s1));
    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1));
    CK(hipEventRecord(e1, s1));
    CK(hipStreamSynchronize(s1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    // kernel alone
    CK(hipEventRecord(k0, s2));
    stream_kernel<<<2048, 256, 0, s2>>>((const uint4*)sa, (uint4*)sbuf, sb / 16);
    CK(hipEventRecord(k1, s2));
    CK(hipStreamSynchronize(s2));
    float kms; CK(hipEventElapsedTime(&kms, k0, k1));
    // both
    CK(hipEventRecord(e0, s1));
    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1));
    CK(hipEventRecord(e1, s1));
    CK(hipEventRecord(k0, s2));
    for (int i = 0; i < 8; ++i) stream_kernel<<<2048, 256, 0, s2>>>((const uint4*)sa, (uint4*)sbuf, sb / 16);
    CK(hipEventRecord(k1, s2));
    CK(hipDeviceSynchronize());
    float ms2, kms2; CK(hipEventElapsedTime(&ms2, e0, e1)); CK(hipEventElapsedTime(&kms2, k0, k1));
    printf("d2h %.2f ms = %.1f GB/s | kernel alone %.3f ms (%.0f GB/s) | together: d2h %.2f ms, 8 kernels %.3f ms (%.3f each)\n",
           ms, bytes / ms / 1e6, kms, 2.0 * sb / kms / 1e6, ms2, kms2, kms2 / 8);
  }
  return 0;
}
