// Is the D2H rate of a stream's copies into page-locked memory a property of the stream (the
// hardware queue / SDMA engine the runtime binds it to)?  Creates streams one after another (the
// way engines created and destroyed in one process do) and times 10 x 64 MB device -> mapped
// page-locked copies (kind DeviceToDeviceNoCU, as el_stream_result) on each, alone and beside a
// bandwidth-bound kernel on a second stream.  argv[1]: streams to try (default 12);
// argv[2] = "d": destroy each stream pair before creating the next.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_streams.hip -o scripts/micro/d2h_streams
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e));         \
      exit(1);                                              \
    }                                                       \
  } while (0)

__global__ void k_read(const uint4* __restrict__ a, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

int main(int argc, char** argv) {
  const int ns = argc > 1 ? atoi(argv[1]) : 12;
  const bool destroy = argc > 2 && argv[2][0] == 'd';
  const size_t cb = 64ull << 20, kb = 2ull << 30;
  void *d, *big, *h;
  unsigned* o;
  CK(hipMalloc(&d, cb));
  CK(hipMalloc(&big, kb));
  CK(hipMalloc(&o, 4));
  CK(hipHostMalloc(&h, cb, hipHostMallocPortable));
  CK(hipMemset(d, 0x5a, cb));
  CK(hipMemset(big, 1, kb));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, h));
  void* hd = at.devicePointer;
  for (int i = 0; i < ns; ++i) {
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    double ms[2];
    for (int busy = 0; busy < 2; ++busy) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int r = 0; r < 10; ++r) {
        if (busy) hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, s0, (const uint4*)big, kb / 16, o);
        CK(hipMemcpyAsync(hd, d, cb, hipMemcpyDeviceToDeviceNoCU, s1));
      }
      CK(hipStreamSynchronize(s1));
      ms[busy] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      CK(hipDeviceSynchronize());
    }
    printf("stream pair %2d: copies alone %6.1f GB/s, beside a kernel %6.1f GB/s\n", i, 10 * cb / ms[0] / 1e6,
           10 * cb / ms[1] / 1e6);
    fflush(stdout);
    if (destroy) {
      CK(hipStreamDestroy(s0));
      CK(hipStreamDestroy(s1));
    }
  }
  return 0;
}
