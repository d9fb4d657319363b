// D2H copy engine check: does hipMemcpyAsync into page-locked host memory run as a shader blit
// (CUs) or on a copy engine, and how much does it slow a bandwidth-bound kernel beside it?
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_engine.hip -o scripts/micro/d2h_engine
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_read(const uint4* __restrict__ a, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

// zero-copy push: a few workgroups store device data straight into mapped page-locked host
// memory (vector stores over PCIe), so the transfer occupies `grid` workgroups, not a blit grid
__global__ void k_push(const uint4* __restrict__ a, uint4* __restrict__ h, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    h[i] = a[i];
}

int main() {
  const size_t cb = 512ull << 20, kb = 4ull << 30;
  void *d, *big, *h;
  unsigned* o;
  CK(hipMalloc(&d, cb));
  CK(hipMalloc(&big, kb));
  CK(hipMalloc(&o, 4));
  CK(hipHostMalloc(&h, cb, hipHostMallocPortable));
  CK(hipMemset(d, 0x5a, cb));
  CK(hipMemset(big, 1, kb));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  auto kern = [&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, s0, (const uint4*)big, kb / 16, o); };
  auto copy = [&](hipMemcpyKind k) { CK(hipMemcpyAsync(h, d, cb, k, s1)); };
  for (int w = 0; w < 2; ++w) {
    kern();
    copy(hipMemcpyDeviceToHost);
    CK(hipDeviceSynchronize());
  }
  float ms;
  struct M {
    const char* name;
    hipMemcpyKind k;
  } modes[] = {{"DeviceToHost", hipMemcpyDeviceToHost}, {"DeviceToDeviceNoCU", hipMemcpyDeviceToDeviceNoCU},
               {"Default", hipMemcpyDefault}};
  // kernel alone
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(a0, s0));
    kern();
    CK(hipEventRecord(a1, s0));
    CK(hipDeviceSynchronize());
    CK(hipEventElapsedTime(&ms, a0, a1));
    printf("kernel alone: %.3f ms (%.0f GB/s)\n", ms, kb / ms / 1e6);
  }
  for (auto& m : modes) {
    memset(h, 0, cb);
    hipError_t e = hipMemcpyAsync(h, d, cb, m.k, s1);
    if (e != hipSuccess) {
      printf("%s: %s\n", m.name, hipGetErrorString(e));
      (void)hipGetLastError();
      continue;
    }
    CK(hipDeviceSynchronize());
    printf("%s: data %s\n", m.name, ((unsigned char*)h)[cb - 1] == 0x5a ? "ok" : "WRONG");
    for (int r = 0; r < 2; ++r) {
      CK(hipEventRecord(b0, s1));
      copy(m.k);
      CK(hipEventRecord(b1, s1));
      CK(hipDeviceSynchronize());
      CK(hipEventElapsedTime(&ms, b0, b1));
      printf("%s alone: %.3f ms (%.1f GB/s)\n", m.name, ms, cb / ms / 1e6);
    }
    for (int r = 0; r < 2; ++r) {
      CK(hipEventRecord(b0, s1));
      copy(m.k);
      CK(hipEventRecord(b1, s1));
      CK(hipEventRecord(a0, s0));
      for (int i = 0; i < 8; ++i) kern();
      CK(hipEventRecord(a1, s0));
      CK(hipDeviceSynchronize());
      float kms;
      CK(hipEventElapsedTime(&kms, a0, a1));
      CK(hipEventElapsedTime(&ms, b0, b1));
      printf("%s beside 8 kernels: copy %.3f ms, kernels %.3f ms (%.3f each)\n", m.name, ms, kms, kms / 8);
    }
  }
  uint4* hd = nullptr;
  CK(hipHostGetDevicePointer((void**)&hd, h, 0));
  for (int g : {8, 16, 32, 64, 128}) {
    memset(h, 0, cb);
    hipLaunchKernelGGL(k_push, dim3(g), dim3(256), 0, s1, (const uint4*)d, hd, cb / 16);
    CK(hipDeviceSynchronize());
    printf("push grid %d: data %s\n", g, ((unsigned char*)h)[cb - 1] == 0x5a ? "ok" : "WRONG");
    CK(hipEventRecord(b0, s1));
    hipLaunchKernelGGL(k_push, dim3(g), dim3(256), 0, s1, (const uint4*)d, hd, cb / 16);
    CK(hipEventRecord(b1, s1));
    CK(hipDeviceSynchronize());
    CK(hipEventElapsedTime(&ms, b0, b1));
    printf("push grid %d alone: %.3f ms (%.1f GB/s)\n", g, ms, cb / ms / 1e6);
    CK(hipEventRecord(b0, s1));
    hipLaunchKernelGGL(k_push, dim3(g), dim3(256), 0, s1, (const uint4*)d, hd, cb / 16);
    CK(hipEventRecord(b1, s1));
    CK(hipEventRecord(a0, s0));
    for (int i = 0; i < 8; ++i) kern();
    CK(hipEventRecord(a1, s0));
    CK(hipDeviceSynchronize());
    float kms;
    CK(hipEventElapsedTime(&kms, a0, a1));
    CK(hipEventElapsedTime(&ms, b0, b1));
    printf("push grid %d beside 8 kernels: copy %.3f ms, kernels %.3f ms (%.3f each)\n", g, ms, kms, kms / 8);
  }
  return 0;
}
