// FETCH_SIZE / WRITE_SIZE calibration for the access patterns of the saturation kernels
// (MI355X_MICROARCH.md "HBM": only 16-B/lane streaming reads are calibrated on gfx950).
// Each kernel touches a known number of distinct lines of an 8 GB array (far past the 256 MiB
// Infinity Cache), one launch each, so `rocprofv3 --pmc FETCH_SIZE` (and, in its own pass,
// `--pmc WRITE_SIZE`) per dispatch divided by the count printed here is the counter's bytes per
// access of that pattern:
//   k_stream16   16 B/lane coalesced streaming read                       (bytes = n · 16)
//   k_stream4    4 B/lane coalesced streaming read                        (bytes = n · 4)
//   k_gather4    random 4-B loads, one per distinct 128-B line            (accesses = n)
//   k_gather8    random 8-B loads (a hash-set probe), one per line        (accesses = n)
//   k_store4     random 4-B stores, one per distinct line                 (accesses = n)
//   k_atomic_or  random returning atomicOr on 4 B, one per distinct line  (accesses = n)
//   k_cas8       random 64-bit CAS (the link-set insert), one per line    (accesses = n)
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/pmc_cal.hip -o scripts/micro/pmc_cal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr uint64_t LINES = (8ull << 30) / 128;  // 128-B lines of the 8 GB array

// line of access i: a bijection of [0, LINES) (odd multiplier mod 2^26), so every access hits a
// distinct line and consecutive lanes hit lines far apart
__device__ __forceinline__ uint64_t line_of(uint64_t i) { return (i * 0x9E3779B1ull) & (LINES - 1); }

__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345679u) out[0] = s;
}

__global__ void k_stream4(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s ^= a[i];
  if (s == 0x12345679u) out[0] = s;
}

__global__ void k_gather4(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s ^= a[line_of(i) * 32 + (i & 31)];
  if (s == 0x12345679u) out[0] = s;
}

__global__ void k_gather8(const uint64_t* __restrict__ a, uint64_t n, uint32_t* out) {
  uint64_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s ^= a[line_of(i) * 16 + (i & 15)];
  if (s == 0x12345679u) out[0] = (uint32_t)s;
}

__global__ void k_store4(uint32_t* a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[line_of(i) * 32 + (i & 31)] = (uint32_t)i;
}

__global__ void k_atomic_or(uint32_t* a, uint64_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s ^= atomicOr(&a[line_of(i) * 32 + (i & 31)], 1u << (i & 31));
  if (s == 0x12345679u) out[0] = s;
}

__global__ void k_cas8(unsigned long long* a, uint64_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long old = atomicCAS(&a[line_of(i) * 16 + (i & 15)], ~0ull, (unsigned long long)i);
    s ^= (uint32_t)old;
  }
  if (s == 0x12345679u) out[0] = s;
}

int main() {
  void* big = nullptr;
  uint32_t* o = nullptr;
  CK(hipMalloc(&big, 8ull << 30));
  CK(hipMalloc(&o, 4));
  CK(hipMemset(big, 0xff, 8ull << 30));
  CK(hipDeviceSynchronize());
  const uint64_t n_rand = 16ull << 20;     // 16 M accesses, 16 M distinct lines (2 GB of lines)
  const uint64_t n16 = (1ull << 30) / 16;  // 1 GB streamed
  const uint64_t n4 = (1ull << 30) / 4;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char* name, uint64_t n, uint64_t bytes, auto launch) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-12s accesses %llu algorithmic_bytes %llu  %.3f ms  %.2f G accesses/s\n", name, (unsigned long long)n,
           (unsigned long long)bytes, ms, n / ms / 1e6);
  };
  const dim3 g(4096), t(256);
  timed("k_stream16", n16, n16 * 16, [&] { hipLaunchKernelGGL(k_stream16, g, t, 0, 0, (const uint4*)big, n16, o); });
  timed("k_stream4", n4, n4 * 4, [&] { hipLaunchKernelGGL(k_stream4, g, t, 0, 0, (const uint32_t*)big, n4, o); });
  timed("k_gather4", n_rand, n_rand * 4,
        [&] { hipLaunchKernelGGL(k_gather4, g, t, 0, 0, (const uint32_t*)big, n_rand, o); });
  timed("k_gather8", n_rand, n_rand * 8,
        [&] { hipLaunchKernelGGL(k_gather8, g, t, 0, 0, (const uint64_t*)big, n_rand, o); });
  timed("k_store4", n_rand, n_rand * 4, [&] { hipLaunchKernelGGL(k_store4, g, t, 0, 0, (uint32_t*)big, n_rand); });
  timed("k_atomic_or", n_rand, n_rand * 8,
        [&] { hipLaunchKernelGGL(k_atomic_or, g, t, 0, 0, (uint32_t*)big, n_rand, o); });
  timed("k_cas8", n_rand, n_rand * 16,
        [&] { hipLaunchKernelGGL(k_cas8, g, t, 0, 0, (unsigned long long*)big, n_rand, o); });
  return 0;
}
