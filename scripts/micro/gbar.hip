// Microbenchmark: grid-barrier cost inside one cooperative launch (k_tail's grid_barrier),
// by grid size and variant.  mode 0: seq_cst atomics + __threadfence on both sides (first
// k_tail); 1: relaxed atomics, no fences (lower bound); 2: relaxed atomics + agent release
// fence before arriving, acquire fence after the wait; 3: as 2, each block dirties 4 KB first.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t SH = 16, STR = 64;
struct Ctl { uint32_t arrive[(SH + 1) * STR]; uint32_t gen; uint32_t pad[STR - 1]; };

__device__ void gbar(Ctl* c, uint32_t& gen, int mode) {
  __shared__ uint32_t last;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (mode == 0) __threadfence();
    if (mode == 2 || mode == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t sh = blockIdx.x % SH, in_shard = (gridDim.x - 1 - sh) / SH + 1, shards = min(gridDim.x, SH);
    const int mo = mode == 0 ? __ATOMIC_SEQ_CST : __ATOMIC_RELAXED;
    last = 0;
    if (__hip_atomic_fetch_add(c->arrive + sh * STR, 1u, mo, __HIP_MEMORY_SCOPE_AGENT) == in_shard - 1) {
      __hip_atomic_store(c->arrive + sh * STR, 0u, mo, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(c->arrive + SH * STR, 1u, mo, __HIP_MEMORY_SCOPE_AGENT) == shards - 1) {
        __hip_atomic_store(c->arrive + SH * STR, 0u, mo, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
  }
  __syncthreads();
  if (last) {
    if (threadIdx.x == 0) {
      if (mode == 0) __threadfence();
      if (mode == 2 || mode == 3) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
      __hip_atomic_store(&c->gen, gen + 1, mode == 0 ? __ATOMIC_SEQ_CST : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (threadIdx.x == 0) {
    while (__hip_atomic_load(&c->gen, mode == 0 ? __ATOMIC_SEQ_CST : __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen)
      __builtin_amdgcn_s_sleep(1);
    if (mode == 0) __threadfence();
    if (mode == 2 || mode == 3) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  ++gen;
  __syncthreads();
}

__global__ void k_bar(Ctl* c, uint32_t* scratch, int n, int mode) {
  uint32_t gen = __hip_atomic_load(&c->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = 0; i < n; ++i) {
    if (mode == 3) scratch[(size_t)blockIdx.x * 1024 + threadIdx.x * 4] = i;
    gbar(c, gen, mode);
  }
}

int main() {
  Ctl* c;
  uint32_t* scratch;
  CK(hipMalloc(&c, sizeof(Ctl)));
  CK(hipMemset(c, 0, sizeof(Ctl)));
  CK(hipMalloc(&scratch, 4096 * 4096));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 4; ++mode)
    for (int grid : {4, 8, 16, 32, 64, 256}) {
      for (int n : {0, 200}) {
        float best = 1e9f;
        for (int t = 0; t < 3; ++t) {
          void* args[] = {&c, &scratch, &n, &mode};
          CK(hipEventRecord(e0, st));
          CK(hipLaunchCooperativeKernel((const void*)k_bar, dim3(grid), dim3(256), args, 0, st));
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        printf("mode %d grid %4d barriers %3d: %8.2f us total%s", mode, grid, n, best * 1e3, n ? "" : "\n");
        if (n) printf("  -> %.2f us/barrier\n", best * 1e3 / n);
      }
    }
  return 0;
}
