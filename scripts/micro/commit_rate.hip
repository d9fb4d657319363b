// What does the S commit's random atomicOr cost, and what would the alternatives cost?
// Table: R rows x W words (the bit matrix, 15 GB); n ops (row, bit), each op = one candidate.
// An op (j, i): row = 8 * h(i, j) % (R / 8) + j (so rows with row % 8 == j form segment j), bit random;
// "grouped": 64 consecutive ops of a segment share their row (one trigger's row walk).
// Modes:
//   agent     atomicOr returning, agent scope (the engine's commit_s today)
//   wg-rand   atomicOr returning, workgroup scope, any block any op (rate only: not coherent)
//   wg-xcd    workgroup scope, op segment j taken only by blocks that run on XCC j (HW_REG_XCC_ID,
//             dynamic tickets per segment): every row's line lives in one XCD's L2
//   load      plain 4-B load of the word (expand's test_bit)
//   ldst      plain load + OR + store (rate only: races)
// grouped = k > 1: the 64 ops of a wave-instruction hit k random 64-B lines of one row (how far do
// same-line lanes of one atomic instruction combine into one memory request?)
// Correctness of wg-xcd: bits set and "new" answers compared with the agent run (popcount).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/micro/commit_rate.hip -o scripts/micro/commit_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s: %s line %d\n", #x, hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

struct P {
  uint32_t* bits;
  uint64_t R, W;
  uint32_t per_seg;  // ops per segment
  uint32_t grouped, seed;
  unsigned long long* nnew;
  uint32_t* tickets;  // 8 segment tickets
};

__device__ __forceinline__ void op_addr(const P& p, uint32_t j, uint32_t i, uint32_t** w, uint32_t* m) {
  const uint64_t hr = mix64(((uint64_t)p.seed << 40) ^ ((uint64_t)j << 32) ^ (p.grouped ? i >> 6 : i));
  const uint64_t hc = mix64(((uint64_t)(p.seed + 7) << 40) ^ ((uint64_t)j << 32) ^ i);
  const uint64_t row = (hr % (p.R / 8)) * 8 + j;
  uint64_t col = hc % (p.W * 32);
  if (p.grouped > 1) {  // k = grouped lines of 64 B per 64 ops (one wave-instruction), same row
    const uint64_t hl = mix64(((uint64_t)(p.seed + 3) << 40) ^ ((uint64_t)j << 32) ^ ((i >> 6) * 64 + (hc >> 40) % p.grouped));
    col = (hl % (p.W / 16)) * 512 + (hc & 511);
  }
  *w = p.bits + row * p.W + (col >> 5);
  *m = 1u << (col & 31);
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

template <int MODE>
__global__ void k_ops(P p) {
  uint32_t cnt = 0;
  const uint64_t n = (uint64_t)p.per_seg * 8;
  if (MODE == 2) {
    __shared__ uint32_t base;
    const uint32_t j = xcc_id() & 7;
    for (;;) {
      if (threadIdx.x == 0) base = atomicAdd(p.tickets + j * 32, 4096u);
      __syncthreads();
      const uint32_t b = base;
      __syncthreads();
      if (b >= p.per_seg) break;
      for (uint32_t k = threadIdx.x; k < 4096u; k += blockDim.x) {
        const uint32_t i = b + k;
        if (i >= p.per_seg) break;
        uint32_t* w;
        uint32_t m;
        op_addr(p, j, i, &w, &m);
        const uint32_t old = __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        cnt += (old & m) == 0;
      }
    }
  } else {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x) {
      // op order: consecutive g walk one segment's ops (as a queue of one trigger's candidates)
      const uint32_t j = (uint32_t)(g / p.per_seg), i = (uint32_t)(g % p.per_seg);
      uint32_t* w;
      uint32_t m;
      op_addr(p, j, i, &w, &m);
      if (MODE == 0) {
        const uint32_t old = atomicOr(w, m);
        cnt += (old & m) == 0;
      } else if (MODE == 1) {
        const uint32_t old = __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        cnt += (old & m) == 0;
      } else if (MODE == 3) {
        cnt += (*w & m) == 0;
      } else {
        const uint32_t old = *w;
        *w = old | m;
        cnt += (old & m) == 0;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(p.nnew, (unsigned long long)cnt);
}

__global__ void k_pop(const uint32_t* __restrict__ b, uint64_t n, unsigned long long* out) {
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += __popc(b[i]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

int main(int argc, char** argv) {
  const uint64_t R = 320ull * 1024, W = 12288;  // 320 k rows x 393 k bits = 15 GiB
  const uint32_t n = argc > 1 ? atoi(argv[1]) : (64u << 20);
  P p{};
  p.R = R;
  p.W = W;
  p.per_seg = n / 8;
  CK(hipMalloc(&p.bits, R * W * 4));
  CK(hipMalloc(&p.nnew, 8));
  CK(hipMalloc(&p.tickets, 8 * 32 * 4));
  unsigned long long* pop;
  CK(hipMalloc(&pop, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"agent", "wg-rand", "wg-xcd", "load", "ldst"};
  for (uint32_t grouped : {0u, 1u, 64u, 16u, 4u, 1u << 30}) {
    if (grouped == (1u << 30)) grouped = 2;
    unsigned long long ref_pop = 0, ref_new = 0;
    for (int mode = 0; mode < 5; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(p.bits, 0, R * W * 4));
        CK(hipMemset(p.nnew, 0, 8));
        CK(hipMemset(p.tickets, 0, 8 * 32 * 4));
        CK(hipMemset(pop, 0, 8));
        p.grouped = grouped;
        p.seed = 11;
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const dim3 g(4096), b(256);
        if (mode == 0) hipLaunchKernelGGL(k_ops<0>, g, b, 0, 0, p);
        if (mode == 1) hipLaunchKernelGGL(k_ops<1>, g, b, 0, 0, p);
        if (mode == 2) hipLaunchKernelGGL(k_ops<2>, g, b, 0, 0, p);
        if (mode == 3) hipLaunchKernelGGL(k_ops<3>, g, b, 0, 0, p);
        if (mode == 4) hipLaunchKernelGGL(k_ops<4>, g, b, 0, 0, p);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        hipLaunchKernelGGL(k_pop, dim3(8192), dim3(256), 0, 0, p.bits, R * W, pop);
        unsigned long long hn = 0, hp = 0;
        CK(hipMemcpy(&hn, p.nnew, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&hp, pop, 8, hipMemcpyDeviceToHost));
        if (mode == 0) {
          ref_pop = hp;
          ref_new = hn;
        }
        printf("k=%-3u %-8s rep %d: %8.3f ms  %6.2f Gop/s  new %llu set %llu%s\n", grouped, names[mode], rep, ms, n / (ms * 1e-3) / 1e9, hn, hp,
               (mode == 2 && (hp != ref_pop || hn != ref_new)) ? "  MISMATCH vs agent" : "");
        fflush(stdout);
      }
    }
  }
  return 0;
}
