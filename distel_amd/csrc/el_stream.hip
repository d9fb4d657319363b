// el_stream.hip — run encoding of the streamed result's log segments (el_stream.h).
#include "el_stream.h"


#include <stdexcept>
#include <string>
#include <vector>

namespace elst {
namespace {

#define SCHK(expr)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr uint32_t WAVES = BLOCK / 64;

uint32_t grid(uint64_t nt) { return (uint32_t)(nt < 1024 ? (nt ? nt : 1) : 1024); }

// A run starts at e when e opens its tile or its key differs from the one before.
__device__ __forceinline__ bool run_head(const uint32_t* __restrict__ keys, uint64_t e, uint64_t t0, uint32_t key) {
  return e == t0 || keys[e - 1] != key;
}

__global__ void __launch_bounds__(BLOCK) k_run_count(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                     uint32_t* __restrict__ cnt) {
  __shared__ uint32_t wsum[WAVES];
  const uint64_t nt = tiles(b - a);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {  // (block-uniform trip count)
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    uint32_t c = 0;
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      if (e < t1) c += run_head(keys, e, t0, keys[e]) ? 1u : 0u;
    }
    for (uint32_t o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0;
      for (uint32_t i = 0; i < WAVES; ++i) s += wsum[i];
      cnt[t] = s;
    }
    __syncthreads();
  }
}

// Tile t's runs are numbered from base + off[t] in log order: the run of a tail element e (the
// last of its run in the tile) is the number of heads up to e, minus one.  Coalesced loads
// (element k·BLOCK + thread of the tile), one ballot per round for the heads.
__global__ void __launch_bounds__(BLOCK) k_run_emit(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                    const uint32_t* __restrict__ off, uint2* out, uint64_t cap,
                                                    const unsigned long long* base) {
  __shared__ uint32_t wtot[WAVES];
  const uint64_t nt = tiles(b - a), b0 = *base;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    const uint64_t run0 = b0 + off[t];
    uint32_t running = 0;  // heads of the tile before this round
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      const bool valid = e < t1;
      const uint32_t key = valid ? keys[e] : 0u;
      const bool head = valid && run_head(keys, e, t0, key);
      const bool tail = valid && (e + 1 == t1 || keys[e + 1] != key);
      const unsigned long long m = __ballot(head);
      if (lane == 0) wtot[w] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, all = 0;
      for (uint32_t i = 0; i < WAVES; ++i) {
        const uint32_t v = wtot[i];
        before += i < w ? v : 0u;
        all += v;
      }
      __syncthreads();  // (wtot is rewritten next round)
      if (tail) {
        const uint64_t r = run0 + running + before + (uint32_t)__popcll(m & below) + (head ? 1u : 0u) - 1u;
        if (r < cap) out[r] = make_uint2(key, (uint32_t)(e + 1));
      }
      running += all;
    }
  }
}

__global__ void k_run_advance(unsigned long long* base, const uint32_t* off, const uint32_t* cnt, uint64_t last,
                              unsigned long long* total) {
  const unsigned long long v = *base + off[last] + cnt[last];
  *base = v;
  *total = v;
}

}  // namespace

void count(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, uint32_t* cnt) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_run_count, dim3(grid(tiles(b - a))), dim3(BLOCK), 0, s, keys, a, b, cnt);
  SCHK(hipGetLastError());
}

void emit(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, const uint32_t* off, const uint32_t* cnt,
          uint2* out, uint64_t cap, unsigned long long* base, unsigned long long* total) {
  if (b <= a) return;
  const uint64_t nt = tiles(b - a);
  hipLaunchKernelGGL(k_run_emit, dim3(grid(nt)), dim3(BLOCK), 0, s, keys, a, b, off, out, cap, base);
  SCHK(hipGetLastError());
  hipLaunchKernelGGL(k_run_advance, dim3(1), dim3(1), 0, s, base, off, cnt, nt - 1, total);
  SCHK(hipGetLastError());
}

}  // namespace elst
