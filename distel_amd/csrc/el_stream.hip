// el_stream.hip — run encoding of the streamed result's log segments (el_stream.h).
#include "el_stream.h"


#include <cstdlib>
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

// Workgroups of an encoding launch: one per tile up to a cap (EL_RUN_GRID, default 1024; the
// encodings run beside the supersteps and share the CUs with them).
uint32_t grid(uint64_t nt) {
  static const uint64_t cap = [] {
    const char* e = getenv("EL_RUN_GRID");
    const unsigned long v = e ? strtoul(e, nullptr, 10) : 1024ul;
    return (uint64_t)(v ? v : 1024ul);
  }();
  return (uint32_t)(nt < cap ? (nt ? nt : 1) : cap);
}

// A run starts at e when e opens its tile or its key differs from the one before.
__device__ __forceinline__ bool run_head(const uint32_t* __restrict__ keys, uint64_t e, uint64_t t0, uint32_t key) {
  return e == t0 || keys[e - 1] != key;
}

// ---- packed fact values (EL_STREAM_PACKED): a value's bit column (col_of of el_gpu.hip: ⊥, ⊤,
// then the window [c_lo, c_hi) in cperm's order) is its 16-bit code when below CODE_ESC; the
// others escape (code CODE_ESC, the value itself in the escape list, in log order).  The column
// order puts the frequent subsumers first (G3: 96.6 % of the facts in the first 65,535 columns).
// The fact log's codes ride on its run encoding: the same two passes read x and the value of an
// entry, count / number its run heads and its escapes, and write its code.
__device__ __forceinline__ uint32_t code_of(uint32_t v, const uint32_t* __restrict__ cperm, uint32_t c_lo,
                                            uint32_t c_hi) {
  const uint32_t c = v < 2u ? v : (v < c_lo || v >= c_hi) ? 0xffffffffu : cperm ? cperm[v] : v - c_lo + 2u;
  return c < CODE_ESC ? c : CODE_ESC;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t c) {
  for (uint32_t o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  return c;
}

template <bool PACK>
__global__ void __launch_bounds__(BLOCK) k_run_count(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                     uint32_t* __restrict__ cnt, Codes pk) {
  __shared__ uint32_t wsum[2][WAVES];
  const uint64_t nt = tiles(b - a);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {  // (block-uniform trip count)
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    uint32_t c = 0, x = 0;
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      if (e < t1) {
        c += run_head(keys, e, t0, keys[e]) ? 1u : 0u;
        if (PACK) x += code_of(pk.vals[e], pk.cperm, pk.c_lo, pk.c_hi) == CODE_ESC ? 1u : 0u;
      }
    }
    c = wave_sum(c);
    if (PACK) x = wave_sum(x);
    if (lane == 0) wsum[0][w] = c, wsum[1][w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0, sx = 0;
      for (uint32_t i = 0; i < WAVES; ++i) s += wsum[0][i], sx += wsum[1][i];
      cnt[t] = s;
      if (PACK) pk.cnt[t] = sx;
    }
    __syncthreads();
  }
}

// Tile t's runs are numbered from base + off[t] in log order: the run of a tail element e (the
// last of its run in the tile) is the number of heads up to e, minus one.  Coalesced loads
// (element k·BLOCK + thread of the tile), one ballot per round for the heads.  PACK: the code of
// every entry at codes[e] (log position), the escapes numbered from pk.base + pk.off[t] alike.
template <bool PACK>
__global__ void __launch_bounds__(BLOCK) k_run_emit(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                    const uint32_t* __restrict__ off, uint2* out, uint64_t cap,
                                                    const unsigned long long* base, Codes pk) {
  __shared__ uint32_t wtot[2][WAVES];
  const uint64_t nt = tiles(b - a), b0 = *base, x0 = PACK ? *pk.base : 0ull;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    const uint64_t run0 = b0 + off[t], esc0 = PACK ? x0 + pk.off[t] : 0ull;
    uint32_t running = 0, xrunning = 0;  // heads / escapes of the tile before this round
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      const bool valid = e < t1;
      const uint32_t key = valid ? keys[e] : 0u;
      const bool head = valid && run_head(keys, e, t0, key);
      const bool tail = valid && (e + 1 == t1 || keys[e + 1] != key);
      const unsigned long long m = __ballot(head);
      uint32_t v = 0, code = 0;
      bool x = false;
      unsigned long long mx = 0;
      if (PACK) {
        v = valid ? pk.vals[e] : 0u;
        code = valid ? code_of(v, pk.cperm, pk.c_lo, pk.c_hi) : 0u;
        x = valid && code == CODE_ESC;
        if (valid && e < pk.code_cap) pk.codes[e] = (uint16_t)code;
        mx = __ballot(x);
      }
      if (lane == 0) wtot[0][w] = (uint32_t)__popcll(m), wtot[1][w] = (uint32_t)__popcll(mx);
      __syncthreads();
      uint32_t before = 0, all = 0, xbefore = 0, xall = 0;
      for (uint32_t i = 0; i < WAVES; ++i) {
        const uint32_t q = wtot[0][i], qx = wtot[1][i];
        before += i < w ? q : 0u;
        all += q;
        xbefore += i < w ? qx : 0u;
        xall += qx;
      }
      __syncthreads();  // (wtot is rewritten next round)
      if (tail) {
        const uint64_t r = run0 + running + before + (uint32_t)__popcll(m & below) + (head ? 1u : 0u) - 1u;
        if (r < cap) out[r] = make_uint2(key, (uint32_t)(e + 1));
      }
      if (PACK && x) {
        const uint64_t r = esc0 + xrunning + xbefore + (uint32_t)__popcll(mx & below);
        if (r < pk.esc_cap) pk.esc[r] = v;
      }
      running += all;
      xrunning += xall;
    }
  }
}

__global__ void k_run_advance(unsigned long long* base, const uint32_t* off, const uint32_t* cnt, uint64_t last,
                              unsigned long long* total, Codes pk) {
  const unsigned long long v = *base + off[last] + cnt[last];
  *base = v;
  *total = v;
  if (pk.base) {
    const unsigned long long x = *pk.base + pk.off[last] + pk.cnt[last];
    *pk.base = x;
    *pk.total = x;
  }
}

}  // namespace

void count(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, uint32_t* cnt, const Codes* pk) {
  if (b <= a) return;
  if (pk)
    hipLaunchKernelGGL(k_run_count<true>, dim3(grid(tiles(b - a))), dim3(BLOCK), 0, s, keys, a, b, cnt, *pk);
  else
    hipLaunchKernelGGL(k_run_count<false>, dim3(grid(tiles(b - a))), dim3(BLOCK), 0, s, keys, a, b, cnt, Codes{});
  SCHK(hipGetLastError());
}

void emit(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, const uint32_t* off, const uint32_t* cnt,
          uint2* out, uint64_t cap, unsigned long long* base, unsigned long long* total, const Codes* pk) {
  if (b <= a) return;
  const uint64_t nt = tiles(b - a);
  if (pk)
    hipLaunchKernelGGL(k_run_emit<true>, dim3(grid(nt)), dim3(BLOCK), 0, s, keys, a, b, off, out, cap, base, *pk);
  else
    hipLaunchKernelGGL(k_run_emit<false>, dim3(grid(nt)), dim3(BLOCK), 0, s, keys, a, b, off, out, cap, base, Codes{});
  SCHK(hipGetLastError());
  hipLaunchKernelGGL(k_run_advance, dim3(1), dim3(1), 0, s, base, off, cnt, nt - 1, total, pk ? *pk : Codes{});
  SCHK(hipGetLastError());
}

}  // namespace elst
