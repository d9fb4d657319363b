// el_rows.hip — row-sorted CSR of an append-only (row, value) log (see el_rows.h).
//
// Integer gather/scatter work, HBM-bound on the device side: the log is read twice (count,
// scatter), the unsorted rows written once and re-read once by the row sorts, which write the
// sorted rows to dst (device memory, or page-locked host memory over PCIe).  Row sorts run in
// registers (≤ 64 entries, one wave; ≤ 4096 entries, one workgroup with the cross-wave stages
// through LDS); the few longer rows are read off the bit matrix in column order when there is
// one.
#include "el_rows.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace elrows {
namespace {

constexpr uint32_t BLOCK = 256;
constexpr uint32_t SMALL = 64;      // register sort: one row per wave
constexpr uint32_t LDS_MAX = 4096;  // workgroup sort: 16 values per lane, 16 KB of LDS
constexpr uint32_t NONE = 0xffffffffu;

#define RCHK(expr)                                                                                  \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
void ensure(T*& p, uint64_t& cap, uint64_t n) {
  if (n <= cap && p) return;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = n + n / 8 + 1024;
  RCHK(hipMalloc((void**)&p, cap * sizeof(T)));
}

uint32_t grid(uint64_t n, uint32_t cap) {
  uint64_t g = (n + BLOCK - 1) / BLOCK;
  return (uint32_t)(g < 1 ? 1 : g > cap ? cap : g);
}

// Per-row counts and ranks.  A wave's 64 consecutive log entries are cut into runs of equal
// rows (the log holds each told closure, each CR4 fan-out of one X, back to back): the run
// head takes the run's slots with one atomic and its lanes take consecutive ranks.  Entries
// of rows outside [lo, lo + R) are skipped (they end runs).
__global__ void __launch_bounds__(BLOCK) k_rows_count(const uint32_t* __restrict__ rows, uint64_t n, uint32_t lo,
                                                      uint32_t R, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ rank) {
  const uint32_t lane = __lane_id();
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i0 = (uint64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < n; i0 += stride) {  // wave-uniform
    const uint64_t i = i0 + lane;
    uint32_t x = i < n ? rows[i] - lo : NONE;
    const bool ok = x < R;
    if (!ok) x = NONE;
    const uint32_t px = __shfl_up(x, 1);
    const bool head = ok && (lane == 0 || px != x);
    const unsigned long long hm = __ballot(head);
    const unsigned long long bm = __ballot(head || !ok);  // a run ends at the next head or skipped entry
    // this lane's run: head h = last head at or below the lane, end = next break above it
    const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const uint32_t h = 63u - (uint32_t)__clzll(hm & le);
    const unsigned long long above = bm & ~le;
    const uint32_t end = above ? (uint32_t)__ffsll((long long)above) - 1 : 64u;
    uint32_t base = 0;
    if (head) base = atomicAdd(cnt + x, end - lane);
    base = __shfl(base, (int)(h & 63u));
    if (ok && rank) rank[i] = base + (lane - h);
  }
}

__global__ void __launch_bounds__(BLOCK) k_rows_scatter(const uint32_t* __restrict__ rows,
                                                        const uint32_t* __restrict__ vals, uint64_t n, uint32_t lo,
                                                        uint32_t R, const uint64_t* __restrict__ ptr,
                                                        const uint32_t* __restrict__ rank,
                                                        const uint32_t* __restrict__ keymap,
                                                        uint32_t* __restrict__ tmp) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    const uint32_t x = rows[i] - lo;
    if (x >= R) continue;
    const uint32_t v = vals ? vals[i] : (uint32_t)i;  // no values: the entry's log index
    tmp[ptr[x] + rank[i]] = keymap ? keymap[v] : v;
  }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global stores (__syncthreads would also drain the row's PCIe stores into a host buffer
// before the next row could start).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace

// Bit matrix the sorts clear as they write (EL_RESULT_RELEASE): row x at bits + x·W.
__device__ void Clear::bit(uint32_t r, uint32_t v) const {
  if (!bits) return;
  const uint32_t c = v < 2u ? v : v - c_lo + 2u;  // (every value of a row lies in the window)
  bits[(uint64_t)(r + lo) * W + (c >> 5)] = 0u;
}

namespace {

// bitonic compare-exchange of a lane's value with the lane j away (j < 64) in stage k, where
// e is the element's index in the padded row
__device__ __forceinline__ uint32_t bitonic_xor(uint32_t v, uint32_t e, uint32_t k, uint32_t j) {
  const uint32_t u = __shfl_xor(v, (int)j);
  const bool up = (e & k) == 0, lower = (e & j) == 0;
  return (lower == up) ? min(v, u) : max(v, u);
}

// Row offsets: exclusive scan of the row counts (uint32) into uint64 offsets, in tiles of
// SCAN_TILE rows: tile sums, one block scans them, then each tile scans itself and lists its
// rows longer than 64 entries for k_rows_lds (<= LDS_MAX) or the long-row kernels (one global
// atomic per tile and list).
constexpr uint32_t SCAN_PER = 16, SCAN_TILE = BLOCK * SCAN_PER;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* wsum, uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (uint32_t k = 0; k < BLOCK / 64; ++k) {
    before += k < wv ? wsum[k] : 0u;
    all += wsum[k];
  }
  __syncthreads();
  if (total) *total = all;
  return before + inc - v;
}

__global__ void __launch_bounds__(BLOCK) k_rows_tiles(const uint32_t* __restrict__ cnt, uint32_t n1,
                                                      uint64_t* __restrict__ tile_sum) {
  __shared__ uint64_t wsum[BLOCK / 64];
  const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
  uint64_t t = 0;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_PER; ++j) t += base + j < n1 ? cnt[base + j] : 0u;
  uint64_t all = 0;
  block_excl_scan(t, wsum, &all);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = all;
}

__global__ void __launch_bounds__(BLOCK) k_rows_tile_scan(uint64_t* __restrict__ tile_sum, uint32_t ntiles) {
  __shared__ uint64_t wsum[BLOCK / 64];
  uint64_t carry = 0;
  for (uint32_t b = 0; b < ntiles; b += BLOCK) {
    const uint32_t i = b + threadIdx.x;
    const uint64_t v = i < ntiles ? tile_sum[i] : 0;
    uint64_t all = 0;
    const uint64_t ex = block_excl_scan(v, wsum, &all);
    if (i < ntiles) tile_sum[i] = carry + ex;
    carry += all;
  }
}

__global__ void __launch_bounds__(BLOCK) k_rows_offsets(const uint32_t* __restrict__ cnt, uint32_t R,
                                                        const uint64_t* __restrict__ tile_pre,
                                                        uint64_t* __restrict__ ptr, uint32_t* __restrict__ lists,
                                                        uint32_t* __restrict__ nlist) {
  __shared__ uint64_t wsum[BLOCK / 64];
  __shared__ uint32_t lmid[SCAN_TILE], lbig[64];
  __shared__ uint32_t nmid, nbig, gmid, gbig;
  if (threadIdx.x == 0) nmid = nbig = 0;
  const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
  uint32_t c[SCAN_PER];
  uint64_t t = 0;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_PER; ++j) {
    c[j] = base + j < R ? cnt[base + j] : 0u;  // row R (the end offset) counts nothing
    t += c[j];
  }
  uint64_t run = tile_pre[blockIdx.x] + block_excl_scan(t, wsum, nullptr);  // (its barriers order the LDS init)
#pragma unroll
  for (uint32_t j = 0; j < SCAN_PER; ++j) {
    const uint32_t r = base + j;
    if (r <= R) ptr[r] = run;
    run += c[j];
    if (c[j] > SMALL && c[j] <= LDS_MAX) lmid[atomicAdd(&nmid, 1u)] = r;
    if (c[j] > LDS_MAX) {
      const uint32_t k = atomicAdd(&nbig, 1u);
      if (k < 64) lbig[k] = r;
      else lists[R + atomicAdd(nlist + 64, 1u)] = r;  // (a tile with > 64 long rows)
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    gmid = nmid ? atomicAdd(nlist, nmid) : 0u;
    gbig = nbig ? atomicAdd(nlist + 64, min(nbig, 64u)) : 0u;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nmid; i += BLOCK) lists[gmid + i] = lmid[i];
  for (uint32_t i = threadIdx.x; i < min(nbig, 64u); i += BLOCK) lists[R + gbig + i] = lbig[i];
}

// Rows of 1..64 entries, sorted in registers (bitonic network over the wave, shuffles only),
// written to dst: a wave sorts the short rows among 64 consecutive rows one after the other.
__global__ void __launch_bounds__(BLOCK) k_rows_small(const uint64_t* __restrict__ ptr, uint32_t R,
                                                      const uint32_t* __restrict__ tmp, uint32_t* __restrict__ dst,
                                                      Clear cl) {
  const uint32_t lane = __lane_id();
  const uint32_t waves = gridDim.x * (BLOCK / 64);
  for (uint32_t g = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6); (uint64_t)g * 64 < R; g += waves) {
    const uint32_t r = g * 64 + lane;
    uint64_t b = 0, len = 0;
    if (r < R) {
      b = ptr[r];
      len = ptr[r + 1] - b;
    }
    if (len == 1) {
      const uint32_t v = tmp[b];
      dst[b] = v;
      cl.bit(r, v);
    }
    const unsigned long long small = __ballot(len > 1 && len <= SMALL);
    for (unsigned long long m = small; m; m &= m - 1) {
      const int src = __ffsll((long long)m) - 1;
      const uint64_t rb = __shfl(b, src);
      const uint32_t rl = (uint32_t)__shfl(len, src);
      uint32_t v = lane < rl ? tmp[rb + lane] : NONE;
#pragma unroll
      for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) v = bitonic_xor(v, lane, k, j);
      }
      if (lane < rl) {
        dst[rb + lane] = v;
        cl.bit(g * 64 + (uint32_t)src, v);
      }
    }
  }
}

// One row of 65..4096 entries padded to P = 256·E: lane l of wave w holds the elements
// e = (w + 4i)·64 + l, i < E.  Network stages whose partner is within 64 elements run on
// registers with shuffles; the others (j >= 64) exchange through LDS (two barriers).
template <uint32_t E>
__device__ __forceinline__ void sort_row(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t len,
                                         uint32_t* s, const Clear& cl, uint32_t r) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  constexpr uint32_t P = 256 * E;
  uint32_t v[E];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t e = (w + 4 * i) * 64 + lane;
    v[i] = e < len ? src[e] : NONE;
  }
#pragma unroll
  for (uint32_t k = 2; k <= P; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        lds_barrier();
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) s[(w + 4 * i) * 64 + lane] = v[i];
        lds_barrier();
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
          const uint32_t e = (w + 4 * i) * 64 + lane, p = e ^ j;
          const uint32_t u = s[p];
          const bool up = (e & k) == 0, lower = e < p;
          v[i] = (lower == up) ? min(v[i], u) : max(v[i], u);
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) v[i] = bitonic_xor(v[i], (w + 4 * i) * 64 + lane, k, j);
      }
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t e = (w + 4 * i) * 64 + lane;
    if (e < len) {
      dst[e] = v[i];
      cl.bit(r, v[i]);
    }
  }
}

// One row of 65..256 entries per wave, in registers only: lane l holds the elements
// e = 64 i + l, i < E (E = 2 up to 128 entries, else 4); stages with j >= 64 compare a lane's
// own registers (no LDS, no barriers), the others shuffle.
template <uint32_t E>
__device__ __forceinline__ void sort_row_wave(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                              uint32_t len, const Clear& cl, uint32_t r) {
  const uint32_t lane = __lane_id();
  constexpr uint32_t P = 64 * E;
  uint32_t v[E];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t e = 64 * i + lane;
    v[i] = e < len ? src[e] : NONE;
  }
#pragma unroll
  for (uint32_t k = 2; k <= P; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const uint32_t d = j / 64;
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
          if (i & d) continue;  // (the pair (i, i + d): the lower element's lane does both)
          const uint32_t e = 64 * i + lane;
          const bool up = (e & k) == 0;
          const uint32_t a = v[i], c = v[i + d];
          v[i] = up ? min(a, c) : max(a, c);
          v[i + d] = up ? max(a, c) : min(a, c);
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) v[i] = bitonic_xor(v[i], 64 * i + lane, k, j);
      }
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    const uint32_t e = 64 * i + lane;
    if (e < len) {
      dst[e] = v[i];
      cl.bit(r, v[i]);
    }
  }
}

// The listed rows of 65..256 entries, one per wave (k_rows_lds takes the longer ones).
__global__ void __launch_bounds__(BLOCK) k_rows_wave(const uint64_t* __restrict__ ptr, const uint32_t* __restrict__ tmp,
                                                     uint32_t* __restrict__ dst, const uint32_t* __restrict__ lists,
                                                     const uint32_t* __restrict__ nlist, Clear cl) {
  const uint32_t nrows = *nlist;
  const uint32_t waves = gridDim.x * (BLOCK / 64);
  for (uint32_t q = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6); q < nrows; q += waves) {
    const uint32_t r = lists[q];
    const uint64_t b = ptr[r];
    const uint32_t len = (uint32_t)(ptr[r + 1] - b);
    if (len <= 128)
      sort_row_wave<2>(tmp + b, dst + b, len, cl, r);
    else if (len <= 256)
      sort_row_wave<4>(tmp + b, dst + b, len, cl, r);
  }
}

__global__ void __launch_bounds__(BLOCK) k_rows_lds(const uint64_t* __restrict__ ptr, const uint32_t* __restrict__ tmp,
                                                    uint32_t* __restrict__ dst, const uint32_t* __restrict__ lists,
                                                    const uint32_t* __restrict__ nlist, Clear cl, bool waves_took_256) {
  __shared__ uint32_t s[LDS_MAX];
  const uint32_t nrows = *nlist;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[q];
    const uint64_t b = ptr[r];
    const uint32_t len = (uint32_t)(ptr[r + 1] - b);
    if (len <= 256 && waves_took_256) continue;  // (block-uniform: k_rows_wave sorted it)
    if (len <= 256)
      sort_row<1>(tmp + b, dst + b, len, s, cl, r);
    else if (len <= 512)
      sort_row<2>(tmp + b, dst + b, len, s, cl, r);
    else if (len <= 1024)
      sort_row<4>(tmp + b, dst + b, len, s, cl, r);
    else if (len <= 2048)
      sort_row<8>(tmp + b, dst + b, len, s, cl, r);
    else
      sort_row<16>(tmp + b, dst + b, len, s, cl, r);
    lds_barrier();  // s is reused by the next row
  }
}

// Long rows with a bit matrix: the row's set bits are its entries, already in column order.
// One workgroup per row: popcounts of 256 words, block scan, then each lane writes its
// word's columns.
__global__ void __launch_bounds__(BLOCK) k_rows_bits(const uint64_t* __restrict__ ptr, uint32_t* __restrict__ dst,
                                                     const uint32_t* __restrict__ lists,
                                                     const uint32_t* __restrict__ nlist, uint32_t R, Clear m,
                                                     bool clear) {
  __shared__ uint32_t wsum[BLOCK / 64];
  const uint32_t nrows = nlist[64], tid = threadIdx.x, lane = __lane_id(), wv = tid >> 6;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[R + q];
    const uint64_t W = m.W;
    uint32_t* __restrict__ row = m.bits + (uint64_t)(r + m.lo) * W;
    uint64_t at = ptr[r];
    for (uint64_t w0 = 0; w0 < W; w0 += BLOCK) {
      const uint64_t w = w0 + tid;
      uint32_t word = w < W ? row[w] : 0u;
      if (clear && word) row[w] = 0u;
      const uint32_t c = (uint32_t)__popc(word);
      uint32_t inc = c;
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (lane == 63) wsum[wv] = inc;
      __syncthreads();
      uint32_t before = 0, total = 0;
#pragma unroll
      for (uint32_t k = 0; k < BLOCK / 64; ++k) {
        before += k < wv ? wsum[k] : 0u;
        total += wsum[k];
      }
      uint64_t o = at + before + inc - c;
      while (word) {
        const uint32_t bit = (uint32_t)__ffs(word) - 1;
        const uint32_t c = (uint32_t)(w * 32 + bit);
        dst[o++] = c < 2u ? c : c + m.c_lo - 2u;  // column -> concept
        word &= word - 1;
      }
      at += total;
      __syncthreads();
    }
  }
}

// Rows [r0, r1) read off the bit matrix whole: the set columns of row r, in order, to
// dst[ptr[r] - out0 ...] (the rows of a copy-back chunk, staged in device memory for a DMA).
// One workgroup per row, 16 words per lane per round (four coalesced 16-B loads in flight:
// with each lane's four loads adjacent instead, every load instruction touched 64 lines and the
// read-out ran at 1.7 TB/s), popcounts and block scans give each lane its output slots.  A row stops at its last entry (ptr says
// how many): the columns are concept ids and a closure's members are mostly older concepts.
// clear: the read words are zeroed (the caller releases its state; only non-zero words are
// written).
__global__ void __launch_bounds__(BLOCK) k_rows_readout(const uint64_t* __restrict__ ptr, uint32_t r0, uint32_t r1,
                                                        uint64_t out0, uint32_t* __restrict__ dst, Clear m,
                                                        bool clear) {
  // loads: segment i of a round is 256 consecutive 16-B words, lane t takes the t-th (each load
  // instruction of a wave covers 1 KB contiguous); the set columns are ordered by (i, t)
  __shared__ uint32_t wsum[4][BLOCK / 64];
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid >> 6;
  const uint64_t W4 = m.W / 4;
  for (uint32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
    const uint64_t b = ptr[r], len = ptr[r + 1] - b;
    if (len == 0) continue;  // (block-uniform)
    uint4* __restrict__ row = reinterpret_cast<uint4*>(m.bits + (uint64_t)(r + m.lo) * m.W);
    uint64_t done = 0;
    for (uint64_t q0 = 0; q0 < W4 && done < len; q0 += BLOCK * 4) {
      uint4 v[4];
      uint32_t c[4], inc[4];
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) {
        const uint64_t q = q0 + i * BLOCK + tid;
        v[i] = q < W4 ? row[q] : make_uint4(0u, 0u, 0u, 0u);
        c[i] = __popc(v[i].x) + __popc(v[i].y) + __popc(v[i].z) + __popc(v[i].w);
        inc[i] = c[i];
      }
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          const uint32_t y = __shfl_up(inc[i], o);
          if (lane >= o) inc[i] += y;
        }
      }
      if (lane == 63) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) wsum[i][wv] = inc[i];
      }
      __syncthreads();
      uint32_t total = 0;  // the round's entries before segment i
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < BLOCK / 64; ++k) {
          before += k < wv ? wsum[i][k] : 0u;
          tot += wsum[i][k];
        }
        uint32_t* o = dst + (b - out0) + done + total + before + inc[i] - c[i];
        const uint64_t q = q0 + i * BLOCK + tid;
        const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          uint32_t word = wd[j];
          const uint32_t cb = (uint32_t)((q * 4 + j) * 32);
          while (word) {
            const uint32_t col = cb + (uint32_t)__ffs(word) - 1;
            *o++ = col < 2u ? col : col + m.c_lo - 2u;  // column -> concept
            word &= word - 1;
          }
        }
        if (clear && c[i]) row[q] = make_uint4(0u, 0u, 0u, 0u);
        total += tot;
      }
      done += total;
      __syncthreads();  // wsum is reused
    }
  }
}

// Long rows without a bit matrix: bitonic sort in place in tmp, one workgroup per row, then
// the row to dst.  The network only ever puts the smaller value at the lower index (the first
// merge step of each stage compares mirrored positions), so positions past the row act as
// +inf and are never touched.
__global__ void __launch_bounds__(BLOCK) k_rows_global(const uint64_t* __restrict__ ptr, uint32_t* tmp,
                                                       uint32_t* __restrict__ dst, const uint32_t* __restrict__ lists,
                                                       const uint32_t* __restrict__ nlist, uint32_t R) {
  const uint32_t nrows = nlist[64], tid = threadIdx.x;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[R + q];
    const uint64_t b = ptr[r];
    const uint64_t len = ptr[r + 1] - b;
    uint32_t* v = tmp + b;
    uint64_t P = 1;
    while (P < len) P <<= 1;
    for (uint64_t k = 2; k <= P; k <<= 1) {
      for (uint64_t j = k >> 1; j > 0; j >>= 1) {
        for (uint64_t t = tid; t < P / 2; t += BLOCK) {
          uint64_t i, p;
          if (j == k >> 1) {  // mirrored compare inside each block of k
            i = (t / j) * k + (t % j);
            p = (i | (k - 1)) - (i & (k - 1));
          } else {
            i = 2 * t - (t & (j - 1));
            p = i + j;
          }
          if (p < len) {
            const uint32_t a = v[i], c = v[p];
            if (a > c) {
              v[i] = c;
              v[p] = a;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint64_t i = tid; i < len; i += BLOCK) dst[b + i] = v[i];
    __syncthreads();
  }
}

}  // namespace

// The read-out's 512-B block k of a summary row: marked if any of its SUMM_SUB bytes is set.
__device__ __forceinline__ bool summ_any(const uint8_t* sr, uint32_t k) {
  if constexpr (SUMM_SUB == 8) return reinterpret_cast<const uint64_t*>(sr)[k] != 0ull;
  if constexpr (SUMM_SUB == 4) return reinterpret_cast<const uint32_t*>(sr)[k] != 0u;
  if constexpr (SUMM_SUB == 2) return reinterpret_cast<const uint16_t*>(sr)[k] != 0u;
  return sr[k] != 0;
}
__device__ __forceinline__ void summ_zero(uint8_t* sr, uint32_t k) {
  if constexpr (SUMM_SUB == 8) reinterpret_cast<uint64_t*>(sr)[k] = 0ull;
  else if constexpr (SUMM_SUB == 4) reinterpret_cast<uint32_t*>(sr)[k] = 0u;
  else if constexpr (SUMM_SUB == 2) reinterpret_cast<uint16_t*>(sr)[k] = 0u;
  else sr[k] = 0;
}

// k_rows_readout over the block summary: a row's non-zero 512-B blocks (summary bytes set by
// every writer of the matrix) are listed in LDS in column order, and the read-out loads only
// those — G3's rows hold their 104 M facts in 9.9 M of 37 M blocks, so the copy-back reads
// ≈5 GB of the 19 GB matrix instead of ≈18.5 GB (every word up to each row's last entry).
// Rounds of 32 listed blocks: segment i = 8 blocks, lane t loads 16 B (block 8i + t/32, quad
// t%32), so each load instruction covers two whole blocks; output slots from popcounts and
// block scans, in (block, word) order = column order.
constexpr uint32_t RB = 32;  // listed blocks per round
constexpr uint32_t NONE32 = 0xffffffffu;
__global__ void __launch_bounds__(BLOCK) k_rows_readout_sparse(const uint64_t* __restrict__ ptr, uint32_t r0,
                                                               uint32_t r1, uint64_t out0, uint32_t* __restrict__ dst,
                                                               Clear m, bool clear) {
  __shared__ uint32_t wsum[4][BLOCK / 64];
  __shared__ uint32_t blk[BLOCK];  // listed blocks of the current chunk of summary bytes
  __shared__ uint32_t nblk;
  const uint32_t tid = threadIdx.x, lane = __lane_id(), wv = tid >> 6;
  const uint64_t W4 = m.W / 4;
  for (uint32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
    const uint64_t b = ptr[r], len = ptr[r + 1] - b;
    if (len == 0) continue;  // (block-uniform)
    uint4* __restrict__ row = reinterpret_cast<uint4*>(m.bits + (uint64_t)(r + m.lo) * m.W);
    uint8_t* __restrict__ sr = m.summ + (uint64_t)(r + m.lo) * m.SB;
    uint64_t done = 0;
    const uint32_t NB = m.SB / SUMM_SUB;  // 512-B blocks of the summary row
    for (uint32_t k0 = 0; k0 < NB && done < len; k0 += BLOCK) {
      // list this chunk's non-zero blocks, ascending (wave ballots, then the waves in order)
      const bool nz = k0 + tid < NB && summ_any(sr, k0 + tid);
      if (clear && nz) summ_zero(sr, k0 + tid);  // (the reset leaves the read-out's rows to it)
      const unsigned long long bal = __ballot(nz);
      if (lane == 0) wsum[0][wv] = (uint32_t)__popcll(bal);
      __syncthreads();
      uint32_t before = 0, total = 0;
#pragma unroll
      for (uint32_t k = 0; k < BLOCK / 64; ++k) {
        before += k < wv ? wsum[0][k] : 0u;
        total += wsum[0][k];
      }
      if (nz) blk[before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = k0 + tid;
      if (tid == 0) nblk = total;
      __syncthreads();
      const uint32_t nb = nblk;
      for (uint32_t j0 = 0; j0 < nb && done < len; j0 += RB) {
        uint4 v[4];
        uint32_t c[4], inc[4];
        uint64_t qq[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          const uint32_t j = j0 + i * 8 + (tid >> 5);
          const uint64_t q = j < nb ? (uint64_t)blk[j] * 32 + (tid & 31u) : W4;
          qq[i] = q;
          v[i] = q < W4 ? row[q] : make_uint4(0u, 0u, 0u, 0u);
          c[i] = __popc(v[i].x) + __popc(v[i].y) + __popc(v[i].z) + __popc(v[i].w);
          inc[i] = c[i];
        }
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
#pragma unroll
          for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t y = __shfl_up(inc[i], o);
            if (lane >= o) inc[i] += y;
          }
        }
        __syncthreads();  // (wsum[0] of the listing is read)
        if (lane == 63) {
#pragma unroll
          for (uint32_t i = 0; i < 4; ++i) wsum[i][wv] = inc[i];
        }
        __syncthreads();
        uint32_t rtot = 0;  // the round's entries before segment i
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          uint32_t bef = 0, tot = 0;
#pragma unroll
          for (uint32_t k = 0; k < BLOCK / 64; ++k) {
            bef += k < wv ? wsum[i][k] : 0u;
            tot += wsum[i][k];
          }
          uint32_t* o = dst + (b - out0) + done + rtot + bef + inc[i] - c[i];
          const uint64_t q = qq[i];
          const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
          for (uint32_t jj = 0; jj < 4; ++jj) {
            uint32_t word = wd[jj];
            const uint32_t cb = (uint32_t)((q * 4 + jj) * 32);
            while (word) {
              const uint32_t col = cb + (uint32_t)__ffs(word) - 1;
              *o++ = col < 2u ? col : col + m.c_lo - 2u;  // column -> concept
              word &= word - 1;
            }
          }
          if (clear && c[i]) row[q] = make_uint4(0u, 0u, 0u, 0u);
          rtot += tot;
        }
        done += rtot;
        __syncthreads();  // wsum / blk are reused
      }
    }
  }
}

// k_rows_readout_sparse with one wave per row (no workgroup barriers): the wave lists 64
// summary bytes at a time with one ballot, takes the marked blocks two per load instruction
// (lanes 0-31: the lower block's 32 quads, lanes 32-63: the next one's), four loads in flight,
// and places the set columns by wave scans.  A row of G3 (≈25 marked blocks, ≈266 entries)
// is a handful of independent loads instead of a chain of block-wide rounds.
__global__ void __launch_bounds__(BLOCK) k_rows_readout_wave(const uint64_t* __restrict__ ptr, uint32_t r0,
                                                             uint32_t r1, uint64_t out0, uint32_t* __restrict__ dst,
                                                             Clear m, bool clear) {
  const uint32_t lane = __lane_id(), wpb = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * wpb + (threadIdx.x >> 6), nw = gridDim.x * wpb;
  const uint64_t W4 = m.W / 4;
  for (uint32_t r = r0 + gw; r < r1; r += nw) {  // (wave-uniform)
    const uint64_t b = ptr[r], len = ptr[r + 1] - b;
    if (len == 0) continue;
    uint4* __restrict__ row = reinterpret_cast<uint4*>(m.bits + (uint64_t)(r + m.lo) * m.W);
    uint8_t* __restrict__ sr = m.summ + (uint64_t)(r + m.lo) * m.SB;
    uint32_t* __restrict__ out = dst + (b - out0);
    uint64_t done = 0;
    const uint32_t NB = m.SB / SUMM_SUB;  // 512-B blocks of the summary row
    for (uint32_t k0 = 0; k0 < NB && done < len; k0 += 64) {
      const bool nz = k0 + lane < NB && summ_any(sr, k0 + lane);
      if (clear && nz) summ_zero(sr, k0 + lane);  // (the reset leaves the read-out's rows to it)
      unsigned long long bal = __ballot(nz);
      while (bal && done < len) {
        uint4 v[4];
        uint64_t q[4];
        uint32_t c[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {  // two marked blocks per load instruction
          uint32_t blkA = NONE32, blkB = NONE32;
          if (bal) {
            blkA = k0 + (uint32_t)__ffsll((long long)bal) - 1;
            bal &= bal - 1;
          }
          if (bal) {
            blkB = k0 + (uint32_t)__ffsll((long long)bal) - 1;
            bal &= bal - 1;
          }
          const uint32_t blk = lane < 32 ? blkA : blkB;
          q[i] = blk != NONE32 ? (uint64_t)blk * 32 + (lane & 31u) : W4;
          v[i] = q[i] < W4 ? row[q[i]] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
          c[i] = __popc(v[i].x) + __popc(v[i].y) + __popc(v[i].z) + __popc(v[i].w);
          uint32_t inc = c[i];
#pragma unroll
          for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
          }
          uint32_t* o = out + done + inc - c[i];
          const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
          for (uint32_t jj = 0; jj < 4; ++jj) {
            uint32_t word = wd[jj];
            const uint32_t cb = (uint32_t)((q[i] * 4 + jj) * 32);
            while (word) {
              const uint32_t col = cb + (uint32_t)__ffs(word) - 1;
              *o++ = col < 2u ? col : col + m.c_lo - 2u;  // column -> concept
              word &= word - 1;
            }
          }
          if (clear && c[i]) row[q[i]] = make_uint4(0u, 0u, 0u, 0u);
          done += __shfl(inc, 63);
        }
      }
    }
  }
}

void Scratch::release() {
  for (void* p : {(void*)rank, (void*)tmp, (void*)cnt, (void*)lists, (void*)nlist, (void*)tile})
    if (p) (void)hipFree(p);
  rank = tmp = cnt = lists = nlist = nullptr;
  tile = nullptr;
  rank_cap = tmp_cap = cnt_cap = list_cap = tile_cap = 0;
}

void build_prep(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
                uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* dst, Clear matrix, bool clear) {
  ensure(sc.rank, sc.rank_cap, n);
  ensure(sc.tmp, sc.tmp_cap, n);
  ensure(sc.cnt, sc.cnt_cap, (uint64_t)R + 1);
  ensure(sc.lists, sc.list_cap, 2 * (uint64_t)R + 2);
  if (!sc.nlist) RCHK(hipMalloc((void**)&sc.nlist, 128 * sizeof(uint32_t)));
  RCHK(hipMemsetAsync(sc.cnt, 0, ((uint64_t)R + 1) * sizeof(uint32_t), s));
  RCHK(hipMemsetAsync(sc.nlist, 0, 128 * sizeof(uint32_t), s));
  if (n) {
    hipLaunchKernelGGL(k_rows_count, dim3(grid(n, 2048)), dim3(BLOCK), 0, s, rows, n, row_lo, R, sc.cnt, sc.rank);
    RCHK(hipGetLastError());
  }
  const uint32_t tiles = (uint32_t)(((uint64_t)R + 1 + SCAN_TILE - 1) / SCAN_TILE);
  ensure(sc.tile, sc.tile_cap, tiles);
  hipLaunchKernelGGL(k_rows_tiles, dim3(tiles), dim3(BLOCK), 0, s, sc.cnt, R + 1, sc.tile);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_tile_scan, dim3(1), dim3(BLOCK), 0, s, sc.tile, tiles);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_offsets, dim3(tiles), dim3(BLOCK), 0, s, sc.cnt, R, sc.tile, ptr, sc.lists, sc.nlist);
  RCHK(hipGetLastError());
  sc.n = n;
  sc.R = R;
  sc.bits = matrix.bits != nullptr;
  if (!n) return;
  hipLaunchKernelGGL(k_rows_scatter, dim3(grid(n, 2048)), dim3(BLOCK), 0, s, rows, vals, n, row_lo, R, ptr, sc.rank,
                     keymap, sc.tmp);
  RCHK(hipGetLastError());
  if (matrix.bits) {
    hipLaunchKernelGGL(k_rows_bits, dim3(512), dim3(BLOCK), 0, s, ptr, dst, sc.lists, sc.nlist, R, matrix, clear);
    RCHK(hipGetLastError());
  }
}

void build_sort(hipStream_t s, Scratch& sc, const uint64_t* ptr, uint32_t* dst, Clear cl) {
  if (!sc.n) return;
  const uint32_t R = sc.R;
  hipLaunchKernelGGL(k_rows_small, dim3(grid(((uint64_t)R + 63) / 64 * 64, 2048)), dim3(BLOCK), 0, s, ptr, R, sc.tmp,
                     dst, cl);
  RCHK(hipGetLastError());
  static const bool no_wave = getenv("EL_ROWS_NO_WAVE") != nullptr;  // A/B: rows <= 256 by the workgroup sort
  if (!no_wave) {
    hipLaunchKernelGGL(k_rows_wave, dim3(1024), dim3(BLOCK), 0, s, ptr, sc.tmp, dst, sc.lists, sc.nlist, cl);
    RCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_rows_lds, dim3(1024), dim3(BLOCK), 0, s, ptr, sc.tmp, dst, sc.lists, sc.nlist, cl, !no_wave);
  RCHK(hipGetLastError());
  if (!sc.bits) {
    hipLaunchKernelGGL(k_rows_global, dim3(512), dim3(BLOCK), 0, s, ptr, sc.tmp, dst, sc.lists, sc.nlist, R);
    RCHK(hipGetLastError());
  }
}

void build_counts(hipStream_t s, Scratch& sc, const uint32_t* rows, uint64_t n, uint32_t row_lo, uint32_t R,
                  uint64_t* ptr) {
  ensure(sc.cnt, sc.cnt_cap, (uint64_t)R + 1);
  ensure(sc.lists, sc.list_cap, 2 * (uint64_t)R + 2);
  if (!sc.nlist) RCHK(hipMalloc((void**)&sc.nlist, 128 * sizeof(uint32_t)));
  RCHK(hipMemsetAsync(sc.cnt, 0, ((uint64_t)R + 1) * sizeof(uint32_t), s));
  RCHK(hipMemsetAsync(sc.nlist, 0, 128 * sizeof(uint32_t), s));
  if (n) {
    hipLaunchKernelGGL(k_rows_count, dim3(grid(n, 2048)), dim3(BLOCK), 0, s, rows, n, row_lo, R, sc.cnt,
                       (uint32_t*)nullptr);
    RCHK(hipGetLastError());
  }
  const uint32_t tiles = (uint32_t)(((uint64_t)R + 1 + SCAN_TILE - 1) / SCAN_TILE);
  ensure(sc.tile, sc.tile_cap, tiles);
  hipLaunchKernelGGL(k_rows_tiles, dim3(tiles), dim3(BLOCK), 0, s, sc.cnt, R + 1, sc.tile);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_tile_scan, dim3(1), dim3(BLOCK), 0, s, sc.tile, tiles);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_offsets, dim3(tiles), dim3(BLOCK), 0, s, sc.cnt, R, sc.tile, ptr, sc.lists, sc.nlist);
  RCHK(hipGetLastError());
}

void readout(hipStream_t s, const uint64_t* ptr, uint32_t r0, uint32_t r1, uint64_t out0, uint32_t* dst, Clear m,
             bool clear) {
  if (r1 <= r0) return;
  static const uint32_t maxb = [] {
    // A/B: workgroups of the read-out (leaves CUs to the DMA blits and, with two classifications
    // in flight, to the other engine's saturation: G3 25.1 -> 24.7 ms per step at 1024, serial
    // latency unchanged; 256 and fewer starve the read-out)
    const char* e = getenv("EL_READOUT_BLOCKS");
    return e ? (uint32_t)std::max(1l, strtol(e, nullptr, 10)) : 1024u;
  }();
  static const bool per_wave = getenv("EL_READOUT_WAVE") != nullptr;  // A/B: one wave per row (no gain)
  if (m.summ && per_wave)
    hipLaunchKernelGGL(k_rows_readout_wave, dim3(std::min<uint32_t>((r1 - r0 + 3) / 4, maxb)), dim3(BLOCK), 0, s, ptr,
                       r0, r1, out0, dst, m, clear);
  else if (m.summ)
    hipLaunchKernelGGL(k_rows_readout_sparse, dim3(std::min<uint32_t>(r1 - r0, maxb)), dim3(BLOCK), 0, s, ptr, r0, r1,
                       out0, dst, m, clear);
  else
    hipLaunchKernelGGL(k_rows_readout, dim3(std::min<uint32_t>(r1 - r0, maxb)), dim3(BLOCK), 0, s, ptr, r0, r1, out0,
                       dst, m, clear);
  RCHK(hipGetLastError());
}

void build(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
           uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* dst, Clear matrix) {
  build_prep(s, sc, rows, vals, n, row_lo, R, keymap, ptr, dst, matrix, false);
  build_sort(s, sc, ptr, dst, Clear{});
}

}  // namespace elrows
