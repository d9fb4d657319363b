// el_rows.hip — row-sorted CSR of an append-only (row, value) log (see el_rows.h).
//
// Integer gather/scatter work, HBM-bound: the log is read twice (count, scatter), the CSR
// written once and re-read once by the row sorts.  Row sorts run in registers (≤ 64 entries,
// one wave) or LDS (≤ 4096 entries, one workgroup); the few longer rows are read off the
// bit matrix in column order when there is one.
#include "el_rows.h"

#include <hipcub/hipcub.hpp>

#include <stdexcept>
#include <string>

namespace elrows {
namespace {

constexpr uint32_t BLOCK = 256;
constexpr uint32_t SMALL = 64;      // register sort: one row per wave
constexpr uint32_t LDS_MAX = 4096;  // LDS sort: one row per workgroup (16 KB)
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
  cap = n + n / 4 + 1024;
  RCHK(hipMalloc((void**)&p, cap * sizeof(T)));
}

uint32_t grid(uint64_t n, uint32_t cap) {
  uint64_t g = (n + BLOCK - 1) / BLOCK;
  return (uint32_t)(g < 1 ? 1 : g > cap ? cap : g);
}

// Per-row counts and ranks.  A wave's 64 consecutive log entries are cut into runs of equal
// rows (the log holds each told closure, each CR4 fan-out of one X, back to back): the run
// head takes the run's slots with one atomic and its lanes take consecutive ranks.
__global__ void __launch_bounds__(BLOCK) k_rows_count(const uint32_t* __restrict__ rows, uint64_t n, uint32_t lo,
                                                      uint32_t* __restrict__ cnt, uint32_t* __restrict__ rank) {
  const uint32_t lane = __lane_id();
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i0 = (uint64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < n; i0 += stride) {  // wave-uniform
    const uint64_t i = i0 + lane;
    const bool ok = i < n;
    const uint32_t x = ok ? rows[i] - lo : NONE;
    const uint32_t px = __shfl_up(x, 1);
    const bool head = ok && (lane == 0 || px != x);
    const unsigned long long hm = __ballot(head);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(ok));  // valid lanes are a prefix
    // this lane's run: head h = last head at or below the lane, end = next head or nvalid
    const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const uint32_t h = 63u - (uint32_t)__clzll(hm & le);
    const unsigned long long above = hm & ~le;
    const uint32_t end = above ? (uint32_t)__ffsll((long long)above) - 1 : nvalid;
    uint32_t base = 0;
    if (head) base = atomicAdd(cnt + x, end - lane);
    base = __shfl(base, (int)h);
    if (ok) rank[i] = base + (lane - h);
  }
}

__global__ void __launch_bounds__(BLOCK) k_rows_scatter(const uint32_t* __restrict__ rows,
                                                        const uint32_t* __restrict__ vals, uint64_t n, uint32_t lo,
                                                        const uint64_t* __restrict__ ptr,
                                                        const uint32_t* __restrict__ rank,
                                                        const uint32_t* __restrict__ keymap,
                                                        uint32_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    const uint32_t v = vals[i];
    out[ptr[rows[i] - lo] + rank[i]] = keymap ? keymap[v] : v;
  }
}

// Rows of <= 64 entries sorted in registers (bitonic network over the wave, shuffles only);
// longer rows are listed for k_rows_lds (<= LDS_MAX) or the long-row kernels.  A wave looks
// at 64 rows at once, so a list append is one atomic per wave.
__global__ void __launch_bounds__(BLOCK) k_rows_small(const uint64_t* __restrict__ ptr, uint32_t R,
                                                      uint32_t* __restrict__ out, uint32_t* __restrict__ lists,
                                                      uint32_t* __restrict__ nlist) {
  const uint32_t lane = __lane_id();
  const uint32_t waves = gridDim.x * (BLOCK / 64);
  for (uint32_t g = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6); (uint64_t)g * 64 < R; g += waves) {
    const uint32_t r = g * 64 + lane;
    uint64_t b = 0, len = 0;
    if (r < R) {
      b = ptr[r];
      len = ptr[r + 1] - b;
    }
    const unsigned long long small = __ballot(len > 1 && len <= SMALL);
    const unsigned long long mid = __ballot(len > SMALL && len <= LDS_MAX);
    const unsigned long long big = __ballot(len > LDS_MAX);
    if (mid) {
      uint32_t at = 0;
      if (lane == 0) at = atomicAdd(nlist, (uint32_t)__popcll(mid));
      at = __shfl(at, 0);
      if (mid >> lane & 1) lists[at + __popcll(mid & ((1ull << lane) - 1))] = r;
    }
    if (big) {
      uint32_t at = 0;
      if (lane == 0) at = atomicAdd(nlist + 64, (uint32_t)__popcll(big));
      at = __shfl(at, 0);
      if (big >> lane & 1) lists[R + at + __popcll(big & ((1ull << lane) - 1))] = r;
    }
    for (unsigned long long m = small; m; m &= m - 1) {
      const int src = __ffsll((long long)m) - 1;
      const uint64_t rb = __shfl(b, src);
      const uint32_t rl = (uint32_t)__shfl(len, src);
      uint32_t v = lane < rl ? out[rb + lane] : NONE;
#pragma unroll
      for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
          const uint32_t u = __shfl_xor(v, (int)j);
          const bool up = (lane & k) == 0, lower = (lane & j) == 0;
          v = (lower == up) ? min(v, u) : max(v, u);
        }
      }
      if (lane < rl) out[rb + lane] = v;
    }
  }
}

// One workgroup per listed row of 65..4096 entries: bitonic sort in LDS, padded to a power of two.
__global__ void __launch_bounds__(BLOCK) k_rows_lds(const uint64_t* __restrict__ ptr, uint32_t* __restrict__ out,
                                                    const uint32_t* __restrict__ lists,
                                                    const uint32_t* __restrict__ nlist) {
  __shared__ uint32_t s[LDS_MAX];
  const uint32_t nrows = *nlist, tid = threadIdx.x;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[q];
    const uint64_t b = ptr[r];
    const uint32_t len = (uint32_t)(ptr[r + 1] - b);
    uint32_t P = 128;
    while (P < len) P <<= 1;
    for (uint32_t i = tid; i < P; i += BLOCK) s[i] = i < len ? out[b + i] : NONE;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t t = tid; t < P / 2; t += BLOCK) {
          const uint32_t i = 2 * t - (t & (j - 1)), p = i + j;
          const uint32_t a = s[i], c = s[p];
          if ((a > c) == ((i & k) == 0)) {
            s[i] = c;
            s[p] = a;
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t i = tid; i < len; i += BLOCK) out[b + i] = s[i];
    __syncthreads();
  }
}

// Long rows with a bit matrix: the row's set bits are its entries, already in column order.
// One workgroup per row: popcounts of 256 words, block scan, then each lane writes its
// word's columns.
__global__ void __launch_bounds__(BLOCK) k_rows_bits(const uint64_t* __restrict__ ptr, uint32_t* __restrict__ out,
                                                     const uint32_t* __restrict__ lists,
                                                     const uint32_t* __restrict__ nlist, uint32_t R, uint32_t lo,
                                                     const uint32_t* __restrict__ bits, uint64_t W) {
  __shared__ uint32_t wsum[BLOCK / 64];
  const uint32_t nrows = nlist[64], tid = threadIdx.x, lane = __lane_id(), wv = tid >> 6;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[R + q];
    const uint32_t* __restrict__ row = bits + (uint64_t)(r + lo) * W;
    uint64_t at = ptr[r];
    for (uint64_t w0 = 0; w0 < W; w0 += BLOCK) {
      const uint64_t w = w0 + tid;
      uint32_t word = w < W ? row[w] : 0u;
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
        out[o++] = (uint32_t)(w * 32 + bit);
        word &= word - 1;
      }
      at += total;
      __syncthreads();
    }
  }
}

// Long rows without a bit matrix: bitonic sort in place in global memory, one workgroup per
// row.  The network only ever puts the smaller value at the lower index (the first merge step
// of each stage compares mirrored positions), so positions past the row act as +inf and are
// never touched.
__global__ void __launch_bounds__(BLOCK) k_rows_global(const uint64_t* __restrict__ ptr, uint32_t* out,
                                                       const uint32_t* __restrict__ lists,
                                                       const uint32_t* __restrict__ nlist, uint32_t R) {
  const uint32_t nrows = nlist[64], tid = threadIdx.x;
  for (uint32_t q = blockIdx.x; q < nrows; q += gridDim.x) {
    const uint32_t r = lists[R + q];
    const uint64_t b = ptr[r];
    const uint64_t len = ptr[r + 1] - b;
    uint32_t* v = out + b;
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
  }
}

struct Widen {
  __host__ __device__ uint64_t operator()(uint32_t v) const { return v; }
};

}  // namespace

void Scratch::release() {
  for (void* p : {(void*)rank, (void*)cnt, (void*)lists, (void*)nlist, cub})
    if (p) (void)hipFree(p);
  rank = cnt = lists = nlist = nullptr;
  cub = nullptr;
  rank_cap = cnt_cap = list_cap = 0;
  cub_bytes = 0;
}

void build(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
           uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* out, const uint32_t* bits, uint64_t W) {
  ensure(sc.rank, sc.rank_cap, n);
  ensure(sc.cnt, sc.cnt_cap, (uint64_t)R + 1);
  ensure(sc.lists, sc.list_cap, 2 * (uint64_t)R + 2);
  if (!sc.nlist) RCHK(hipMalloc((void**)&sc.nlist, 128 * sizeof(uint32_t)));
  RCHK(hipMemsetAsync(sc.cnt, 0, ((uint64_t)R + 1) * sizeof(uint32_t), s));
  RCHK(hipMemsetAsync(sc.nlist, 0, 128 * sizeof(uint32_t), s));
  if (n) {
    hipLaunchKernelGGL(k_rows_count, dim3(grid(n, 2048)), dim3(BLOCK), 0, s, rows, n, row_lo, sc.cnt, sc.rank);
    RCHK(hipGetLastError());
  }
  hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t*> in(sc.cnt, Widen{});
  size_t bytes = 0;
  RCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, ptr, (int)(R + 1), s));
  if (bytes > sc.cub_bytes) {
    if (sc.cub) (void)hipFree(sc.cub);
    sc.cub = nullptr;
    sc.cub_bytes = bytes;
    RCHK(hipMalloc(&sc.cub, bytes));
  }
  RCHK(hipcub::DeviceScan::ExclusiveSum(sc.cub, bytes, in, ptr, (int)(R + 1), s));
  if (!n) return;
  hipLaunchKernelGGL(k_rows_scatter, dim3(grid(n, 2048)), dim3(BLOCK), 0, s, rows, vals, n, row_lo, ptr, sc.rank,
                     keymap, out);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_small, dim3(grid(((uint64_t)R + 63) / 64 * 64, 2048)), dim3(BLOCK), 0, s, ptr, R, out,
                     sc.lists, sc.nlist);
  RCHK(hipGetLastError());
  hipLaunchKernelGGL(k_rows_lds, dim3(2048), dim3(BLOCK), 0, s, ptr, out, sc.lists, sc.nlist);
  RCHK(hipGetLastError());
  if (bits)
    hipLaunchKernelGGL(k_rows_bits, dim3(512), dim3(BLOCK), 0, s, ptr, out, sc.lists, sc.nlist, R, row_lo, bits, W);
  else
    hipLaunchKernelGGL(k_rows_global, dim3(512), dim3(BLOCK), 0, s, ptr, out, sc.lists, sc.nlist, R);
  RCHK(hipGetLastError());
}

}  // namespace elrows
