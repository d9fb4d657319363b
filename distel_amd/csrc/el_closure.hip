// el_closure.hip — the told closure (told*, exr*, exl* rows) and the state derived from it,
// built on the device per classification (see el_closure.h).
//
// Kahn levels, top down: a launch per level; each wave takes one ready concept A at a time,
// gathers the rows of its told supers (and the supers themselves, and A's own existential
// axioms) into its LDS, sorts them (bitonic), drops duplicates, and appends the three rows.
// Integer work: the gathers are row reads (coalesced per super), the sorts stay in LDS, and the
// writes are coalesced appends into per-wave reserved chunks (one atomic per 4096 entries, not
// one per concept: a counter hit by 390 k concepts would serialise at ~12 ns a hit,
// MI355X_MICROARCH.md "fanin").
#include "el_closure.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>

namespace elcl {
namespace {

constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t CAPW = 2048;   // LDS per wave: 2048 32-bit keys = 1024 64-bit keys (8 KB)
constexpr uint32_t CHUNK = 4096;  // per-wave row reservation (entries)
constexpr uint32_t TOP = 1, BOT = 0;
constexpr uint8_t KIND_DATATYPE = 3;
constexpr uint32_t WAVES = BLOCK / 64;

#define CCHK(expr)                                                                                   \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }

__device__ __forceinline__ unsigned long long wsum(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Memory of a row being sorted: the wave's LDS (in-order per wave: a compiler fence between the
// stages keeps the lanes' accesses in program order), or global scratch for a row beyond the
// LDS (coherent accesses and a full fence per stage; rare).
struct Lds {
  template <class K>
  __device__ static K ld(K* p) {
    return *p;
  }
  template <class K>
  __device__ static void st(K* p, K v) {
    *p = v;
  }
  __device__ static void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
};
struct Glb {
  template <class K>
  __device__ static K ld(K* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  template <class K>
  __device__ static void st(K* p, K v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ static void sync() { __threadfence(); }
};

// The concatenation of the lanes' segments (lane i: len_i entries), 64 entries a round: every
// lane runs every round; f(valid, owner lane, offset in the owner's segment, index in the
// concatenation).  Owners by binary lifting over the inclusive scan of the lengths.
template <class F>
__device__ __forceinline__ uint32_t wave_concat(uint32_t len, F&& f) {
  const uint32_t ln = lane();
  uint32_t inc = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (ln >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, 63), excl = inc - len;
  for (uint32_t base = 0; base < total; base += 64) {
    const uint32_t k = base + ln;
    uint32_t own = 0;
#pragma unroll
    for (uint32_t step = 32; step > 0; step >>= 1)
      if (__shfl(inc, (int)(own + step - 1)) <= k) own += step;
    const bool valid = k < total;
    own = valid ? own : 0u;
    f(valid, own, k - __shfl(excl, (int)own), k);
  }
  return total;
}

// Sort b[0, n) ascending (bitonic, padded to a power of two with ~0), then keep one copy of
// each value except `excl`, in place.  Returns the count (wave-uniform).
template <class M, class K>
__device__ uint32_t sort_unique(K* b, uint32_t n, K excl) {
  if (n == 0) return 0;
  const K PAD = ~K(0);
  uint32_t m = 1;
  while (m < n) m <<= 1;
  for (uint32_t i = n + lane(); i < m; i += 64) M::st(b + i, PAD);
  M::sync();
  for (uint32_t k = 2; k <= m; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = lane(); t < (m >> 1); t += 64) {
        const uint32_t i = 2 * t - (t & (j - 1)), p = i + j;  // i: bit j clear
        const K x = M::ld(b + i), y = M::ld(b + p);
        if ((x > y) == ((i & k) == 0)) {
          M::st(b + i, y);
          M::st(b + p, x);
        }
      }
      M::sync();
    }
  uint32_t cnt = 0;
  K prev = PAD;
  for (uint32_t base = 0; base < n; base += 64) {  // (writes land at or below the entries read)
    const uint32_t i = base + lane();
    const K v = i < n ? M::ld(b + i) : PAD;
    K pv = __shfl_up(v, 1);
    if (lane() == 0) pv = prev;
    const bool keep = i < n && v != PAD && v != excl && v != pv;
    const unsigned long long mk = __ballot(keep);
    prev = __shfl(v, 63);
    M::sync();
    if (keep) M::st(b + cnt + (uint32_t)__popcll(mk & ((1ull << lane()) - 1ull)), v);
    cnt += (uint32_t)__popcll(mk);
  }
  M::sync();
  return cnt;
}

// Row space: a wave appends its rows into a chunk it reserved (one atomic per CHUNK entries);
// a row larger than a quarter chunk gets its own reservation.  NONE (and the overflow flag) when
// the row array is full: the host grows it and builds again.
__device__ uint32_t reserve(const Out& o, uint32_t which, uint32_t n, uint32_t cap, uint32_t* tail) {
  if (n == 0) return 0;
  uint32_t r = 0;
  if (lane() == 0) {
    const uint32_t slot = blockIdx.x * WAVES + (threadIdx.x >> 6);
    uint32_t* st = o.rsv + 6 * slot + 2 * which;
    if (n > CHUNK / 4) {
      r = atomicAdd(tail, n);
    } else {
      uint32_t nx = st[0], en = st[1];
      if (en - nx < n) {
        nx = atomicAdd(tail, CHUNK);
        en = nx + CHUNK;
      }
      r = nx;
      st[0] = nx + n;
      st[1] = en;
    }
    if ((uint64_t)r + n > cap) {
      atomicOr(&o.ctr->ovf, 1u);
      r = NONE;
    }
  }
  return __shfl(r, 0);
}

// global scratch for a row that does not fit the LDS: pow2(n) keys of K (nullptr: overflow)
template <class K>
__device__ K* scratch_take(const Out& o, uint32_t n) {
  uint64_t m = 1;
  while (m < n) m <<= 1;
  const uint64_t words = (m * sizeof(K) + 7) / 8 * 2;  // 8-B aligned
  unsigned long long r = 0;
  if (lane() == 0) {
    r = atomicAdd(&o.ctr->s_tail, (unsigned long long)(words / 2));
    if (2 * r + words > o.scratch_cap) {
      atomicOr(&o.ctr->ovf, 1u);
      r = ~0ull;
    }
  }
  r = __shfl(r, 0);
  return r == ~0ull ? nullptr : reinterpret_cast<K*>(o.scratch + 2 * r);
}

template <class M>
__device__ void copy_out(uint32_t* dst, uint32_t* src, uint32_t n) {
  for (uint32_t i = lane(); i < n; i += 64) dst[i] = M::ld(src + i);
}

// told*(A): the supers themselves and their rows
template <class M>
__device__ void gather_told(const Axioms& ax, const Out& o, uint32_t pb, uint32_t pe, uint32_t* buf) {
  uint32_t off = 0;
  for (uint32_t q0 = pb; q0 < pe; q0 += 64) {
    const uint32_t q = q0 + lane();
    uint32_t p = 0, rb = 0, len = 0;
    if (q < pe) {
      p = ax.par[q];
      const uint4 b = o.meta[2 * p], e = o.meta[2 * p + 1];
      rb = b.x;
      len = 1 + e.x - b.x;
    }
    off += wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t k) {
      const uint32_t po = __shfl(p, (int)own), ro = __shfl(rb, (int)own);
      if (v) M::st(buf + off + k, j == 0 ? po : o.t_val[ro + j - 1]);
    });
  }
}

// exr*(A): A's own pairs, then the supers' rows
template <class M>
__device__ void gather_exr(const Axioms& ax, const Out& o, uint32_t A, uint32_t pb, uint32_t pe, uint32_t* buf) {
  const uint32_t xb = ax.xr_ptr[A], xn = ax.xr_ptr[A + 1] - xb;
  for (uint32_t i = lane(); i < xn; i += 64) M::st(buf + i, ax.xr[xb + i]);
  uint32_t off = xn;
  for (uint32_t q0 = pb; q0 < pe; q0 += 64) {
    const uint32_t q = q0 + lane();
    uint32_t rb = 0, len = 0;
    if (q < pe) {
      const uint32_t p = ax.par[q];
      const uint4 b = o.meta[2 * p], e = o.meta[2 * p + 1];
      rb = b.z;
      len = e.z - b.z;
    }
    off += wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t k) {
      const uint32_t ro = __shfl(rb, (int)own);
      if (v) M::st(buf + off + k, o.e_val[ro + j]);
    });
  }
}

// exl*(A) as 64-bit keys (r << 32 | B)
template <class M>
__device__ void gather_exl(const Axioms& ax, const Out& o, uint32_t A, uint32_t pb, uint32_t pe,
                           unsigned long long* buf) {
  const uint32_t yb = ax.xl_ptr[A], yn = ax.xl_ptr[A + 1] - yb;
  for (uint32_t i = lane(); i < yn; i += 64)
    M::st(buf + i, ((unsigned long long)ax.xl_r[yb + i] << 32) | ax.xl_b[yb + i]);
  uint32_t off = yn;
  for (uint32_t q0 = pb; q0 < pe; q0 += 64) {
    const uint32_t q = q0 + lane();
    uint32_t rb = 0, len = 0;
    if (q < pe) {
      const uint32_t p = ax.par[q];
      const uint4 b = o.meta[2 * p], e = o.meta[2 * p + 1];
      rb = b.w;
      len = e.w - b.w;
    }
    off += wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t k) {
      const uint32_t ro = __shfl(rb, (int)own);
      if (v) M::st(buf + off + k, ((unsigned long long)o.l_r[ro + j] << 32) | o.l_b[ro + j]);
    });
  }
}

// pid of (r, Y) by a binary search of Y's pair range (sorted by role), or NONE
__device__ __forceinline__ uint32_t pid_of(const Axioms& ax, uint32_t r, uint32_t fb, uint32_t fe) {
  while (fb < fe) {
    const uint32_t mid = (fb + fe) >> 1, rr = ax.pair_role[mid];
    if (rr == r) return mid;
    if (rr < r)
      fb = mid + 1;
    else
      fe = mid;
  }
  return NONE;
}

__device__ __forceinline__ bool two_of(const Axioms& ax, uint32_t x) {
  return x != TOP && x != BOT && ax.kind[x] != KIND_DATATYPE;
}

// One concept's three rows and statistics (a wave; A wave-uniform).  RELAX: a relaxation round
// (told cycles): the concept's current rows are in meta; a row is rewritten only when it grew,
// and the new ranges go to meta2 (committed after the round).
template <bool RELAX>
__device__ void node(const Axioms& ax, const Out& o, uint32_t A, uint32_t L, bool props, uint32_t* lbuf,
                     bool& any) {
  const uint32_t pb = ax.par_ptr[A], pe = ax.par_ptr[A + 1];
  unsigned long long st = 0, se = 0, sl = 0;
  for (uint32_t q = pb + lane(); q < pe; q += 64) {
    const uint32_t p = ax.par[q];
    const uint4 b = o.meta[2 * p], e = o.meta[2 * p + 1];
    st += 1 + e.x - b.x;
    se += e.z - b.z;
    sl += e.w - b.w;
  }
  st = wsum(st);
  se = wsum(se) + (ax.xr_ptr[A + 1] - ax.xr_ptr[A]);
  sl = wsum(sl) + (ax.xl_ptr[A + 1] - ax.xl_ptr[A]);
  const uint4 ob = o.meta[2 * A], oe = o.meta[2 * A + 1];
  uint4 nb = ob, ne = oe;
  bool grew = false;
  const uint32_t N1 = ax.N + 1;
  uint32_t ninit = 0, cz = 0, sc = 0, sc0 = 0, lift = 0, np = 0;
  const bool two = two_of(ax, A);
  // ---- told*(A)
  {
    const bool big = st > CAPW;
    uint32_t* buf = big ? scratch_take<uint32_t>(o, (uint32_t)st) : lbuf;
    uint32_t n = 0;
    if (buf) {
      if (big) {
        gather_told<Glb>(ax, o, pb, pe, buf);
        n = sort_unique<Glb>(buf, (uint32_t)st, A);
      } else {
        gather_told<Lds>(ax, o, pb, pe, buf);
        n = sort_unique<Lds>(buf, (uint32_t)st, A);
      }
      unsigned long long c = 0;
      bool top = false;
      for (uint32_t i = lane(); i < n; i += 64) {
        const uint32_t v = big ? Glb::ld(buf + i) : buf[i];
        c += ax.cidx_ptr[v + 1] - ax.cidx_ptr[v];
        top |= i < 2 && v == TOP;
      }
      cz = (uint32_t)wsum(c);
      top = __ballot(top) != 0;
      ninit = 1 + (two ? 1u : 0u) + n - ((two && top) ? 1u : 0u);
      if (!RELAX || n != oe.x - ob.x) {
        grew = true;
        const uint32_t r = reserve(o, 0, n, o.t_cap, &o.ctr->t_tail);
        if (r != NONE) {
          if (big)
            copy_out<Glb>(o.t_val + r, buf, n);
          else
            copy_out<Lds>(o.t_val + r, buf, n);
          nb.x = r;
          ne.x = r + n;
        }
      }
    }
    Lds::sync();
  }
  // ---- exr*(A)
  {
    const bool big = se > CAPW;
    uint32_t* buf = big ? scratch_take<uint32_t>(o, (uint32_t)se) : lbuf;
    uint32_t n = 0;
    if (buf) {
      if (big) {
        gather_exr<Glb>(ax, o, A, pb, pe, buf);
        n = sort_unique<Glb>(buf, (uint32_t)se, NONE);
      } else {
        gather_exr<Lds>(ax, o, A, pb, pe, buf);
        n = sort_unique<Lds>(buf, (uint32_t)se, NONE);
      }
      unsigned long long a = 0, b = 0, c = 0;
      for (uint32_t i = lane(); i < n; i += 64) {
        const uint32_t p = big ? Glb::ld(buf + i) : buf[i];
        a += ax.sc_w[p];
        b += ax.sc_self[p];
        c += ax.psup_ptr[p + 1] - ax.psup_ptr[p];
      }
      sc = (uint32_t)wsum(a);
      sc0 = (uint32_t)wsum(b);
      lift = (uint32_t)wsum(c);
      if (!RELAX || n != oe.z - ob.z) {
        grew = true;
        const uint32_t r = reserve(o, 1, n, o.e_cap, &o.ctr->e_tail);
        if (r != NONE) {
          if (big)
            copy_out<Glb>(o.e_val + r, buf, n);
          else
            copy_out<Lds>(o.e_val + r, buf, n);
          nb.z = r;
          ne.z = r + n;
        }
      }
    }
    Lds::sync();
  }
  // ---- exl*(A)
  {
    const bool big = sl > CAPW / 2;
    unsigned long long* buf =
        big ? scratch_take<unsigned long long>(o, (uint32_t)sl) : reinterpret_cast<unsigned long long*>(lbuf);
    uint32_t n = 0;
    if (buf) {
      if (big) {
        gather_exl<Glb>(ax, o, A, pb, pe, buf);
        n = sort_unique<Glb>(buf, (uint32_t)sl, ~0ull);
      } else {
        gather_exl<Lds>(ax, o, A, pb, pe, buf);
        n = sort_unique<Lds>(buf, (uint32_t)sl, ~0ull);
      }
      const uint32_t fb = ax.fp_ptr[A], fe = ax.fp_ptr[A + 1];
      const bool write = !RELAX || n != oe.w - ob.w;
      const uint32_t r = write ? reserve(o, 2, n, o.l_cap, &o.ctr->l_tail) : NONE;
      unsigned long long m = 0;
      for (uint32_t i = lane(); i < n; i += 64) {
        const unsigned long long k = big ? Glb::ld(buf + i) : buf[i];
        if (r != NONE) {
          o.l_r[r + i] = (uint32_t)(k >> 32);
          o.l_b[r + i] = (uint32_t)k;
        }
        if (props && fb < fe) m += pid_of(ax, (uint32_t)(k >> 32), fb, fe) != NONE;
      }
      np = (uint32_t)wsum(m);
      if (write) {
        grew = true;
        if (r != NONE) {
          nb.w = r;
          ne.w = r + n;
        }
      }
    }
    Lds::sync();
  }
  if (lane() == 0) {
    o.nd[ND_INIT * N1 + A] = ninit;
    o.nd[ND_EXR * N1 + A] = ne.z - nb.z;
    o.nd[ND_PROPS * N1 + A] = np;
    o.nd[ND_CZ * N1 + A] = cz;
    o.nd[ND_SC * N1 + A] = sc;
    o.nd[ND_SC0 * N1 + A] = sc0;
    o.nd[ND_LIFT * N1 + A] = lift;
    if (!RELAX) {
      o.meta[2 * A] = nb;
      o.meta[2 * A + 1] = ne;
    } else if (grew) {
      o.meta2[2 * A] = nb;
      o.meta2[2 * A + 1] = ne;
      o.changed[A] = 1;
      o.ctr->dirty = 1;
    }
  }
  const uint32_t cb = ax.chi_ptr[A], ce = ax.chi_ptr[A + 1];
  if (!RELAX) {  // a sub whose last super this was is ready for the next level
    for (uint32_t q = cb + lane(); q < ce; q += 64) {
      const uint32_t c = ax.chi[q];
      if (atomicSub(o.indeg + c, 1u) == 1u) {
        o.level[c] = L + 1;
        any = true;
      }
    }
  } else if (grew) {  // subs still being relaxed see the grown rows next round
    for (uint32_t q = cb + lane(); q < ce; q += 64) {
      const uint32_t c = ax.chi[q];
      if (o.level[c] == NONE) o.dirty2[c] = 1;
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_start(Axioms ax, Out o) {
  const uint32_t stride = gridDim.x * blockDim.x;
  bool root = false;
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += stride) {
    const uint32_t d = ax.par_ptr[A + 1] - ax.par_ptr[A];
    o.indeg[A] = d;
    o.level[A] = d ? NONE : 0u;
    root |= d == 0;
    o.meta[2 * A] = make_uint4(0u, ax.cidx_ptr[A], 0u, 0u);
    o.meta[2 * A + 1] = make_uint4(0u, ax.cidx_ptr[A + 1], 0u, 0u);
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < RSV_WORDS; i += stride) o.rsv[i] = 0;
  if (root) o.lvl_flag[0] = 1;  // (zeroed by the host before this launch)
}

__global__ void __launch_bounds__(BLOCK) k_level(Axioms ax, Out o, uint32_t L, uint32_t props) {
  if (o.lvl_flag[L] == 0) return;  // (block-uniform: nothing at this level)
  __shared__ unsigned long long lds[WAVES * (CAPW / 2)];
  __shared__ uint32_t sany;
  if (threadIdx.x == 0) sany = 0;
  __syncthreads();
  uint32_t* lbuf = reinterpret_cast<uint32_t*>(lds + (threadIdx.x >> 6) * (CAPW / 2));
  bool any = false;
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t base = w * 64; base < ax.N; base += nw * 64) {  // (wave-uniform)
    const uint32_t A0 = base + lane();
    unsigned long long m = __ballot(A0 < ax.N && o.level[A0] == L);
    while (m) {
      const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      node<false>(ax, o, base + i, L, props != 0, lbuf, any);
    }
  }
  if (any) sany = 1;
  __syncthreads();
  if (threadIdx.x == 0 && sany) o.lvl_flag[L + 1] = 1;
}

// after the levels: concepts never ready (told cycles and everything below them) are stuck;
// they start the relaxation dirty.  Clears the relaxation flags of every other concept.
__global__ void __launch_bounds__(BLOCK) k_check(Axioms ax, Out o) {
  unsigned long long c = 0;
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += gridDim.x * blockDim.x) {
    const bool stuck = o.level[A] == NONE;
    o.dirty[A] = stuck;
    o.dirty2[A] = 0;
    o.changed[A] = 0;
    c += stuck;
  }
  __shared__ unsigned long long part[WAVES];
  c = wsum(c);
  if (lane() == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (uint32_t w = 0; w < WAVES; ++w) s += part[w];
    if (s) atomicAdd(&o.ctr->tot[T_STUCK], s);
  }
}

__global__ void __launch_bounds__(BLOCK) k_relax(Axioms ax, Out o, uint32_t props) {
  __shared__ unsigned long long lds[WAVES * (CAPW / 2)];
  uint32_t* lbuf = reinterpret_cast<uint32_t*>(lds + (threadIdx.x >> 6) * (CAPW / 2));
  bool any = false;
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t base = w * 64; base < ax.N; base += nw * 64) {
    const uint32_t A0 = base + lane();
    unsigned long long m = __ballot(A0 < ax.N && o.dirty[A0]);
    while (m) {
      const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      node<true>(ax, o, base + i, 0, props != 0, lbuf, any);
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_relax_commit(Axioms ax, Out o) {
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += gridDim.x * blockDim.x) {
    if (o.changed[A]) {
      o.meta[2 * A] = o.meta2[2 * A];
      o.meta[2 * A + 1] = o.meta2[2 * A + 1];
      o.changed[A] = 0;
    }
    o.dirty[A] = o.dirty2[A];
    o.dirty2[A] = 0;
  }
}

// Totals over the own rows [lo, hi) and the closure events over every concept: per concept A
// one trigger, rows: its supers, subs, own exr / exl rows and the three rows of every super;
// entries: the supers, the subs, the rows gathered (the supers' rows, its own axioms) and the
// rows written; one pending-count decrement per sub.  (The CPU oracle counts the same.)
__global__ void __launch_bounds__(BLOCK) k_totals(Axioms ax, Out o, uint32_t lo, uint32_t hi) {
  unsigned long long t[T_NUM - 1] = {}, e[E_NUM] = {};
  const uint32_t N1 = ax.N + 1;
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += gridDim.x * blockDim.x) {
    const uint4 b = o.meta[2 * A], f = o.meta[2 * A + 1];
    const uint32_t tl = f.x - b.x, el = f.z - b.z, ll = f.w - b.w;
    const uint32_t pb = ax.par_ptr[A], pe = ax.par_ptr[A + 1], nch = ax.chi_ptr[A + 1] - ax.chi_ptr[A];
    unsigned long long g = 0;
    for (uint32_t q = pb; q < pe; ++q) {
      const uint32_t p = ax.par[q];
      const uint4 pb4 = o.meta[2 * p], pf4 = o.meta[2 * p + 1];
      g += (pf4.x - pb4.x) + (pf4.z - pb4.z) + 2ull * (pf4.w - pb4.w);
    }
    const uint32_t np = pe - pb;
    e[E_TRIG] += 1;
    e[E_ROW] += 4 + 3ull * np;
    e[E_ENT] += np + nch + g + (ax.xr_ptr[A + 1] - ax.xr_ptr[A]) + 2ull * (ax.xl_ptr[A + 1] - ax.xl_ptr[A]) + tl + el +
                2ull * ll;
    e[E_RMW] += nch;
    if (A >= lo && A < hi) {
      t[T_INIT] += o.nd[ND_INIT * N1 + A];
      t[T_TOLD] += tl;
      t[T_EXR] += el;
      t[T_EXL] += ll;
      t[T_PROPS] += o.nd[ND_PROPS * N1 + A];
      t[T_CZ] += o.nd[ND_CZ * N1 + A];
      t[T_CIDX] += f.y - b.y;
      t[T_TWO] += two_of(ax, A);
      t[T_SC] += o.nd[ND_SC * N1 + A];
      t[T_SC0] += o.nd[ND_SC0 * N1 + A];
      t[T_LIFT] += o.nd[ND_LIFT * N1 + A];
      t[T_OWN] += 1;
    }
  }
  __shared__ unsigned long long part[WAVES][T_NUM - 1 + E_NUM];
  for (uint32_t i = 0; i < T_NUM - 1; ++i) {
    const unsigned long long s = wsum(t[i]);
    if (lane() == 0) part[threadIdx.x >> 6][i] = s;
  }
  for (uint32_t i = 0; i < E_NUM; ++i) {
    const unsigned long long s = wsum(e[i]);
    if (lane() == 0) part[threadIdx.x >> 6][T_NUM - 1 + i] = s;
  }
  __syncthreads();
  if (threadIdx.x < T_NUM - 1 + E_NUM) {
    unsigned long long s = 0;
    for (uint32_t w = 0; w < WAVES; ++w) s += part[w][threadIdx.x];
    if (s) {
      if (threadIdx.x < T_NUM - 1)
        atomicAdd(&o.ctr->tot[threadIdx.x], s);
      else
        atomicAdd(&o.ctr->ev[threadIdx.x - (T_NUM - 1)], s);
    }
  }
}

// ---- state pass: the own rows' init facts, base links and base propagations

// Rows [a, b), one lane per row, slots [pos[x - a], pos[x - a + 1]) + base of the log: the
// wave walks the concatenation of its lanes' slot ranges 64 at a time (coalesced stores).
template <class F>
__device__ __forceinline__ void rows_by_slot(uint32_t a, uint32_t b, const uint32_t* pos, F&& f) {
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t r0 = a + w * 64; r0 < b; r0 += nw * 64) {  // (wave-uniform)
    const uint32_t x = r0 + lane();
    uint32_t s = 0, len = 0;
    if (x < b) {
      s = pos[x - a];
      len = pos[x - a + 1] - s;
    }
    wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t) {
      const uint32_t xo = r0 + own, so = __shfl(s, (int)own);
      f(v, xo, j, so + j);
    });
  }
}

// S(X) = {X, ⊤} for classes and individuals, {X} for ⊤, ⊥ and datatypes
// (AxiomLoader.java:1237-1245 classes, :1281-1289 individuals), with the told closure of X —
// what CR1 derives from the init fact X ∈ S(X) — in one go: X (flag 2: its closure is written
// here), ⊤ (flag 0), told*(X) (flag 1) without a second ⊤.  Bits by atomicOr (no return).
__global__ void __launch_bounds__(BLOCK) k_init_facts(Axioms ax, Out o, uint32_t a, uint32_t b, const uint32_t* pos,
                                                      uint32_t base, uint32_t* slog_x, uint32_t* slog_a,
                                                      uint8_t* slog_f, uint32_t* bits, uint64_t W, uint32_t c_lo,
                                                      uint32_t c_hi, uint8_t* summ, uint32_t SB) {
  rows_by_slot(a, b, pos, [&](bool v, uint32_t x, uint32_t j, uint32_t slot) {
    if (!v) return;
    const bool two = two_of(ax, x);
    const uint32_t t0 = o.meta[2 * x].x, t1 = o.meta[2 * x + 1].x;
    uint32_t val;
    uint8_t f = 1;
    if (j == 0) {
      val = x;
      f = 2;
    } else if (two && j == 1) {
      val = TOP;
      f = 0;
    } else {
      uint32_t c = j - 1 - (two ? 1u : 0u);
      if (two) {  // ⊤ sorts first or right after ⊥ in told*(X): skip it there
        const uint32_t ptop = (t0 < t1 && o.t_val[t0] == TOP) ? 0u : (t0 + 1 < t1 && o.t_val[t0 + 1] == TOP) ? 1u : NONE;
        if (c >= ptop) ++c;
      }
      val = o.t_val[t0 + c];
    }
    slog_x[base + slot] = x;
    slog_a[base + slot] = val;
    slog_f[base + slot] = f;
    const uint32_t col = val < 2u ? val : (val >= c_lo && val < c_hi ? val - c_lo + 2u : NONE);
    if (col != NONE) {
      __hip_atomic_fetch_or(bits + (uint64_t)x * W + (col >> 5), 1u << (col & 31u), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
      if (summ) summ[(uint64_t)x * SB + (col >> 12)] = 1;
    }
  });
}

// the base links {(X, p) : p ∈ exr*(X)} in X order
__global__ void __launch_bounds__(BLOCK) k_base_links(Axioms ax, Out o, uint32_t a, uint32_t b, const uint32_t* pos,
                                                      uint32_t* llog_x, uint32_t* llog_p) {
  rows_by_slot(a, b, pos, [&](bool v, uint32_t x, uint32_t j, uint32_t slot) {
    if (!v) return;
    llog_x[slot] = x;
    llog_p[slot] = o.e_val[o.meta[2 * x].z + j];
  });
}

// the base propagations {((r, Y), B) : (r, B) ∈ exl*(Y), (r, Y) a pair}: pid-major (pids sort by
// (Y, r), exl*(Y) by (r, B)), B ascending within a pid; one wave per Y
__global__ void __launch_bounds__(BLOCK) k_base_props(Axioms ax, Out o, uint32_t a, uint32_t b, const uint32_t* pos,
                                                      uint32_t* plog_p, uint32_t* plog_b) {
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t y = a + w; y < b; y += nw) {
    const uint32_t fb = ax.fp_ptr[y], fe = ax.fp_ptr[y + 1];
    if (fb == fe) continue;
    const uint32_t l0 = o.meta[2 * y].w, l1 = o.meta[2 * y + 1].w;
    uint32_t out = pos[y - a];
    for (uint32_t j0 = l0; j0 < l1; j0 += 64) {
      const uint32_t j = j0 + lane();
      uint32_t pid = NONE, B = 0;
      if (j < l1) {
        pid = pid_of(ax, o.l_r[j], fb, fe);
        B = o.l_b[j];
      }
      const unsigned long long m = __ballot(pid != NONE);
      if (pid != NONE) {
        const uint32_t s = out + (uint32_t)__popcll(m & ((1ull << lane()) - 1ull));
        plog_p[s] = pid;
        plog_b[s] = B;
      }
      out += (uint32_t)__popcll(m);
    }
  }
}

// first / last + 1 index of each key's run in keys[0, n) (each key one run)
__global__ void __launch_bounds__(BLOCK) k_runs(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* first,
                                                uint32_t* last) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    if (i == 0 || keys[i - 1] != k) first[k] = i;
    if (i + 1 == n || keys[i + 1] != k) last[k] = i + 1;
  }
}

// row capacities: cap[p] = last[p] - first[p] (+ the CR5 lifts: every super-role pair u of p
// receives p's count, when psup_ptr is given); cap zeroed by the host
__global__ void __launch_bounds__(BLOCK) k_caps(const uint32_t* first, const uint32_t* last, uint32_t n,
                                                const uint32_t* psup_ptr, const uint32_t* psup, uint32_t* cap,
                                                uint32_t* len) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const uint32_t c = last[p] - first[p];
    if (len) len[p] = c;
    if (!c || !cap) continue;
    atomicAdd(cap + p, c);
    if (psup_ptr)
      for (uint32_t k = psup_ptr[p]; k < psup_ptr[p + 1]; ++k) atomicAdd(cap + psup[k], c);
  }
}

// entries i of a key-grouped list into their gapped rows: val[start[key] + i - first[key]]
__global__ void __launch_bounds__(BLOCK) k_group_fill(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ vals, uint32_t n,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ start, uint32_t* __restrict__ val) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    val[start[k] + i - first[k]] = vals[i];
  }
}

// successor rows of the base links: X's chain-second pids (exr*(X) filtered), one wave per X
__global__ void __launch_bounds__(BLOCK) k_succ_fill(Axioms ax, Out o, uint32_t a, uint32_t b,
                                                     const uint32_t* __restrict__ start, uint32_t* __restrict__ len,
                                                     uint32_t* __restrict__ val) {
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t x = a + w; x < b; x += nw) {
    const uint32_t e0 = o.meta[2 * x].z, e1 = o.meta[2 * x + 1].z;
    uint32_t out = 0;
    const uint32_t s = start[x];
    for (uint32_t j0 = e0; j0 < e1; j0 += 64) {
      const uint32_t j = j0 + lane();
      const uint32_t p = j < e1 ? o.e_val[j] : 0u;
      const bool keep = j < e1 && ax.sc_self[p];
      const unsigned long long m = __ballot(keep);
      if (keep) val[s + out + (uint32_t)__popcll(m & ((1ull << lane()) - 1ull))] = p;
      out += (uint32_t)__popcll(m);
    }
    if (lane() == 0) len[x] = out;
  }
}

uint32_t grid_for(uint64_t n, uint32_t cap = 1024) {
  uint64_t g = (n + BLOCK - 1) / BLOCK;
  return (uint32_t)(g < 1 ? 1 : g > cap ? cap : g);
}

}  // namespace

void start(hipStream_t s, const Axioms& ax, const Out& o) {
  CCHK(hipMemsetAsync(o.ctr, 0, sizeof(Ctr), s));
  CCHK(hipMemsetAsync(o.lvl_flag, 0, ((uint64_t)ax.N + 2) * sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_start, dim3(grid_for(std::max<uint64_t>(ax.N, RSV_WORDS))), dim3(BLOCK), 0, s, ax, o);
  CCHK(hipGetLastError());
}

void level(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L, bool props) {
  hipLaunchKernelGGL(k_level, dim3(GRID), dim3(BLOCK), 0, s, ax, o, L, props ? 1u : 0u);
  CCHK(hipGetLastError());
}

void check(hipStream_t s, const Axioms& ax, const Out& o) {
  hipLaunchKernelGGL(k_check, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o);
  CCHK(hipGetLastError());
}

void relax(hipStream_t s, const Axioms& ax, const Out& o, bool props) {
  CCHK(hipMemsetAsync(&o.ctr->dirty, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_relax, dim3(GRID), dim3(BLOCK), 0, s, ax, o, props ? 1u : 0u);
  hipLaunchKernelGGL(k_relax_commit, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o);
  CCHK(hipGetLastError());
}

void totals(hipStream_t s, const Axioms& ax, const Out& o, uint32_t lo, uint32_t hi) {
  hipLaunchKernelGGL(k_totals, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o, lo, hi);
  CCHK(hipGetLastError());
}

size_t scan_temp_bytes(uint32_t n) {
  size_t b = 0;
  CCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n));
  return b;
}

void scan(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n) {
  CCHK(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s));
}

size_t sort_temp_bytes(uint32_t n) {
  size_t b = 0;
  CCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                          (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n));
  return b;
}

void sort_pairs(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                uint32_t* vout, uint32_t n, uint32_t key_bits) {
  CCHK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, kin, kout, vin, vout, (int)n, 0, (int)key_bits, s));
}

void init_facts(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t base, uint32_t* slog_x, uint32_t* slog_a, uint8_t* slog_f, uint32_t* bits, uint64_t W,
                uint32_t c_lo, uint32_t c_hi, uint8_t* summ, uint32_t SB) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_init_facts, dim3(grid_for((uint64_t)(b - a) * 64, 2048)), dim3(BLOCK), 0, s, ax, o, a, b, pos,
                     base, slog_x, slog_a, slog_f, bits, W, c_lo, c_hi, summ, SB);
  CCHK(hipGetLastError());
}

void base_links(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t* llog_x, uint32_t* llog_p) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_base_links, dim3(grid_for((uint64_t)(b - a) * 64, 2048)), dim3(BLOCK), 0, s, ax, o, a, b, pos,
                     llog_x, llog_p);
  CCHK(hipGetLastError());
}

void base_props(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t* plog_p, uint32_t* plog_b) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_base_props, dim3(grid_for((uint64_t)(b - a) * 64, 2048)), dim3(BLOCK), 0, s, ax, o, a, b, pos,
                     plog_p, plog_b);
  CCHK(hipGetLastError());
}

void runs(hipStream_t s, const uint32_t* keys, uint32_t n, uint32_t* first, uint32_t* last) {
  if (!n) return;
  hipLaunchKernelGGL(k_runs, dim3(grid_for(n, 2048)), dim3(BLOCK), 0, s, keys, n, first, last);
  CCHK(hipGetLastError());
}

void caps(hipStream_t s, const uint32_t* first, const uint32_t* last, uint32_t n, const uint32_t* psup_ptr,
          const uint32_t* psup, uint32_t* cap, uint32_t* len) {
  if (!n) return;
  hipLaunchKernelGGL(k_caps, dim3(grid_for(n)), dim3(BLOCK), 0, s, first, last, n, psup_ptr, psup, cap, len);
  CCHK(hipGetLastError());
}

void group_fill(hipStream_t s, const uint32_t* keys, const uint32_t* vals, uint32_t n, const uint32_t* first,
                const uint32_t* start, uint32_t* val) {
  if (!n) return;
  hipLaunchKernelGGL(k_group_fill, dim3(grid_for(n, 2048)), dim3(BLOCK), 0, s, keys, vals, n, first, start, val);
  CCHK(hipGetLastError());
}

void succ_fill(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* start,
               uint32_t* len, uint32_t* val) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_succ_fill, dim3(grid_for((uint64_t)(b - a) * 64, 2048)), dim3(BLOCK), 0, s, ax, o, a, b, start,
                     len, val);
  CCHK(hipGetLastError());
}

}  // namespace elcl
