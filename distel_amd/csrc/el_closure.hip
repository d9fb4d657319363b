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
#include "el_rows.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>

namespace elcl {
namespace {

constexpr uint32_t NONE = 0xffffffffu;
#ifndef EL_CLOSURE_CAPW
#define EL_CLOSURE_CAPW 2048
#endif
constexpr uint32_t CAPW = EL_CLOSURE_CAPW;  // LDS per wave: 2048 32-bit keys = 1024 64-bit keys (8 KB)
// (a power of two: the LDS bitonic sort pads a row of up to CAPW keys to the next power of two in place)
static_assert((CAPW & (CAPW - 1)) == 0, "CAPW must be a power of two");
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

// Rows of up to 64·E keys sort in registers: lane l holds the keys 64 i + l (i < E); network
// stages with a partner 64 or more keys away compare a lane's own registers, the others
// shuffle (no LDS round trip per stage: a 128-key row is 28 stages of a few cycles each instead
// of 28 LDS load / store rounds).  Then duplicates (and `excl`) drop out and the unique keys
// are written back to b[0, cnt) in order.
template <class K>
__device__ __forceinline__ K bitonic_cx(K v, uint32_t e, uint32_t k, uint32_t j) {
  const K u = __shfl_xor(v, (int)j);
  const bool up = (e & k) == 0, lower = (e & j) == 0;
  return (lower == up) ? (v < u ? v : u) : (v < u ? u : v);
}

template <uint32_t E, class K>
__device__ uint32_t sort_unique_regs(K* b, uint32_t n, K excl) {
  const K PAD = ~K(0);
  const uint32_t ln = lane();
  K v[E];
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) v[i] = 64 * i + ln < n ? b[64 * i + ln] : PAD;
#pragma unroll
  for (uint32_t k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {  // partner in the same lane, register i ^ (j / 64)
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) {
          const uint32_t i2 = i ^ (j / 64);
          if (i2 > i) {
            const uint32_t e = 64 * i + ln;
            const bool up = (e & k) == 0;
            const K x = v[i], y = v[i2];
            if ((x > y) == up) {
              v[i] = y;
              v[i2] = x;
            }
          }
        }
      } else {
#pragma unroll
        for (uint32_t i = 0; i < E; ++i) v[i] = bitonic_cx(v[i], 64 * i + ln, k, j);
      }
    }
  }
  Lds::sync();  // (every lane has read b before any writes back)
  uint32_t cnt = 0;
  K prev = PAD;
#pragma unroll
  for (uint32_t i = 0; i < E; ++i) {
    K pv = __shfl_up(v[i], 1);
    if (ln == 0) pv = prev;
    const bool keep = v[i] != PAD && v[i] != excl && v[i] != pv;
    const unsigned long long mk = __ballot(keep);
    prev = __shfl(v[i], 63);
    if (keep) b[cnt + (uint32_t)__popcll(mk & ((1ull << ln) - 1ull))] = v[i];
    cnt += (uint32_t)__popcll(mk);
  }
  Lds::sync();
  return cnt;
}

// LDS rows: in registers up to 512 32-bit / 256 64-bit keys, else the LDS network
template <class K>
__device__ uint32_t sort_unique_lds(K* b, uint32_t n, K excl) {
  if (n == 0) return 0;
  if (n <= 64) return sort_unique_regs<1>(b, n, excl);
  if (n <= 128) return sort_unique_regs<2>(b, n, excl);
  if (n <= 256) return sort_unique_regs<4>(b, n, excl);
  if (sizeof(K) == 4 && n <= 512) return sort_unique_regs<8>(b, n, excl);
  return sort_unique<Lds>(b, n, excl);
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

// Row space: a wave appends its rows into a chunk it reserved (one atomic per CHUNK entries);
// a row larger than a quarter chunk gets its own reservation.  A wave's chunk state stays in
// registers for the launch (Out::rsv keeps it between launches).  NONE (and the overflow flag)
// when the row array is full: the host grows it and builds again.
struct Rsv {
  uint32_t nx[3], en[3];
};

__device__ __forceinline__ uint32_t slot_id() { return blockIdx.x * WAVES + (threadIdx.x >> 6); }

__device__ Rsv rsv_load(const Out& o) {
  Rsv r;
  const uint32_t* s = o.rsv + 6 * slot_id();
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.nx[i] = __builtin_amdgcn_readfirstlane(s[2 * i]);
    r.en[i] = __builtin_amdgcn_readfirstlane(s[2 * i + 1]);
  }
  return r;
}

__device__ void rsv_store(const Out& o, const Rsv& r) {
  if (lane() == 0) {
    uint32_t* s = o.rsv + 6 * slot_id();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      s[2 * i] = r.nx[i];
      s[2 * i + 1] = r.en[i];
    }
  }
}

__device__ uint32_t reserve(const Out& o, Rsv& rs, uint32_t which, uint32_t n, uint32_t cap, uint32_t* tail) {
  if (n == 0) return 0;
  uint32_t r;
  if (n > CHUNK / 4) {
    uint32_t b = 0;
    if (lane() == 0) b = atomicAdd(tail, n);
    r = __builtin_amdgcn_readfirstlane(b);
  } else {
    if (rs.en[which] - rs.nx[which] < n) {
      uint32_t b = 0;
      if (lane() == 0) b = atomicAdd(tail, CHUNK);
      b = __builtin_amdgcn_readfirstlane(b);
      rs.nx[which] = b;
      rs.en[which] = b + CHUNK;
    }
    r = rs.nx[which];
    rs.nx[which] += n;
  }
  if ((uint64_t)r + n > cap) {
    if (lane() == 0) atomicOr(&o.ctr->ovf, 1u);
    return NONE;
  }
  return r;
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

// The three row types.  Each depends only on the rows of the same type of the told supers (and
// the concept's own axioms), so the three of a concept are independent tasks.
enum : uint32_t { R_TOLD = 0, R_EXR = 1, R_EXL = 2 };
// meta word of a row type: told* -> .x, exr* -> .z, exl* -> .w (of the begin / end uint4)
template <uint32_t T>
struct RowT {
  static constexpr uint32_t comp = T == R_TOLD ? 0u : T == R_EXR ? 2u : 3u;
  using K = typename std::conditional<T == R_EXL, unsigned long long, uint32_t>::type;
  static constexpr uint32_t lds_cap = T == R_EXL ? CAPW / 2 : CAPW;
};

__device__ __forceinline__ uint32_t meta_word(const uint4* meta, uint32_t A, uint32_t end, uint32_t comp) {
  return reinterpret_cast<const uint32_t*>(meta + 2 * A + end)[comp];
}

// The rows of type T of the supers [pb, pe) (with each super itself first, for told*) after
// A's own axioms, concatenated into buf.
template <uint32_t T, class M>
__device__ void gather(const Axioms& ax, const Out& o, uint32_t A, uint32_t pb, uint32_t pe,
                       typename RowT<T>::K* buf) {
  using K = typename RowT<T>::K;
  uint32_t off = 0;
  if (T == R_TOLD && ax.tx_ptr) {  // a told cycle's representative: the other members
    const uint32_t b0 = ax.tx_ptr[A], n0 = ax.tx_ptr[A + 1] - b0;
    for (uint32_t i = lane(); i < n0; i += 64) M::st(buf + i, (K)ax.tx[b0 + i]);
    off = n0;
  } else if (T == R_EXR) {
    const uint32_t b0 = ax.xr_ptr[A], n0 = ax.xr_ptr[A + 1] - b0;
    for (uint32_t i = lane(); i < n0; i += 64) M::st(buf + i, (K)ax.xr[b0 + i]);
    off = n0;
  } else if (T == R_EXL) {
    const uint32_t b0 = ax.xl_ptr[A], n0 = ax.xl_ptr[A + 1] - b0;
    for (uint32_t i = lane(); i < n0; i += 64) M::st(buf + i, ((K)ax.xl_r[b0 + i] << 32) | ax.xl_b[b0 + i]);
    off = n0;
  }
  for (uint32_t q0 = pb; q0 < pe; q0 += 64) {
    const uint32_t q = q0 + lane();
    uint32_t p = 0, rb = 0, len = 0;
    if (q < pe) {
      p = ax.par[q];
      rb = meta_word(o.meta, p, 0, RowT<T>::comp);
      len = meta_word(o.meta, p, 1, RowT<T>::comp) - rb + (T == R_TOLD ? 1u : 0u);
    }
    off += wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t k) {
      const uint32_t po = __shfl(p, (int)own), ro = __shfl(rb, (int)own);
      if (!v) return;
      K key;
      if (T == R_TOLD)
        key = j == 0 ? po : o.t_val[ro + j - 1];
      else if (T == R_EXR)
        key = o.e_val[ro + j];
      else
        key = ((K)o.l_r[ro + j] << 32) | o.l_b[ro + j];
      M::st(buf + off + k, key);
    });
  }
}

// A level task's head values, loaded for 64 tasks at once (one lane each) before the wave runs
// them one by one: the told supers (≤ 2 of them), their rows of the task's type, and the
// concept's own list (xr / xl range; for told*, its subs).  Each was a dependent global load at the
// head of every task (par_ptr -> par -> meta, xr_ptr), ~1-2 µs apiece under load.
struct Pre {
  uint32_t pb, pe;     // told supers [pb, pe) in par
  uint32_t P1, P2;     // the first two supers
  uint32_t b1, n1, b2, n2;  // their rows of the task's type
  uint32_t ob, on;     // own list: xr / xl range (exr* / exl*), subs in chi (told*)
};

__device__ __forceinline__ Pre pre_load(const Axioms& ax, const Out& o, uint32_t A, uint32_t T) {
  Pre p{};
  p.pb = ax.par_ptr[A];
  p.pe = ax.par_ptr[A + 1];
  const uint32_t comp = T == R_TOLD ? 0u : T == R_EXR ? 2u : 3u;
  if (p.pe > p.pb) {
    p.P1 = ax.par[p.pb];
    p.b1 = meta_word(o.meta, p.P1, 0, comp);
    p.n1 = meta_word(o.meta, p.P1, 1, comp) - p.b1;
  }
  if (p.pe - p.pb == 2) {
    p.P2 = ax.par[p.pb + 1];
    p.b2 = meta_word(o.meta, p.P2, 0, comp);
    p.n2 = meta_word(o.meta, p.P2, 1, comp) - p.b2;
  }
  const uint32_t* op = T == R_TOLD ? ax.chi_ptr : T == R_EXR ? ax.xr_ptr : ax.xl_ptr;
  p.ob = op[A];
  p.on = op[A + 1] - p.ob;
  return p;
}

// lane i's Pre, wave-uniform
__device__ __forceinline__ Pre pre_of(const Pre& p, int i) {
  Pre q;
  q.pb = __shfl(p.pb, i), q.pe = __shfl(p.pe, i);
  q.P1 = __shfl(p.P1, i), q.P2 = __shfl(p.P2, i);
  q.b1 = __shfl(p.b1, i), q.n1 = __shfl(p.n1, i), q.b2 = __shfl(p.b2, i), q.n2 = __shfl(p.n2, i);
  q.ob = __shfl(p.ob, i), q.on = __shfl(p.on, i);
  return q;
}

// A concept with at most one told super P (in the Kahn levels: no cycle through A, so A is not in
// P's rows): its row of type T is P's row merged with a short sorted list — {P} for told*, A's own
// axioms xr(A) / xl(A) (sorted, unique) for exr* / exl*.  A merge, not a sort: each list entry
// finds its place in P's row by a binary search (and drops out if P's row holds it), each entry
// of P's row moves up by the list entries below it, and the row is written straight into its
// reservation (coalesced).  Returns false when the list has more than 64 entries (the caller
// sorts).  Writes meta like task().  P's row is staged in the wave's LDS first (one coalesced read)
// when it fits, so the binary searches cost LDS latency, not a chain of dependent global loads.
template <uint32_t T>
__device__ bool task_merge1(const Axioms& ax, const Out& o, uint32_t A, const Pre& pr, uint32_t* lbuf, Rsv& rs) {
  using K = typename RowT<T>::K;
  const uint32_t pb = pr.pb, pe = pr.pe;
  uint32_t s = 0;
  K sv = 0;
  if (T == R_TOLD) {
    s = pe > pb ? 1u : 0u;
    if (s && lane() == 0) sv = (K)pr.P1;
  } else if (T == R_EXR) {
    const uint32_t b0 = pr.ob;
    s = pr.on;
    if (s > 64) return false;
    if (lane() < s) sv = (K)ax.xr[b0 + lane()];
  } else {
    const uint32_t b0 = pr.ob;
    s = pr.on;
    if (s > 64) return false;
    if (lane() < s) sv = ((K)ax.xl_r[b0 + lane()] << 32) | ax.xl_b[b0 + lane()];
  }
  uint32_t lb = 0, n = 0;
  if (pe > pb) {
    lb = pr.b1;
    n = pr.n1;
  }
#ifndef EL_NO_ROW_SHARE  // (A/B build: every row copied, as round 4)
  if (T != R_TOLD && s == 0) {
    // no own axioms of this type: the row IS the super's row (exr*(A) = exr*(P), exl*(A) =
    // exl*(P)), so A's meta points at it — no copy.  Rows are read-only once built and every
    // reader goes through meta; the closure events are counted from the final row sizes
    // (k_totals), so they are unchanged.  G3: 193 k of the 900 k non-root tasks, 21 M of the
    // 86 M row entries.
    if (lane() == 0) {
      reinterpret_cast<uint32_t*>(o.meta + 2 * A)[RowT<T>::comp] = lb;
      reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1)[RowT<T>::comp] = lb + n;
    }
    return true;
  }
#endif
  auto at_g = [&](uint32_t j) -> K {
    if (T == R_TOLD) return (K)o.t_val[lb + j];
    if (T == R_EXR) return (K)o.e_val[lb + j];
    return ((K)o.l_r[lb + j] << 32) | o.l_b[lb + j];
  };
  K* rowl = reinterpret_cast<K*>(lbuf);
  const bool staged = n <= RowT<T>::lds_cap;
  if (staged) {
    for (uint32_t j = lane(); j < n; j += 64) rowl[j] = at_g(j);
    Lds::sync();
  }
  auto at = [&](uint32_t j) -> K { return staged ? rowl[j] : at_g(j); };
  // the list entries: rank in P's row, dropped when P's row holds them
  uint32_t rank = 0;
  bool kept = false;
  if (lane() < s) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (at(mid) < sv)
        lo = mid + 1;
      else
        hi = mid;
    }
    rank = lo;
    kept = !(lo < n && at(lo) == sv);
  }
  const unsigned long long km = __ballot(kept);
  const uint32_t nk = (uint32_t)__popcll(km), nout = n + nk;
  const uint32_t cap = T == R_TOLD ? o.t_cap : T == R_EXR ? o.e_cap : o.l_cap;
  uint32_t* tail = T == R_TOLD ? &o.ctr->t_tail : T == R_EXR ? &o.ctr->e_tail : &o.ctr->l_tail;
  const uint32_t r = reserve(o, rs, T, nout, cap, tail);
  if (r == NONE) {  // (overflow flagged: the build is redone larger)
    Lds::sync();
    return true;
  }
  auto put = [&](uint32_t i, K v) {
    if (T == R_TOLD) {
      o.t_val[r + i] = (uint32_t)v;
    } else if (T == R_EXR) {
      o.e_val[r + i] = (uint32_t)v;
    } else {
      o.l_r[r + i] = (uint32_t)((unsigned long long)v >> 32);
      o.l_b[r + i] = (uint32_t)v;
    }
  };
  if (kept) put(rank + (uint32_t)__popcll(km & ((1ull << lane()) - 1ull)), sv);
  for (uint32_t j0 = 0; j0 < n; j0 += 64) {  // (wave-uniform)
    const uint32_t j = j0 + lane();
    K v = 0;
    if (j < n) v = at(j);
    uint32_t below = 0;  // kept list entries below v
    for (unsigned long long m = km; m;) {
      const uint32_t i = (uint32_t)__ffsll((long long)m) - 1u;
      m &= m - 1ull;
      below += __shfl(sv, (int)i) < v ? 1u : 0u;
    }
    if (j < n) put(j + below, v);
  }
  if (lane() == 0) {
    reinterpret_cast<uint32_t*>(o.meta + 2 * A)[RowT<T>::comp] = r;
    reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1)[RowT<T>::comp] = r + nout;
  }
  Lds::sync();  // (lbuf is reused by the wave's next task)
  return true;
}

// Two told supers P1, P2: the row is the union of their rows (sorted, unique) and a short sorted
// list ({P1, P2} for told*, A's own axioms for exr* / exl*), found by ranks instead of a sort.  An
// entry's place in the row is the number of distinct values below it: those of P1's row, those of
// P2's row not in P1's (a prefix count over P2's row, in the wave's LDS), and the list entries in
// neither row below it.  An entry of P2's row or of the list that an earlier source holds drops
// out.  Returns false (the caller sorts) when the list has more than 64 entries or P2's row does
// not fit the LDS prefix.  Both rows are staged in the wave's LDS beside the prefix array when
// they fit, so the binary searches cost LDS latency instead of chains of dependent global loads.
template <uint32_t T>
__device__ bool task_merge2(const Axioms& ax, const Out& o, uint32_t A, const Pre& pr, uint32_t* lbuf, Rsv& rs) {
  using K = typename RowT<T>::K;
  const uint32_t P1 = pr.P1, P2 = pr.P2;
  const uint32_t b1 = pr.b1, n1 = pr.n1;
  const uint32_t b2 = pr.b2, n2 = pr.n2;
  if (n2 + 1 > CAPW) return false;
  uint32_t s = 0;
  K sv = 0;
  if (T == R_TOLD) {
    s = 2;
    if (lane() < 2) sv = (K)(lane() ? P2 : P1);  // (par is sorted: P1 < P2)
  } else if (T == R_EXR) {
    const uint32_t b0 = pr.ob;
    s = pr.on;
    if (s > 64) return false;
    if (lane() < s) sv = (K)ax.xr[b0 + lane()];
  } else {
    const uint32_t b0 = pr.ob;
    s = pr.on;
    if (s > 64) return false;
    if (lane() < s) sv = ((K)ax.xl_r[b0 + lane()] << 32) | ax.xl_b[b0 + lane()];
  }
  auto at_g = [&](uint32_t b, uint32_t j) -> K {
    if (T == R_TOLD) return (K)o.t_val[b + j];
    if (T == R_EXR) return (K)o.e_val[b + j];
    return ((K)o.l_r[b + j] << 32) | o.l_b[b + j];
  };
  constexpr uint32_t KW = sizeof(K) / 4;  // 32-bit words per key
  const bool staged = (uint64_t)(n1 + n2) * KW + n2 + 1 <= CAPW;
  K* row1 = reinterpret_cast<K*>(lbuf);
  K* row2 = row1 + n1;
  if (staged) {
    for (uint32_t j = lane(); j < n1; j += 64) row1[j] = at_g(b1, j);
    for (uint32_t j = lane(); j < n2; j += 64) row2[j] = at_g(b2, j);
    Lds::sync();
  }
  // (rows are named by their base in the global arrays: b1 or b2)
  auto at = [&](uint32_t b, uint32_t j) -> K { return staged ? (b == b1 && n1 ? row1[j] : row2[j]) : at_g(b, j); };
  auto lower = [&](uint32_t b, uint32_t n, K v) {  // entries of row [b, b + n) below v
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (at(b, mid) < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  // P2's row: which entries P1's row holds; pre[j] = entries of P2's row before j it does not
  uint32_t* pre = staged ? reinterpret_cast<uint32_t*>(row2 + n2) : lbuf;
  uint32_t run = 0;
  for (uint32_t j0 = 0; j0 < n2; j0 += 64) {  // (wave-uniform)
    const uint32_t j = j0 + lane();
    bool fresh = false;
    if (j < n2) {
      const K v = at(b2, j);
      const uint32_t r = lower(b1, n1, v);
      fresh = !(r < n1 && at(b1, r) == v);
    }
    const unsigned long long m = __ballot(fresh);
    if (j < n2) pre[j] = run + (uint32_t)__popcll(m & ((1ull << lane()) - 1ull));
    run += (uint32_t)__popcll(m);
  }
  if (lane() == 0) pre[n2] = run;
  Lds::sync();
  // the list entries in neither row
  uint32_t r1 = 0, r2 = 0;
  bool kept = false;
  if (lane() < s) {
    r1 = lower(b1, n1, sv);
    r2 = lower(b2, n2, sv);
    kept = !(r1 < n1 && at(b1, r1) == sv) && !(r2 < n2 && at(b2, r2) == sv);
  }
  const unsigned long long km = __ballot(kept);
  const uint32_t nout = n1 + run + (uint32_t)__popcll(km);
  const uint32_t cap = T == R_TOLD ? o.t_cap : T == R_EXR ? o.e_cap : o.l_cap;
  uint32_t* tail = T == R_TOLD ? &o.ctr->t_tail : T == R_EXR ? &o.ctr->e_tail : &o.ctr->l_tail;
  const uint32_t r = reserve(o, rs, T, nout, cap, tail);
  if (r != NONE) {
    auto put = [&](uint32_t i, K v) {
      if (T == R_TOLD) {
        o.t_val[r + i] = (uint32_t)v;
      } else if (T == R_EXR) {
        o.e_val[r + i] = (uint32_t)v;
      } else {
        o.l_r[r + i] = (uint32_t)((unsigned long long)v >> 32);
        o.l_b[r + i] = (uint32_t)v;
      }
    };
    auto list_below = [&](K v) {  // kept list entries below v
      uint32_t c = 0;
      for (unsigned long long m = km; m;) {
        const uint32_t i = (uint32_t)__ffsll((long long)m) - 1u;
        m &= m - 1ull;
        c += __shfl(sv, (int)i) < v ? 1u : 0u;
      }
      return c;
    };
    if (kept) put(r1 + pre[r2] + (uint32_t)__popcll(km & ((1ull << lane()) - 1ull)), sv);
    for (uint32_t j0 = 0; j0 < n1; j0 += 64) {  // P1's row (wave-uniform)
      const uint32_t j = j0 + lane();
      K v = 0;
      uint32_t q = 0;
      if (j < n1) {
        v = at(b1, j);
        q = pre[lower(b2, n2, v)];
      }
      const uint32_t lb = list_below(v);
      if (j < n1) put(j + q + lb, v);
    }
    for (uint32_t j0 = 0; j0 < n2; j0 += 64) {  // P2's row: the entries P1's row does not hold
      const uint32_t j = j0 + lane();
      K v = 0;
      bool fresh = false;
      uint32_t q = 0;
      if (j < n2) {
        v = at(b2, j);
        fresh = pre[j + 1] != pre[j];
        if (fresh) q = lower(b1, n1, v);
      }
      const uint32_t lb = list_below(v);
      if (fresh) put(q + pre[j] + lb, v);
    }
    if (lane() == 0) {
      reinterpret_cast<uint32_t*>(o.meta + 2 * A)[RowT<T>::comp] = r;
      reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1)[RowT<T>::comp] = r + nout;
    }
  }
  Lds::sync();  // (lbuf is reused by the wave's next task)
  return true;
}

// Row type T of concept A (a wave; A wave-uniform): gather, sort, drop duplicates (and A itself
// from told*: a told cycle would put it there), append, record the range.  RELAX: a row is only
// appended when it grew; its range goes to meta2 (committed after the round).  Returns whether
// the row was written.
template <uint32_t T, bool RELAX>
__device__ bool task(const Axioms& ax, const Out& o, uint32_t A, uint32_t* lbuf, Rsv& rs, const Pre* pr = nullptr) {
  using K = typename RowT<T>::K;
  const uint32_t pb = pr ? pr->pb : ax.par_ptr[A], pe = pr ? pr->pe : ax.par_ptr[A + 1];
  // a told cycle's representative: its told row also holds the component's other members (the
  // extras), gathered and sorted with the rest
  const uint32_t nx = T == R_TOLD && ax.tx_ptr ? ax.tx_ptr[A + 1] - ax.tx_ptr[A] : 0u;
  if (!RELAX && !nx && pe - pb <= 1 && task_merge1<T>(ax, o, A, *pr, lbuf, rs)) return true;
  if (!RELAX && !nx && pe - pb == 2 && task_merge2<T>(ax, o, A, *pr, lbuf, rs)) return true;
  unsigned long long raw = 0;
  for (uint32_t q = pb + lane(); q < pe; q += 64) {
    const uint32_t p = ax.par[q];
    raw += meta_word(o.meta, p, 1, RowT<T>::comp) - meta_word(o.meta, p, 0, RowT<T>::comp) + (T == R_TOLD ? 1u : 0u);
  }
  raw = wsum(raw) + nx;  // (the extras once, not per lane)
  if (T == R_EXR) raw += ax.xr_ptr[A + 1] - ax.xr_ptr[A];
  if (T == R_EXL) raw += ax.xl_ptr[A + 1] - ax.xl_ptr[A];
  if (raw > 0x7fffffffull) {
    if (lane() == 0) atomicOr(&o.ctr->ovf, 1u);
    return false;
  }
  const bool big = raw > RowT<T>::lds_cap;
  K* buf = big ? scratch_take<K>(o, (uint32_t)raw) : reinterpret_cast<K*>(lbuf);
  if (!buf) return false;
  const K excl = T == R_TOLD ? (K)A : ~K(0);
  uint32_t n;
  if (big) {
    gather<T, Glb>(ax, o, A, pb, pe, buf);
    n = sort_unique<Glb>(buf, (uint32_t)raw, excl);
  } else {
    gather<T, Lds>(ax, o, A, pb, pe, buf);
    n = sort_unique_lds(buf, (uint32_t)raw, excl);
  }
  bool wrote = false;
  const uint32_t ob = meta_word(o.meta, A, 0, RowT<T>::comp), oe = meta_word(o.meta, A, 1, RowT<T>::comp);
  if (!RELAX || n != oe - ob) {
    const uint32_t cap = T == R_TOLD ? o.t_cap : T == R_EXR ? o.e_cap : o.l_cap;
    uint32_t* tail = T == R_TOLD ? &o.ctr->t_tail : T == R_EXR ? &o.ctr->e_tail : &o.ctr->l_tail;
    const uint32_t r = reserve(o, rs, T, n, cap, tail);
    if (r != NONE) {
      for (uint32_t i = lane(); i < n; i += 64) {
        const K v = big ? Glb::ld(buf + i) : buf[i];
        if (T == R_TOLD) {
          o.t_val[r + i] = (uint32_t)v;
        } else if (T == R_EXR) {
          o.e_val[r + i] = (uint32_t)v;
        } else {
          o.l_r[r + i] = (uint32_t)((unsigned long long)v >> 32);
          o.l_b[r + i] = (uint32_t)v;
        }
      }
      if (lane() == 0) {
        uint4* m = RELAX ? o.meta2 : o.meta;
        reinterpret_cast<uint32_t*>(m + 2 * A)[RowT<T>::comp] = r;
        reinterpret_cast<uint32_t*>(m + 2 * A + 1)[RowT<T>::comp] = r + n;
      }
      wrote = true;
    }
  }
  Lds::sync();  // (lbuf is reused by the wave's next task)
  return wrote;
}

// Tasks (A, T) of the concepts of one level (or of the dirty concepts: relaxation) are spread
// over all waves: task t = 3A + T goes to wave t mod nw, so a level's concepts (often a
// contiguous id range) and their three row types all run side by side.
template <class Sel, class Run>
__device__ __forceinline__ void for_tasks(uint32_t N, Sel&& sel, Run&& run) {
  const uint32_t nw = gridDim.x * WAVES, w = slot_id();
  const uint64_t ntask = 3ull * N;
  for (uint64_t base = 0; base * nw + w < ntask; base += 64) {  // (wave-uniform)
    const uint64_t t0 = (base + lane()) * nw + w;
    const bool in = t0 < ntask && sel((uint32_t)(t0 / 3), (uint32_t)(t0 % 3));
    unsigned long long m = __ballot(in);
    while (m) {
      const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      const uint64_t t = (base + i) * nw + w;
      run((uint32_t)(t / 3), (uint32_t)(t % 3));
    }
  }
}

// a concept outside the built set (Axioms::w_lo/w_hi): never ready, never stuck
constexpr uint32_t SKIP = NONE - 1u;
static_assert(SKIP == LVL_SKIP, "level marks");
// a told cycle's follower: its rows come from its representative's (k_follow), never ready, never stuck
constexpr uint32_t FOLLOW = NONE - 2u;
static_assert(FOLLOW == LVL_FOLLOW, "level marks");
constexpr uint32_t FOLLOWED = NONE - 3u;  // (k_follow wrote its rows)
__device__ __forceinline__ bool built(const Axioms& ax, uint32_t A) { return A < 2u || (A >= ax.w_lo && A < ax.w_hi); }

__global__ void __launch_bounds__(BLOCK) k_start(Axioms ax, Out o) {
  const uint32_t stride = gridDim.x * blockDim.x;
  bool root = false, root1 = false;
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += stride) {
    const uint32_t d = ax.par_ptr[A + 1] - ax.par_ptr[A];
    const bool in = built(ax, A);
    // told cycles: a follower's rows come from its representative's (k_follow); a representative
    // without outside supers still gathers its component's members into its told row, so it is a
    // level-1 task (level 0 copies own axiom lists only)
    const bool fol = ax.rep && ax.rep[A] != A;
    const bool xt = ax.tx_ptr && ax.tx_ptr[A + 1] > ax.tx_ptr[A];
    o.indeg[A] = fol || ax.slevel ? 0u : d;
    o.level[A] = ax.slevel ? ax.slevel[A] : !in ? SKIP : fol ? FOLLOW : d ? NONE : xt ? 1u : 0u;
    root |= in && !fol && d == 0 && !xt;
    root1 |= in && !fol && d == 0 && xt;
    o.meta[2 * A] = make_uint4(0u, ax.cidx_ptr[A], 0u, 0u);
    o.meta[2 * A + 1] = make_uint4(0u, ax.cidx_ptr[A + 1], 0u, 0u);
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < RSV_WORDS; i += stride) o.rsv[i] = 0;
  if (root) o.lvl_flag[0] = 1;  // (zeroed by the host before this launch)
  if (root1) o.lvl_flag[1] = 1;
}

#ifdef EL_LEVEL_WAVES  // (A/B builds: a VGPR budget for more waves per SIMD; CAPW sets the LDS one)
__global__ void __attribute__((amdgpu_flat_work_group_size(BLOCK, BLOCK), amdgpu_waves_per_eu(EL_LEVEL_WAVES, 8)))
k_level(Axioms ax, Out o, uint32_t L) {
#else
__global__ void __launch_bounds__(BLOCK) k_level(Axioms ax, Out o, uint32_t L) {
#endif
  if (o.lvl_flag[L] == 0) return;  // (block-uniform: nothing at this level)
  __shared__ unsigned long long lds[WAVES * (CAPW / 2)];
  __shared__ uint32_t sany;
  if (threadIdx.x == 0) sany = 0;
  __syncthreads();
  uint32_t* lbuf = reinterpret_cast<uint32_t*>(lds + (threadIdx.x >> 6) * (CAPW / 2));
  Rsv rs = rsv_load(o);
  bool any = false;
  // for_tasks with each selected task's head values loaded by its lane first (pre_load)
  const uint32_t nw = gridDim.x * WAVES, w = slot_id();
  const uint64_t ntask = 3ull * ax.N;
  for (uint64_t base = 0; base * nw + w < ntask; base += 64) {  // (wave-uniform)
    const uint64_t t0 = (base + lane()) * nw + w;
    const uint32_t A0 = (uint32_t)(t0 / 3), T0 = (uint32_t)(t0 % 3);
    const bool in = t0 < ntask && o.level[A0] == L;
    const Pre mine = in ? pre_load(ax, o, A0, T0) : Pre{};
    unsigned long long m = __ballot(in);
    while (m) {
      const int i = __ffsll((long long)m) - 1;
      m &= m - 1;
      const uint32_t A = __shfl(A0, i), T = __shfl(T0, i);
      const Pre pr = pre_of(mine, i);
      if (T == R_EXR) {
        task<R_EXR, false>(ax, o, A, lbuf, rs, &pr);
      } else if (T == R_EXL) {
        task<R_EXL, false>(ax, o, A, lbuf, rs, &pr);
      } else {
        // the first 64 subs are loaded before the merge, so their loads overlap it
        const uint32_t cb = pr.ob, ce = pr.ob + pr.on;
        const uint32_t c0 = cb + lane() < ce ? ax.chi[cb + lane()] : NONE;
        task<R_TOLD, false>(ax, o, A, lbuf, rs, &pr);
        // a sub whose last super this was is ready for the next level.  The count first: the level
        // word is read only for the sub that reaches zero (a skipped concept's count is never read)
        auto ready = [&](uint32_t c) {
          if (atomicSub(o.indeg + c, 1u) == 1u && o.level[c] != SKIP) {
            o.level[c] = L + 1;
            any = true;
          }
        };
        if (c0 != NONE) ready(c0);
        for (uint32_t q = cb + 64 + lane(); q < ce; q += 64) ready(ax.chi[q]);
      }
    }
  }
  rsv_store(o, rs);
  if (any) sany = 1;
  __syncthreads();
  if (threadIdx.x == 0 && sany) o.lvl_flag[L + 1] = 1;
}

// One static level L (Axioms::slevel): the 3n tasks of its n concepts ids[0, n) spread over the
// launch's waves as in k_level, read off the list instead of a scan of every concept's level; no
// pending counts (every super is in an earlier level, done by an earlier launch).
__global__ void __launch_bounds__(BLOCK) k_level_list(Axioms ax, Out o, uint32_t L, const uint32_t* __restrict__ ids,
                                                      uint32_t n) {
  __shared__ unsigned long long lds[WAVES * (CAPW / 2)];
  uint32_t* lbuf = reinterpret_cast<uint32_t*>(lds + (threadIdx.x >> 6) * (CAPW / 2));
  Rsv rs = rsv_load(o);
  const uint32_t nw = gridDim.x * WAVES, w = slot_id();
  const uint64_t ntask = 3ull * n;
  for (uint64_t base = 0; base * nw + w < ntask; base += 64) {  // (wave-uniform)
    const uint64_t t0 = (base + lane()) * nw + w;
    const bool in = t0 < ntask;
    const uint32_t A0 = in ? ids[t0 / 3] : 0u, T0 = (uint32_t)(t0 % 3);
    const Pre mine = in ? pre_load(ax, o, A0, T0) : Pre{};
    unsigned long long m = __ballot(in);
    while (m) {
      const int i = __ffsll((long long)m) - 1;
      m &= m - 1;
      const uint32_t A = __shfl(A0, i), T = __shfl(T0, i);
      const Pre pr = pre_of(mine, i);
      if (T == R_EXR)
        task<R_EXR, false>(ax, o, A, lbuf, rs, &pr);
      else if (T == R_EXL)
        task<R_EXL, false>(ax, o, A, lbuf, rs, &pr);
      else
        task<R_TOLD, false>(ax, o, A, lbuf, rs, &pr);
    }
  }
  rsv_store(o, rs);
  (void)L;
}

// Level 0 — the concepts without told supers: told* is empty and exr* / exl* are the concept's
// own axiom lists (sorted, unique), so a lane per concept copies them (the wave reserves its
// lanes' rows with one atomic per row type), and the subs whose last super it was are counted
// down with the wave walking its lanes' child lists together.  As wave-per-concept tasks of
// k_level each root cost a chain of dependent loads (G3: 90 k roots, 0.7 ms).
__global__ void __launch_bounds__(BLOCK) k_level0(Axioms ax, Out o) {
  if (o.lvl_flag[0] == 0) return;  // (block-uniform)
  __shared__ uint32_t sany;
  if (threadIdx.x == 0) sany = 0;
  __syncthreads();
  bool any = false;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t base = blockIdx.x * blockDim.x; base < ax.N; base += stride) {  // (uniform trip count)
    const uint32_t A = base + threadIdx.x;
    const bool on = A < ax.N && o.level[A] == 0u;
    uint32_t xb = 0, ne = 0, lb = 0, nl = 0, cb = 0, nc = 0;
    if (on) {
      xb = ax.xr_ptr[A];
      ne = ax.xr_ptr[A + 1] - xb;
      lb = ax.xl_ptr[A];
      nl = ax.xl_ptr[A + 1] - lb;
      cb = ax.chi_ptr[A];
      nc = ax.chi_ptr[A + 1] - cb;
    }
    uint32_t ie = ne, il = nl;  // inclusive wave scans of the row sizes
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t ve = __shfl_up(ie, d), vl = __shfl_up(il, d);
      if (lane() >= d) ie += ve, il += vl;
    }
    const uint32_t te = __shfl(ie, 63), tl = __shfl(il, 63);
    uint32_t re = 0, rl = 0;
    if (lane() == 0) {
      if (te) re = atomicAdd(&o.ctr->e_tail, te);
      if (tl) rl = atomicAdd(&o.ctr->l_tail, tl);
    }
    re = __shfl(re, 0);
    rl = __shfl(rl, 0);
    const bool eok = (uint64_t)re + te <= o.e_cap, lok = (uint64_t)rl + tl <= o.l_cap;
    if (lane() == 0 && ((te && !eok) || (tl && !lok))) atomicOr(&o.ctr->ovf, 1u);  // (redone larger)
    if (on && ne && eok) {
      const uint32_t e0 = re + ie - ne;
      for (uint32_t j = 0; j < ne; ++j) o.e_val[e0 + j] = ax.xr[xb + j];
      reinterpret_cast<uint32_t*>(o.meta + 2 * A)[RowT<R_EXR>::comp] = e0;
      reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1)[RowT<R_EXR>::comp] = e0 + ne;
    }
    if (on && nl && lok) {
      const uint32_t l0 = rl + il - nl;
      for (uint32_t j = 0; j < nl; ++j) {
        o.l_r[l0 + j] = ax.xl_r[lb + j];
        o.l_b[l0 + j] = ax.xl_b[lb + j];
      }
      reinterpret_cast<uint32_t*>(o.meta + 2 * A)[RowT<R_EXL>::comp] = l0;
      reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1)[RowT<R_EXL>::comp] = l0 + nl;
    }
    if (!ax.slevel)  // (static levels: the next levels are known already)
      wave_concat(nc, [&](bool v, uint32_t own, uint32_t j, uint32_t) {
        const uint32_t cbo = __shfl(cb, (int)own);
        if (!v) return;
        const uint32_t c = ax.chi[cbo + j];
        if (atomicSub(o.indeg + c, 1u) == 1u && o.level[c] != SKIP) {  // (as in k_level)
          o.level[c] = 1u;
          any = true;
        }
      });
  }
  if (any) sany = 1;
  __syncthreads();
  if (threadIdx.x == 0 && sany) o.lvl_flag[1] = 1;
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

// The followers of the told cycles (el_index.h): member m of a component with representative r
// has told*(m) = told*(r) ∪ {r} \ {m} (the representative's row holds every other member) and
// the same exr* / exl* rows as r, which it shares (meta points at them).  One wave per follower:
// m's place in r's sorted row and r's insertion point by binary searches, then a coalesced copy.
// Runs after every batch of levels (closure_tail): a follower is copied once, when its
// representative's row is final — the representative was a task of a level already launched
// (level < L), or `all` after the relaxation rounds — and is then marked FOLLOWED.  (Round 5 ran
// every follower at every tail: one whose representative sat in a later batch read an empty row
// (n = 0), reserved 0 slots and still stored the representative at t_val[base] — the first slot
// of another wave's row, or one past t_cap: the kat_cycle illegal access and a wrong closure.)
// A representative's row must hold the follower (its component's other members): anything else
// is a broken condensation and fails the build (ctr->bad) instead of writing.
__global__ void __launch_bounds__(BLOCK) k_follow(Axioms ax, Out o, uint32_t L, uint32_t all) {
  const uint32_t nw = gridDim.x * WAVES;
  for (uint32_t i = slot_id(); i < ax.nfol; i += nw) {  // (wave-uniform)
    const uint32_t m = ax.fol[i];
    if (m >= ax.N || !built(ax, m) || o.level[m] != FOLLOW) continue;
    const uint32_t r = ax.rep[m];
    const uint32_t lr = r < ax.N ? o.level[r] : NONE;
    // a representative outside the built window (a partition's window is a contiguous id range,
    // so it may hold a follower no owned row reaches while its representative lies below the
    // range): the follower's rows are never read — left empty
    if (lr == SKIP) continue;
    if (!all && !(lr < L)) continue;  // (the representative's row is not built yet)
    const uint4 rb = o.meta[2 * r], re = o.meta[2 * r + 1];
    const uint32_t b = rb.x, n = re.x - rb.x;
    if (r >= m || n == 0 || re.x < rb.x) {
      if (lane() == 0) atomicOr(&o.ctr->bad, 1u);
      continue;
    }
    auto lower = [&](uint32_t v) {
      uint32_t lo = 0, hi = n;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (o.t_val[b + mid] < v)
          lo = mid + 1;
        else
          hi = mid;
      }
      return lo;
    };
    const uint32_t im = lower(m), ir = lower(r);  // (r < m: the representative is the smallest member)
    if (im >= n || o.t_val[b + im] != m || ir > im) {  // (wave-uniform: every lane read the same row)
      if (lane() == 0) atomicOr(&o.ctr->bad, 1u);
      continue;
    }
    uint32_t base = 0;
    if (lane() == 0) base = atomicAdd(&o.ctr->t_tail, n);
    base = __shfl(base, 0);
    if ((uint64_t)base + n > o.t_cap) {
      if (lane() == 0) atomicOr(&o.ctr->ovf, 1u);  // (the build is redone larger)
      continue;
    }
    for (uint32_t j = lane(); j < n; j += 64) {
      const uint32_t v = o.t_val[b + j];
      if (j != im) o.t_val[base + j - (j > im ? 1u : 0u) + (v > r ? 1u : 0u)] = v;
    }
    if (lane() == 0) {
      o.t_val[base + ir] = r;
      uint32_t* mb = reinterpret_cast<uint32_t*>(o.meta + 2 * m);
      uint32_t* me = reinterpret_cast<uint32_t*>(o.meta + 2 * m + 1);
      mb[0] = base;
      me[0] = base + n;
      mb[2] = rb.z;
      me[2] = re.z;
      mb[3] = rb.w;
      me[3] = re.w;
      o.level[m] = FOLLOWED;
    }
  }
}

// One Jacobi relaxation round over the dirty concepts: each row type recomputed from the
// committed rows (meta); a grown row lands in meta2, its concept's changed bit for the type is
// set, and its subs still being relaxed are dirty next round.
__global__ void __launch_bounds__(BLOCK) k_relax(Axioms ax, Out o) {
  __shared__ unsigned long long lds[WAVES * (CAPW / 2)];
  uint32_t* lbuf = reinterpret_cast<uint32_t*>(lds + (threadIdx.x >> 6) * (CAPW / 2));
  Rsv rs = rsv_load(o);
  for_tasks(ax.N, [&](uint32_t A, uint32_t) { return o.dirty[A] != 0; }, [&](uint32_t A, uint32_t T) {
    const bool grew = T == R_TOLD  ? task<R_TOLD, true>(ax, o, A, lbuf, rs)
                      : T == R_EXR ? task<R_EXR, true>(ax, o, A, lbuf, rs)
                                   : task<R_EXL, true>(ax, o, A, lbuf, rs);
    if (!grew) return;
    if (lane() == 0) {
      atomicOr(o.changed + A, 1u << T);
      o.ctr->dirty = 1;
    }
    const uint32_t cb = ax.chi_ptr[A], ce = ax.chi_ptr[A + 1];
    for (uint32_t q = cb + lane(); q < ce; q += 64) {
      const uint32_t c = ax.chi[q];
      if (o.level[c] == NONE) o.dirty2[c] = 1;
    }
  });
  rsv_store(o, rs);
}

__global__ void __launch_bounds__(BLOCK) k_relax_commit(Axioms ax, Out o) {
  for (uint32_t A = blockIdx.x * blockDim.x + threadIdx.x; A < ax.N; A += gridDim.x * blockDim.x) {
    const uint32_t ch = o.changed[A];
    if (ch) {
      uint32_t* b = reinterpret_cast<uint32_t*>(o.meta + 2 * A);
      uint32_t* e = reinterpret_cast<uint32_t*>(o.meta + 2 * A + 1);
      const uint32_t* b2 = reinterpret_cast<const uint32_t*>(o.meta2 + 2 * A);
      const uint32_t* e2 = reinterpret_cast<const uint32_t*>(o.meta2 + 2 * A + 1);
      for (uint32_t T = 0; T < 3; ++T)
        if ((ch >> T) & 1u) {
          const uint32_t c = T == R_TOLD ? 0u : T == R_EXR ? 2u : 3u;
          b[c] = b2[c];
          e[c] = e2[c];
        }
      o.changed[A] = 0;
    }
    o.dirty[A] = o.dirty2[A];
    o.dirty2[A] = 0;
  }
}

// Per-concept statistics of the final rows (for the state pass and the host's buffer sizes):
// init facts, CR2 candidates over told*, successor-row weights and CR5 lifts over exr*, base
// propagations over exl*.  Lanes own concepts; the wave walks the concatenation of its 64
// concepts' rows (coalesced) and adds each entry's contribution to its owner in LDS.
// acc[own] += v over a wave_concat round: the lanes of one owner are consecutive, so a segmented
// scan leaves each owner's sum in its last lane, which adds it alone (an LDS atomic per lane on a
// handful of owner words serialised, k_stats 0.68 ms on G3).  Invalid lanes: own = 64 (no owner).
__device__ __forceinline__ void seg_add(uint32_t* acc, uint32_t own, uint32_t v) {
  const uint32_t ln = lane();
  uint32_t sum = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(sum, d), ow = __shfl_up(own, d);
    if (ln >= d && ow == own) sum += t;
  }
  const uint32_t next = __shfl_down(own, 1);
  if (own < 64 && (ln == 63 || next != own) && sum) acc[own] += sum;
}

// wave_concat four rounds at a time, the rounds' loads in flight together: first(v, own, j)
// returns a round's first load, second(v, own, x) its dependent load, use(v, own, y) consumes it.
// (k_stats' per-entry lookups were one dependent chain per round: ~220 rounds per wave on G3.)
template <class First, class Second, class Use>
__device__ __forceinline__ void wave_concat4(uint32_t len, First&& first, Second&& second, Use&& use) {
  const uint32_t ln = lane();
  uint32_t inc = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (ln >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, 63), excl = inc - len;
  for (uint32_t base = 0; base < total; base += 256) {  // (wave-uniform)
    uint32_t own[4], x[4];
    bool v[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
      const uint32_t k = base + r * 64 + ln;
      uint32_t ow = 0;
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1)
        if (__shfl(inc, (int)(ow + step - 1)) <= k) ow += step;
      v[r] = k < total;
      own[r] = v[r] ? ow : 0u;
      x[r] = first(v[r], own[r], k - __shfl(excl, (int)own[r]));
    }
    decltype(second(false, 0u, 0u)) y[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) y[r] = second(v[r], own[r], x[r]);
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) use(v[r], own[r], x[r], y[r]);
  }
}

// Concepts per wave chunk: a chunk's rows are walked as one dependent chain of rounds, so smaller
// chunks (more of them, spread over every resident wave) shorten the longest chain.
#ifndef EL_STATS_CH
#define EL_STATS_CH 16
#endif
constexpr uint32_t STATS_CH = EL_STATS_CH;
static_assert(STATS_CH >= 1 && STATS_CH <= 64, "k_stats chunk: 1..64 concepts (lanes)");

__global__ void __launch_bounds__(BLOCK) k_stats(Axioms ax, Out o, uint32_t lo, uint32_t hi, uint32_t props) {
  __shared__ uint32_t acc[WAVES][6][64];
  uint32_t(&a)[6][64] = acc[threadIdx.x >> 6];
  const uint32_t N1 = ax.N + 1, nw = gridDim.x * WAVES, w = slot_id();
  for (uint32_t x0 = lo + w * STATS_CH; x0 < hi; x0 += nw * STATS_CH) {  // (wave-uniform)
    const uint32_t x = x0 + lane();
    const bool ok = lane() < STATS_CH && x < hi;
    uint4 b = make_uint4(0, 0, 0, 0), e = b;
    uint32_t fb = 0, fe = 0;
    if (ok) {
      b = o.meta[2 * x];
      e = o.meta[2 * x + 1];
      fb = ax.fp_ptr[x];
      fe = ax.fp_ptr[x + 1];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) a[k][lane()] = 0;
    Lds::sync();
    // told*: CR2 candidates (|cidx| of every entry), ⊤ among the first two entries
    // (the entry's position among the first two of its row: j < 2 ⇔ the row's begin + j < begin + 2)
    wave_concat4(
        e.x - b.x,
        [&](bool v, uint32_t own, uint32_t j) {
          const uint32_t ro = __shfl(b.x, (int)own);
          return v ? (o.t_val[ro + j] | (j < 2 ? 0x80000000u : 0u)) : 0u;  // (concept ids < 2^31)
        },
        [&](bool v, uint32_t, uint32_t t) { return v ? ax.cz[t & 0x7fffffffu] : 0u; },
        [&](bool v, uint32_t own, uint32_t t, uint32_t cz) {
          if (v && (t >> 31) && (t & 0x7fffffffu) == TOP) a[1][own] = 1;
          seg_add(a[0], v ? own : 64u, cz);
        });
    // exr*: successor-row weight, chain-second base links, CR5 lifts
    wave_concat4(
        e.z - b.z,
        [&](bool v, uint32_t own, uint32_t j) {
          const uint32_t ro = __shfl(b.z, (int)own);
          return v ? o.e_val[ro + j] : 0u;
        },
        [&](bool v, uint32_t, uint32_t p) { return v ? ax.pstat[p] : make_uint2(0u, 0u); },
        [&](bool v, uint32_t own, uint32_t, uint2 ps) {
          const uint32_t ow = v ? own : 64u;
          seg_add(a[2], ow, ps.x);
          seg_add(a[3], ow, ps.y & 1u);
          seg_add(a[4], ow, ps.y >> 1);
        });
    // exl*: base propagations ((r, x), B) with (r, x) a pair
    wave_concat4(
        props && fe > fb ? e.w - b.w : 0u,
        [&](bool v, uint32_t own, uint32_t j) {
          const uint32_t ro = __shfl(b.w, (int)own);
          return v ? o.l_r[ro + j] : 0u;
        },
        [&](bool v, uint32_t own, uint32_t r) {
          const uint32_t f0 = __shfl(fb, (int)own), f1 = __shfl(fe, (int)own);
          return (v && pid_of(ax, r, f0, f1) != NONE) ? 1u : 0u;
        },
        [&](bool v, uint32_t own, uint32_t, uint32_t hit) { seg_add(a[5], v ? own : 64u, hit); });
    Lds::sync();
    if (ok) {
      const bool two = two_of(ax, x);
      const uint32_t tl = e.x - b.x;
      o.nd[ND_INIT * N1 + x] = 1 + (two ? 1u : 0u) + tl - ((two && a[1][lane()]) ? 1u : 0u);
      o.nd[ND_EXR * N1 + x] = e.z - b.z;
      o.nd[ND_CZ * N1 + x] = a[0][lane()];
      o.nd[ND_SC * N1 + x] = a[2][lane()];
      o.nd[ND_SC0 * N1 + x] = a[3][lane()];
      o.nd[ND_LIFT * N1 + x] = a[4][lane()];
      o.nd[ND_PROPS * N1 + x] = a[5][lane()];
    }
    Lds::sync();
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
    if (!built(ax, A)) continue;
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
// row(x) -> uint3 loads what a row's entries need once, by the row's lane (round 4 re-read it per
// entry: a chain of dependent loads in every round); f(valid, x, j, slot, the owner's row value).
template <class Row, class F>
__device__ __forceinline__ void rows_by_slot(uint32_t a, uint32_t b, const uint32_t* pos, Row&& row, F&& f) {
  const uint32_t nw = gridDim.x * WAVES, w = blockIdx.x * WAVES + (threadIdx.x >> 6);
  for (uint32_t r0 = a + w * 64; r0 < b; r0 += nw * 64) {  // (wave-uniform)
    const uint32_t x = r0 + lane();
    uint32_t s = 0, len = 0;
    uint3 rv = make_uint3(0u, 0u, 0u);
    if (x < b) {
      s = pos[x - a];
      len = pos[x - a + 1] - s;
      if (len) rv = row(x);
    }
    wave_concat(len, [&](bool v, uint32_t own, uint32_t j, uint32_t) {
      const uint32_t xo = r0 + own, so = __shfl(s, (int)own);
      const uint3 ro = make_uint3(__shfl(rv.x, (int)own), __shfl(rv.y, (int)own), __shfl(rv.z, (int)own));
      f(v, xo, j, so + j, ro);
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
  rows_by_slot(
      a, b, pos,
      [&](uint32_t x) {  // told*(X)'s start, where ⊤ sits in it (NONE: X has no ⊤ fact), ⊤ is a fact
        const bool two = two_of(ax, x);
        const uint32_t t0 = o.meta[2 * x].x, t1 = o.meta[2 * x + 1].x;
        // ⊤ sorts first or right after ⊥ in told*(X): its entry is skipped there
        const uint32_t ptop = !two ? NONE
                              : (t0 < t1 && o.t_val[t0] == TOP)          ? 0u
                              : (t0 + 1 < t1 && o.t_val[t0 + 1] == TOP) ? 1u
                                                                         : NONE;
        return make_uint3(t0, ptop, two ? 1u : 0u);
      },
      [&](bool v, uint32_t x, uint32_t j, uint32_t slot, uint3 r) {
        if (!v) return;
        const bool two = r.z;
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
          if (c >= r.y) ++c;  // (r.y = NONE when there is no ⊤ entry to skip)
          val = o.t_val[r.x + c];
        }
        slog_x[base + slot] = x;
        slog_a[base + slot] = val;
        slog_f[base + slot] = f;
        const uint32_t col =
            val < 2u ? val : (val >= c_lo && val < c_hi ? (ax.cperm ? ax.cperm[val] : val - c_lo + 2u) : NONE);
        if (col != NONE) {
          __hip_atomic_fetch_or(bits + (uint64_t)x * W + (col >> 5), 1u << (col & 31u), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
          if (summ) summ[(uint64_t)x * SB + (col >> elrows::SUMM_SHIFT)] = 1;
        }
      });
}

// the base links {(X, p) : p ∈ exr*(X)} in X order
__global__ void __launch_bounds__(BLOCK) k_base_links(Axioms ax, Out o, uint32_t a, uint32_t b, const uint32_t* pos,
                                                      uint32_t* llog_x, uint32_t* llog_p) {
  rows_by_slot(
      a, b, pos, [&](uint32_t x) { return make_uint3(o.meta[2 * x].z, 0u, 0u); },
      [&](bool v, uint32_t x, uint32_t j, uint32_t slot, uint3 r) {
        if (!v) return;
        llog_x[slot] = x;
        llog_p[slot] = o.e_val[r.x + j];
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

void level(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L) {
  if (L == 0)
    hipLaunchKernelGGL(k_level0, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o);
  else
    hipLaunchKernelGGL(k_level, dim3(GRID), dim3(BLOCK), 0, s, ax, o, L);
  CCHK(hipGetLastError());
}

void level_list(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L, uint32_t first, uint32_t n) {
  if (!n) return;
  // (a small level gets a small grid: its ramp is the launch's cost, not its few tasks)
  const uint32_t g = std::min<uint32_t>(GRID, std::max<uint32_t>(1, (3 * n + WAVES - 1) / WAVES));
  hipLaunchKernelGGL(k_level_list, dim3(g), dim3(BLOCK), 0, s, ax, o, L, ax.lvl_ids + first, n);
  CCHK(hipGetLastError());
}

void check(hipStream_t s, const Axioms& ax, const Out& o) {
  hipLaunchKernelGGL(k_check, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o);
  CCHK(hipGetLastError());
}

void follow(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L, bool all) {
  if (!ax.nfol) return;
  hipLaunchKernelGGL(k_follow, dim3(std::min<uint32_t>((ax.nfol + WAVES - 1) / WAVES, 2048)), dim3(BLOCK), 0, s, ax, o, L,
                     all ? 1u : 0u);
  CCHK(hipGetLastError());
}

void relax(hipStream_t s, const Axioms& ax, const Out& o) {
  CCHK(hipMemsetAsync(&o.ctr->dirty, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_relax, dim3(GRID), dim3(BLOCK), 0, s, ax, o);
  hipLaunchKernelGGL(k_relax_commit, dim3(grid_for(ax.N)), dim3(BLOCK), 0, s, ax, o);
  CCHK(hipGetLastError());
}

void stats(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, bool props) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_stats, dim3(grid_for((uint64_t)(b - a) * (64 / STATS_CH), 2048)), dim3(BLOCK), 0, s, ax, o, a, b,
                     props ? 1u : 0u);
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
