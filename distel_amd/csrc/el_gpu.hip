// el_gpu.hip — MI355X (gfx950) EL+ saturation engine behind the C-ABI of include/el_gpu.h.
//
// What the reference does: eight rule-type JVM processes run
// Lua scripts against Redis shards and funnel every new subsumption into a
// single result node, each iteration closed by an all-to-all "anything new?"
// barrier (CommunicationHandler.java:49-84).  Here the whole state lives in HBM:
//
//   S(X)      dense bit rows, N × W uint32 words      (dedup: atomicOr, test: 1 word)
//             + append-only fact log                  (semi-naive Δ = log[wm, end))
//             + CSR of the facts by row X, built lazily for export only
//   R(r)      link set {(X, pid)} as an open-addressing hash of 64-bit keys,
//             pid = dense (role, filler) pair id (el_index.cpp), + predecessor
//             CSR keyed by pid and successor CSR keyed by X, + link log
//   CR4       propagation set {((r, Y), B)} (hash) + log + CSR keyed by pid
//
// One Jacobi superstep t (all rules, or one rule type for el_step) = 5 launches:
//   generation  k_expand (roles: Δ S-facts, Δ links, Δ range activations, leftover
//               propagations) and k_jobs (wide fan-outs) read ONLY the state of
//               step t-1 and append candidate facts that are not yet present;
//   commit      k_commit (roles: S, links, activations, propagations) dedups the
//               candidates against the bit rows / hash sets, appends the new ones
//               to the logs and publishes the counters to pinned host memory;
//   (relocation) only when a gapped CSR row overflowed: k_reloc_claim / _move / _commit move
//               that row alone to the end of the CSR's slot array.
// Result rows (export, copy-back) are built from the logs on demand (el_rows.hip).
// Generation never writes state, so a step can be re-run after growing a buffer,
// and the delta of every step is exactly {candidates} \ S_{t-1}: the same sets
// and the same algorithmic event counts as the CPU oracle (oracle/el_oracle.c).
//
// Everything is integer/bitset work: no MFMA.  The roofline is HBM bandwidth
// (SURVEY.md §8(d)); kernels use wave-aggregated appends (one atomic per wave via
// __ballot/popcount) and per-wave event-counter reduction.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <dlfcn.h>
#include <sys/mman.h>
#include <rccl/rccl.h>  // types only: librccl is opened on first use (EL_XCHG_RCCL)

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <numeric>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "el_closure.h"
#include "el_stream.h"

#include <type_traits>
#include "el_gpu.h"
#include "el_index.h"
#include "el_rows.h"

namespace {

constexpr uint32_t NONE = 0xffffffffu;
constexpr unsigned long long EMPTY_KEY = ~0ull;
constexpr int BLOCK = 256;
static_assert(BLOCK <= 512, "commit kernels stage one block round in LDS");

// sub-rule mask bits
enum : uint32_t {
  M_R1 = 1u << 0,    // CR1
  M_R2 = 1u << 1,    // CR2
  M_R3 = 1u << 2,    // CR3
  M_R4Y = 1u << 3,   // CR4 half-1 (new A ∈ S(Y))
  M_R4L = 1u << 4,   // CR4 half-2 (new link)
  M_R5 = 1u << 5,    // CR5
  M_R6 = 1u << 6,    // CR6
  M_RBOT = 1u << 7,  // ⊥
  M_RDOM = 1u << 8,  // domain
  M_RRNG = 1u << 9,  // range
  M_R4P = 1u << 10,  // CR4: new propagations × existing predecessors (per-rule stepping)
  M_R4D = 1u << 11,  // CR4: fused mode — a new propagation fans out to predecessors at once
  M_LEMPTY = 1u << 12,  // no link committed before this step: link probes would all miss
  M_PEMPTY = 1u << 13,  // no propagation committed before this step: idem
  M_ALL = M_R1 | M_R2 | M_R3 | M_R4Y | M_R4L | M_R5 | M_R6 | M_RBOT | M_RDOM | M_RRNG | M_R4D
};

// el_rule → sub-rules it owns (see el_gpu.h)
const uint32_t kRuleMask[EL_NUM_RULE_TYPES] = {
    M_R1, M_R2, M_R3 | M_RDOM | M_RRNG, M_R4Y, M_R4L | M_R4P, M_R5, M_R6, M_RBOT};

// JOB_PRED_U: JOB_PRED_S without the B ∈ S(x) probe, for the first superstep over the base
// links (M_LEMPTY): S(x) holds only the told closure then, so nearly every conclusion of the
// fan-out is new (G3: 96 M candidates) and the probe was one random read each that the
// commit's atomicOr repeats anyway
enum : uint32_t { JOB_PRED_S = 0, JOB_PRED_L = 1, JOB_PRED_U = 2, JOB_R6A = 3 };

struct ElError {
  int code;
  std::string msg;
};

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      throw ElError{e_ == hipErrorOutOfMemory ? EL_ENOMEM : EL_EHIP,                  \
                    std::string(#expr) + ": " + hipGetErrorString(e_)};               \
  } while (0)

// (EL_TRACE_INIT: host wall time since el_init's entry at each phase's end, on stderr; no syncs
// are added, so it shows where el_init's host side spends its time)
thread_local std::chrono::steady_clock::time_point init_t0;
void init_lap(const char* what) {
  static const bool trace = getenv("EL_TRACE_INIT") != nullptr;
  if (trace)
    fprintf(stderr, "init %-16s %8.3f ms\n", what,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - init_t0).count());
}

// ---------------------------------------------------------------- device views

struct DIndex {
  uint32_t N, R, P;
  uint64_t W;  // uint32 words per bit row
  const uint8_t* kind;
  // the rows over the told closure (el_closure.h, rebuilt by every el_init): told*(A), exr*(A),
  // exl*(A) at [begin, end) of meta below
  const uint32_t* told_b;
  const uint32_t *cidx_ptr, *cidx_c;
  // per cidx entry j of A: a binary conjunction {A, p} ⊑ B as {p | (p sorts before A) << 31, B,
  // column of p, column of B} (x = NONE: another arity, walked through conj_ptr / conj_ops).  The
  // columns (col_of at el_load: window and column order applied) let both bit words load at once
  // instead of the chain entry -> cperm[p] -> word -> cperm[B] -> word (round 6)
  const uint4* cidx_q;
  const uint32_t *conj_ptr, *conj_ops, *conj_b;
  const uint32_t* exr_pid;
  const uint32_t *exl_r, *exl_b;
  const uint32_t *fp_ptr, *pair_role, *pair_y;
  const uint32_t *psup_ptr, *psup_pid;
  // pid -> {role, filler, psup begin, psup end}: what a link trigger reads of its pair, one 16-B
  // load instead of three random lines (k_expand's link role)
  const uint4* pinfo;
  const uint32_t *chf_ptr, *chf_s, *chf_t;
  const uint32_t *chs_ptr, *chs_p, *chs_t;
  const uint32_t *dom_ptr, *dom_c;
  const uint32_t *rng_ptr, *rng_c;
  const uint8_t* role_has_exl;
  // per concept A, 32 B: meta[2A] = row begins {told*, cidx, exr*, exl*}, meta[2A + 1] = ends
  const uint4* meta;
  uint32_t has_range;
  uint32_t has_bot;  // some axiom concludes ⊥ (or ∃r.⊥): else ⊥ ∈ S(Y) only for Y = ⊥, no link reaches ⊥
  // row partition (el_config.exchange != NONE): this context owns rows [lo, hi)
  uint32_t lo, hi;
  // bit-row columns: ⊥, ⊤, then the concepts [c_lo, c_hi) — every concept an owned row can
  // hold (el_ctx::column_window; the whole ontology: 2, N) — in window order (column = concept -
  // c_lo + 2) or, for a whole ontology, in cperm's order (el_index.h column_order: the expected
  // frequent CR4 conclusions first, so a row's new facts share lines)
  uint32_t c_lo, c_hi;
  const uint32_t* cperm;
  uint32_t part;               // 1 = partitioned protocol (oracle/partition_model.py)
  uint32_t base;               // 1 = the base links {(X, p) : p ∈ exr(X)} and base propagations
                               // are in their logs and rows but not in their sets (install_base)
  // base propagations of pid: the propagation log's [bpp_s[pid], bpp_e[pid]) (B ascending)
  const uint32_t *bpp_s, *bpp_e;
  const uint8_t* role_chs;     // r -> r is the second role of some chain (its links are exchanged)
  // partitioned: every rank's column window [x, y) (el_ctx::exchange_windows); a record keyed by
  // concept Y is sent only when some OTHER rank's window holds Y (its rows can reach Y)
  const uint2* xwin;
  uint32_t nranks, me;
};

// some other rank's rows can reach concept y (⊥ and ⊤ are in every window)
__device__ __forceinline__ bool remote(const DIndex& ix, uint32_t y) {
  if (ix.nranks < 2) return false;
  if (y < 2u) return true;
  for (uint32_t q = 0; q < ix.nranks; ++q)
    if (q != ix.me && y >= ix.xwin[q].x && y < ix.xwin[q].y) return true;
  return false;
}

// Event counters: one partial row per block index, updated with plain read-modify-writes
// (a block index is unique within a launch and launches on the stream do not overlap), so
// counting costs no atomics at all; blocks beyond EV_BLOCKS share an atomic overflow row.
// k_ev_reduce folds the rows into EV_TOTAL words when the host asks.
constexpr uint32_t EV_BLOCKS = 4096;
constexpr size_t EV_TOTAL = (size_t)EL_NUM_KERNELS * EL_NUM_EVENTS;
constexpr size_t EV_WORDS = (EV_BLOCKS + 1) * EV_TOTAL;

// Step counters.  On the device every counter sits on a 256-B line of its own: appends of
// different queues then do not serialise on one L2 line (MI355X_MICROARCH.md, "fanin":
// ≈12 ns per atomic on one line).  The host copy (HCounters) is compact.
constexpr uint32_t CTR_STRIDE = 64;  // words
// Counters [0, CTR_KEEP) persist across steps; the rest are per-step (zeroed by k_commit).
// x_log / x_send / x_sp / x_sa / g_delta / g_max belong to the partitioned exchange (k_ximport):
// x_send, x_sp, x_sa count this step's records routed to other ranks (chain links, propagations,
// activations; k_commit appends, the import zeroes them once they went out).
// ov_* count the entries of this step that did not fit their slack row (gapped CSRs below).
// cand_t counts the CR1 told-closure candidates (committed first, by k_commit_told).
#define EL_COUNTERS(X) X(s_log) X(l_log) X(a_log) X(p_log) X(x_log) X(x_send) X(x_sp) X(x_sa) X(ov_pr) X(ov_sc) X(ov_pp) \
  X(cand_s) X(cand_l) X(cand_a) X(jobs) X(cand_p) X(cand_t) X(g_delta) X(g_max) X(g_ovf) X(g_pown) X(ticket) X(seq)
constexpr uint32_t CTR_KEEP = 11;
#define EL_CTR_DEV(n) uint32_t n; uint32_t n##_pad[CTR_STRIDE - 1];
#define EL_CTR_HOST(n) uint32_t n;
struct DCounters {
  EL_COUNTERS(EL_CTR_DEV)
};
struct HCounters {  // ticket: k_gap_scan tile dispenser; seq: host copy only
  EL_COUNTERS(EL_CTR_HOST)
};
constexpr uint32_t NUM_CTRS = sizeof(HCounters) / 4;
static_assert(sizeof(DCounters) == NUM_CTRS * CTR_STRIDE * 4, "counter layout");

// Gapped ("slack") CSR: row r owns the slots [start[r], end[r]) and holds len[r] entries.
// An entry is appended where its row's keyed atomic on len places it, so a superstep needs no
// CSR merge; an entry past its row's capacity goes to the overflow queue (row, value, rank)
// and the host relocates the rows that overflowed — each to gap_cap(len) fresh slots at the
// end of the slot array, its in-place entries moved and the overflow entries placed by rank —
// before the next step reads them; every other row stays where it is.  Readers of step t see
// len at the end of step t-1 (appends happen only in commit / import launches, which no reader
// shares).
struct DGap {
  const uint32_t* start;  // rows + 1 (the initial layout's scan; start[rows] is its end)
  const uint32_t* end;    // rows: end of row r's slots
  uint32_t* len;          // rows
  uint32_t* val;
  uint32_t* ovq;          // 3 words per overflowing entry
  uint32_t ovq_cap;
  uint32_t* ov_count;     // DCounters::ov_*
};

// row r of a gapped CSR as (begin, length); a CSR the ontology never fills is not allocated
// and reads as empty rows
__device__ __forceinline__ uint2 gap_row(const DGap& g, uint32_t r) {
  return g.start ? make_uint2(g.start[r], g.len[r]) : make_uint2(0u, 0u);
}

// capacity of a row with n entries after a re-layout (the CPU oracle mirrors it)
constexpr uint32_t GAP_MUL = 8;    // slack factor: a row re-laid out with n entries has room for GAP_MUL·n + GAP_BASE
constexpr uint32_t GAP_BASE = 64;  // (16 left G3 / G5 a late re-layout for a handful of entries)
__host__ __device__ constexpr uint32_t gap_cap(uint32_t n) { return GAP_MUL * n + GAP_BASE; }

struct DState {
  uint32_t* bits;
  uint8_t* summ;  // block summary of the bits (virtual row base like bits): row x, 512-B block k
  uint32_t SB;    // at summ[x·SB + k]; nullptr: none (EL_NO_SUMMARY)
  uint32_t *slog_x, *slog_a;
  uint8_t* slog_f;  // 1: the fact came out of a CR1 told closure (its own closure, links and
                    // propagations are already out); 2: an init fact X ∈ S(X) whose closure
                    // k_init wrote (its links and propagations are not out yet); 0: neither
  unsigned long long* lhash;
  unsigned long long lmask;
  uint32_t *llog_x, *llog_p;
  unsigned long long* ahash;
  unsigned long long amask;
  uint32_t *alog_y, *alog_c;
  uint8_t* has_act;
  const uint64_t* act_ptr;  // activations by Y: log indices, ascending (rebuilt between supersteps)
  const uint32_t* act_k;
  unsigned long long* phash;  // CR4 propagations (pid, B)
  unsigned long long pmask;
  uint32_t *plog_p, *plog_b;
  DGap pp;                          // propagations per pid
  uint32_t *cp_p, *cp_b, cp_cap;
  DGap pr;                          // predecessors per pid
  DGap sc;                          // successors per X (chain-second links in partitioned mode)
  uint32_t need_pred, need_succ;  // CSRs with readers: only those get delta counts
  uint32_t dedup;                 // in-wave S-candidate filter on (EL_DEDUP_OFF: off)
  uint32_t csort;                 // S commit in sorted chunks (commit_s_sorted; EL_COMMIT_SORT=0: off)
  unsigned long long* lines;      // diagnostic (EL_TRACE_CANDS): S-commit atomics, distinct 64-B lines per
                                  // wave-instruction summed, instructions (nullptr: off)
  uint32_t succ_at_commit;        // successor counts taken by k_commit (whole-ontology mode)
  // partitioned exchange: replicated chain-second link log; this step's records for other ranks:
  // chain-second links (xs), propagations (xp), activations (xa)
  uint32_t *xlog_x, *xlog_p;
  uint32_t *xs_x, *xs_p, xs_cap;
  uint32_t *xp_p, *xp_b, xp_cap;
  uint32_t *xa_y, *xa_c, xa_cap;
  uint32_t *cs_x, *cs_a, cs_cap;
  uint32_t cs_chunk;  // S-queue reservation per wave (wq_publish_s; 0: one atomic per publish)
  uint32_t *ct_x, *ct_a, ct_cap;  // CR1 told-closure candidates
  uint32_t *cl_x, *cl_p, cl_cap;
  uint32_t *ca_y, *ca_c, ca_cap;
  uint4* jobs;
  uint32_t job_cap;
  DCounters* ctr;
  unsigned long long* ev;  // [EV_BLOCKS + 1][kernel][event] per-block partials
};

// ---------------------------------------------------------------- device helpers

struct Ev {
  uint32_t v[EL_NUM_EVENTS];
  uint32_t dup;  // S candidates dropped as in-wave duplicates: charged to the S commit (ev_flush)
  __device__ Ev() : dup(0) {
#pragma unroll
    for (int i = 0; i < EL_NUM_EVENTS; ++i) v[i] = 0;
  }
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned long long wave_sum(uint32_t x) {
  unsigned long long v = x;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Block-level reduction of the event counters: one LDS atomic per wave, then one global
// atomic per (event, block) into a sharded slot.  Every thread of the block must call it.
// A candidate dropped as an in-wave duplicate (emit_s) is charged to the S commit as the
// commit would have counted it: a trigger read and a bit-word RMW that finds the bit set.
__device__ __forceinline__ void ev_flush(unsigned long long* evg, int k, const Ev& e) {
  __shared__ unsigned long long sev[EL_NUM_EVENTS + 1];
  if (threadIdx.x <= EL_NUM_EVENTS) sev[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i <= EL_NUM_EVENTS; ++i) {
    unsigned long long s = wave_sum(i < EL_NUM_EVENTS ? e.v[i] : e.dup);
    if (lane_id() == 0 && s) atomicAdd(&sev[i], s);
  }
  __syncthreads();
  const auto add = [&](int kk, int ev, unsigned long long v) {
    if (blockIdx.x < EV_BLOCKS) {
      evg[((size_t)blockIdx.x * EL_NUM_KERNELS + kk) * EL_NUM_EVENTS + ev] += v;
    } else {
      atomicAdd(&evg[((size_t)EV_BLOCKS * EL_NUM_KERNELS + kk) * EL_NUM_EVENTS + ev], v);
    }
  };
  if (threadIdx.x < EL_NUM_EVENTS && sev[threadIdx.x]) add(k, threadIdx.x, sev[threadIdx.x]);
  if (threadIdx.x == EL_NUM_EVENTS && sev[EL_NUM_EVENTS]) {
    add(EL_K_COMMIT_S, EL_EV_TRIG, sev[EL_NUM_EVENTS]);
    add(EL_K_COMMIT_S, EL_EV_RMW, sev[EL_NUM_EVENTS]);
  }
}

// out[w] = Σ_slots ev[slot][w]: one block per word
__global__ void k_ev_reduce(const unsigned long long* __restrict__ ev, unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[4];
  unsigned long long s = 0;
  for (uint32_t q = threadIdx.x; q <= EV_BLOCKS; q += blockDim.x) s += ev[(size_t)q * EV_TOTAL + blockIdx.x];
  s = wave_sum_u64(s);
  if (lane_id() == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// Wave-aggregated append: one atomic per wave; returns this lane's slot when pred.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
  unsigned long long m = __ballot(pred);
  if (m == 0) return NONE;
  int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
  return pred ? base + rank : NONE;
}

// Keyed counter update: the lanes of a wave are grouped by key (a match-any built from
// ballots and v_readlane: scalar-latency ALU work, one round per distinct key — a shuffle
// per round would put an LDS round trip on this chain), then ONE atomic instruction is issued
// in which each group's first lane adds the group size; the members read their slot from
// the returned value by a shuffle.  Same-key lanes of one atomic instruction would
// otherwise serialise at the L2 atomic unit, and hub rows (a pid that gains hundreds of
// predecessors in a step) make that the common case.
// Returns, per lane, the value an individual atomic on that lane would have returned
// in some serialisation (old + rank for add, old - rank for sub).
__device__ __forceinline__ uint32_t wave_keyed_atomic(uint32_t* base, uint32_t key, bool pred, bool sub) {
  unsigned long long pending = __ballot(pred);
  if (pending == 0) return 0;
  const uint32_t lane = lane_id();
  unsigned long long group = 0;  // this lane's key group (lanes with the same key)
  while (pending) {              // scalar loop: leader by s_ff1, its key by v_readlane
    const int leader = __ffsll((long long)pending) - 1;
    const uint32_t lkey = __builtin_amdgcn_readlane(key, leader);
    const unsigned long long same = __ballot(pred && key == lkey) & pending;
    if ((same >> lane) & 1ull) group = same;
    pending &= ~same;
  }
  const uint32_t first = pred ? (uint32_t)__ffsll((long long)group) - 1 : lane;
  const uint32_t rank = (uint32_t)__popcll(group & ((1ull << lane) - 1ull));
  uint32_t old = 0;
  if (pred && first == lane) {
    const uint32_t cnt = (uint32_t)__popcll(group);
    old = sub ? atomicSub(base + key, cnt) : atomicAdd(base + key, cnt);
  }
  old = __shfl(old, (int)first);
  return sub ? old - rank : old + rank;
}

// Append v to row `row` of a gapped CSR (every lane calls it; pred selects the lanes that
// append).  Events: the len atomic (RMW), the row bounds (ROW), the value (ENT); an entry
// past the row's capacity writes a 3-word overflow record instead (3 ENT).
__device__ __forceinline__ void gap_append(const DGap& g, uint32_t row, uint32_t v, bool pred, uint32_t* ev) {
  const uint32_t rank = wave_keyed_atomic(g.len, row, pred, false);
  bool ovf = false;
  if (pred) {
    ev[EL_EV_RMW]++;
    ev[EL_EV_ROW]++;
    ev[EL_EV_ENT]++;
    const uint32_t s = g.start[row] + rank;
    ovf = s >= g.end[row];
    if (!ovf) g.val[s] = v;
  }
  const uint32_t q = wave_append(g.ov_count, ovf);
  if (ovf) {
    ev[EL_EV_ENT] += 2;
    if (q < g.ovq_cap) {
      g.ovq[3 * (size_t)q] = row;
      g.ovq[3 * (size_t)q + 1] = v;
      g.ovq[3 * (size_t)q + 2] = rank;
    }
  }
}

// bit-row column of concept a, NONE when no owned row can hold a (outside the window)
__device__ __forceinline__ uint32_t col_of(const DIndex& ix, uint32_t a) {
  if (a < 2u) return a;
  if (a < ix.c_lo || a >= ix.c_hi) return NONE;
  return ix.cperm ? ix.cperm[a] : a - ix.c_lo + 2u;
}

__device__ __forceinline__ bool test_bit(const DIndex& ix, const uint32_t* bits, uint32_t x, uint32_t b) {
  const uint32_t c = col_of(ix, b);
  return c != NONE && ((bits[(uint64_t)x * ix.W + (c >> 5)] >> (c & 31u)) & 1u);
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

__device__ __forceinline__ unsigned long long link_key(uint32_t pid, uint32_t x) {
  return ((unsigned long long)pid << 32) | x;
}

__device__ __forceinline__ bool hash_contains(const unsigned long long* t, unsigned long long mask,
                                              unsigned long long key) {
  unsigned long long h = mix64(key) & mask;
  while (true) {
    unsigned long long k = t[h];
    if (k == key) return true;
    if (k == EMPTY_KEY) return false;
    h = (h + 1) & mask;
  }
}

// true when the key was not present and this thread inserted it
__device__ __forceinline__ bool hash_insert(unsigned long long* t, unsigned long long mask,
                                            unsigned long long key) {
  unsigned long long h = mix64(key) & mask;
  while (true) {
    unsigned long long prev = atomicCAS(&t[h], EMPTY_KEY, key);
    if (prev == EMPTY_KEY) return true;
    if (prev == key) return false;
    h = (h + 1) & mask;
  }
}

// Base links: the links every init fact X ∈ S(X) implies by CR3 over its told closure,
// {(X, p) : p ∈ exr*(X)} (G3: 25 M of 33 M links).  el_saturate writes them into the link log
// and the predecessor / successor rows before the first superstep, with coalesced stores,
// instead of deriving them as 25 M candidates that the commit would hash one by one; the
// set of them is exr* itself, so membership is a binary search of the row exr*(X) (sorted).
__device__ __forceinline__ bool base_has(const DIndex& ix, uint32_t x, uint32_t pid, Ev& ev) {
  ev.v[EL_EV_ROW]++;
  uint32_t lo = ix.meta[2 * x].z, hi = ix.meta[2 * x + 1].z;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    ev.v[EL_EV_ENT]++;
    const uint32_t v = ix.exr_pid[mid];
    if (v == pid) return true;
    if (v < pid)
      lo = mid + 1;
    else
      hi = mid;
  }
  return false;
}

// (x, pid) known at t-1: a base link, or in the link set (lempty: the set is empty, no probe)
__device__ __forceinline__ bool link_known(const DIndex& ix, const DState& st, uint32_t x, uint32_t pid,
                                           bool lempty, Ev& ev) {
  if (ix.base && base_has(ix, x, pid, ev)) return true;
  if (lempty) return false;
  ev.v[EL_EV_HASH]++;
  return hash_contains(st.lhash, st.lmask, link_key(pid, x));
}

// ((r, Y), B) known at t-1: a base propagation (binary search of bpp(pid)), or in the set
__device__ __forceinline__ bool prop_known(const DIndex& ix, const DState& st, uint32_t pid, uint32_t b,
                                           bool pempty, Ev& ev) {
  if (ix.base) {
    ev.v[EL_EV_ROW]++;
    uint32_t lo = ix.bpp_s[pid], hi = ix.bpp_e[pid];
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      ev.v[EL_EV_ENT]++;
      const uint32_t v = st.plog_b[mid];
      if (v == b) return true;
      if (v < b)
        lo = mid + 1;
      else
        hi = mid;
    }
  }
  if (pempty) return false;
  ev.v[EL_EV_HASH]++;
  return hash_contains(st.phash, st.pmask, link_key(pid, b));
}

// (role, filler) -> pid by a scan of the filler's pair range (sorted by role)
__device__ __forceinline__ uint32_t pair_lookup(const DIndex& ix, uint32_t r, uint32_t y, Ev& ev) {
  ev.v[EL_EV_ROW]++;
  uint32_t b = ix.fp_ptr[y], e = ix.fp_ptr[y + 1];
  for (uint32_t p = b; p < e; ++p) {
    ev.v[EL_EV_ENT]++;
    uint32_t rr = ix.pair_role[p];
    if (rr == r) return p;
    if (rr > r) return NONE;
  }
  return NONE;
}

// pair_lookup over a pair range [b, e) of the filler already read (same events)
__device__ __forceinline__ uint32_t pair_scan(const DIndex& ix, uint32_t r, uint32_t b, uint32_t e, Ev& ev) {
  ev.v[EL_EV_ROW]++;
  for (uint32_t p = b; p < e; ++p) {
    ev.v[EL_EV_ENT]++;
    uint32_t rr = ix.pair_role[p];
    if (rr == r) return p;
    if (rr > r) return NONE;
  }
  return NONE;
}

// LDS staging of the commit roles (new facts / links of a block round)
constexpr uint32_t QS_CAP = 2048;  // (a block flushes ~QS_CAP/2 new facts per log atomic)
constexpr uint32_t QL_CAP = 2048;

// LDS slot for each predicated lane (one LDS atomic per wave)
__device__ __forceinline__ uint32_t lds_reserve(uint32_t* qn, bool pred) {
  unsigned long long m = __ballot(pred);
  if (m == 0) return NONE;
  int leader = __ffsll((long long)m) - 1;
  uint32_t off = 0;
  if ((int)lane_id() == leader) off = atomicAdd(qn, (uint32_t)__popcll(m));
  off = __shfl(off, leader);
  return pred ? off + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull)) : NONE;
}

// Wave-private staging of appended records in LDS.  A single global append counter
// serialises same-address atomics (MI355X_MICROARCH.md, "fanin": ≈12 ns each), so each
// wave stages its candidates in its own LDS queues and publishes a full queue with ONE
// global atomic (WQ records).  No block barrier is involved, so a wave may flush in the
// middle of a divergent inner loop (a told closure, a fan-out row): only the wave's
// active lanes take part, and LDS accesses of one wave execute in program order.
// 128 records: 20.7 KB of LDS per block, so VGPRs (not LDS) bound k_expand's occupancy at 7 waves
// per SIMD instead of 4 (G3 A/B, round 4: 26.09 / 25.93 vs 26.19 / 26.51 ms per classification).
#ifndef EL_WQ
#define EL_WQ 128
#endif
constexpr uint32_t WQ = EL_WQ;  // (x, a) / (x, pid) records per wave and queue
constexpr uint32_t WQJ = 64;   // fan-out job records per wave

// In-wave duplicate filter for S candidates: a direct-mapped cache of the wave's recent
// (x, a) keys.  Duplicates of one conclusion within a step are common (G3 step 1: 96 M S
// candidates for 13 M new facts — the links of one X reach fillers with overlapping
// subsumers) and each would cost a queue slot, a global write and read and a bit-word
// atomic; the cache drops those it still holds.  Lossy by design: a key evicted or raced
// by another lane just reaches the commit, whose atomicOr dedups exactly.
#ifndef EL_DEDUP_BITS
#define EL_DEDUP_BITS 7
#endif
constexpr uint32_t DEDUP_SLOTS = 1u << EL_DEDUP_BITS;

struct WaveQ {
  unsigned long long seen[DEDUP_SLOTS];  // S-candidate keys (x << 32 | a), ~0 = empty
  uint32_t sx[WQ], sa[WQ];  // S candidates
  uint32_t tx[WQ], ta[WQ];  // CR1 told-closure candidates
  uint32_t lx[WQ], lp[WQ];  // link candidates
  uint32_t px[WQ], pb[WQ];  // CR4 propagation candidates (pid, B)
  uint4 jb[WQJ];            // fan-out jobs
  uint32_t ns, nt, nl, nj, np;
  uint32_t rs_base, rs_left, rs_next;  // S queue: this wave's reserved slots, next reservation size
};
struct BlockQ {
  WaveQ w[BLOCK / 64];
};

__device__ __forceinline__ WaveQ& wave_q(BlockQ& q) { return q.w[threadIdx.x >> 6]; }

__device__ __forceinline__ void q_init(BlockQ& q) {
  WaveQ& w = wave_q(q);
  if (lane_id() == 0) w.ns = w.nt = w.nl = w.nj = w.np = w.rs_left = w.rs_next = 0;
  for (uint32_t i = lane_id(); i < DEDUP_SLOTS; i += 64) w.seen[i] = ~0ull;
  __syncthreads();
}

// Publish n staged records of this wave: one atomic, the active lanes copy.
template <class T>
__device__ __forceinline__ void wq_publish(const T* qa, const uint32_t* qb, uint32_t n, uint32_t* gcnt, T* ga,
                                           uint32_t* gb, uint32_t gcap) {
  if (n == 0) return;
  const unsigned long long act = __ballot(true);
  const int leader = __ffsll((long long)act) - 1;
  uint32_t base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(gcnt, n);
  base = __shfl(base, leader);
  const uint32_t na = (uint32_t)__popcll(act), r = (uint32_t)__popcll(act & ((1ull << lane_id()) - 1ull));
  for (uint32_t k = r; k < n; k += na) {
    const uint32_t slot = base + k;
    if (slot < gcap) {
      ga[slot] = qa[k];
      if (gb) gb[slot] = qb[k];
    }
  }
}

// The S-candidate queue of a big step (G3's first superstep: 96 M candidates): a wave reserves
// queue slots in growing chunks (its first publish exactly, then 512, 1024, … up to cs_chunk)
// and fills them over several publishes, instead of one atomic on the queue counter per 256
// records — 375 k same-address atomics at ~12 ns each (MI355X_MICROARCH.md "fanin") were 4.5 ms
// of that step's k_jobs.  The last reservation's unused tail is marked x = NONE when the wave
// finishes (q_flush) and the commit skips such holes; growing chunks keep the holes below the
// wave's own output (a wave of a small step that publishes once leaves none).
__device__ __forceinline__ void wq_publish_s(WaveQ& w, const DState& st, uint32_t n) {
  if (n == 0) return;
  const uint32_t chunk = st.cs_chunk;
  if (chunk == 0) {
    wq_publish(w.sx, w.sa, n, &st.ctr->cand_s, st.cs_x, st.cs_a, st.cs_cap);
    return;
  }
  const unsigned long long act = __ballot(true);
  const int leader = __ffsll((long long)act) - 1;
  const uint32_t na = (uint32_t)__popcll(act), r = (uint32_t)__popcll(act & ((1ull << lane_id()) - 1ull));
  uint32_t base = w.rs_base, left = w.rs_left, next = w.rs_next, size = 0;
  for (uint32_t done = 0; done < n;) {
    if (left == 0) {
      size = next == 0 ? n - done : next;  // (the first reservation: exactly this publish)
      next = next == 0 ? min(2u * WQ, chunk) : min(2u * next, chunk);
      uint32_t b = 0;
      if ((int)lane_id() == leader) b = atomicAdd(&st.ctr->cand_s, size);
      base = __shfl(b, leader) + size;  // base: the reservation's end
      left = size;
    }
    const uint32_t take = min(n - done, left), off = base - left;
    for (uint32_t k = r; k < take; k += na) {
      const uint32_t slot = off + k;
      if (slot < st.cs_cap) {
        st.cs_x[slot] = w.sx[done + k];
        st.cs_a[slot] = w.sa[done + k];
      }
    }
    done += take;
    left -= take;
  }
  if ((int)lane_id() == leader) {
    w.rs_base = base;
    w.rs_left = left;
    w.rs_next = next;
  }
}

// Stage (a, b) for the predicated lanes; a full queue is published first.
__device__ __forceinline__ void wq_push(uint32_t* qa, uint32_t* qb, uint32_t& qn, bool pred, uint32_t a, uint32_t b,
                                        uint32_t* gcnt, uint32_t* ga, uint32_t* gb, uint32_t gcap) {
  const unsigned long long m = __ballot(pred);
  if (m == 0) return;
  const uint32_t cnt = (uint32_t)__popcll(m);
  uint32_t n = qn;
  if (n + cnt > WQ) {
    wq_publish(qa, qb, n, gcnt, ga, gb, gcap);
    n = 0;
  }
  if (pred) {
    const uint32_t r = n + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
    qa[r] = a;
    qb[r] = b;
  }
  if ((int)lane_id() == __ffsll((long long)__ballot(true)) - 1) qn = n + cnt;
}

__device__ __forceinline__ void emit_s(const DState& st, BlockQ& q, bool pred, uint32_t x, uint32_t a, Ev& ev) {
  WaveQ& w = wave_q(q);
  if (pred) ev.v[EL_EV_EMIT]++;
  if (pred && st.dedup) {
    const unsigned long long key = ((unsigned long long)x << 32) | a;
    const uint32_t slot = ((x * 2654435761u) ^ (a * 2246822519u)) >> (32 - EL_DEDUP_BITS);
    if (w.seen[slot] == key) {
      pred = false;  // the wave queued (x, a) already in this launch
      ev.dup++;
    } else {
      w.seen[slot] = key;
    }
  }
  const unsigned long long m = __ballot(pred);
  if (m == 0) return;
  const uint32_t cnt = (uint32_t)__popcll(m);
  uint32_t n = w.ns;
  if (n + cnt > WQ) {
    wq_publish_s(w, st, n);
    n = 0;
  }
  if (pred) {
    const uint32_t r = n + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
    w.sx[r] = x;
    w.sa[r] = a;
  }
  if ((int)lane_id() == __ffsll((long long)__ballot(true)) - 1) w.ns = n + cnt;
}

__device__ __forceinline__ void emit_t(const DState& st, BlockQ& q, bool pred, uint32_t x, uint32_t a, Ev& ev) {
  WaveQ& w = wave_q(q);
  if (pred) ev.v[EL_EV_EMIT]++;
  wq_push(w.tx, w.ta, w.nt, pred, x, a, &st.ctr->cand_t, st.ct_x, st.ct_a, st.ct_cap);
}

__device__ __forceinline__ void emit_l(const DState& st, BlockQ& q, bool pred, uint32_t x, uint32_t pid, Ev& ev) {
  WaveQ& w = wave_q(q);
  if (pred) ev.v[EL_EV_EMIT]++;
  wq_push(w.lx, w.lp, w.nl, pred, x, pid, &st.ctr->cand_l, st.cl_x, st.cl_p, st.cl_cap);
}

__device__ __forceinline__ void emit_job1(const DState& st, BlockQ& q, bool pred, uint32_t type, uint32_t begin,
                                          uint32_t len, uint32_t a, uint32_t b, Ev& ev) {
  WaveQ& w = wave_q(q);
  const unsigned long long m = __ballot(pred);
  if (m == 0) return;
  const uint32_t cnt = (uint32_t)__popcll(m);
  uint32_t n = w.nj;
  if (n + cnt > WQJ) {
    wq_publish<uint4>(w.jb, nullptr, n, &st.ctr->jobs, st.jobs, nullptr, st.job_cap);
    n = 0;
  }
  if (pred) {
    ev.v[EL_EV_JOB]++;
    w.jb[n + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull))] = make_uint4(begin, len | (type << 28), a, b);
  }
  if ((int)lane_id() == __ffsll((long long)__ballot(true)) - 1) w.nj = n + cnt;
}

// A fan-out list of len items becomes ceil(len / JOB_CHUNK) job records, so one hub
// (a filler with 10^4 predecessors) is spread over many waves instead of serialising one.
constexpr uint32_t JOB_CHUNK = 256;
__device__ __forceinline__ void emit_job(const DState& st, BlockQ& q, bool pred, uint32_t type, uint32_t begin,
                                         uint32_t len, uint32_t a, uint32_t b, Ev& ev) {
  const uint32_t n = pred ? (len + JOB_CHUNK - 1) / JOB_CHUNK : 0u;
  for (uint32_t c = 0; __ballot(c < n) != 0; ++c) {
    const bool pc = c < n;
    const uint32_t cb = begin + c * JOB_CHUNK;
    const uint32_t cl = pc ? min(JOB_CHUNK, len - c * JOB_CHUNK) : 0u;
    emit_job1(st, q, pc, type, cb, cl, a, b, ev);
  }
}

// activations are rare: plain wave-aggregated global append
__device__ __forceinline__ void emit_a(const DState& st, bool pred, uint32_t y, uint32_t c, Ev& ev) {
  uint32_t slot = wave_append(&st.ctr->cand_a, pred);
  if (pred) {
    ev.v[EL_EV_EMIT]++;
    if (slot < st.ca_cap) {
      st.ca_y[slot] = y;
      st.ca_c[slot] = c;
    }
  }
}

// CR4 propagations, staged in the wave's queue like the links (round 6: a wave-aggregated global
// append per wave-instruction put every emitting round of the CR4 half-1 walk on one counter —
// same-address atomics serialise at ~12 ns)
__device__ __forceinline__ void emit_p(const DState& st, BlockQ& q, bool pred, uint32_t pid, uint32_t b, Ev& ev) {
  WaveQ& w = wave_q(q);
  if (pred) ev.v[EL_EV_EMIT]++;
  wq_push(w.px, w.pb, w.np, pred, pid, b, &st.ctr->cand_p, st.cp_p, st.cp_b, st.cp_cap);
}

// Publish what this wave still has staged (every lane of the block calls it at the end
// of its role, so the staged records of the step are all in the global queues).
__device__ void q_flush(BlockQ& q, const DState& st) {
  WaveQ& w = wave_q(q);
  wq_publish_s(w, st, w.ns);
  if (st.cs_chunk) {  // the reservation's unused tail becomes holes
    const unsigned long long act = __ballot(true);
    const uint32_t na = (uint32_t)__popcll(act), r = (uint32_t)__popcll(act & ((1ull << lane_id()) - 1ull));
    const uint32_t left = w.rs_left, off = w.rs_base - left;
    for (uint32_t k = r; k < left; k += na)
      if (off + k < st.cs_cap) st.cs_x[off + k] = NONE;
    if ((int)lane_id() == __ffsll((long long)act) - 1) w.rs_left = 0;
  }
  wq_publish(w.tx, w.ta, w.nt, &st.ctr->cand_t, st.ct_x, st.ct_a, st.ct_cap);
  wq_publish(w.lx, w.lp, w.nl, &st.ctr->cand_l, st.cl_x, st.cl_p, st.cl_cap);
  wq_publish(w.px, w.pb, w.np, &st.ctr->cand_p, st.cp_p, st.cp_b, st.cp_cap);
  wq_publish<uint4>(w.jb, nullptr, w.nj, &st.ctr->jobs, st.jobs, nullptr, st.job_cap);
  if (lane_id() == 0) w.ns = w.nt = w.nl = w.nj = w.np = 0;
}

// The wave queues publish themselves when full: nothing to do between loop rounds.
__device__ __forceinline__ void q_maybe_flush(BlockQ&, const DState&) {}

// ---------------------------------------------------------------- kernels

// State reset for el_init in one launch (instead of a dozen fill launches): each segment
// is filled with a repeated 32-bit pattern, 16 B per store.
struct FillSeg {
  void* p;
  uint64_t bytes;
  uint32_t pattern;
};
struct FillArgs {
  FillSeg seg[16];
  uint32_t n;
};
__global__ void k_fill(FillArgs f) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint32_t k = 0; k < f.n; ++k) {
    const FillSeg g = f.seg[k];
    const uint32_t v = g.pattern;
    uint4* q = reinterpret_cast<uint4*>(g.p);
    const uint64_t n16 = g.bytes / 16;
    for (uint64_t i = tid; i < n16; i += stride) q[i] = make_uint4(v, v, v, v);
    uint8_t* b = reinterpret_cast<uint8_t*>(g.p);
    for (uint64_t i = n16 * 16 + tid; i < g.bytes; i += stride) b[i] = (uint8_t)(v >> (8 * (i & 3)));
  }
}

__global__ void k_set_u32(uint32_t* p, uint32_t v) { *p = v; }

// The block summary of whole rows from the matrix (after an increment re-laid the matrix out).
__global__ void k_summ_build(const uint32_t* __restrict__ bits, uint64_t W, uint64_t words, uint8_t* __restrict__ summ,
                             uint32_t SB) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    if (bits[i]) summ[(i / W) * SB + (i % W) / elrows::SUMM_WORDS] = 1;
}

// Wave-cooperative loop over one CSR row per lane, [b, e) (an idle lane passes b = e): the
// wave walks the concatenation of its lanes' rows 64 entries at a time, so a lane with a
// long row (a told closure, the links of a whole closure) does not serialise its wave while
// the other lanes idle.  Every lane runs every round (the emitters ballot); f(valid, owner,
// j) gets the lane that owns entry j.  Owners are found by binary lifting over the
// inclusive scan of the row lengths (6 lane shuffles).
template <class F>
__device__ __forceinline__ void wave_rows(uint32_t b, uint32_t e, F&& f) {
  const uint32_t lane = lane_id(), len = e - b;
  uint32_t inc = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, 63), excl = inc - len;
  for (uint32_t base = 0; base < total; base += 64) {
    const uint32_t k = base + lane;
    uint32_t own = 0;  // the number of lanes whose rows end at or before entry k
#pragma unroll
    for (uint32_t step = 32; step > 0; step >>= 1)
      if (__shfl(inc, (int)(own + step - 1)) <= k) own += step;
    const bool valid = k < total;
    own = valid ? own : 0u;
    const uint32_t j = __shfl(b, (int)own) + (k - __shfl(excl, (int)own));
    f(valid, own, j);
  }
}

// wave_rows four rounds at a time, each round's loads issued before any is used: first(valid,
// owner, j) makes a round's first load, second(valid, owner, x) its dependent load, use(valid,
// owner, x, y) the rest.  A round of a row walk is otherwise a chain (entry -> bit word) the wave
// waits out alone; four in flight quadruple its memory-level parallelism.
template <class First, class Second, class Use>
__device__ __forceinline__ void wave_rows4(uint32_t b, uint32_t e, First&& first, Second&& second, Use&& use) {
  const uint32_t lane = lane_id(), len = e - b;
  uint32_t inc = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, 63), excl = inc - len;
  for (uint32_t base = 0; base < total; base += 256) {  // (wave-uniform)
    uint32_t own[4];
    bool valid[4];
    decltype(first(false, 0u, 0u)) x[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
      const uint32_t k = base + r * 64 + lane;
      uint32_t ow = 0;
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1)
        if (__shfl(inc, (int)(ow + step - 1)) <= k) ow += step;
      valid[r] = k < total;
      own[r] = valid[r] ? ow : 0u;
      x[r] = first(valid[r], own[r], __shfl(b, (int)own[r]) + (k - __shfl(excl, (int)own[r])));
    }
    decltype(second(false, 0u, x[0])) y[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) y[r] = second(valid[r], own[r], x[r]);
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) use(valid[r], own[r], x[r], y[r]);
  }
}

// wave_rows NR rounds at a time: f(valid[NR], own[NR], j[NR]) gets NR rounds of entries (every
// lane, every call) and runs their chains in lockstep, NR dependent loads in flight per step.
#ifndef EL_XR
#define EL_XR 2  // (4: 106 VGPRs, 4 waves per SIMD, slower; 2: 87 VGPRs, 5 waves — G3 A/B, round 6)
#endif
constexpr uint32_t XR = EL_XR;
template <uint32_t NR, class F>
__device__ __forceinline__ void wave_rows_x(uint32_t b, uint32_t e, F&& f) {
  const uint32_t lane = lane_id(), len = e - b;
  uint32_t inc = len;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  const uint32_t total = __shfl(inc, 63), excl = inc - len;
  for (uint32_t base = 0; base < total; base += NR * 64) {  // (wave-uniform)
    uint32_t own[NR], j[NR];
    bool valid[NR];
#pragma unroll
    for (uint32_t r = 0; r < NR; ++r) {
      const uint32_t k = base + r * 64 + lane;
      uint32_t ow = 0;
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1)
        if (__shfl(inc, (int)(ow + step - 1)) <= k) ow += step;
      valid[r] = k < total;
      own[r] = valid[r] ? ow : 0u;
      j[r] = __shfl(b, (int)own[r]) + (k - __shfl(excl, (int)own[r]));
    }
    f(valid, own, j);
  }
}

// NR binary searches of sorted a[lo, hi) for v in lockstep (one probe of each per step: NR
// loads in flight); the probe sequence of each is base_has's, so are its events (one entry per probe)
template <uint32_t NR>
__device__ __forceinline__ void bsearch_x(const uint32_t* a, uint32_t (&lo)[NR], uint32_t (&hi)[NR],
                                          const uint32_t (&v)[NR], bool (&found)[NR], Ev& ev) {
  bool any = false;
#pragma unroll
  for (uint32_t r = 0; r < NR; ++r) any |= lo[r] < hi[r];
  while (any) {
    uint32_t mid[NR], x[NR];
#pragma unroll
    for (uint32_t r = 0; r < NR; ++r) {
      mid[r] = (lo[r] + hi[r]) >> 1;
      x[r] = lo[r] < hi[r] ? a[mid[r]] : 0u;
    }
    any = false;
#pragma unroll
    for (uint32_t r = 0; r < NR; ++r) {
      if (lo[r] < hi[r]) {
        ev.v[EL_EV_ENT]++;
        if (x[r] == v[r]) {
          found[r] = true;
          lo[r] = hi[r];
        } else if (x[r] < v[r]) {
          lo[r] = mid[r] + 1;
        } else {
          hi[r] = mid[r];
        }
      }
      any |= lo[r] < hi[r];
    }
  }
}

// NR open-addressing probes in lockstep (hash_contains each)
template <uint32_t NR>
__device__ __forceinline__ void hash_contains_x(const unsigned long long* t, unsigned long long mask,
                                                const unsigned long long (&key)[NR], const bool (&ask)[NR],
                                                bool (&found)[NR]) {
  unsigned long long h[NR];
  bool pend[NR], any = false;
#pragma unroll
  for (uint32_t r = 0; r < NR; ++r) {
    pend[r] = ask[r];
    found[r] = false;
    h[r] = mix64(key[r]) & mask;
    any |= pend[r];
  }
  while (any) {
    unsigned long long k[NR];
#pragma unroll
    for (uint32_t r = 0; r < NR; ++r) k[r] = pend[r] ? t[h[r]] : EMPTY_KEY;
    any = false;
#pragma unroll
    for (uint32_t r = 0; r < NR; ++r) {
      if (!pend[r]) continue;
      if (k[r] == key[r]) {
        found[r] = true;
        pend[r] = false;
      } else if (k[r] == EMPTY_KEY) {
        pend[r] = false;
      } else {
        h[r] = (h[r] + 1) & mask;
        any = true;
      }
    }
  }
}

// the bit word holding (x, b)'s bit, and the bit (NONE-column: no word, bit 32 = never set)
__device__ __forceinline__ uint32_t bit_word(const DIndex& ix, const uint32_t* bits, uint32_t x, uint32_t b) {
  const uint32_t c = col_of(ix, b);
  return c != NONE ? bits[(uint64_t)x * ix.W + (c >> 5)] : 0u;
}
__device__ __forceinline__ bool bit_in(const DIndex& ix, uint32_t word, uint32_t b) {
  const uint32_t c = col_of(ix, b);
  return c != NONE && ((word >> (c & 31u)) & 1u);
}

// Rules triggered by new S-facts (X, A) = log[begin, end).
//  CR1  Type1_1AxiomProcessorBase.java:22-43      CR2  Type1_2AxiomProcessorBase.java:45-66
//  CR3  Type2AxiomProcessorBase.java:45-75        CR4½ Type3_1AxiomProcessorBase.java:194-239
//  ⊥    TypeBottomAxiomProcessorBase.java:62-123  range RolePairHandler.java:471-479 + K10
// The index rows of CR1, CR3 and CR4 half-1 (told closure, its links, its propagations) are
// walked wave-cooperatively (wave_rows); the short CR2 rows per lane.
// tpw: triggers per wave (lanes [0, tpw) take one each) — see wave_triggers.
__device__ __forceinline__ void expand_s(const DIndex& ix, const DState& st, BlockQ& q, uint32_t bid, uint32_t nb,
                         uint32_t begin, uint32_t end, uint32_t mask, uint32_t a_end, uint32_t tpw) {
  Ev ev;
  const uint32_t w0 = bid * (blockDim.x >> 6) + (threadIdx.x >> 6), nw = nb * (blockDim.x >> 6);
  const uint32_t step = nw * tpw;
  // A software pipeline over the wave's trigger batches: while a batch walks its rows, the
  // batch after it has its fact and its meta rows in flight and the one after that its fact,
  // so the two dependent loads (log -> meta) at the head of a batch are off the wave's chain.
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  auto live = [&](uint64_t b) { return lane_id() < tpw && b + lane_id() < end; };
  uint32_t X1 = 0, A1 = 0, f1 = 1, X2 = 0, A2 = 0, f2 = 1;
  uint4 n0 = z4, n1 = z4;
  {
    const uint64_t b0 = begin + (uint64_t)w0 * tpw;
    if (live(b0)) {
      const uint32_t i = (uint32_t)b0 + lane_id();
      X1 = st.slog_x[i], A1 = st.slog_a[i], f1 = st.slog_f[i];
      n0 = ix.meta[2 * A1];  // the four rows of A at once: begins, ends
      n1 = ix.meta[2 * A1 + 1];
    }
    if (live(b0 + step)) {
      const uint32_t i = (uint32_t)(b0 + step) + lane_id();
      X2 = st.slog_x[i], A2 = st.slog_a[i], f2 = st.slog_f[i];
    }
  }
  for (uint32_t base = begin + w0 * tpw; base < end; base += step) {  // (wave-uniform)
    const bool act = live(base);
    const uint32_t X = act ? X1 : 0u, A = act ? A1 : 0u, f = act ? f1 : 1u;
    const uint4 m0 = act ? n0 : z4, m1 = act ? n1 : z4;
    if (act) ev.v[EL_EV_TRIG]++;
    X1 = X2, A1 = A2, f1 = f2;
    n0 = n1 = z4;
    if (live((uint64_t)base + step)) {
      n0 = ix.meta[2 * A1];
      n1 = ix.meta[2 * A1 + 1];
    }
    if (live((uint64_t)base + 2ull * step)) {
      const uint32_t i = base + 2 * step + lane_id();
      X2 = st.slog_x[i], A2 = st.slog_a[i], f2 = st.slog_f[i];
    }
    // A ∈ S(X), A ⊑* B  =>  B ∈ S(X), over the told closure at once; a fact that came out
    // of a closure is not re-expanded (its closure is a subset of the one that produced it)
    {
      const bool on = act && (mask & M_R1) && f == 0;
      if (on) ev.v[EL_EV_ROW]++;
      wave_rows4(
          on ? m0.x : 0u, on ? m1.x : 0u,
          [&](bool v, uint32_t own, uint32_t j) {
            const uint32_t Xo = __shfl(X, (int)own);
            return make_uint2(Xo, v ? ix.told_b[j] : 0u);
          },
          [&](bool v, uint32_t, uint2 xb) { return v ? bit_word(ix, st.bits, xb.x, xb.y) : 0u; },
          [&](bool v, uint32_t, uint2 xb, uint32_t word) {
            bool nw = false;
            if (v) {
              ev.v[EL_EV_ENT]++;
              ev.v[EL_EV_TEST]++;
              nw = !bit_in(ix, word, xb.y);
            }
            emit_t(st, q, nw, xb.x, xb.y, ev);
          });
    }
    if (act && (mask & M_R2)) {  // A1..An ∈ S(X), ⊓Ai ⊑ B  =>  B ∈ S(X)
      ev.v[EL_EV_ROW]++;
      for (uint32_t j = m0.y; j < m1.y; ++j) {
        const uint4 cq = ix.cidx_q[j];
        ev.v[EL_EV_ENT]++;
        ev.v[EL_EV_ROW]++;
        if (cq.x != NONE) {
          // binary A ⊓ p ⊑ B from the entry itself: one 16-B load instead of the chain conj id ->
          // operand row -> operands, and the two bit words (p's and B's) loaded together from
          // the entry's columns.  Events as the operand walk counts them (the sorted operands:
          // A's entry is read before p's, or after it only if p ∈ S(X)); B's word is a
          // speculative load, counted only when the walk would test it
          const uint32_t B = cq.y;
          const bool p_first = cq.x >> 31;
          const uint32_t* row = st.bits + (uint64_t)X * ix.W;
          const uint32_t wp = cq.z != NONE ? row[cq.z >> 5] : 0u;
          const uint32_t wb = cq.w != NONE ? row[cq.w >> 5] : 0u;
          ev.v[EL_EV_ENT]++;
          ev.v[EL_EV_TEST]++;
          const bool ok = cq.z != NONE && ((wp >> (cq.z & 31u)) & 1u);
          if (ok || !p_first) ev.v[EL_EV_ENT]++;
          bool nw = false;
          if (ok) {
            ev.v[EL_EV_ENT]++;
            ev.v[EL_EV_TEST]++;
            nw = !(cq.w != NONE && ((wb >> (cq.w & 31u)) & 1u));
          }
          emit_s(st, q, nw, X, B, ev);
          continue;
        }
        const uint32_t c = ix.cidx_c[j];
        const uint32_t o1 = ix.conj_ptr[c + 1];
        bool ok = true;
        for (uint32_t k = ix.conj_ptr[c]; k < o1; ++k) {
          const uint32_t op = ix.conj_ops[k];
          ev.v[EL_EV_ENT]++;
          if (op == A) continue;
          ev.v[EL_EV_TEST]++;
          if (!test_bit(ix, st.bits, X, op)) {
            ok = false;
            break;
          }
        }
        bool nw = false;
        const uint32_t B = ix.conj_b[c];
        if (ok) {
          ev.v[EL_EV_ENT]++;
          ev.v[EL_EV_TEST]++;
          nw = !test_bit(ix, st.bits, X, B);
        }
        emit_s(st, q, nw, X, B, ev);
      }
    }
    // CR3 / CR4 half-1 run over the told closure too (index rows exr / exl of A cover
    // {A} ∪ told*(A)): the facts of a closure were covered by the fact that emitted it
    const bool star = act && f != 1;
    {  // A ∈ S(X), A ⊑ ∃r.B  =>  (X, B) ∈ R(r)
      // (an init fact's own links are the base links, already in place)
      const bool on = star && (mask & M_R3) && !(ix.base && f == 2);
      if (on) ev.v[EL_EV_ROW]++;
      // X's own exr* row (the base links {(X, p) : p ∈ exr*(X)}), read once per trigger
      uint32_t xb = 0, xe = 0;
      if (on && ix.base) {
        xb = ix.meta[2 * X].z;
        xe = ix.meta[2 * X + 1].z;
      }
      const bool lempty = mask & M_LEMPTY;
      // XR rounds of entries at a time, their chains (entry -> base-link search -> set probe) in
      // lockstep: XR dependent loads in flight per lane instead of one (round 6)
      wave_rows_x<XR>(on ? m0.z : 0u, on ? m1.z : 0u, [&](const bool (&v)[XR], const uint32_t (&own)[XR],
                                                          const uint32_t (&j)[XR]) {
        uint32_t Xo[XR], pid[XR], lo[XR], hi[XR];
        bool known[XR], ask[XR], found[XR];
        unsigned long long key[XR];
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          Xo[k] = __shfl(X, (int)own[k]);
          lo[k] = __shfl(xb, (int)own[k]);
          hi[k] = __shfl(xe, (int)own[k]);
        }
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          pid[k] = v[k] ? ix.exr_pid[j[k]] : 0u;
          known[k] = false;
          if (v[k]) ev.v[EL_EV_ENT]++;
          if (v[k] && ix.base)
            ev.v[EL_EV_ROW]++;  // (base_has: the row lookup)
          else
            lo[k] = hi[k];
        }
        bsearch_x<XR>(ix.exr_pid, lo, hi, pid, known, ev);
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          ask[k] = v[k] && !known[k] && !lempty;
          if (ask[k]) ev.v[EL_EV_HASH]++;
          key[k] = link_key(pid[k], Xo[k]);
        }
        hash_contains_x<XR>(st.lhash, st.lmask, key, ask, found);
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) emit_l(st, q, v[k] && !known[k] && !found[k], Xo[k], pid[k], ev);
      });
    }
    {  // A ∈ S(Y=X) new, ∃r.A ⊑ B  =>  propagation ((r, Y), B)
       // (Type3_1AxiomProcessorBase.java:208-234 writes "Yr" -> B)
      // (an init fact's own propagations are the base propagations, already in place)
      bool on = star && (mask & M_R4Y) && !(ix.base && f == 2);
      if (on) ev.v[EL_EV_ROW]++;
      // Y's pair range (the roles r with (r, Y) a link target), read once per trigger; when Y
      // is no link target at all, no entry can find a pair: the row is not walked, and its
      // events — two entries and one pair-row lookup per entry, as the walk counts them — are
      // added at once
      uint32_t fpb = 0, fpe = 0;
      if (on && m1.w > m0.w) {
        fpb = ix.fp_ptr[X];
        fpe = ix.fp_ptr[X + 1];
        if (fpb == fpe) {
          ev.v[EL_EV_ENT] += 2 * (m1.w - m0.w);
          ev.v[EL_EV_ROW] += m1.w - m0.w;
          on = false;
        }
      }
      // Y's first PR_REG pair roles in registers, loaded once per trigger (round 6): an entry's
      // pair lookup is then a comparison against its owner's roles (shuffled) instead of a loop
      // of dependent pair_role loads per entry; longer ranges keep the loop.  Events as the
      // loop counts them: one pair-row lookup, and the roles read up to the first >= r.
      constexpr uint32_t PR_REG = 4;
      uint32_t prr[PR_REG];
#pragma unroll
      for (uint32_t k = 0; k < PR_REG; ++k) prr[k] = on && fpb + k < fpe ? ix.pair_role[fpb + k] : NONE;
      const bool pempty = mask & M_PEMPTY;
      // XR rounds in lockstep, as CR3 above: entry -> pair -> base-propagation search -> set
      // probe -> predecessor row (fused fan-out)
      wave_rows_x<XR>(on ? m0.w : 0u, on ? m1.w : 0u, [&](const bool (&v)[XR], const uint32_t (&own)[XR],
                                                          const uint32_t (&j)[XR]) {
        uint32_t pid[XR], B[XR], rr[XR], lo[XR], hi[XR], pb[XR], pl[XR];
        bool known[XR], ask[XR], found[XR];
        unsigned long long key[XR];
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          rr[k] = v[k] ? ix.exl_r[j[k]] : 0u;
          B[k] = v[k] ? ix.exl_b[j[k]] : 0u;
          if (v[k]) ev.v[EL_EV_ENT] += 2;
        }
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          const uint32_t pb0 = __shfl(fpb, (int)own[k]), pe0 = __shfl(fpe, (int)own[k]);
          uint32_t ro[PR_REG];
#pragma unroll
          for (uint32_t i = 0; i < PR_REG; ++i) ro[i] = __shfl(prr[i], (int)own[k]);
          pid[k] = NONE;
          if (v[k]) {
            const uint32_t K = pe0 - pb0, r = rr[k];
            if (K <= PR_REG) {
              uint32_t idx = 0;
#pragma unroll
              for (uint32_t i = 0; i < PR_REG; ++i) idx += (i < K && ro[i] < r) ? 1u : 0u;
              ev.v[EL_EV_ROW]++;
              ev.v[EL_EV_ENT] += idx < K ? idx + 1 : K;
              bool hit = false;
#pragma unroll
              for (uint32_t i = 0; i < PR_REG; ++i) hit |= i == idx && i < K && ro[i] == r;
              pid[k] = hit ? pb0 + idx : NONE;
            } else {
              pid[k] = pair_scan(ix, r, pb0, pe0, ev);
            }
          }
        }
        // prop_known: a base propagation (binary search of bpp(pid), B ascending), else the set
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          known[k] = false;
          lo[k] = hi[k] = 0;
          if (pid[k] != NONE && ix.base) {
            ev.v[EL_EV_ROW]++;
            lo[k] = ix.bpp_s[pid[k]];
            hi[k] = ix.bpp_e[pid[k]];
          }
        }
        bsearch_x<XR>(st.plog_b, lo, hi, B, known, ev);
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          ask[k] = pid[k] != NONE && !known[k] && !pempty;
          if (ask[k]) ev.v[EL_EV_HASH]++;
          key[k] = link_key(pid[k], B[k]);
        }
        hash_contains_x<XR>(st.phash, st.pmask, key, ask, found);
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          const bool fresh = pid[k] != NONE && !known[k] && !found[k];
          pb[k] = pl[k] = 0;
          if (fresh && (mask & M_R4D)) {  // fused mode: B reaches today's predecessors now
            ev.v[EL_EV_ROW]++;
            const uint2 row = gap_row(st.pr, pid[k]);
            pb[k] = row.x;
            pl[k] = row.y;
          }
          found[k] = fresh;
        }
#pragma unroll
        for (uint32_t k = 0; k < XR; ++k) {
          emit_p(st, q, found[k], pid[k], B[k], ev);
          emit_job(st, q, pl[k] > 0, (mask & M_LEMPTY) ? JOB_PRED_U : JOB_PRED_S, pb[k], pl[k], 0, B[k], ev);
        }
      });
    }
    if (act && (mask & M_RBOT) && ix.has_bot && A == EL_BOTTOM) {  // ⊥ ∈ S(Y=X) new, (X', Y) ∈ R(*)  =>  ⊥ ∈ S(X')
      ev.v[EL_EV_ROW]++;
      const uint32_t p1 = ix.fp_ptr[X + 1];
      for (uint32_t p = ix.fp_ptr[X]; p < p1; ++p) {
        if (ix.part) {  // partitioned: ⊥ rides the propagation set ((r, Y), ⊥) to every rank
          ev.v[EL_EV_HASH]++;
          const bool fresh = !hash_contains(st.phash, st.pmask, link_key(p, EL_BOTTOM));
          emit_p(st, q, fresh, p, EL_BOTTOM, ev);
          if (!fresh || !(mask & M_R4D)) continue;
          // fused: this rank's own predecessors now (the other ranks' after the import)
        }
        ev.v[EL_EV_ROW]++;
        const uint2 row = gap_row(st.pr, p);
        emit_job(st, q, row.y > 0, (mask & M_LEMPTY) ? JOB_PRED_U : JOB_PRED_S, row.x, row.y, 0, EL_BOTTOM, ev);
      }
    }
    if (act && (mask & M_RRNG) && ix.has_range) {  // Y=A ∈ S(X) new, active range (Y, C)  =>  C ∈ S(X)
      ev.v[EL_EV_ENT]++;
      if (st.has_act[A]) {  // A's activations: its row of the activation index
        ev.v[EL_EV_ROW]++;
        const uint64_t e = st.act_ptr[A + 1];
        for (uint64_t j = st.act_ptr[A]; j < e; ++j) {
          const uint32_t k = st.act_k[j];
          if (k >= a_end) break;
          ev.v[EL_EV_ENT] += 2;
          const uint32_t C = st.alog_c[k];
          ev.v[EL_EV_TEST]++;
          emit_s(st, q, !test_bit(ix, st.bits, X, C), X, C, ev);
        }
      }
    }
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_EXPAND_S, ev);
}


// CR6 with the new link (X, r, Y) in second position: (X', X) ∈ R(p), p ∘ r ⊑ t  =>  (X', Y) ∈ R(t)
// (Type5AxiomProcessorBase.java:115-154, DB4 "Xp" -> Y of RolePairHandler.java:428-443, s checked).
__device__ __forceinline__ void r6_second(const DIndex& ix, const DState& st, BlockQ& q, uint32_t X, uint32_t r,
                                          uint32_t Y, Ev& ev) {
  ev.v[EL_EV_ROW]++;
  const uint32_t h1 = ix.chs_ptr[r + 1];
  for (uint32_t j = ix.chs_ptr[r]; j < h1; ++j) {
    const uint32_t p = ix.chs_p[j], t = ix.chs_t[j];
    ev.v[EL_EV_ENT] += 2;
    const uint32_t pq = pair_lookup(ix, p, X, ev);
    uint32_t pb = 0, pl = 0, pt = NONE;
    if (pq != NONE) {
      ev.v[EL_EV_ROW]++;
      const uint2 row = gap_row(st.pr, pq);
      pb = row.x;
      pl = row.y;
      if (pl) pt = pair_lookup(ix, t, Y, ev);
    }
    emit_job(st, q, pl > 0, JOB_PRED_L, pb, pl, pt, 0, ev);
  }
}

// Rules triggered by new links (X, pid = (r, Y)) = link log[begin, end).
//  CR4½ Type3_2AxiomProcessorBase.java:67-96,182-224   CR5 Type4AxiomProcessorBase.java:38-76
//  CR6  Type5AxiomProcessorBase.java:115-154           ⊥   RolePairHandler.java:358-372
//  domain/range RolePairHandler.java:456-491
__device__ __forceinline__ void expand_l(const DIndex& ix, const DState& st, BlockQ& q, uint32_t bid, uint32_t nb,
                         uint32_t begin, uint32_t end, uint32_t mask, uint32_t tpw) {
  Ev ev;
  const uint32_t w0 = bid * (blockDim.x >> 6) + (threadIdx.x >> 6), nw = nb * (blockDim.x >> 6);
  for (uint32_t base = begin + w0 * tpw; base < end; base += nw * tpw) {  // (wave-uniform)
    const uint32_t i = base + lane_id();
    const bool act = lane_id() < tpw && i < end;
    uint32_t X = 0, pid = 0, r = 0, Y = 0, q0 = 0, q1 = 0;
    if (act) {
      X = st.llog_x[i];
      pid = st.llog_p[i];
      ev.v[EL_EV_TRIG]++;
      const uint4 pi = ix.pinfo[pid];  // (role, filler; the CR5 lift range below)
      r = pi.x;
      Y = pi.y;
      q0 = pi.z;
      q1 = pi.w;
      ev.v[EL_EV_ENT] += 2;
    }
    {  // (X, Y) ∈ R(r) new, propagation ((r, Y), B)  =>  B ∈ S(X)
       // (Type3_2AxiomProcessorBase.java:67-96, part 2: all B × ΔX; rows walked by the wave)
      const bool on = act && (mask & M_R4L);
      uint2 row = make_uint2(0u, 0u);
      if (on) {
        ev.v[EL_EV_ROW]++;
        row = gap_row(st.pp, pid);  // (no propagation CSR without ∃r.A ⊑ B: rows are empty)
      }
      // No probe of B ∈ S(X) here: a new link's conclusions are nearly all new (G3: 103 M of
      // 107 M), so the probe was one random line read per conclusion that the commit's
      // atomicOr repeats anyway; the commit drops the few already present.
      // (four rounds' entries loaded before the first is emitted: wave_rows4)
      wave_rows4(
          row.x, row.x + row.y,
          [&](bool v, uint32_t own, uint32_t j) { return make_uint2(__shfl(X, (int)own), v ? st.pp.val[j] : 0u); },
          [&](bool, uint32_t, uint2) { return 0u; },
          [&](bool v, uint32_t, uint2 xb, uint32_t) {
            if (v) ev.v[EL_EV_ENT]++;
            emit_s(st, q, v, xb.x, xb.y, ev);
          });
    }
    if (act) {
      if ((mask & M_RBOT) && ix.has_bot && !ix.part) {  // ⊥ ∈ S(Y) => ⊥ ∈ S(X)  (partitioned: via propagations)
        ev.v[EL_EV_TEST]++;
        bool nw = false;
        if (test_bit(ix, st.bits, Y, EL_BOTTOM)) {
          ev.v[EL_EV_TEST]++;
          nw = !test_bit(ix, st.bits, X, EL_BOTTOM);
        }
        emit_s(st, q, nw, X, EL_BOTTOM, ev);
      }
      if (mask & M_R5) {  // r ⊑ s  =>  (X, Y) ∈ R(s)
        ev.v[EL_EV_ROW]++;
        for (uint32_t j = q0; j < q1; ++j) {
          const uint32_t sp = ix.psup_pid[j];
          ev.v[EL_EV_ENT]++;
          emit_l(st, q, !link_known(ix, st, X, sp, mask & M_LEMPTY, ev), X, sp, ev);
        }
      }
      if (mask & M_R6) {  // r ∘ s ⊑ t
        ev.v[EL_EV_ROW]++;
        const bool first = ix.chf_ptr[r + 1] > ix.chf_ptr[r];
        uint32_t sb = 0, sl = 0;
        if (first) {  // r first: (Y, Z) ∈ R(s)  =>  (X, Z) ∈ R(t)
          ev.v[EL_EV_ROW]++;
          const uint2 row = gap_row(st.sc, Y);
          sb = row.x;
          sl = row.y;
        }
        emit_job(st, q, first && sl > 0, JOB_R6A, sb, sl, X, r, ev);
        if (!ix.part) r6_second(ix, st, q, X, r, Y, ev);  // partitioned: over the exchanged chain links
      }
      if (mask & M_RDOM) {  // domain(r) = D  =>  D ∈ S(X)   (X ≠ ⊤, not a datatype)
        ev.v[EL_EV_ROW]++;
        const uint32_t d0 = ix.dom_ptr[r], d1 = ix.dom_ptr[r + 1];
        bool ok = false;
        if (d1 > d0) {
          ev.v[EL_EV_ENT]++;
          ok = X != EL_TOP && ix.kind[X] != EL_KIND_DATATYPE;
        }
        for (uint32_t j = d0; j < d1; ++j) {
          const uint32_t D = ix.dom_c[j];
          ev.v[EL_EV_ENT]++;
          bool nw = false;
          if (ok) {
            ev.v[EL_EV_TEST]++;
            nw = !test_bit(ix, st.bits, X, D);
          }
          emit_s(st, q, nw, X, D, ev);
        }
      }
      if (mask & M_RRNG) {  // range(r) = C  =>  activate Y ⊑ C  (Y ≠ ⊤, not a datatype; H1)
        ev.v[EL_EV_ROW]++;
        const uint32_t g0 = ix.rng_ptr[r], g1 = ix.rng_ptr[r + 1];
        bool ok = false;
        if (g1 > g0) {
          ev.v[EL_EV_ENT]++;
          ok = Y != EL_TOP && ix.kind[Y] != EL_KIND_DATATYPE;
        }
        for (uint32_t j = g0; j < g1; ++j) {
          const uint32_t C = ix.rng_c[j];
          ev.v[EL_EV_ENT]++;
          bool nw = false;
          if (ok) {
            ev.v[EL_EV_HASH]++;
            nw = !hash_contains(st.ahash, st.amask, link_key(C, Y));
          }
          emit_a(st, nw, Y, C, ev);
        }
      }
    }
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_EXPAND_L, ev);
}

// Wide fan-outs: one wave per job record, lanes stride over the list.
//  JOB_PRED_S  preds(pid) × {B}         (CR4 half-1, ⊥)
//  JOB_PRED_L  preds(pq)  × {pid_t}     (CR6, r second)
//  JOB_R6A     succ(Y)    × chains of r (CR6, r first)
__global__ void k_jobs(DIndex ix, DState st, uint32_t mask) {
  const bool lempty = mask & M_LEMPTY;
  __shared__ BlockQ q;
  q_init(q);
  Ev ev;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t nwaves = gridDim.x * wpb;
  const uint32_t njobs = min(st.ctr->jobs, st.job_cap);
  // 64 job records per wave, one per lane, their lists walked wave-cooperatively: most
  // records are short (a fresh propagation meets a few predecessors), and one wave per
  // record left most lanes idle (G5 step 1: 1.6 M records, 0.85 ms)
  // (a step with few jobs spreads them over every wave, as wave_triggers does for triggers)
  const uint32_t tpw = min(64u, max(1u, (njobs + nwaves - 1) / nwaves));
  for (uint32_t base = (blockIdx.x * wpb + (threadIdx.x >> 6)) * tpw; base < njobs; base += nwaves * tpw) {
    const uint32_t j = base + lane;
    uint4 jb = make_uint4(0u, 0u, 0u, 0u);
    uint32_t len = 0;
    if (lane < tpw && j < njobs) {
      jb = st.jobs[j];
      len = jb.y & 0x0fffffffu;
      ev.v[EL_EV_JOB]++;
    }
    const uint32_t type = jb.y >> 28;
    // the column of a JOB_PRED_S's B, once per job (every entry tests the same column)
    const uint32_t jcol = (lane < tpw && j < njobs && type == JOB_PRED_S) ? col_of(ix, jb.w) : NONE;
    // (four rounds of entries at a time: the list entry, then the bit word a JOB_PRED_S tests)
    wave_rows4(
        jb.x, jb.x + len,
        [&](bool v, uint32_t own, uint32_t k) {
          const uint32_t t = __shfl(type, (int)own);
          return v ? ((t == JOB_R6A) ? st.sc.val[k] : st.pr.val[k]) : 0u;
        },
        [&](bool v, uint32_t own, uint32_t val) {
          const uint32_t c = __shfl(jcol, (int)own);
          return (v && c != NONE) ? st.bits[(uint64_t)val * ix.W + (c >> 5)] : 0u;
        },
        [&](bool v, uint32_t own, uint32_t val, uint32_t word) {
      const uint32_t t = __shfl(type, (int)own), a = __shfl(jb.z, (int)own), b = __shfl(jb.w, (int)own);
      const uint32_t jc = __shfl(jcol, (int)own);
      const uint4 e = make_uint4(val, t, a, b);
      if (t == JOB_PRED_S || t == JOB_PRED_U) {  // preds(pid) × {B}
        uint32_t xp = 0;
        bool nw = false;
        if (v) {
          xp = e.x;
          ev.v[EL_EV_ENT]++;
          nw = true;
          if (t == JOB_PRED_S) {
            ev.v[EL_EV_TEST]++;
            nw = !(jc != NONE && ((word >> (jc & 31u)) & 1u));
          }
        }
        emit_s(st, q, nw, xp, b, ev);
      } else if (t == JOB_PRED_L) {  // preds(pq) × {pid_t}
        uint32_t xp = 0;
        bool nw = false;
        if (v) {
          xp = e.x;
          ev.v[EL_EV_ENT]++;
          nw = !link_known(ix, st, xp, a, lempty, ev);
        }
        emit_l(st, q, nw, xp, a, ev);
      } else {  // JOB_R6A: succ(Y) × chains of r
        const uint32_t X = a, r = b;
        uint32_t s2 = NONE, Z = 0, f0 = 0, f1 = 0;
        if (v) {
          const uint32_t sq = e.x;
          ev.v[EL_EV_ENT]++;
          s2 = ix.pair_role[sq];
          Z = ix.pair_y[sq];
          ev.v[EL_EV_ENT] += 2;
          ev.v[EL_EV_ROW]++;
          f0 = ix.chf_ptr[r];
          f1 = ix.chf_ptr[r + 1];
        }
        for (uint32_t f = f0; f < f1; ++f) {
          const uint32_t s = ix.chf_s[f], tt = ix.chf_t[f];
          ev.v[EL_EV_ENT] += 2;
          bool nw = false;
          uint32_t pt = NONE;
          if (s == s2) {
            pt = pair_lookup(ix, tt, Z, ev);
            nw = !link_known(ix, st, X, pt, lempty, ev);
          }
          emit_l(st, q, nw, X, pt, ev);
        }
      }
    });
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_JOBS, ev);
}

// Range activations (Y, C) = act log[a_begin, a_end): every X with Y ∈ S(X) gets C
// (ScriptsCollection.insertClassAssertions1 :45-62 copies result[Y] into result[C]).  The
// X's holding Y are found in the fact log (one coalesced pass over the facts known at t-1,
// each fact (X, Y) meeting the new activations of Y through the activation index), not by
// sweeping column Y of the bit matrix (one random line per row and activation).
__device__ __forceinline__ void expand_a(const DIndex& ix, const DState& st, BlockQ& q, uint32_t bid, uint32_t nb,
                         uint32_t s_end, uint32_t a_begin, uint32_t a_end) {
  Ev ev;
  for (uint32_t base = bid * blockDim.x; base < s_end; base += nb * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    if (i < s_end) {
      const uint32_t x = st.slog_x[i], Y = st.slog_a[i];
      ev.v[EL_EV_TRIG]++;
      ev.v[EL_EV_ENT]++;
      if (st.has_act[Y]) {
        ev.v[EL_EV_ROW]++;
        const uint64_t b = st.act_ptr[Y];
        for (uint64_t j = st.act_ptr[Y + 1]; j > b; --j) {  // the newest activations are last
          const uint32_t k = st.act_k[j - 1];
          if (k < a_begin) break;
          if (k >= a_end) continue;
          ev.v[EL_EV_ENT] += 2;
          const uint32_t C = st.alog_c[k];
          ev.v[EL_EV_TEST]++;
          emit_s(st, q, !test_bit(ix, st.bits, x, C), x, C, ev);
        }
      }
    }
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_EXPAND_A, ev);
}

// S candidates per chunk of the sorted S commit (commit_s_sorted)
#ifndef EL_CC_BITS
#define EL_CC_BITS 11  // (12: 48 KB of LDS per block, G3 21.9 ms; 10: 19.8-20.1 ms; 11: 19.8 — round 6)
#endif
constexpr uint32_t CC_BITS = EL_CC_BITS, CC = 1u << CC_BITS;
static_assert(CC % BLOCK == 0, "chunk per thread");
constexpr uint32_t CSORT_MIN = 1u << 18;  // smaller commits: plain order (the sort's barriers cost more)

// LDS of the commit roles (one role per block): staging of new facts / links, or the S role's
// counting sort of a candidate chunk (bin counts, then the chunk in bin order)
struct CommitLds {
  union {
    struct {
      uint32_t x[QS_CAP > QL_CAP ? QS_CAP : QL_CAP], v[QS_CAP > QL_CAP ? QS_CAP : QL_CAP];
    } q;
    struct {
      uint32_t bin[CC];
      unsigned long long srt[CC];  // x << 32 | a
      uint32_t part[BLOCK / 64];
    } c;
  };
  uint32_t n, base, total;
};

// Diagnostic (EL_TRACE_CANDS): count this wave-instruction's atomics and the distinct 64-B lines
// they address (the memory-side requests of the atomic, commit_s_sorted)
__device__ void count_lines(unsigned long long* out, bool valid, uint32_t x, uint32_t c) {
  const unsigned long long k = valid ? ((unsigned long long)x << 24) | (c >> 9) : ~0ull;
  bool first = valid;
  for (int j = 0; j < 64; ++j) {
    const unsigned long long o = __shfl(k, j);
    if (j < (int)lane_id() && o == k) first = false;
  }
  const unsigned long long v = __ballot(valid), f = __ballot(first);
  if (lane_id() == 0 && v) {
    atomicAdd(out, (unsigned long long)__popcll(v));
    atomicAdd(out + 1, (unsigned long long)__popcll(f));
    atomicAdd(out + 2, 1ull);
  }
}

// Dedup S candidates against the bit rows; new facts go to the log (the versioned
// ZADD of every Lua kernel, e.g. Type1_1AxiomProcessorBase.java:36-41).
// (x, a) = the candidate queue; flag = slog_f of the facts it adds; kev = the work phase
__device__ void commit_s(const DIndex& ix, const DState& st, CommitLds& sm, uint32_t bid, uint32_t nb,
                         uint32_t n, const uint32_t* __restrict__ qx, const uint32_t* __restrict__ qa,
                         uint8_t flag, int kev) {
  uint32_t* lx = sm.q.x;
  uint32_t* la = sm.q.v;
  uint32_t& ln = sm.n;
  uint32_t& lbase = sm.base;
  if (threadIdx.x == 0) ln = 0;
  __syncthreads();
  Ev ev;
  for (uint32_t base = bid * blockDim.x; base < n; base += nb * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    bool nw = false;
    uint32_t x = 0, a = 0;
    if (i < n && qx[i] != NONE) {  // (NONE: a hole of a wave's reservation, wq_publish_s)
      x = qx[i];
      a = qa[i];
      ev.v[EL_EV_TRIG]++;
      ev.v[EL_EV_RMW]++;
      const uint32_t c = col_of(ix, a);  // (every candidate of an owned row lies inside the window)
      const uint32_t m = 1u << (c & 31u);
      const uint32_t old = c != NONE ? atomicOr(st.bits + (uint64_t)x * ix.W + (c >> 5), m) : m;
      nw = (old & m) == 0;
      if (nw && st.summ) st.summ[(uint64_t)x * st.SB + (c >> elrows::SUMM_SHIFT)] = 1;  // (idempotent: plain store)
      if (nw) ev.v[EL_EV_EMIT]++;
    }
    if (st.lines) count_lines(st.lines, i < n && qx[i] != NONE, x, col_of(ix, a));
    // one LDS slot per new fact; blockDim <= QS_CAP/2 so a round never overflows
    const uint32_t off = lds_reserve(&ln, nw);
    if (nw) {
      lx[off] = x;
      la[off] = a;
    }
    __syncthreads();
    if (ln > QS_CAP / 2 || base + nb * blockDim.x >= n) {
      const uint32_t cnt = ln;
      if (threadIdx.x == 0) lbase = cnt ? atomicAdd(&st.ctr->s_log, cnt) : 0u;
      __syncthreads();
      for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) {
        st.slog_x[lbase + k] = lx[k];
        st.slog_a[lbase + k] = la[k];
        st.slog_f[lbase + k] = flag;
      }
      __syncthreads();
      if (threadIdx.x == 0) ln = 0;
      __syncthreads();
    }
  }
  ev_flush(st.ev, kev, ev);
}

// Block-wide exclusive scan of one value per thread (thread order); *total = the sum.
// Uses sm.c.part; every thread must call it.
__device__ __forceinline__ uint32_t block_excl(CommitLds& sm, uint32_t v, uint32_t* total) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) sm.c.part[wv] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < BLOCK / 64; ++w) {
    const uint32_t u = sm.c.part[w];
    base += w < wv ? u : 0u;
    tot += u;
  }
  __syncthreads();  // (part is reused by the next call)
  *total = tot;
  return base + inc - v;
}

// The S commit in sorted chunks.  A commit is bound by the bit-word atomics, which run at the
// memory side, one 64-B request per distinct line of a wave-instruction: 64 lanes in 64 random
// lines made 20 G atomics/s, the same 64 lanes in 16 / 4 lines 54 / 80 G/s (MI355X,
// scripts/micro/commit_rate.hip, profiles/r04_commit_rate_micro.txt).  The candidates of one
// row arrive together in the queue (a wave's triggers are consecutive log entries, mostly of one
// X) and a row's subsumers cluster in its columns (G3 at scale 0.25: 8.6 facts per 128-B line at
// the fixpoint), so a block counting-sorts each chunk of CC candidates in LDS before its atomics:
// bin = (x-run of the chunk, hash of the column's 64-B line) — the chunk's runs of one x keep their
// order (the log stays in x-runs: the streamed result's run encoding depends on it) and inside a
// run the candidates of one line become adjacent, so the lanes of a wave-instruction meet few
// lines.  New facts reach the log in sorted order (a block scan, no LDS atomics).  Same facts and
// events as commit_s: a step's delta is a set.
__device__ void commit_s_sorted(const DIndex& ix, const DState& st, CommitLds& sm, uint32_t bid, uint32_t nb,
                                uint32_t n, const uint32_t* __restrict__ qx, const uint32_t* __restrict__ qa,
                                uint8_t flag, int kev) {
  constexpr uint32_t PER = CC / BLOCK;
  Ev ev;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  for (uint32_t c0 = bid * CC; c0 < n; c0 += nb * CC) {  // (block-uniform)
    for (uint32_t k = tid; k < CC; k += BLOCK) sm.c.bin[k] = 0;
    // 1. this thread's PER consecutive candidates, the x-runs that start among them
    uint32_t hx[PER], ha[PER], hb[PER], hr[PER];
    const uint32_t e0 = c0 + tid * PER;
    uint32_t prev = (e0 > c0 && e0 - 1 < n) ? qx[e0 - 1] : NONE;
    uint32_t heads = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t i = e0 + k;
      hx[k] = i < n ? qx[i] : NONE;  // (NONE: a hole of a wave's reservation, wq_publish_s)
      ha[k] = hx[k] != NONE ? qa[i] : 0u;
      hr[k] = hx[k] != NONE && (i == c0 || hx[k] != prev);  // (a run head)
      heads += hr[k];
      if (hx[k] != NONE) prev = hx[k];
    }
    uint32_t nruns;
    uint32_t run = block_excl(sm, heads, &nruns);  // heads before this thread's first candidate
    // 2. bins: run-major, then the line hash; sbits = the line-hash bits a run gets
    uint32_t lg = 0;
    while ((1u << lg) < nruns) ++lg;
    const uint32_t sbits = lg < CC_BITS ? CC_BITS - lg : 0u;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      run += hr[k];
      hb[k] = NONE;
      if (hx[k] != NONE) {
        const uint32_t c = col_of(ix, ha[k]);
        // (the line's hash, then the word inside the 64-B line: one word's candidates adjacent)
        const uint32_t h = sbits > 4u ? (((hx[k] * 769u + (c >> 9)) * 2654435761u) >> (36 - sbits)) << 4 | ((c >> 5) & 15u)
                           : sbits ? ((hx[k] * 769u + (c >> 9)) * 2654435761u) >> (32 - sbits) : 0u;
        hb[k] = ((run - 1) << sbits) | h;
        hr[k] = atomicAdd(&sm.c.bin[hb[k]], 1u);
      }
    }
    __syncthreads();
    // 3. exclusive scan of the bin counts (PER consecutive bins per thread), then the chunk in bin order
    uint32_t loc[PER], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      loc[k] = sum;
      sum += sm.c.bin[tid * PER + k];
    }
    uint32_t total;
    const uint32_t excl = block_excl(sm, sum, &total);
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) sm.c.bin[tid * PER + k] = excl + loc[k];
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k)
      if (hb[k] != NONE) sm.c.srt[sm.c.bin[hb[k]] + hr[k]] = ((unsigned long long)hx[k] << 32) | ha[k];
    __syncthreads();
    // 4. the atomics, 64 consecutive sorted candidates per wave-instruction.  The lanes holding
    // the same (row, word) — adjacent in the sorted chunk — OR their bits together first (a
    // segmented scan over the wave) and the segment's last lane issues one atomic for them: with
    // the column order (DIndex::cperm) a row's frequent subsumers share a few words, whose
    // atomics would otherwise serialise on one address.  A lane's bit is new if neither the word
    // nor an earlier lane of its segment had it.
    bool nw[PER];
    unsigned long long key[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t i = k * BLOCK + tid;
      const bool v = i < total;
      uint32_t x = 0, c = NONE;
      key[k] = 0;
      if (v) {
        key[k] = sm.c.srt[i];
        x = (uint32_t)(key[k] >> 32);
        c = col_of(ix, (uint32_t)key[k]);  // (every candidate of an owned row lies inside the window)
        ev.v[EL_EV_TRIG]++;
        ev.v[EL_EV_RMW]++;
      }
      const bool on = v && c != NONE;
      const uint32_t m = on ? 1u << (c & 31u) : 0u;
      // word id (row, word); lanes without one never match a neighbour
      const uint32_t wx = on ? x : NONE, ww = on ? c >> 5 : NONE - lane;
      const uint32_t px = __shfl_up(wx, 1), pw = __shfl_up(ww, 1);
      const uint32_t head = lane == 0 || px != wx || pw != ww;
      uint32_t incl = m, f = head;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d), of = __shfl_up(f, d);
        if (lane >= d) {
          if (!f) incl |= o;
          f |= of;
        }
      }
      const uint32_t before = __shfl_up(incl, 1);
      const uint32_t excl = head ? 0u : before;
      const uint32_t next = __shfl_down(head, 1);  // (every lane takes part: not under a short-circuit)
      const uint32_t tail = lane == 63u || next;
      uint32_t old = 0;
      if (tail && incl) old = atomicOr(st.bits + (uint64_t)wx * ix.W + ww, incl);
      const unsigned long long tails = __ballot(tail != 0);
      const uint32_t last = lane + (uint32_t)__ffsll((long long)(tails >> lane)) - 1u;
      const uint32_t seen = __shfl(old, (int)last) | excl;
      nw[k] = on && (seen & m) == 0;
      if (nw[k] && st.summ) st.summ[(uint64_t)x * st.SB + (c >> elrows::SUMM_SHIFT)] = 1;  // (idempotent: plain store)
      if (nw[k]) ev.v[EL_EV_EMIT]++;
      if (st.lines) count_lines(st.lines, v, x, c);
    }
    // 5. the new facts, in sorted order: per round k, the waves' counts in LDS (one barrier)
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const unsigned long long m = __ballot(nw[k]);
      if (lane == 0) sm.c.bin[k * (BLOCK / 64) + wv] = (uint32_t)__popcll(m);  // (bins are free again)
      hr[k] = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    __syncthreads();  // (also: every sorted entry has been read)
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < PER * (BLOCK / 64); ++j) {
      const uint32_t v = sm.c.bin[j];
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k)
        if (j < k * (BLOCK / 64) + wv) hr[k] += v;
      cnt += v;
    }
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k)
      if (nw[k]) sm.c.srt[hr[k]] = key[k];
    if (tid == 0) sm.base = cnt ? atomicAdd(&st.ctr->s_log, cnt) : 0u;
    __syncthreads();
    const uint32_t lbase = sm.base;
    for (uint32_t k = tid; k < cnt; k += BLOCK) {
      const unsigned long long v = sm.c.srt[k];
      st.slog_x[lbase + k] = (uint32_t)(v >> 32);
      st.slog_a[lbase + k] = (uint32_t)v;
      st.slog_f[lbase + k] = flag;
    }
    __syncthreads();  // (the next chunk reuses the bins and the sorted entries)
  }
  ev_flush(st.ev, kev, ev);
}

// Dedup link candidates against the link set (checkAndInsertScript,
// RolePairHandler.java:133-168); new links feed the predecessor/successor CSRs.
__device__ void commit_l(const DIndex& ix, const DState& st, CommitLds& sm, uint32_t bid, uint32_t nb,
                         uint32_t n) {
  uint32_t* lx = sm.q.x;
  uint32_t* lp = sm.q.v;
  uint32_t& ln = sm.n;
  uint32_t& lbase = sm.base;
  if (threadIdx.x == 0) ln = 0;
  __syncthreads();
  Ev ev;
  for (uint32_t base = bid * blockDim.x; base < n; base += nb * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    bool nw = false;
    uint32_t x = 0, p = 0;
    if (i < n) {
      x = st.cl_x[i];
      p = st.cl_p[i];
      ev.v[EL_EV_TRIG]++;
      ev.v[EL_EV_HASH]++;
      nw = hash_insert(st.lhash, st.lmask, link_key(p, x));
      if (nw) ev.v[EL_EV_EMIT]++;
    }
    // the new link joins its predecessor / successor rows in place
    if (st.need_pred) gap_append(st.pr, p, x, nw, ev.v);
    // successor rows are read only by CR6 with the row's role second: other links stay out
    if (st.succ_at_commit) gap_append(st.sc, x, p, nw && ix.role_chs[ix.pair_role[p]], ev.v);
    if (ix.part) {
      // partitioned: a new link (x, s, z) of a chain-second role joins this rank's replicated
      // chain-link log and successor rows now (CR6 with s second, expand_x), and goes to the ranks
      // whose rows can reach x (a link (x', r, x) of theirs) in the exchange
      const bool ch = nw && ix.role_chs[ix.pair_role[p]];
      const uint32_t xsl = wave_append(&st.ctr->x_log, ch);
      if (st.need_succ) gap_append(st.sc, x, p, ch, ev.v);
      if (ch) {
        st.xlog_x[xsl] = x;
        st.xlog_p[xsl] = p;
      }
      const bool xs = ch && remote(ix, x);
      const uint32_t slot = wave_append(&st.ctr->x_send, xs);
      if (xs && slot < st.xs_cap) {
        st.xs_x[slot] = x;
        st.xs_p[slot] = p;
      }
    }
    const uint32_t off = lds_reserve(&ln, nw);
    if (nw) {
      lx[off] = x;
      lp[off] = p;
    }
    __syncthreads();
    if (ln > QL_CAP / 2 || base + nb * blockDim.x >= n) {
      const uint32_t cnt = ln;
      if (threadIdx.x == 0) lbase = cnt ? atomicAdd(&st.ctr->l_log, cnt) : 0u;
      __syncthreads();
      for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) {
        st.llog_x[lbase + k] = lx[k];
        st.llog_p[lbase + k] = lp[k];
      }
      __syncthreads();
      if (threadIdx.x == 0) ln = 0;
      __syncthreads();
    }
  }
  ev_flush(st.ev, EL_K_COMMIT_L, ev);
}

__device__ void commit_a(const DIndex& ix, const DState& st, uint32_t bid, uint32_t nb, uint32_t n) {
  Ev ev;
  const uint32_t stride = nb * blockDim.x;
  for (uint32_t i = bid * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t y = st.ca_y[i], c = st.ca_c[i];
    ev.v[EL_EV_TRIG]++;
    ev.v[EL_EV_HASH]++;
    const bool nw = hash_insert(st.ahash, st.amask, link_key(c, y));
    const uint32_t slot = wave_append(&st.ctr->a_log, nw);
    if (nw) {
      ev.v[EL_EV_EMIT]++;
      st.alog_y[slot] = y;
      st.alog_c[slot] = c;
      st.has_act[y] = 1;
    }
    if (ix.part) {  // to the ranks whose rows can hold y
      const bool xs = nw && remote(ix, y);
      const uint32_t q = wave_append(&st.ctr->x_sa, xs);
      if (xs && q < st.xa_cap) {
        st.xa_y[q] = y;
        st.xa_c[q] = c;
      }
    }
  }
  ev_flush(st.ev, EL_K_COMMIT_A, ev);
}

// New CR4 propagations ((r, Y), B) = prop log[begin, end) × existing predecessors of (r, Y)
// (per-rule stepping: Type3_2AxiomProcessor part 1, ΔB × all X).  In fused saturation the
// fan-out happens when the propagation is generated (M_R4D), so this kernel is idle there.
__device__ __forceinline__ void expand_p(const DIndex& ix, const DState& st, BlockQ& q, uint32_t bid, uint32_t nb,
                         uint32_t begin, uint32_t end) {
  Ev ev;
  for (uint32_t base = begin + bid * blockDim.x; base < end; base += nb * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    if (i < end) {
      const uint32_t pid = st.plog_p[i], B = st.plog_b[i];
      ev.v[EL_EV_TRIG]++;
      ev.v[EL_EV_ROW]++;
      const uint2 row = gap_row(st.pr, pid);
      const uint32_t pb = row.x, pl = row.y;
      emit_job(st, q, pl > 0, JOB_PRED_S, pb, pl, 0, B, ev);
    }
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_EXPAND_P, ev);
}

// Dedup propagation candidates (checkAndInsertScript, Type3_1AxiomProcessorBase.java:88-121)
__device__ void commit_p(const DIndex& ix, const DState& st, uint32_t bid, uint32_t nb, uint32_t n) {
  Ev ev;
  const uint32_t stride = nb * blockDim.x;
  for (uint32_t i = bid * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t pid = st.cp_p[i], b = st.cp_b[i];
    ev.v[EL_EV_TRIG]++;
    ev.v[EL_EV_HASH]++;
    const bool nw = hash_insert(st.phash, st.pmask, link_key(pid, b));
    const uint32_t slot = wave_append(&st.ctr->p_log, nw);
    gap_append(st.pp, pid, b, nw, ev.v);
    if (nw) {
      ev.v[EL_EV_EMIT]++;
      st.plog_p[slot] = pid;
      st.plog_b[slot] = b;
    }
    if (ix.part) {  // ((r, Y), B) to the ranks whose rows can link to Y
      const bool xs = nw && remote(ix, ix.pair_y[pid]);
      const uint32_t q = wave_append(&st.ctr->x_sp, xs);
      if (xs && q < st.xp_cap) {
        st.xp_p[q] = pid;
        st.xp_b[q] = b;
      }
    }
  }
  ev_flush(st.ev, EL_K_COMMIT_P, ev);
}

// Generation of one superstep in ONE launch: blocks [0, gs) take ΔS triggers, then gl
// blocks Δlinks, ga blocks range activations, gp blocks leftover propagations.  The roles
// read only state t-1 and append to disjoint candidate queues, so they run side by side.
struct ExpandArgs {
  uint32_t gs, gl, ga, gp, gx;
  uint32_t ts, tl;  // triggers per wave of the S and link roles (wave_triggers)
  uint32_t sb, se, lb, le, ab, ae, pb, pe, xb, xe;
  uint32_t mask, a_end;
};

// Partitioned mode: new chain-second links of every rank = xlog[begin, end) meet this
// rank's predecessors (CR6, r second; oracle/partition_model.py Rank.step).
__device__ __forceinline__ void expand_x(const DIndex& ix, const DState& st, BlockQ& q, uint32_t bid, uint32_t nb,
                         uint32_t begin, uint32_t end) {
  Ev ev;
  for (uint32_t base = begin + bid * blockDim.x; base < end; base += nb * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    if (i < end) {
      const uint32_t X = st.xlog_x[i], pid = st.xlog_p[i];
      ev.v[EL_EV_TRIG]++;
      r6_second(ix, st, q, X, ix.pair_role[pid], ix.pair_y[pid], ev);
    }
    q_maybe_flush(q, st);
  }
  q_flush(q, st);
  ev_flush(st.ev, EL_K_EXPAND_L, ev);
}
#ifdef EL_EXPAND_WAVES  // (A/B builds: a VGPR budget for more waves per SIMD)
__global__ void __attribute__((amdgpu_waves_per_eu(EL_EXPAND_WAVES, 8))) k_expand(DIndex ix, DState st, ExpandArgs a) {
#else
__global__ void k_expand(DIndex ix, DState st, ExpandArgs a) {
#endif
  __shared__ BlockQ q;
  q_init(q);
  uint32_t b = blockIdx.x;
  if (b < a.gs) {
    expand_s(ix, st, q, b, a.gs, a.sb, a.se, a.mask, a.a_end, a.ts);
    return;
  }
  b -= a.gs;
  if (b < a.gl) {
    expand_l(ix, st, q, b, a.gl, a.lb, a.le, a.mask, a.tl);
    return;
  }
  b -= a.gl;
  if (b < a.ga) {
    expand_a(ix, st, q, b, a.ga, a.se, a.ab, a.ae);
    return;
  }
  b -= a.ga;
  if (b < a.gp) {
    expand_p(ix, st, q, b, a.gp, a.pb, a.pe);
    return;
  }
  expand_x(ix, st, q, b - a.gp, a.gx, a.xb, a.xe);
}

constexpr uint32_t DONE_SHARDS = 16;
struct PubArgs {
  HCounters* host;  // device view of the pinned host copy
  uint32_t* done;   // [(DONE_SHARDS + 1) * CTR_STRIDE], zero between launches
  uint32_t seq;     // written last to host->seq: the host spins on it
};

// Completion protocol shared by k_commit and k_ximport: the last block of the launch runs
// last_fn (block-wide), copies every counter but seq to the pinned host mirror (unless
// last_fn did), then writes seq.  Every thread of every block must call it.
template <class LastFn>
__device__ __forceinline__ void publish_last(const DState& st, const PubArgs& a, bool copy, LastFn last_fn) {
  __shared__ uint32_t last;
  // The barrier waits for this block's memory operations; every counter update is a
  // returning device-scope atomic, so it has been performed before the block reports done.
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t sh = blockIdx.x % DONE_SHARDS;
    const uint32_t in_shard = (gridDim.x - 1 - sh) / DONE_SHARDS + 1;
    const uint32_t shards = min(gridDim.x, DONE_SHARDS);
    last = 0;
    if (__hip_atomic_fetch_add(a.done + sh * CTR_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        in_shard - 1)
      last = __hip_atomic_fetch_add(a.done + DONE_SHARDS * CTR_STRIDE, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == shards - 1;
  }
  __syncthreads();
  if (!last) return;
  last_fn();
  __syncthreads();
  constexpr uint32_t NW = NUM_CTRS - 1;  // every counter but seq
  if (copy && threadIdx.x < NW) {
    uint32_t* dc = reinterpret_cast<uint32_t*>(st.ctr) + threadIdx.x * CTR_STRIDE;
    reinterpret_cast<volatile uint32_t*>(a.host)[threadIdx.x] =
        __hip_atomic_load(dc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x <= DONE_SHARDS) a.done[threadIdx.x * CTR_STRIDE] = 0;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    reinterpret_cast<volatile uint32_t*>(a.host)[NW] = a.seq;  // counters are visible first
    __threadfence_system();
  }
}

// The CR1 told-closure candidates of a superstep, committed before every other candidate
// (a fact that is also a closure candidate is therefore marked closed, whatever else
// derived it — the same order as the CPU oracle, so per-step deltas and events agree).
// A generation that overflowed a candidate or job queue lost candidates: its commit is
// skipped whole (state t-1 stays untouched) and the host re-runs the step with larger
// queues, so every step's delta is exactly {candidates} \ S_{t-1} even then.
__device__ __forceinline__ bool gen_overflowed(const DState& st) {
  const DCounters* c = st.ctr;
  return c->cand_s > st.cs_cap || c->cand_t > st.ct_cap || c->cand_l > st.cl_cap || c->cand_a > st.ca_cap ||
         c->cand_p > st.cp_cap || c->jobs > st.job_cap;
}

__global__ void k_commit_told(DIndex ix, DState st, uint32_t cap) {
  __shared__ CommitLds sm;
  if (gen_overflowed(st)) return;
  const uint32_t n = min(st.ctr->cand_t, cap);
  if (st.csort && n >= CSORT_MIN)
    commit_s_sorted(ix, st, sm, blockIdx.x, gridDim.x, n, st.ct_x, st.ct_a, 1, EL_K_COMMIT_T);
  else
    commit_s(ix, st, sm, blockIdx.x, gridDim.x, n, st.ct_x, st.ct_a, 1, EL_K_COMMIT_T);
}

// Block-wide: copy every counter but seq to the host mirror, then zero those in zero_mask
// (bit i = counter i).  Each thread owns one counter, so each is read before it is zeroed.
__device__ __forceinline__ void copy_and_zero(const DState& st, HCounters* host, uint32_t zero_mask) {
  constexpr uint32_t NW = NUM_CTRS - 1;
  static_assert(NW <= 32, "zero mask width");
  if (threadIdx.x < NW) {
    uint32_t* dc = reinterpret_cast<uint32_t*>(st.ctr) + threadIdx.x * CTR_STRIDE;
    reinterpret_cast<volatile uint32_t*>(host)[threadIdx.x] =
        __hip_atomic_load(dc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((zero_mask >> threadIdx.x) & 1u) __hip_atomic_store(dc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Commit of one superstep in ONE launch (roles as in k_expand: S, links, activations,
// propagations; each dedups into its own set).  The last block to finish publishes the
// step's counters to pinned host memory and zeroes the per-step counters for the next
// step, so the host learns everything with the step's single sync.
// Blocks that finished are counted in 16 sharded words, then per shard in one word: a
// single same-address counter hit by every block of a 2k-block launch would serialise.
struct CommitArgs {
  uint32_t gs, gl, ga, gp;
  uint32_t cs_cap, cl_cap, ca_cap, cp_cap;
  PubArgs pub;
  uint32_t publish; // 0: a partial launch (diagnostic split): no completion protocol
};
__global__ void k_commit(DIndex ix, DState st, CommitArgs a) {
  __shared__ CommitLds sm;
  uint32_t b = blockIdx.x;
  if (gen_overflowed(st)) {
    // nothing committed (see gen_overflowed); the counters still reach the host
  } else if (b < a.gs) {
    const uint32_t n = min(st.ctr->cand_s, a.cs_cap);
    if (st.csort && n >= CSORT_MIN)
      commit_s_sorted(ix, st, sm, b, a.gs, n, st.cs_x, st.cs_a, 0, EL_K_COMMIT_S);
    else
      commit_s(ix, st, sm, b, a.gs, n, st.cs_x, st.cs_a, 0, EL_K_COMMIT_S);
  } else if ((b -= a.gs) < a.gl) {
    commit_l(ix, st, sm, b, a.gl, min(st.ctr->cand_l, a.cl_cap));
  } else if ((b -= a.gl) < a.ga) {
    commit_a(ix, st, b, a.ga, min(st.ctr->cand_a, a.ca_cap));
  } else {
    commit_p(ix, st, b - a.ga, a.gp, min(st.ctr->cand_p, a.cp_cap));
  }
  if (!a.publish) return;
  publish_last(st, a.pub, false, [&] { copy_and_zero(st, a.pub.host, ~0u << CTR_KEEP); });
}

// ---- partitioned exchange (protocol: oracle/partition_model.py)
// Each rank's slot of the all-gather: XH header words, then up to cap records (a, b):
// its new propagations (pid, B), then new activations (Y, C), then new chain-second
// links (X, pid) — only those some other rank's rows can reach (remote(), routed by the commit).
// Records past cap wait for a larger exchange (the host redoes it).
constexpr uint32_t XH = 16;
// header words: records sent (NP, NA, NX); this step's local deltas — facts, links, propagations,
// activations, chain links (DS, DL, DP, DA, DX: their sum over ranks, with the records sent, is
// the termination test); a candidate queue overflowed (OVF: redo); a send queue overflowed (QOVF)
enum : uint32_t { XH_NP = 0, XH_NA = 1, XH_NX = 2, XH_DS = 3, XH_DL = 4, XH_OVF = 5, XH_QOVF = 6, XH_DP = 7, XH_DA = 8,
                  XH_DX = 9 };
struct XchgArgs {
  uint32_t* send;        // this rank's slot: XH + 2 * cap words
  const uint32_t* recv;  // nranks slots
  uint32_t cap, nranks, me;
  uint32_t s0, l0, a0, p0, x0;  // log counts at the start of the attempt
  uint32_t cs_cap, cl_cap, ca_cap, cp_cap, job_cap, ct_cap;  // a candidate queue past its cap = redo
};
// per-step counters the import zeroes once the exchange went through: x_send, x_sp, x_sa,
// cand_*, jobs
constexpr uint32_t XCHG_ZERO = (1u << 5) | (1u << 6) | (1u << 7) | (1u << 11) | (1u << 12) | (1u << 13) | (1u << 14) |
                               (1u << 15) | (1u << 16);
static_assert(offsetof(DCounters, x_send) == 5 * CTR_STRIDE * 4 && offsetof(DCounters, x_sa) == 7 * CTR_STRIDE * 4 &&
                  offsetof(DCounters, cand_s) == 11 * CTR_STRIDE * 4 && offsetof(DCounters, cand_t) == 16 * CTR_STRIDE * 4,
              "XCHG_ZERO bits");

__global__ void k_xpack(DState st, XchgArgs x) {
  const uint32_t np = st.ctr->x_sp, na = st.ctr->x_sa, nx = st.ctr->x_send;
  const uint32_t tot = np + na + nx, n = min(tot, x.cap);
  if (blockIdx.x == 0 && threadIdx.x < XH) {
    uint32_t v = 0;
    if (threadIdx.x == XH_NP) v = np;
    if (threadIdx.x == XH_NA) v = na;
    if (threadIdx.x == XH_NX) v = nx;
    if (threadIdx.x == XH_DS) v = st.ctr->s_log - x.s0;
    if (threadIdx.x == XH_DL) v = st.ctr->l_log - x.l0;
    if (threadIdx.x == XH_DP) v = st.ctr->p_log - x.p0;
    if (threadIdx.x == XH_DA) v = st.ctr->a_log - x.a0;
    if (threadIdx.x == XH_DX) v = st.ctr->x_log - x.x0;
    if (threadIdx.x == XH_OVF)
      v = st.ctr->cand_s > x.cs_cap || st.ctr->cand_l > x.cl_cap || st.ctr->cand_a > x.ca_cap ||
          st.ctr->cand_p > x.cp_cap || st.ctr->jobs > x.job_cap || st.ctr->cand_t > x.ct_cap;
    if (threadIdx.x == XH_QOVF)  // a send queue lost records (sized to never do so): fatal
      v = np > st.xp_cap || na > st.xa_cap || nx > st.xs_cap;
    x.send[threadIdx.x] = v;
  }
  uint2* rec = reinterpret_cast<uint2*>(x.send + XH);
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < n; g += gridDim.x * blockDim.x) {
    uint2 r;
    if (g < np) r = make_uint2(st.xp_p[g], st.xp_b[g]);
    else if (g < np + na) r = make_uint2(st.xa_y[g - np], st.xa_c[g - np]);
    else r = make_uint2(st.xs_x[g - np - na], st.xs_p[g - np - na]);
    rec[g] = r;
  }
}

// Import the other ranks' records: propagations and activations into the replicated sets
// (dedup), chain links into the replicated chain-link log and the successor rows (this rank's
// own went there at its commit).  If any rank's records exceeded the cap
// nothing is imported (g_max tells the host; it re-runs the exchange with a larger cap).
// The last block publishes: g_delta = Σ over ranks of all deltas (0 = global fixpoint).
__global__ void k_ximport(DIndex ix, DState st, XchgArgs x, PubArgs pub) {
  Ev ev;  // not accounted (the import has no oracle counterpart)
  const uint32_t stride = XH + 2 * x.cap;
  uint32_t gmax = 0;
  for (uint32_t q = 0; q < x.nranks; ++q) {
    const uint32_t* h = x.recv + (size_t)q * stride;
    gmax = max(gmax, h[XH_NP] + h[XH_NA] + h[XH_NX]);
  }
  const bool ok = gmax <= x.cap;
  const uint32_t total = ok ? x.nranks * x.cap : 0u;
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gs) {  // wave-uniform trip count
    const uint32_t i = base + threadIdx.x;
    uint32_t q = 0, j = 0, np = 0, na = 0, nx = 0;
    uint2 r = make_uint2(0, 0);
    if (i < total) {
      q = i / x.cap;
      j = i - q * x.cap;
      const uint32_t* h = x.recv + (size_t)q * stride;
      np = h[XH_NP], na = h[XH_NA], nx = h[XH_NX];
      if (j < np + na + nx) r = reinterpret_cast<const uint2*>(h + XH)[j];
    }
    const bool live = i < total && j < np + na + nx;
    const bool is_p = live && j < np && q != x.me;
    const bool is_a = live && j >= np && j < np + na && q != x.me;
    const bool is_x = live && j >= np + na && q != x.me;
    // propagations (unique per owner of Y, so a remote one is new unless re-imported)
    const bool nwp = is_p && hash_insert(st.phash, st.pmask, link_key(r.x, r.y));
    const uint32_t ps = wave_append(&st.ctr->p_log, nwp);
    gap_append(st.pp, r.x, r.y, nwp, ev.v);
    if (nwp) {
      st.plog_p[ps] = r.x;
      st.plog_b[ps] = r.y;
    }
    // activations (two ranks may have made the same one)
    const bool nwa = is_a && hash_insert(st.ahash, st.amask, link_key(r.y, r.x));
    const uint32_t as = wave_append(&st.ctr->a_log, nwa);
    if (nwa) {
      st.alog_y[as] = r.x;
      st.alog_c[as] = r.y;
      st.has_act[r.x] = 1;
    }
    // chain-second links: every rank's, successor CSR keyed by the link's source
    const uint32_t xsl = wave_append(&st.ctr->x_log, is_x);
    if (st.need_succ) gap_append(st.sc, r.x, r.y, is_x, ev.v);
    if (is_x) {
      st.xlog_x[xsl] = r.x;
      st.xlog_p[xsl] = r.y;
    }
  }
  publish_last(st, pub, false, [&] {
    if (threadIdx.x == 0) {
      uint32_t gd = 0, go = 0;
      for (uint32_t q = 0; q < x.nranks; ++q) {
        const uint32_t* h = x.recv + (size_t)q * stride;
        gd += h[XH_NP] + h[XH_NA] + h[XH_NX] + h[XH_DS] + h[XH_DL] + h[XH_DP] + h[XH_DA] + h[XH_DX];
        go += h[XH_OVF] + (h[XH_QOVF] << 16);  // (a lost send-queue record: the host throws)
      }
      auto put = [](uint32_t* w, uint32_t v) { __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
      put(&st.ctr->g_delta, gd);
      put(&st.ctr->g_max, gmax);
      put(&st.ctr->g_ovf, go);
      put(&st.ctr->g_pown, x.recv[(size_t)x.me * stride + XH_DP]);  // this rank's own new propagations
    }
    __syncthreads();
    // sent: the send queue and the candidate counters start over (on an exchange overflow
    // the redo packs the same records again)
    copy_and_zero(st, pub.host, ok ? XCHG_ZERO : 0u);
  });
}

// Partitioned install of the base links / propagations (el_ctx::install_base): what the commit
// routes for a new link or propagation (commit_l, commit_p), done for the base ones.  The
// chain-second base links join the replicated chain-link log (the successor rows already hold
// them: succ_fill) and, when another rank's rows can reach their x, the send queue; a base
// propagation ((r, Y), B) goes to the send queue when another rank's rows can link to Y.
__global__ void k_base_route(DIndex ix, DState st, uint32_t nb, uint32_t nbp) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t base = blockIdx.x * blockDim.x; base < nb; base += stride) {  // (uniform trip count)
    const uint32_t i = base + threadIdx.x;
    uint32_t x = 0, p = 0;
    bool ch = false;
    if (i < nb) {
      x = st.llog_x[i];
      p = st.llog_p[i];
      ch = ix.role_chs[ix.pair_role[p]];
    }
    const uint32_t xsl = wave_append(&st.ctr->x_log, ch);
    if (ch) {
      st.xlog_x[xsl] = x;
      st.xlog_p[xsl] = p;
    }
    const bool xs = ch && remote(ix, x);
    const uint32_t q = wave_append(&st.ctr->x_send, xs);
    if (xs && q < st.xs_cap) {
      st.xs_x[q] = x;
      st.xs_p[q] = p;
    }
  }
  for (uint32_t base = blockIdx.x * blockDim.x; base < nbp; base += stride) {
    const uint32_t i = base + threadIdx.x;
    bool xs = false;
    uint32_t pid = 0, b = 0;
    if (i < nbp) {
      pid = st.plog_p[i];
      b = st.plog_b[i];
      xs = remote(ix, ix.pair_y[pid]);
    }
    const uint32_t q = wave_append(&st.ctr->x_sp, xs);
    if (xs && q < st.xp_cap) {
      st.xp_p[q] = pid;
      st.xp_b[q] = b;
    }
  }
}

// Re-layout scan of a gapped CSR: new row starts = exclusive scan of gap_cap(len[r]).
// Single pass with decoupled look-back: tiles are handed out by an atomic ticket, so every
// predecessor tile of a block is owned by a block that is already running (look-back cannot
// wait on an unscheduled block).  Look-back flags carry the launch epoch: stale words from
// earlier launches never match, so they need no reset.
constexpr uint32_t SCAN_ITEMS = 8;
constexpr uint32_t SCAN_TILE = 256 * SCAN_ITEMS;
constexpr uint32_t FLAG_AGG = 1, FLAG_INC = 2;
struct ScanArgs {
  const uint32_t* len;  // rows: start_out = exclusive scan of gap_cap(len[r])
  uint32_t* start_out;  // rows + 1
  uint32_t n1;          // rows + 1
  uint32_t tiles;
  uint32_t epoch;
  unsigned long long* flags;
  uint32_t* ticket;
};

__device__ __forceinline__ unsigned long long flag_word(uint32_t epoch, uint32_t state, uint32_t v) {
  return ((unsigned long long)((epoch << 2) | state) << 32) | v;
}

__global__ void __launch_bounds__(256) k_gap_scan(ScanArgs sa) {
  __shared__ uint32_t buf[SCAN_TILE];
  __shared__ uint32_t wtot[4];
  __shared__ uint32_t s_tile, s_excl;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(sa.ticket, 1u);
  __syncthreads();
  const uint32_t t = __builtin_amdgcn_readfirstlane(s_tile);
  if (t == sa.tiles - 1 && tid == 0) *sa.ticket = 0;  // every other tile is already taken
  const uint32_t r0 = t * SCAN_TILE;
#pragma unroll
  for (uint32_t i = 0; i < SCAN_ITEMS; ++i) {
    const uint32_t idx = r0 + i * 256 + tid;
    buf[i * 256 + tid] = idx + 1 >= sa.n1 ? 0u : gap_cap(sa.len[idx]);  // row capacities
  }
  __syncthreads();
  uint32_t v[SCAN_ITEMS], run = 0;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) {
    v[j] = run;
    run += buf[tid * SCAN_ITEMS + j];
  }
  // wave-inclusive scan of the per-thread totals
  uint32_t inc = run;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wtot[wv] = inc;
  __syncthreads();
  uint32_t wbase = 0, agg = 0;
#pragma unroll
  for (uint32_t w = 0; w < 4; ++w) {
    if (w < wv) wbase += wtot[w];
    agg += wtot[w];
  }
  if (wv == 0) {  // look-back over the earlier tiles, 64 at a time
    unsigned long long* fl = sa.flags;
    const uint32_t ep = sa.epoch & 0x3fffffffu;
    uint32_t excl = 0;
    if (t == 0) {
      if (lane == 0) __hip_atomic_store(fl + t, flag_word(ep, FLAG_INC, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(fl + t, flag_word(ep, FLAG_AGG, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t j = (int64_t)t - 1;
      while (true) {
        const int64_t idx = j - (int64_t)lane;
        const bool valid = idx >= 0;
        uint32_t state = valid ? 0u : FLAG_INC, val = 0;
        while (true) {
          if (valid && state == 0) {
            const unsigned long long f = __hip_atomic_load(fl + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t hi = (uint32_t)(f >> 32);
            if ((hi >> 2) == ep) {
              state = hi & 3u;
              val = (uint32_t)f;
            }
          }
          if (__ballot(state == 0) == 0) break;
        }
        const unsigned long long incm = __ballot(state == FLAG_INC);
        if (incm) {
          const uint32_t first = (uint32_t)__ffsll((long long)incm) - 1;
          excl += (uint32_t)wave_sum(lane <= first ? val : 0u);
          break;
        }
        excl += (uint32_t)wave_sum(val);
        j -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(fl + t, flag_word(ep, FLAG_INC, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const uint32_t tbase = s_excl + wbase + inc - run;
#pragma unroll
  for (uint32_t j = 0; j < SCAN_ITEMS; ++j) buf[tid * SCAN_ITEMS + j] = tbase + v[j];
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < SCAN_ITEMS; ++i) {
    const uint32_t idx = r0 + i * 256 + tid;
    if (idx < sa.n1) sa.start_out[idx] = buf[i * 256 + tid];
  }
}

__global__ void k_rehash(unsigned long long* t, unsigned long long mask, const uint32_t* kx,
                         const uint32_t* kp, uint32_t n) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    hash_insert(t, mask, link_key(kp[i], kx[i]));
}

// el_init after a classification: only the words the fact log names can be non-zero, and
// when the log is small next to the matrix, clearing those words beats streaming it all
// Clear the bit matrix by its block summary: every marked block is zeroed (512-B blocks: by one
// wave, 8 B per lane, one coalesced store; smaller blocks: SUMM_WORDS / 4 lanes of 16 B each, so
// one store instruction zeroes 64 / (SUMM_WORDS / 4) whole blocks), its summary byte with it.
// Reads the summary and writes only the blocks that hold a bit: G3's 104 M facts lie in 10.0 M
// of 37 M 512-B blocks (5.1 GB of stores), 27.9 M 128-B blocks (3.6 GB) or 43.0 M 64-B lines
// (2.8 GB), instead of 104 M scattered stores (k_clear_logged) or a 19 GB memset.
// rows: the summary's rows (relative to the matrix base), SB bytes each.
__device__ __forceinline__ uint32_t nth_set(unsigned long long m, uint32_t k) {  // k-th set bit of m
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
    if (k >= c) {
      k -= c;
      m >>= w;
      pos += w;
    }
  }
  return pos;
}

__global__ void k_clear_summ(uint32_t* __restrict__ bits, uint64_t W, uint8_t* __restrict__ summ, uint32_t SB,
                             uint64_t rows) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t dwords = rows * SB / 4;  // (SB is a multiple of 16)
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  uint32_t* sw = reinterpret_cast<uint32_t*>(summ);
  constexpr uint32_t G = elrows::SUMM_WORDS / 4, PER = 64 / G;  // lanes per block, blocks per store
  for (uint64_t base = wave * 64; base < dwords; base += waves * 64) {  // (wave-uniform)
    const uint64_t d = base + lane;
    const uint32_t v = d < dwords ? sw[d] : 0u;
    for (uint32_t j = 0; j < 4; ++j) {
      unsigned long long m = __ballot(((v >> (8 * j)) & 0xffu) != 0u);
      if constexpr (G == 32) {  // 512-B blocks
        while (m) {
          const uint32_t L = (uint32_t)__ffsll((long long)m) - 1u;
          m &= m - 1ull;
          const uint64_t sb = (base + L) * 4 + j;  // summary byte: row sb / SB, block sb % SB
          const uint64_t row = sb / SB, w0 = (sb - row * SB) * 128 + 2 * lane;
          uint32_t* p = bits + row * W + w0;
          if (w0 + 1 < W) {
            *reinterpret_cast<uint2*>(p) = make_uint2(0u, 0u);
          } else if (w0 < W) {
            *p = 0u;
          }
        }
      } else {
        const uint32_t n = (uint32_t)__popcll(m);
        for (uint32_t r = 0; r < n; r += PER) {  // (wave-uniform)
          const uint32_t k = r + lane / G;
          if (k < n) {
            const uint64_t sb = (base + nth_set(m, k)) * 4 + j;
            const uint64_t row = sb / SB, w0 = (sb - row * SB) * elrows::SUMM_WORDS + (lane % G) * 4;
            if (w0 < W) *reinterpret_cast<uint4*>(bits + row * W + w0) = make_uint4(0u, 0u, 0u, 0u);  // (W % 4 == 0)
          }
        }
      }
    }
    if (d < dwords && v) sw[d] = 0u;
  }
}

__global__ void k_clear_logged(DIndex ix, uint32_t* bits_base, const uint32_t* __restrict__ lx,
                               const uint32_t* __restrict__ la, uint32_t n, uint32_t row_from) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (lx[i] < row_from) continue;  // (rows a releasing copy-back already cleared)
    const uint32_t c = col_of(ix, la[i]);
    if (c != NONE) bits_base[(uint64_t)lx[i] * ix.W + (c >> 5)] = 0u;
  }
}

// ---- gapped-CSR layout kernels (rare: initial layout, re-layout after an overflow)
__global__ void k_gap_init(uint32_t* start, uint32_t* end, uint32_t* len, uint32_t rows,
                           const uint32_t* __restrict__ start0) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r <= rows; r += stride) {
    const uint32_t v = start0 ? start0[r] : r * gap_cap(0);
    start[r] = v;
    if (r > 0) end[r - 1] = v;
    if (r < rows) len[r] = 0;
  }
}

// end[r] = start[r + 1]: the slots of a layout made by a scan (gap_build_from_log)
__global__ void k_gap_ends(const uint32_t* __restrict__ start, uint32_t* __restrict__ end, uint32_t rows) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) end[r] = start[r + 1];
}

// ---- relocation of the rows that overflowed in a step (el_ctx::gap_relocate).  rc[0] = the
// slot array's next free slot (64-bit), rc[1] = rows claimed, rc[2] = their in-place entries.
struct Reloc {
  uint64_t base;  // the slot array's tail before this relocation (new slots start there)
  uint32_t* start;
  uint32_t* end;
  const uint32_t* len;
  uint32_t* val;
  const uint32_t* ovq;  // (row, value, rank) per overflowing entry
  uint32_t n_ovf;
  uint32_t* nstart;  // rows: new start of a claimed row
  uint32_t* rlist;   // claimed rows (≤ n_ovf)
  unsigned long long* rc;
};

// The first overflow record of each row claims the row and reserves gap_cap(len) slots for it:
// one atomic per wave on the tail (a prefix sum of the wave's claims), not one per row.
__global__ void k_reloc_claim(Reloc a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t base = blockIdx.x * blockDim.x; base < a.n_ovf; base += stride) {  // (uniform trip count)
    const uint32_t i = base + threadIdx.x;
    uint32_t row = 0, sz = 0, old = 0;
    bool won = false;
    if (i < a.n_ovf) {
      // the record whose rank is the row's capacity claims it: ranks come from the row's len
      // atomic, so exactly one overflow record per row has it (an atomicExch on a per-row flag
      // put every record of a hub row on one word: 173 µs in G3's first superstep)
      row = a.ovq[3 * (size_t)i];
      const uint32_t cap = a.end[row] - a.start[row];
      won = a.ovq[3 * (size_t)i + 2] == cap;
      if (won) {
        sz = gap_cap(a.len[row]);
        old = cap;  // (an overflowing row is full: every slot holds an entry)
      }
    }
    uint32_t inc = sz;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o);
      if (lane_id() >= o) inc += v;
    }
    const uint32_t total = __shfl(inc, 63);
    const unsigned long long moved = wave_sum(old);
    unsigned long long b = 0;
    if (lane_id() == 0 && total) b = atomicAdd(a.rc, (unsigned long long)total);
    if (lane_id() == 0 && moved) atomicAdd(a.rc + 2, moved);
    b = __shfl(b, 0);
    const uint32_t k = wave_append(reinterpret_cast<uint32_t*>(a.rc + 1), won);
    if (won) {
      // (truncated to 32 bits here: the host reads the claims' total before any move and throws
      // when the tail passes 2^32, so k_reloc_move never runs on a wrapped start)
      a.nstart[row] = (uint32_t)(a.base + b + inc - sz);
      a.rlist[k] = row;
    }
  }
}

// Claimed rows: the in-place entries to the new slots (a block per row), then the overflow
// entries by rank (roles: blocks [0, nb) rows, the rest overflow records).
__global__ void k_reloc_move(Reloc a, uint32_t nb) {
  const uint32_t nrows = (uint32_t)a.rc[1];
  if (blockIdx.x < nb) {
    for (uint32_t k = blockIdx.x; k < nrows; k += nb) {
      const uint32_t row = a.rlist[k], s0 = a.start[row], n = a.end[row] - s0, d = a.nstart[row];
      for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) a.val[d + j] = a.val[s0 + j];
    }
    return;
  }
  const uint32_t stride = (gridDim.x - nb) * blockDim.x;
  for (uint32_t i = (blockIdx.x - nb) * blockDim.x + threadIdx.x; i < a.n_ovf; i += stride) {
    const uint32_t row = a.ovq[3 * (size_t)i];
    a.val[a.nstart[row] + a.ovq[3 * (size_t)i + 2]] = a.ovq[3 * (size_t)i + 1];
  }
}

// Before the claims: the relocation counters of the three CSRs and the step's overflow counts
// (DCounters ov_pr, ov_sc, ov_pp: the host read them with the step's counters) start over.
__global__ void k_reloc_reset(unsigned long long* rc, uint32_t* ov) {
  if (threadIdx.x < 9) rc[threadIdx.x] = 0;
  if (threadIdx.x < 3) ov[threadIdx.x * CTR_STRIDE] = 0;
}

// After the claims: the counters to coherent pinned host memory, then the sequence word (the
// host spins on it instead of a stream synchronisation).
__global__ void k_reloc_publish(const unsigned long long* rc, volatile unsigned long long* host, uint32_t seq) {
  if (threadIdx.x == 0) {
    for (int i = 0; i < 9; ++i) host[i] = rc[i];
    __threadfence_system();
    host[9] = seq;
    __threadfence_system();
  }
}

__global__ void k_reloc_commit(Reloc a) {
  const uint32_t nrows = (uint32_t)a.rc[1], stride = gridDim.x * blockDim.x;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nrows; k += stride) {
    const uint32_t row = a.rlist[k];
    a.start[row] = a.nstart[row];
    a.end[row] = a.nstart[row] + gap_cap(a.len[row]);
  }
}

// rows[i] -> map[rows[i]] (pair ids after an increment re-numbered the pair universe)
// The re-trigger lists of an increment (el_ctx::migrate_state): facts i < s_old whose A or X is
// marked, the links whose pid is marked.
// dA[A] bit 0: re-trigger the facts (X, A) over all of A's rows (flag 2: the closed rows exr*,
// exl*); bit 1: the told closure too (flag 0: A is the source of a new told axiom).  The facts
// re-triggered because their X is a new link target (dX) keep flag 1 — their parent fact, of the
// same X, is re-triggered too — and walk no told closure (flag 2): A's told* did not change unless
// A lies below a source A', and then (X, A') is in S(X) and re-walks its own.  (The migrated
// context has no base links, so flag 2 means "closed rows, no told walk" to k_expand.)  Order is
// irrelevant to the fixpoint.
constexpr uint32_t RT_TILE = 8192;  // entries per block of k_retrigger (one counter atomic per tile)
__global__ void __launch_bounds__(256) k_retrigger(const uint32_t* __restrict__ sx, const uint32_t* __restrict__ sa,
                                                   const uint8_t* __restrict__ sf, uint32_t s_old, uint32_t s_n,
                                                   const uint32_t* __restrict__ lx, const uint32_t* __restrict__ lp,
                                                   uint32_t l_n, const uint8_t* __restrict__ dA,
                                                   const uint8_t* __restrict__ dX, const uint8_t* __restrict__ dP,
                                                   uint32_t* rx, uint32_t* ra, uint8_t* rf, uint32_t* rlx, uint32_t* rlp,
                                                   const uint4* __restrict__ meta, unsigned long long* cnt) {
  // two passes over the block's tile: count the kept entries (per wave, then a block prefix and
  // one atomic per tile and list), then write them at their places
  __shared__ uint32_t wcnt[2][4];
  __shared__ unsigned long long gbase[2];
  const uint32_t t0 = blockIdx.x * RT_TILE, wid = threadIdx.x >> 6;
  // (facts from s_old on — the new concepts' init facts — lie above the watermarks: the
  // supersteps after the re-trigger step expand them)
  auto keep_s = [&](uint32_t i) { return i < s_old && (dA[sa[i]] || dX[sx[i]]); };
  auto keep_l = [&](uint32_t i) { return i < l_n && dP[lp[i]]; };
  uint32_t cs = 0, cl = 0;
  for (uint32_t k = 0; k < RT_TILE; k += 256) {
    const uint32_t i = t0 + k + threadIdx.x;
    cs += (uint32_t)__popcll(__ballot(keep_s(i)));
    cl += (uint32_t)__popcll(__ballot(keep_l(i)));
  }
  if (lane_id() == 0) wcnt[0][wid] = cs, wcnt[1][wid] = cl;
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t* w = wcnt[threadIdx.x];
    const unsigned long long tot = (unsigned long long)w[0] + w[1] + w[2] + w[3];
    gbase[threadIdx.x] = tot ? atomicAdd(cnt + threadIdx.x, tot) : 0ull;
  }
  __syncthreads();
  unsigned long long os = gbase[0], ol = gbase[1];
  for (uint32_t w = 0; w < wid; ++w) os += wcnt[0][w], ol += wcnt[1][w];
  const unsigned long long below = (1ull << lane_id()) - 1ull;
  unsigned long long told = 0;  // told candidates the kept facts can emit (the rows they re-walk)
  for (uint32_t k = 0; k < RT_TILE; k += 256) {  // (block-uniform trip count; each wave in order)
    const uint32_t i = t0 + k + threadIdx.x;
    const bool ks = keep_s(i), kl = keep_l(i);
    const unsigned long long ms = __ballot(ks), ml = __ballot(kl);
    if (ks) {
      const uint64_t o = os + __popcll(ms & below);
      const uint32_t a = sa[i];
      const uint8_t d = dA[a];
      rx[o] = sx[i];
      ra[o] = a;
      rf[o] = d & 2u ? 0 : d ? 2 : sf[i] == 1 ? 1 : 2;
      if (d & 2u) told += meta[2 * a + 1].x - meta[2 * a].x;
    }
    if (kl) {
      const uint64_t o = ol + __popcll(ml & below);
      rlx[o] = lx[i];
      rlp[o] = lp[i];
    }
    os += __popcll(ms);
    ol += __popcll(ml);
  }
  for (int k = 32; k >= 1; k >>= 1) told += __shfl_xor(told, k);
  if (lane_id() == 0 && told) atomicAdd(cnt + 2, told);
}

__global__ void k_remap(uint32_t* __restrict__ v, uint64_t n, const uint32_t* __restrict__ map) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) v[i] = map[v[i]];
}

// keep (optional): entry i is kept iff keep[role[vals[i]]] (the successor rows' role filter)
struct GapKeep {
  const uint8_t* keep;
  const uint32_t* role;
  __device__ __forceinline__ bool operator()(uint32_t v) const { return !keep || keep[role[v]]; }
};

__global__ void k_gap_count(uint32_t* __restrict__ len, const uint32_t* __restrict__ rows,
                            const uint32_t* __restrict__ vals, uint64_t n, GapKeep keep) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    if (keep(vals[i])) atomicAdd(len + rows[i], 1u);
}

// every logged entry appended to its row (the layout already fits every row)
__global__ void k_gap_fill(DGap g, const uint32_t* __restrict__ rows, const uint32_t* __restrict__ vals, uint64_t n,
                           GapKeep keep) {
  uint32_t ev[EL_NUM_EVENTS] = {};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    const bool p = i < n && keep(vals[i]);
    gap_append(g, p ? rows[i] : 0u, p ? vals[i] : 0u, p, ev);
  }
}

// ---------------------------------------------------------------- host side

// Launch that carries a work phase: expand roles run in k_expand (timed as EXPAND_S),
// commit roles in k_commit (COMMIT_S), the re-layout scan in k_gap_scan.
uint32_t kernel_group(int k) {
  switch (k) {
    case EL_K_EXPAND_L:
    case EL_K_EXPAND_A:
    case EL_K_EXPAND_P:
      return EL_K_EXPAND_S;
    case EL_K_COMMIT_L:
    case EL_K_COMMIT_A:
    case EL_K_COMMIT_P:
      return EL_K_COMMIT_S;
    case EL_K_MERGE_PTR:
      return EL_K_SCAN;
    default:
      return (uint32_t)k;
  }
}

template <class T>
T* dalloc(size_t n) {
  void* p = nullptr;
  if (n == 0) n = 1;
  HIPCHK(hipMalloc(&p, n * sizeof(T)));
  return (T*)p;
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <class T>
T* dupload(const std::vector<T>& v) {
  T* p = dalloc<T>(v.size());
  if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}
// grow a device array to cap elements keeping the first used ones
template <class T>
void dgrow(T*& p, size_t used, size_t cap) {
  T* q = dalloc<T>(cap);
  if (used) HIPCHK(hipMemcpy(q, p, used * sizeof(T), hipMemcpyDeviceToDevice));
  dfree(p);
  p = q;
}

// Grid-stride kernels: at most 1024 blocks (4 per CU) — enough to fill the chip and few
// enough that the per-block flush atomics of a launch stay cheap.
uint32_t grid_for(uint64_t n, uint32_t cap = 1024) {
  uint64_t g = (n + BLOCK - 1) / BLOCK;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (uint32_t)g;
}

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

// a log's new capacity for n entries: 1/8 slack in 4 M-entry steps.  The logs must hold every
// candidate of a step that could be new (count + the candidate queues), which the queues' own
// headroom already overstates; round 4 grew them to the next power of two of 1.5× that (G3's fact
// log: 2^30 entries = 9.7 GB for 104 M facts).
static uint64_t log_cap(uint64_t n) {
  const uint64_t step = 1ull << 22;
  return (n + n / 8 + step - 1) / step * step;
}
// The fact and link logs, which the streamed result reads, keep power-of-two growth with
// half again as slack: with log_cap's slack (G3's fact log 4.3 GB instead of 9.7 GB) the
// result's copy-back tail grew by 7-8 ms in every A/B run, the supersteps unchanged (the
// cause was not found: after the first classification neither sizing regrows the log).
static uint64_t stream_log_cap(uint64_t n) { return next_pow2(n + n / 2); }

// Triggers per wave and grid of an expand role with n triggers: a small step's triggers
// spread over up to maxb·4 waves, T = ceil(n / waves) each (64, a lane per trigger, once n
// fills them).  Each wave walks its triggers' index rows 64 entries a round with a dependent
// random read per round (a link-set probe, a bit test), so a step of 10 k triggers on 40
// blocks of 64-trigger waves took ~65 rounds of latency (G3's late supersteps: 60–100 µs of
// CR3 each); at 3 triggers per wave on 834 blocks it takes a few.
static void wave_triggers(uint64_t n, uint32_t maxb, uint32_t& grid, uint32_t& tpw) {
  const uint64_t waves = (uint64_t)maxb * (BLOCK / 64);
  tpw = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, (n + waves - 1) / waves));
  const uint64_t per_block = (uint64_t)tpw * (BLOCK / 64);
  grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(maxb, (n + per_block - 1) / per_block));
}

// Gapped CSR (DGap) on the host side: the layout buffers, the overflow queue, relocation scratch.
struct GapCsr {
  uint32_t rows = 0;
  uint32_t *start = nullptr, *end = nullptr, *len = nullptr;
  uint32_t* val = nullptr;
  uint64_t val_cap = 0;
  uint64_t used = 0;  // slots in use: the layout's, then every relocated row's (val[used, val_cap) is free)
  uint32_t* ovq = nullptr;
  uint64_t ovq_cap = 0;
  uint32_t* nstart = nullptr;  // relocation: a claimed row's new start
  uint32_t* rlist = nullptr;                    // relocation: claimed rows (ovq_cap)
  bool live = false;  // maintained for this ontology (it has readers)
  // The classification's initial layout (el_init: a device scan of the row capacities the
  // first supersteps ask for — the base links and their CR5 lifts; el_ctx::closure_state), or
  // r · gap_cap(0) when `laid` is false.  Reset restores it (k_gap_init).
  uint32_t* start0 = nullptr;
  bool laid = false;
  uint64_t total0 = 0;  // slots of the initial layout
  void alloc(uint32_t n, uint64_t ovq_entries) {
    rows = n;
    start = dalloc<uint32_t>(n + 1);
    end = dalloc<uint32_t>(n);
    len = dalloc<uint32_t>(n);
    start0 = dalloc<uint32_t>(n + 1);
    nstart = dalloc<uint32_t>(n);
    laid = false;
    total0 = (uint64_t)gap_cap(0) * n;
    val_cap = total0;
    used = total0;
    val = dalloc<uint32_t>(val_cap);
    live = true;
    set_ovq(ovq_entries);
  }
  // An increment's re-build (el_ctx::migrate_state) for n rows: the row arrays follow n, the
  // slot array is kept (gap_build_from_log grows it if the logs need more) — freeing and
  // re-allocating gigabytes of slots cost more than the build itself.
  void reshape(uint32_t n, uint64_t ovq_entries) {
    if (!live || n != rows) {
      for (uint32_t** p : {&start, &end, &len, &start0, &nstart}) dfree(*p);
      rows = n;
      start = dalloc<uint32_t>(n + 1);
      end = dalloc<uint32_t>(n);
      len = dalloc<uint32_t>(n);
      start0 = dalloc<uint32_t>(n + 1);
      nstart = dalloc<uint32_t>(n);
    }
    laid = false;
    total0 = used = (uint64_t)gap_cap(0) * n;
    live = true;
    set_ovq(ovq_entries);
  }
  void set_ovq(uint64_t entries) {
    if (!live || entries <= ovq_cap) return;
    dfree(ovq);
    dfree(rlist);
    ovq_cap = entries;
    ovq = dalloc<uint32_t>(3 * entries);
    rlist = dalloc<uint32_t>(entries);
  }
  void release() {
    dfree(start);
    dfree(end);
    dfree(len);
    dfree(val);
    dfree(ovq);
    dfree(rlist);
    dfree(nstart);
    dfree(start0);
    val_cap = ovq_cap = total0 = used = 0;
    live = laid = false;
  }
  DGap view(uint32_t* ov_count) const {
    return DGap{start, end, len, val, ovq, (uint32_t)ovq_cap, ov_count};
  }
};

struct PendingEvent {
  int kernel;
  hipEvent_t a, b;
};

// ---- delta exchange transports.  allgather is stream-ordered: it
// reads `send` after the work already queued on s and later work on s sees `recv`.
struct Exchange {
  int rank = 0, size = 1;
  virtual ~Exchange() {}
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
};

// RCCL over xGMI.  librccl is opened on first use, so a whole-ontology context (and the
// CPU-side ABI checks) never need it; the header provides the types only.
struct RcclApi {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
};
const RcclApi& rccl_api() {
  static RcclApi api;
  static std::once_flag once;
  static std::string why;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
      why = dlerror() ? dlerror() : "librccl not found";
      return;
    }
    api.get_id = (decltype(api.get_id))dlsym(h, "ncclGetUniqueId");
    api.init_rank = (decltype(api.init_rank))dlsym(h, "ncclCommInitRank");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.destroy = (decltype(api.destroy))dlsym(h, "ncclCommDestroy");
    api.err = (decltype(api.err))dlsym(h, "ncclGetErrorString");
  });
  if (!api.get_id || !api.init_rank || !api.all_gather || !api.destroy || !api.err)
    throw ElError{EL_EHIP, "RCCL unavailable: " + why};
  return api;
}
#define RCCLCHK(expr)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (expr);                                                                      \
    if (r_ != ncclSuccess) throw ElError{EL_EHIP, std::string(#expr) + ": " + rccl_api().err(r_)}; \
  } while (0)

struct RcclExchange : Exchange {
  ncclComm_t comm = nullptr;
  RcclExchange(int r, int n, const uint8_t id[128]) {
    rank = r;
    size = n;
    ncclUniqueId uid;
    static_assert(sizeof(uid) == 128, "ncclUniqueId");
    memcpy(&uid, id, sizeof uid);
    RCCLCHK(rccl_api().init_rank(&comm, n, uid, r));
  }
  ~RcclExchange() override {
    if (comm) (void)rccl_api().destroy(comm);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    RCCLCHK(rccl_api().all_gather(send, recv, bytes, ncclUint8, comm, s));
  }
};

// The caller's transport (EL_XCHG_HOST): the send block is staged through page-locked host
// memory, the caller all-gathers it, and the gathered blocks go back to the device.
struct HostExchange : Exchange {
  el_allgather_fn fn;
  void* user;
  void *hsend = nullptr, *hrecv = nullptr;
  size_t cap = 0;
  HostExchange(int r, int n, el_allgather_fn f, void* u) : fn(f), user(u) {
    rank = r;
    size = n;
  }
  ~HostExchange() override {
    if (hsend) (void)hipHostFree(hsend);
    if (hrecv) (void)hipHostFree(hrecv);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (bytes > cap) {
      HIPCHK(hipStreamSynchronize(s));  // (the last gather's upload has read hrecv)
      if (hsend) HIPCHK(hipHostFree(hsend));
      if (hrecv) HIPCHK(hipHostFree(hrecv));
      hsend = hrecv = nullptr;
      HIPCHK(hipHostMalloc(&hsend, bytes, hipHostMallocDefault));
      HIPCHK(hipHostMalloc(&hrecv, bytes * (size_t)size, hipHostMallocDefault));
      cap = bytes;
    }
    HIPCHK(hipMemcpyAsync(hsend, send, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));  // (also: the last gather's upload has read hrecv)
    if (fn(user, hsend, hrecv, bytes) != 0)
      throw ElError{EL_ESTATE, "EL_XCHG_HOST: the caller's all-gather failed"};
    HIPCHK(hipMemcpyAsync(recv, hrecv, bytes * (size_t)size, hipMemcpyHostToDevice, s));
  }
};

}  // namespace

// In-process group: n contexts driven by n host threads (tests, and one process driving
// several GPUs).  Peers copy each other's send buffers device-to-device between barriers.
struct el_group {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const void*> src;
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (broken) throw ElError{EL_ESTATE, "exchange group broken by a failed rank"};
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) || broken) {
      broken = true;
      cv.notify_all();
      throw ElError{EL_ESTATE, "exchange group barrier timed out or broken"};
    }
  }
  void fail() {
    std::lock_guard<std::mutex> lk(m);
    broken = true;
    cv.notify_all();
  }
};

namespace {
struct LocalExchange : Exchange {
  el_group* g;
  LocalExchange(el_group* grp, int r) : g(grp) {
    rank = r;
    size = grp->n;
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    try {
      HIPCHK(hipStreamSynchronize(s));  // send is complete
      g->src[rank] = send;
      g->barrier();
      for (int q = 0; q < size; ++q)
        HIPCHK(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)q * bytes, g->src[q], bytes,
                              hipMemcpyDeviceToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
      g->barrier();  // nobody reuses its send buffer before every peer has copied it
    } catch (...) {
      g->fail();
      throw;
    }
  }
};
}  // namespace

namespace {
uint32_t* mapped_for_device(void* h);
}

struct el_ctx {
  int device = 0;
  int profile = 0;
  uint32_t flags = 0;  // EL_FLAG_* (el_config.flags)
  hipStream_t stream = nullptr;
  std::string err;
  bool loaded = false, inited = false;

  el::HostIndex hx;
  DIndex ix{};
  std::vector<void*> index_bufs;

  // state
  uint32_t* bits = nullptr;
  uint64_t W = 0;
  // Block summary of the bit rows: one byte per block of SUMM_WORDS words (512 B by default,
  // EL_SUMM_SHIFT) of each owned row, set
  // with a plain store by every writer of a bit (k_commit, k_init, k_init_bits), cleared with
  // the matrix; the copy-back read-out loads only the blocks it marks.
  uint8_t* summ = nullptr;
  uint32_t SB = 0;
  bool no_summary = getenv("EL_NO_SUMMARY") != nullptr;  // A/B: dense read-out
  // one byte per SUMM_WORDS words, rows padded to 16 B (k_fill clears from any row with 16-B
  // stores; whole 512-B blocks of the read-out)
  static uint32_t summ_stride(uint64_t w) {
    return (uint32_t)((((w + elrows::SUMM_WORDS - 1) / elrows::SUMM_WORDS) + 15) & ~15ull);
  }
  uint32_t *slog_x = nullptr, *slog_a = nullptr;
  uint8_t* slog_f = nullptr;  // told-closure flags of the facts (slog_cap)
  uint64_t slog_cap = 0;
  uint32_t *ct_x = nullptr, *ct_a = nullptr;  // CR1 told-closure candidates
  uint64_t ct_cap = 0;
  unsigned long long* lhash = nullptr;
  uint64_t lhash_cap = 0;
  uint32_t *llog_x = nullptr, *llog_p = nullptr;
  uint64_t llog_cap = 0;
  unsigned long long* ahash = nullptr;
  uint64_t ahash_cap = 0;
  uint32_t *alog_y = nullptr, *alog_c = nullptr;
  uint64_t alog_cap = 0;
  uint8_t* has_act = nullptr;
  // activation index: log indices of the activations (Y, C) by Y, ascending (el_rows build)
  uint64_t* act_ptr = nullptr;  // N + 1
  uint32_t* act_k = nullptr;
  uint64_t act_k_cap = 0, act_n = ~0ull;  // entries indexed (~0: rebuild)
  elrows::Scratch asc;
  void refresh_acts();
  unsigned long long* phash = nullptr;
  uint64_t phash_cap = 0;
  uint32_t *plog_p = nullptr, *plog_b = nullptr;
  uint64_t plog_cap = 0;
  uint32_t *cp_p = nullptr, *cp_b = nullptr;
  uint64_t cp_cap = 0;
  // result rows for export / copy-back (el_rows.h), rebuilt from the logs when they changed
  struct Rows {
    uint64_t* ptr = nullptr;  // owned rows + 1
    uint32_t* val = nullptr;
    uint64_t cap = 0;
    uint64_t n = ~0ull;  // entries the rows were built from (~0: stale)
    void release() {
      if (ptr) (void)hipFree(ptr);
      if (val) (void)hipFree(val);
      ptr = nullptr;
      val = nullptr;
      cap = 0;
      n = ~0ull;
    }
  };
  Rows rs, rl;  // S rows X -> {B}; link rows X -> {q}, q = pair rank in (role, filler) order
  elrows::Scratch rsc, rsc_l;  // row-build scratch (S rows, link rows: built concurrently)
  const uint32_t* pid_rank = nullptr;        // device: pid -> q (an index buffer)
  std::vector<uint32_t> rank_role, rank_y;   // host: the pair (role, filler) of rank q
  hipStream_t cstream = nullptr;             // copy-back DMA, beside the row builds
  // S-row read-out copy-back (el_copy_result): device staging chunks and their DMA stream
  hipStream_t dstream = nullptr;
  // EL_STREAM_PRIO (A/B): the copy-back streams and the read-out's own stream at the lowest
  // priority, the engine stream at the highest, so a copy-back in flight beside another
  // engine's saturation yields the dispatcher to it.  Measured with two engines in flight: G3
  // 29.7 -> 27.2 ms while the host enqueued the copy-back before starting the other engine;
  // once a helper thread enqueues it, 25.07 vs 25.12 ms, and G2 loses (1.26 vs 1.01 ms): off.
  hipStream_t ostream = nullptr;
  hipEvent_t ev_out = nullptr;
  static constexpr uint32_t NSTAGE = 4;  // staging buffers: the read-out runs up to 3 chunks ahead of the DMA
  hipEvent_t ev_stage[NSTAGE] = {}, ev_dma[NSTAGE] = {};
  uint32_t* stage[NSTAGE] = {};
  uint64_t stage_cap = 0;
  bool readout_off = getenv("EL_NO_READOUT") != nullptr;  // A/B: S rows by the log sort instead
  uint64_t readout_min = env_u32("EL_READOUT_MIN", 16u << 20);  // tests: the read-out for small results too
  bool links_direct = getenv("EL_LINKS_DIRECT") != nullptr;  // A/B: link-row sorts write the host buffer
  bool s_dma = getenv("EL_S_DMA") != nullptr;                // A/B: small S results by device sort + DMA
  uint64_t readout_chunk = (uint64_t)env_u32("EL_READOUT_CHUNK_MB", 32) << 18;  // entries per read-out DMA
  hipEvent_t ev_rows[2] = {nullptr, nullptr};
  GapCsr PR, SC, PP;   // predecessors per pid, successors per X, propagations per pid
  uint32_t* pin_word = nullptr;  // pinned scratch for the rare synchronous readbacks
  bool need_pred = true;      // predecessor CSR has readers (CR4, ⊥, CR6)
  bool need_succ = true;      // successor CSR has readers (CR6)
  uint32_t *cs_x = nullptr, *cs_a = nullptr, *cl_x = nullptr, *cl_p = nullptr, *ca_y = nullptr,
           *ca_c = nullptr;
  uint64_t cs_cap = 0, cl_cap = 0, ca_cap = 0;
  uint32_t max_rng = 0;  // most ranges of one role: activation candidates per new link
  uint4* jobs = nullptr;
  uint64_t job_cap = 0;
  DCounters* ctr = nullptr;
  unsigned long long* ev = nullptr;
  unsigned long long hev[EL_NUM_KERNELS][EL_NUM_EVENTS] = {};
  unsigned long long* scan_flags = nullptr;  // k_gap_scan look-back words (epoch-tagged)
  uint32_t* commit_done = nullptr;           // k_commit finished-block counters
  uint64_t scan_tiles = 0;
  uint32_t scan_epoch = 0;

  // host mirrors
  HCounters hc{};
  HCounters* hc_pinned = nullptr;  // counters published by k_commit (hipHostMalloc)
  HCounters* hc_dev = nullptr;     // device view of hc_pinned
  uint32_t commit_seq = 0;         // k_commit launches so far (published with the counters)
  bool stats_stale = false;        // el_init ran without a sync: `last` is filled on demand
  bool split_commit = getenv("EL_SPLIT_COMMIT") != nullptr;  // diagnostic only
  bool split_expand = getenv("EL_SPLIT_EXPAND") != nullptr;  // diagnostic: one k_expand launch per role
  unsigned long long* ev_sum = nullptr;   // k_ev_reduce output
  unsigned long long* lines_dbg = nullptr;  // EL_TRACE_CANDS: DState::lines
  unsigned long long* ev_host = nullptr;  // pinned copy of ev_sum
  bool events_queued = false;
  uint64_t s_count = 0, l_count = 0, a_count = 0, p_count = 0, s_init = 0;
  uint64_t l_base = 0;  // base links at the head of the link log (ix.base; install_base)
  uint64_t p_base = 0;  // base propagations at the head of the propagation log
  bool fresh = false;   // el_init ran and no superstep since: el_saturate installs the base links
  void install_base();

  // ---- the told closure and what it derives (el_closure.h), rebuilt by every el_init
  elcl::Axioms cax{};   // the told axiom rows on the device (index buffers)
  elcl::Axioms caxk{};  // what the Kahn levels walk: cax, or its told-cycle condensation (el_index.h)
  elcl::Out cl{};      // rows told*, exr*, exl*, meta, per-concept statistics, working storage
  struct ClHost {      // pinned readback of a build: counters, the next level's flag, meta of ⊤
    elcl::Ctr ctr;
    uint32_t flag, pad[3];
    uint4 top[2];
  };
  ClHost* clh = nullptr;
  elcl::Ctr clt{};          // the last build's totals
  uint32_t* cpos[3] = {};   // exclusive scans over the rows [a, b) of the last build: init facts,
                            // base links, base propagations (b - a + 1 entries)
  void* cscan_tmp = nullptr;
  size_t cscan_bytes = 0;
  void* csort_tmp = nullptr;
  size_t csort_bytes = 0;
  uint32_t *sk = nullptr, *sv = nullptr;  // the base links by pid (radix sort): predecessor rows
  uint64_t sk_cap = 0;
  uint32_t *pr_first = nullptr, *pr_last = nullptr;  // pid -> its run in sk
  uint32_t *bpp_s = nullptr, *bpp_e = nullptr;       // pid -> its base propagations in the log
  uint32_t *cap_pr = nullptr, *cap_pp = nullptr;     // first-superstep row capacities per pid
  uint32_t key_bits = 1;     // bits of a pid (radix sort)
  uint32_t level_hint = 32;  // Kahn levels launched before the first readback (grows to the depth seen)
  uint64_t nb = 0, nbp = 0, nc = 0;  // base links, base propagations, chain-second base links
  void alloc_closure();
  void free_closure();
  uint64_t cl_alloc_n = 0, cl_alloc_p = 0;
  // the bit matrix's columns are not in concept order (DIndex::cperm): a row read off the matrix
  // would not come out ascending, so S rows come from the log sorts only, and the reset clears the
  // matrix itself (no copy-back clears it as it reads)
  bool colperm() const { return ix.cperm != nullptr; }
  std::chrono::steady_clock::time_point inc_t0;  // (EL_TRACE_INC: el_saturate's start)  // the concept / pair counts the closure buffers were allocated for
  void set_closure_ix();
  void closure_grow();
  void closure_tail(uint32_t a, uint32_t b, uint32_t L, bool all);
  void closure_rows(uint32_t a, uint32_t b);
  // static Kahn levels of the built window (elcl::Axioms::slevel): concepts of level L >= 1 at
  // lvl_ids[lvl_ptr[L], lvl_ptr[L + 1]); empty: the dynamic levels
  std::vector<uint32_t> lvl_ptr;
  void static_levels();
  void closure_state();
  // The logs are indexed by uint32 counters on the device (DCounters): a step whose logs could
  // pass 2^32 entries (count + every candidate new) fails with EL_ENOMEM instead of wrapping.
  void check_u32_room() const {
    const uint64_t lim = 0xffffffffull;
    if (s_count + cs_cap + ct_cap > lim || l_count + cl_cap + remote_bound() > lim ||
        a_count + ca_cap + remote_bound() > lim || p_count + cp_cap + remote_bound() > lim)
      throw ElError{EL_ENOMEM, "a log would pass 2^32 entries (uint32 device counters)"};
  }
  uint64_t wm_s[EL_NUM_RULE_TYPES] = {}, wm_l[EL_NUM_RULE_TYPES] = {}, wm_a[EL_NUM_RULE_TYPES] = {},
           wm_p[EL_NUM_RULE_TYPES] = {}, wm_x = 0;
  // Incremental classification (el_add_axioms): the logged facts and links an increment's axioms
  // reach, compacted (their index rows changed: the first superstep after the increment takes its
  // triggers from here instead of the logs — migrate_state, retrigger_step)
  uint32_t *rt_x = nullptr, *rt_a = nullptr, *rt_lx = nullptr, *rt_lp = nullptr;
  uint8_t* rt_f = nullptr;
  uint64_t rt_ns = 0, rt_nl = 0, rt_scap = 0, rt_lcap = 0;
  bool inc_pending = false;
  // the masks (dA, dX by concept, dP by pair id) of the increments carried over since the last
  // saturation: a second el_add_axioms before el_saturate re-triggers what either reaches
  std::vector<uint8_t> pend_dA, pend_dX, pend_dP;
  double inc_ms[3] = {0, 0, 0};  // the last el_add_axioms: host index build, upload, state migration
  bool trig_override = false;  // superstep(): k_expand reads the rt_* triggers
  void retrigger_step();
  void mem_report() const;  // (EL_TRACE_MEM: device bytes per structure on stderr)
  void retrigger_all();  // (el_step after an increment: every logged fact once, as round 4)
  el_stats last{};
  std::vector<uint64_t> tr_s, tr_l, tr_a;
  // host-side per-kernel accounting (merge kernels, launches, times)
  uint64_t launches[EL_NUM_KERNELS] = {};
  uint64_t host_ev[EL_NUM_KERNELS][EL_NUM_EVENTS] = {};
  double kms[EL_NUM_KERNELS] = {};
  std::vector<PendingEvent> pending;
  std::vector<hipEvent_t> event_pool;

  // row partition + delta exchange
  int xmode = EL_XCHG_NONE;
  uint32_t part_rank = 0, part_count = 1, cfg_lo = 0, cfg_hi = 0;
  uint32_t lo = 0, hi = 0;  // owned rows (whole ontology: [0, N))
  std::unique_ptr<Exchange> xchg;
  bool use_props = false;   // propagation set in use (CR4 axioms, or ⊥ in partitioned mode)
  uint32_t *xlog_x = nullptr, *xlog_p = nullptr;  // replicated chain-second links
  uint64_t xlog_cap = 0, x_count = 0;
  // this step's records for other ranks (routed by the commit, remote()): chain-second links,
  // propagations, activations; sized for a step's candidates (+ the base ones, el_init)
  uint32_t *xs_x = nullptr, *xs_p = nullptr, *xp_p = nullptr, *xp_b = nullptr, *xa_y = nullptr, *xa_c = nullptr;
  uint64_t xs_cap = 0, xp_cap = 0, xa_cap = 0;
  void fit_xqueues(uint64_t xs, uint64_t xp, uint64_t xa);  // (only while they are empty)
  uint2* xwin = nullptr;       // every rank's column window (device; exchange_windows)
  void exchange_windows();     // collective, once per el_load
  uint32_t* sc_own = nullptr;  // partitioned: successor-row capacities of the own rows only (layout)
  uint32_t* xsend = nullptr;                      // exchange slot: XH + 2 * xcap words
  uint32_t* xrecv = nullptr;                      // part_count slots
  uint64_t xcap = 0;                              // records per rank per exchange (grows on overflow)
  uint64_t xspec = 0;                             // records per rank of the next round (exchange_round)
  uint64_t p_import = 0;                          // propagation log: where the last import's records begin
  uint64_t xrounds_bytes = 0;                     // bytes all-gathered (received) since el_init
  bool part() const { return xmode != EL_XCHG_NONE; }
  bool part_fixpoint = false;  // partitioned: the last el_saturate reached the global fixpoint (el_init clears)
  bool bits_logged = false;
  bool trace_xchg = getenv("EL_TRACE_XCHG") != nullptr;    // diagnostic: per-superstep exchange rounds
  bool trace_cands = getenv("EL_TRACE_CANDS") != nullptr;  // every set bit of the matrix is in the fact log (not after el_load)

  // launch shapes (workgroups per role): a workgroup costs dispatch time even when its
  // grid-stride loop is empty, so the capacity-sized roles are capped
  static uint32_t env_u32(const char* n, uint32_t d) {
    const char* e = getenv(n);
    return e ? (uint32_t)std::max(1ul, strtoul(e, nullptr, 10)) : d;
  }
  uint32_t tune_commit = env_u32("EL_COMMIT_BLOCKS", 1024);
  uint32_t tune_expand = env_u32("EL_EXPAND_BLOCKS", 1024);
  uint32_t tune_jobs = env_u32("EL_JOBS_BLOCKS", 1024);
  uint32_t tune_scatter = env_u32("EL_SCATTER_BLOCKS", 512);
  bool small_queues = getenv("EL_QUEUE_CAP") != nullptr;
  bool commit_sort = !getenv("EL_COMMIT_SORT") || getenv("EL_COMMIT_SORT")[0] != '0';
  // workgroups of the summary clear.  It runs beside the told closure (rstream): with 2048
  // workgroups it held every CU and the closure's small launches queued behind it (a 5-µs fill
  // took 615 µs in the trace); 256 leave room (G3 A/B: 25.55 / 25.68 vs 25.86 ms, init 6.38 vs
  // 6.67 ms; 512: 25.83 / 25.93)
  uint32_t clear_grid = getenv("EL_CLEAR_GRID") ? (uint32_t)std::max(1, atoi(getenv("EL_CLEAR_GRID"))) : 256u;
  bool dedup_off = getenv("EL_DEDUP_OFF") != nullptr;  // diagnostic A/B of the in-wave filter  // tests: queues start small, grow only on demand

  DState dstate() const {
    DState s{};
    // virtual row base: row x of the owned range [lo, hi) is bits + (x - lo) * W
    s.bits = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(bits) - (uintptr_t)lo * W * sizeof(uint32_t));
    s.summ = summ ? summ - (uintptr_t)lo * SB : nullptr;
    s.SB = SB;
    s.slog_x = slog_x;
    s.slog_a = slog_a;
    s.slog_f = slog_f;
    s.ct_x = ct_x;
    s.ct_a = ct_a;
    s.ct_cap = (uint32_t)ct_cap;
    s.lhash = lhash;
    s.lmask = lhash_cap - 1;
    s.llog_x = llog_x;
    s.llog_p = llog_p;
    s.ahash = ahash;
    s.amask = ahash_cap - 1;
    s.alog_y = alog_y;
    s.alog_c = alog_c;
    s.has_act = has_act;
    s.act_ptr = act_ptr;
    s.act_k = act_k;
    s.phash = phash;
    s.pmask = phash_cap - 1;
    s.plog_p = plog_p;
    s.plog_b = plog_b;
    s.pp = PP.view(&ctr->ov_pp);
    s.cp_p = cp_p;
    s.cp_b = cp_b;
    s.cp_cap = (uint32_t)cp_cap;
    s.pr = PR.view(&ctr->ov_pr);
    s.sc = SC.view(&ctr->ov_sc);
    s.need_pred = need_pred ? 1u : 0u;
    s.need_succ = need_succ ? 1u : 0u;
    s.dedup = dedup_off ? 0u : 1u;
    s.csort = commit_sort ? 1u : 0u;
    s.lines = lines_dbg;
    s.succ_at_commit = (need_succ && !part()) ? 1u : 0u;
    s.xlog_x = xlog_x;
    s.xlog_p = xlog_p;
    s.xs_x = xs_x;
    s.xs_p = xs_p;
    s.xs_cap = (uint32_t)std::min<uint64_t>(xs_cap, 0xffffffffu);
    s.xp_p = xp_p;
    s.xp_b = xp_b;
    s.xp_cap = (uint32_t)std::min<uint64_t>(xp_cap, 0xffffffffu);
    s.xa_y = xa_y;
    s.xa_c = xa_c;
    s.xa_cap = (uint32_t)std::min<uint64_t>(xa_cap, 0xffffffffu);

    s.cs_x = cs_x;
    s.cs_a = cs_a;
    s.cs_cap = (uint32_t)cs_cap;
    s.cl_x = cl_x;
    s.cl_p = cl_p;
    s.cl_cap = (uint32_t)cl_cap;
    s.ca_y = ca_y;
    s.ca_c = ca_c;
    s.ca_cap = (uint32_t)ca_cap;
    s.jobs = jobs;
    s.job_cap = (uint32_t)job_cap;
    s.ctr = ctr;
    s.ev = ev;
    return s;
  }

  hipEvent_t take_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
  }
  // bracket one kernel launch with HIP events on the launch stream (profile mode)
  template <class F>
  void launch(int k, F&& f) {
    launches[k]++;
    if (!profile) {
      f();
      HIPCHK(hipGetLastError());
      return;
    }
    PendingEvent pe{k, take_event(), take_event()};
    HIPCHK(hipEventRecord(pe.a, stream));
    f();
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(pe.b, stream));
    pending.push_back(pe);
  }
  void sync() {
    HIPCHK(hipStreamSynchronize(stream));
    for (auto& pe : pending) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, pe.a, pe.b));
      kms[pe.kernel] += ms;
      event_pool.push_back(pe.a);
      event_pool.push_back(pe.b);
    }
    pending.clear();
  }
  void read_counters() {
    static thread_local std::vector<uint32_t> tmp(sizeof(DCounters) / 4);
    HIPCHK(hipMemcpy(tmp.data(), ctr, sizeof(DCounters), hipMemcpyDeviceToHost));
    uint32_t* h = reinterpret_cast<uint32_t*>(&hc);
    for (uint32_t i = 0; i < NUM_CTRS; ++i) h[i] = tmp[i * CTR_STRIDE];
  }
  // Wait until k_commit #seq has published the step's counters (the merge kernels of the
  // step may still be running: the next step is enqueued behind them on the stream).
  void wait_commit(uint32_t seq) {
    volatile HCounters* p = hc_pinned;
    for (uint64_t it = 1;; ++it) {
      if (p->seq == seq) break;
      if ((it & 1023) == 0) {  // a faulted or finished stream must not leave us spinning
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) {
          if (p->seq == seq) break;
          throw std::runtime_error("k_commit did not publish its counters");
        }
        if (e != hipErrorNotReady) HIPCHK(e);
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    uint32_t* h = reinterpret_cast<uint32_t*>(&hc);
    const volatile uint32_t* src = reinterpret_cast<const volatile uint32_t*>(hc_pinned);
    for (size_t i = 0; i < NUM_CTRS; ++i) h[i] = src[i];
  }
  // Event counters travel with the stream (pinned target): a caller that syncs anyway
  // enqueues them first and sums after its sync, without a second round trip.
  void enqueue_events() {
    hipLaunchKernelGGL(k_ev_reduce, dim3(EV_TOTAL), dim3(256), 0, stream, ev, ev_sum);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ev_host, ev_sum, EV_TOTAL * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    events_queued = true;
  }
  void read_events() {
    if (!events_queued) enqueue_events();
    sync();
    events_queued = false;
    const unsigned long long* h = ev_host;
    for (int k = 0; k < EL_NUM_KERNELS; ++k)
      for (int e = 0; e < EL_NUM_EVENTS; ++e) hev[k][e] = h[(size_t)k * EL_NUM_EVENTS + e];
  }

  void free_state();
  void free_index();
  void alloc_state();
  void reset_state();
  void ensure_capacity();
  void ensure_rows(bool facts, bool links);
  void readout_rows(uint64_t* dptr, uint64_t* ptr_out, uint32_t* val_out, bool clear, hipEvent_t counted);
  // half: 0 = whole build, 1 = the part that reads the state, 2 = the rest (el_rows.h);
  // clear: the S-row build zeroes the bit matrix as it writes (a releasing copy-back)
  void build_rows(bool facts, hipStream_t s, uint64_t* ptr, uint32_t* dst, int half = 0, bool clear = false);
  hipStream_t rstream = nullptr;  // state reset behind a releasing copy-back; the base links' set fill
  hipEvent_t ev_reset = nullptr;
  hipEvent_t ev_copied[3] = {nullptr, nullptr, nullptr};  // an async copy-back's streams drained
  bool copy_pending = false;
  // (copy_pending is cleared only once every stream has drained: a failed copy keeps failing)
  void wait_copy() {
    if (!copy_pending) return;
    for (hipEvent_t e : ev_copied) HIPCHK(hipEventSynchronize(e));
    copy_pending = false;
  }
  // Streamed result (el_stream_result): the committed segments of the fact and link logs cross
  // PCIe while the saturation goes on: their values (b, pid) by DMA on dstream, their runs of x
  // (el_stream.h) encoded on nstream into device run buffers, which follow by DMA once a later
  // stream_out finds the encoding done (an event query: the host never waits for it there)
  el_stream* strm = nullptr;      // armed for the next el_saturate
  uint64_t strm_s = 0, strm_l = 0;  // log entries already enqueued
  bool strm_ovf = false;          // a buffer was too small (el_result_wait: EL_ERANGE)
  hipEvent_t ev_strm = nullptr;   // recorded right behind a superstep's commit
  bool dma_hostptr = getenv("EL_DMA_HOSTPTR") != nullptr;  // A/B: copies to the host pointers, kind DeviceToHost
  bool strm_marked = false;       // ev_strm was recorded right behind this step's commit
  hipStream_t nstream = nullptr;  // run encoding (never queued behind the DMAs)
  uint2 *s_run_dev = nullptr, *l_run_dev = nullptr;  // device addresses of the caller's run buffers
  uint32_t *s_b_dev = nullptr, *l_p_dev = nullptr;     // ... and of its value buffers (null: pageable)
  uint2 *srun = nullptr, *lrun = nullptr;              // the runs, encoded in device memory
  uint64_t srun_cap = 0, lrun_cap = 0;
  uint64_t run_sent[2] = {0, 0};                       // runs DMA'd so far: S, links
  unsigned long long* rtot_h = nullptr;                // runs encoded so far (mapped, written by the device)
  unsigned long long* rtot_d = nullptr;                // its device address
  hipEvent_t ev_run = nullptr;                         // after the last encoding enqueued
  bool run_pending = false;
  void runs_out(bool wait);
  uint32_t *rcnt = nullptr, *roff = nullptr;  // per-tile run counts / their scan (packed: escapes from rtiles_cap)
  uint64_t rtiles_cap = 0;
  void* rscan_tmp = nullptr;
  size_t rscan_bytes = 0;
  unsigned long long* rbase = nullptr;    // runs written so far: S, links (device)
  void stream_runs(const uint32_t* keys, uint64_t a, uint64_t b, uint2* out, uint64_t cap, int which);
  void stream_tiles(uint64_t nt);  // (the per-tile scratch of the encodings: rcnt, roff)
  // EL_STREAM_PACKED: the facts' values as 16-bit codes (their bit column) + escapes, encoded on
  // nstream beside the runs into device buffers, DMA'd with the runs (runs_out)
  bool packed = false;
  uint16_t* scode = nullptr;           // codes at log positions (device), scode_cap = the caller's s_cap
  uint64_t scode_cap = 0;
  uint32_t* sesc = nullptr;            // escape values (device)
  uint64_t sesc_cap = 0;
  uint16_t* s_code_dev = nullptr;      // device addresses of the caller's code / escape buffers
  uint32_t* s_esc_dev = nullptr;
  uint64_t code_enc = 0, code_sent = 0, esc_sent = 0;  // codes encoded (behind ev_run) / DMA'd; escapes DMA'd
  unsigned long long *ebase = nullptr, *etot_h = nullptr, *etot_d = nullptr;  // escapes written (device / mapped)
  std::vector<uint32_t> code_table;    // code -> concept (el_stream_codes), per index
  void stream_out();    // stream_mark + stream_flush
  void stream_mark();
  // force: flush whatever is marked; else only a segment of stream_min entries or more (a late
  // superstep's few entries wait for a later flush: the host's enqueue work for copies and run
  // encodings — a dozen API calls — would otherwise sit between two short supersteps)
  void stream_flush(bool force = true);
  uint64_t stream_min = env_u32("EL_STREAM_MIN", 1u << 17);
  uint64_t mark_s = 0, mark_l = 0;  // the marked segment ends [strm_s, mark_s), [strm_l, mark_l)
  bool mark_pending = false;
  void stream_end(bool release);
  hipEvent_t ev_base[2] = {nullptr, nullptr};  // base links logged (stream) / in the link set (rstream)
  hipEvent_t ev_init[2] = {nullptr, nullptr};  // closure rows ready (stream) / init facts written (rstream)
  bool base_filling = false;                   // the set fill runs beside the first superstep
  void join_base();
  bool pre_reset = false;         // the device part of the next reset_state is already enqueued
  bool reset_wait = false;        // ... and the engine stream has not waited for it yet
  // clear_from: the first row whose bits the reset clears (lo: all; hi: none — a releasing
  // copy-back cleared the rows it read)
  // summ_from: the first row whose block summary the reset clears (a releasing read-out
  // cleared the summary of the rows it read, and may still be reading it: the reset must not
  // touch those rows)
  void reset_device(hipStream_t s, uint32_t clear_from, uint32_t summ_from);
  void reset_device(hipStream_t s) { reset_device(s, lo, lo); }
  void rehash_links(uint64_t cap);
  void rehash_acts(uint64_t cap);
  void rehash_props(uint64_t cap);
  bool superstep(uint32_t mask, uint64_t sb, uint64_t se, uint64_t lb, uint64_t le, uint64_t ab,
                 uint64_t ae, uint64_t pb, uint64_t pe);
  // partitioned mode: one superstep + the delta exchange; returns Σ over ranks of the deltas
  uint64_t superstep_part(uint32_t mask, uint64_t sb, uint64_t se, uint64_t lb, uint64_t le, uint64_t ab,
                          uint64_t ae, uint64_t pb, uint64_t pe, uint64_t xb, uint64_t xe);
  void grow_part(uint64_t new_xcap);
  uint32_t exchange_round(uint32_t s0, uint32_t l0, uint32_t a0, uint32_t p0, uint32_t x0);
  uint64_t remote_bound() const { return part() ? (uint64_t)(part_count - 1) * xcap : 0u; }
  // successor-row appends of one step: the own new chain links (+ the imported ones)
  uint64_t sc_ovq() const { return cl_cap + (part() ? (uint64_t)part_count * xcap : 0u); }
  void fill_stats(el_stats* st, double ms);
  void gap_relocate_all();
  // relocation counters (device; their published copy in coherent pinned memory + sequence word)
  unsigned long long *reloc_rc = nullptr, *reloc_h = nullptr, *reloc_hd = nullptr;
  unsigned long long reloc_seq = 0;
  void gap_build_from_log(GapCsr& g, const uint32_t* rows, const uint32_t* vals, uint64_t n,
                          const uint8_t* keep = nullptr);
  void gap_build_sorted(GapCsr& g, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t bits);
  void launch_gap_scan(const uint32_t* len, uint32_t R, uint32_t* start_out);
  std::string install_index(el::HostIndex&& h);
  void column_window();
  void migrate_state(uint32_t N0, const std::vector<uint32_t>& pmap, const std::vector<uint8_t>& dA,
                     const std::vector<uint8_t>& dX, const std::vector<uint8_t>& dP);
  el::AxiomStore store;  // the loaded axioms (increments append to them)
  // ELK range fillers (el_index.h elk_ranges): concepts [n_user, N) are internal; the result
  // rows cover the caller's concepts [lo, uhi()) only
  uint32_t n_user = 0;
  std::vector<uint32_t> fresh_b, fresh_r;
  uint32_t uhi() const { return std::max(lo, std::min(hi, n_user)); }
  uint64_t user_count(bool facts);  // facts / links of the result rows (= the log's without fresh rows)
  uint64_t uc_s_n = ~0ull, uc_s = 0, uc_l_n = ~0ull, uc_l = 0;  // (reset with every state and index)
};

// Upload the indexes of hx and derive what the kernels need from them (which CSRs have
// readers, the owned rows).  The state is not touched.
std::string el_ctx::install_index(el::HostIndex&& hnew) {
  hx = std::move(hnew);
  const el::HostIndex& h = hx;
  auto up32 = [&](const std::vector<uint32_t>& v) {
    uint32_t* p = dupload(v);
    index_bufs.push_back(p);
    return (const uint32_t*)p;
  };
  auto up8 = [&](const std::vector<uint8_t>& v) {
    uint8_t* p = dupload(v);
    index_bufs.push_back(p);
    return (const uint8_t*)p;
  };
  DIndex& d = ix;
  d.N = h.N;
  d.R = h.R;
  d.P = h.P;
  d.kind = up8(h.kind);
  d.cidx_ptr = up32(h.cidx.ptr);
  d.cidx_c = up32(h.cidx.a);
  d.conj_ptr = up32(h.conj.ptr);
  d.conj_ops = up32(h.conj.a);
  d.conj_b = up32(h.conj_b);
  d.fp_ptr = up32(h.fp_ptr);
  d.pair_role = up32(h.pair_role);
  d.pair_y = up32(h.pair_y);
  {
    std::vector<uint4> pi(h.P);
    for (uint32_t q = 0; q < h.P; ++q) pi[q] = make_uint4(h.pair_role[q], h.pair_y[q], h.psup.ptr[q], h.psup.ptr[q + 1]);
    uint4* pp = dupload(pi);
    index_bufs.push_back(pp);
    d.pinfo = pp;
  }
  d.psup_ptr = up32(h.psup.ptr);
  d.psup_pid = up32(h.psup.a);
  d.chf_ptr = up32(h.chf.ptr);
  d.chf_s = up32(h.chf.a);
  d.chf_t = up32(h.chf.b);
  d.chs_ptr = up32(h.chs.ptr);
  d.chs_p = up32(h.chs.a);
  d.chs_t = up32(h.chs.b);
  d.dom_ptr = up32(h.dom.ptr);
  d.dom_c = up32(h.dom.a);
  d.rng_ptr = up32(h.rng.ptr);
  d.rng_c = up32(h.rng.a);
  d.role_has_exl = up8(h.role_has_exl);
  {  // the told axiom rows the device closure is built from (el_closure.h)
    elcl::Axioms& a = cax;
    a.N = h.N;
    a.P = h.P;
    a.par_ptr = up32(h.told.ptr);
    a.par = up32(h.told.a);
    a.chi_ptr = up32(h.toldT.ptr);
    a.chi = up32(h.toldT.a);
    a.xr_ptr = up32(h.exr.ptr);
    a.xr = up32(h.exr.a);
    a.xl_ptr = up32(h.exl.ptr);
    a.xl_r = up32(h.exl.a);
    a.xl_b = up32(h.exl.b);
    a.cidx_ptr = d.cidx_ptr;
    a.psup_ptr = d.psup_ptr;
    a.sc_self = up8(h.sc_self);
    a.sc_w = up32(h.sc_w);
    {
      std::vector<uint2> ps(h.P);
      for (uint32_t q = 0; q < h.P; ++q)
        ps[q] = make_uint2(h.sc_w[q], ((h.psup.ptr[q + 1] - h.psup.ptr[q]) << 1) | (h.sc_self[q] ? 1u : 0u));
      std::vector<uint32_t> cz(h.N);
      for (uint32_t q = 0; q < h.N; ++q) cz[q] = h.cidx.ptr[q + 1] - h.cidx.ptr[q];
      uint2* pp = dupload(ps);
      index_bufs.push_back(pp);
      a.pstat = pp;
      a.cz = up32(cz);
    }
    a.fp_ptr = d.fp_ptr;
    a.pair_role = d.pair_role;
    a.kind = d.kind;
    caxk = a;
    if (!h.scc_rep.empty()) {  // told cycles: the levels run over the condensed told graph
      caxk.par_ptr = up32(h.told_c.ptr);
      caxk.par = up32(h.told_c.a);
      caxk.chi_ptr = up32(h.toldT_c.ptr);
      caxk.chi = up32(h.toldT_c.a);
      caxk.xr_ptr = up32(h.exr_c.ptr);
      caxk.xr = up32(h.exr_c.a);
      caxk.xl_ptr = up32(h.exl_c.ptr);
      caxk.xl_r = up32(h.exl_c.a);
      caxk.xl_b = up32(h.exl_c.b);
      caxk.rep = up32(h.scc_rep);
      caxk.tx_ptr = up32(h.told_x.ptr);
      caxk.tx = up32(h.told_x.a);
      caxk.fol = up32(h.followers);
      caxk.nfol = (uint32_t)h.followers.size();
    }
    key_bits = 1;
    while (key_bits < 32 && (1ull << key_bits) < h.P) ++key_bits;
  }
  uc_s_n = uc_l_n = ~0ull;
  {  // link export order: pair ids ranked by (role, filler)
    std::vector<uint32_t> ord(h.P), rank(h.P);
    std::iota(ord.begin(), ord.end(), 0u);
    std::sort(ord.begin(), ord.end(), [&](uint32_t u, uint32_t v) {
      return h.pair_role[u] != h.pair_role[v] ? h.pair_role[u] < h.pair_role[v] : h.pair_y[u] < h.pair_y[v];
    });
    rank_role.resize(h.P);
    rank_y.resize(h.P);
    for (uint32_t q = 0; q < h.P; ++q) {
      rank[ord[q]] = q;
      rank_role[q] = h.pair_role[ord[q]];
      rank_y[q] = h.pair_y[ord[q]];
    }
    pid_rank = up32(rank);
  }
  d.has_range = h.rng.a.empty() ? 0u : 1u;
  {
    // ⊥ derivable only if some axiom mentions it (as a conclusion or a CR3 filler)
    auto has0 = [](const std::vector<uint32_t>& v) { return std::find(v.begin(), v.end(), EL_BOTTOM) != v.end(); };
    const bool bot = has0(store.sub_b) || has0(store.conj_b) || has0(store.exr_b) || has0(store.exl_b) ||
                     has0(store.dom_c) || has0(store.rng_c);
    need_succ = !h.chf.a.empty();
    need_pred = !h.exl.a.empty() || need_succ || bot;
    ix.has_bot = bot ? 1u : 0u;
    use_props = !h.exl.a.empty() || (part() && bot);
  }
  // owned rows: the configured range, or the equal split of [0, N)
  if (part()) {
    if (cfg_lo == 0 && cfg_hi == 0) {
      lo = (uint32_t)((uint64_t)h.N * part_rank / part_count);
      hi = (uint32_t)((uint64_t)h.N * (part_rank + 1) / part_count);
    } else {
      if (cfg_hi > h.N) return "partition rows beyond n_concepts";
      lo = cfg_lo;
      hi = cfg_hi == n_user ? h.N : cfg_hi;  // the last rank also owns the ELK range fillers
    }
  } else {
    lo = 0;
    hi = h.N;
  }
  if (part() || need_succ) {  // chain-second roles: their links are exchanged and feed the succ rows
    std::vector<uint8_t> chs(h.R + 1, 0);
    for (uint32_t r = 0; r < h.R; ++r) chs[r] = h.chs.ptr[r + 1] > h.chs.ptr[r];
    d.role_chs = up8(chs);
  } else {
    d.role_chs = nullptr;
  }
  d.lo = lo;
  d.hi = hi;
  column_window();
  // the column order (el_index.h column_order; EL_COLUMN_ORDER=0: id order, a diagnostic): a
  // whole ontology's, or a partition's over its own column window
  static const bool col_order = !getenv("EL_COLUMN_ORDER") || getenv("EL_COLUMN_ORDER")[0] != '0';
  d.cperm = nullptr;
  std::vector<uint32_t> perm;
  if (col_order && !part() && h.cperm.size() == h.N && ix.c_lo == 2u)
    perm = h.cperm;
  else if (col_order && part() && h.cscore.size() == h.N && ix.c_hi > ix.c_lo)
    perm = el::column_perm(h, ix.c_lo, ix.c_hi);
  if (!perm.empty()) d.cperm = up32(perm);
  cax.cperm = caxk.cperm = d.cperm;
  {  // code -> concept of a packed stream: the concept of bit column c < 0xFFFF (elst::code_of)
    code_table.assign(elst::CODE_ESC, NONE);
    for (uint32_t a = 0; a < h.N; ++a) {
      const uint32_t c = a < 2u ? a : (a < ix.c_lo || a >= ix.c_hi) ? NONE : perm.empty() ? a - ix.c_lo + 2u : perm[a];
      if (c < elst::CODE_ESC) code_table[c] = a;
    }
  }
  {  // binary conjunctions per cidx entry, with the bit columns of p and B (DIndex::cidx_q)
    auto col = [&](uint32_t a) -> uint32_t {  // (col_of on the host)
      if (a < 2u) return a;
      if (a < ix.c_lo || a >= ix.c_hi) return NONE;
      return d.cperm ? perm[a] : a - ix.c_lo + 2u;
    };
    std::vector<uint4> cq(std::max<size_t>(h.cidx.a.size(), 1), make_uint4(NONE, 0u, NONE, NONE));
    for (uint32_t a = 0; a < h.N; ++a)
      for (uint32_t j = h.cidx.ptr[a]; j < h.cidx.ptr[a + 1]; ++j) {
        const uint32_t c = h.cidx.a[j], o0 = h.conj.ptr[c];
        cq[j].y = h.conj_b[c];
        if (h.conj.ptr[c + 1] - o0 != 2 || h.N > 0x7fffffffu) continue;
        const uint32_t u = h.conj.a[o0], v = h.conj.a[o0 + 1];  // (sorted, distinct)
        if (u != a && v != a) continue;
        const uint32_t p = a == u ? v : u;
        cq[j] = make_uint4(a == u ? v : u | 0x80000000u, h.conj_b[c], col(p), col(h.conj_b[c]));
      }
    uint4* pq = dupload(cq);
    index_bufs.push_back(pq);
    d.cidx_q = pq;
  }
  d.part = part() ? 1u : 0u;
  d.xwin = nullptr;  // (the windows of the other ranks: exchange_windows, at the first el_saturate)
  d.nranks = part() ? part_count : 1u;
  d.me = part_rank;
  static_levels();
  return "";
}

// The Kahn levels of the told closure are a property of the told axioms and of the built window:
// computed here once per index (O(N + told edges) on the host), uploaded as each concept's level
// and the concepts of every level >= 1 in level order (elcl::Axioms::slevel / lvl_ids).  The same
// marks as k_start: ⊥ / ⊤ and the window built, a told cycle's follower FOLLOW, level 0 without
// condensed supers (1 for a representative with members), else 1 + the largest super level; a
// concept never reached (a super outside the window) stays NONE and goes to the relaxation.
void el_ctx::static_levels() {
  lvl_ptr.clear();
  caxk.slevel = caxk.lvl_ids = nullptr;
  static const bool dynamic = getenv("EL_DYNAMIC_LEVELS") && getenv("EL_DYNAMIC_LEVELS")[0] == '1';
  if (dynamic) return;
  const el::HostIndex& h = hx;
  const uint32_t N = h.N;
  const bool scc = !h.scc_rep.empty();
  const el::Csr& par = scc ? h.told_c : h.told;
  const el::Csr& chi = scc ? h.toldT_c : h.toldT;
  const uint32_t w_lo = part() ? ix.c_lo : 2u, w_hi = part() ? ix.c_hi : 0xffffffffu;
  std::vector<uint32_t> lev(N), pend(N, 0), stk;
  for (uint32_t A = 0; A < N; ++A) {
    const bool in = A < 2u || (A >= w_lo && A < w_hi);
    const bool fol = scc && h.scc_rep[A] != A;
    const uint32_t d = par.ptr[A + 1] - par.ptr[A];
    const bool xt = scc && h.told_x.ptr[A + 1] > h.told_x.ptr[A];
    lev[A] = !in ? elcl::LVL_SKIP : fol ? elcl::LVL_FOLLOW : d ? elcl::LVL_NONE : xt ? 1u : 0u;
    pend[A] = (in && !fol) ? d : 0u;
    if (lev[A] == 0u || lev[A] == 1u) stk.push_back(A);
  }
  std::vector<uint32_t> cand(N, 0);
  uint32_t depth = 0;
  while (!stk.empty()) {  // (any order: a concept is pushed once, when its last super is done)
    const uint32_t A = stk.back();
    stk.pop_back();
    depth = std::max(depth, lev[A]);
    for (uint32_t j = chi.ptr[A]; j < chi.ptr[A + 1]; ++j) {
      const uint32_t c = chi.a[j];
      if (lev[c] != elcl::LVL_NONE) continue;  // (skipped, followers)
      cand[c] = std::max(cand[c], lev[A] + 1);
      if (--pend[c] == 0) {
        lev[c] = cand[c];
        stk.push_back(c);
      }
    }
  }
  lvl_ptr.assign(depth + 2, 0);
  for (uint32_t A = 0; A < N; ++A)
    if (lev[A] >= 1u && lev[A] <= depth) lvl_ptr[lev[A] + 1]++;
  for (uint32_t L = 0; L <= depth; ++L) lvl_ptr[L + 1] += lvl_ptr[L];
  std::vector<uint32_t> ids(std::max<uint32_t>(lvl_ptr[depth + 1], 1)), at(lvl_ptr.begin(), lvl_ptr.end() - 1);
  for (uint32_t A = 0; A < N; ++A)
    if (lev[A] >= 1u && lev[A] <= depth) ids[at[lev[A]]++] = A;
  auto up = [&](const std::vector<uint32_t>& v) {
    uint32_t* p = dupload(v);
    index_bufs.push_back(p);
    return (const uint32_t*)p;
  };
  caxk.slevel = up(lev);
  caxk.lvl_ids = up(ids);
}

// Every rank's column window, all-gathered once per el_load (the first el_saturate: collective).
// A record keyed by concept y (a propagation ((r, y), B), an activation (y, C), a chain-second
// link (y, s, z)) can only matter to a rank whose rows can reach y — y in its window — so the
// commit routes to the exchange only those some other rank's window holds (remote()).  For
// OntologyMultiplier copies aligned with the partition nothing crosses but the header words.
void el_ctx::exchange_windows() {
  if (ix.xwin || part_count < 2) {
    if (!ix.xwin) ix.nranks = 1;
    return;
  }
  uint32_t* buf = dalloc<uint32_t>(4 + 4 * (uint64_t)part_count);
  index_bufs.push_back(buf);
  const uint32_t mine[4] = {ix.c_lo, ix.c_hi, lo, hi};
  HIPCHK(hipMemcpyAsync(buf, mine, sizeof mine, hipMemcpyHostToDevice, stream));
  xchg->allgather(buf, buf + 4, 4 * sizeof(uint32_t), stream);
  std::vector<uint32_t> all(4 * (uint64_t)part_count);
  HIPCHK(hipMemcpyAsync(all.data(), buf + 4, all.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  std::vector<uint32_t> win(2 * (uint64_t)part_count);
  for (uint32_t q = 0; q < part_count; ++q) {
    win[2 * q] = all[4 * q];
    win[2 * q + 1] = all[4 * q + 1];
  }
  uint32_t* d = dupload(win);
  index_bufs.push_back(d);
  ix.xwin = reinterpret_cast<const uint2*>(d);
}

void el_ctx::fit_xqueues(uint64_t xs, uint64_t xp, uint64_t xa) {
  auto fit = [&](uint64_t want, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
    if (want <= cap && a) return;
    HIPCHK(hipStreamSynchronize(stream));
    dfree(a);
    dfree(b);
    cap = std::max<uint64_t>(want, 1024);
    a = dalloc<uint32_t>(cap);
    b = dalloc<uint32_t>(cap);
  };
  fit(xs, xs_cap, xs_x, xs_p);
  fit(xp, xp_cap, xp_p, xp_b);
  fit(xa, xa_cap, xa_y, xa_c);
}

// Bit-row columns of this context (SURVEY.md §7 "hard parts": columns compacted per
// partition).  A whole-ontology context keeps column = concept id.  A partition keeps ⊥, ⊤
// and the id window spanning every concept an owned row can ever hold: the closure of the
// owned rows under the ways a concept enters S(X) — told supers (CR1), conjunctions with an
// operand in it (CR2), the fillers of its existentials (CR4 reads S(Y) of a filler Y), the B
// of ∃r.A ⊑ B for A in it (CR4), the domains and ranges of every role its links can carry
// (CR3, CR5 supers, CR6 results), and the ranges of every role a link into it can carry
// (DistEL's range rule puts them into each S(X) that holds the link's target).  For OntologyMultiplier copies aligned with the partition
// (G4) the window is the rank's own copy: 8 × 19 GB for SNOMED×8 instead of 8 × 152 GB.
void el_ctx::column_window() {
  const el::HostIndex& h = hx;
  uint32_t c_lo = 2, c_hi = std::max<uint32_t>(h.N, 2);
  if (part()) {
    std::vector<uint8_t> seen(h.N, 0), role_seen(h.R + 1, 0);
    std::vector<uint32_t> st, rst;
    auto add = [&](uint32_t a) {
      if (!seen[a]) seen[a] = 1, st.push_back(a);
    };
    auto add_role = [&](uint32_t r) {
      if (!role_seen[r]) role_seen[r] = 1, rst.push_back(r);
    };
    for (uint32_t x = lo; x < hi; ++x) add(x);
    add(EL_BOTTOM);
    add(EL_TOP);
    while (!st.empty() || !rst.empty()) {
      if (!st.empty()) {
        const uint32_t a = st.back();
        st.pop_back();
        for (uint32_t j = h.told.ptr[a]; j < h.told.ptr[a + 1]; ++j) add(h.told.a[j]);
        for (uint32_t j = h.cidx.ptr[a]; j < h.cidx.ptr[a + 1]; ++j) add(h.conj_b[h.cidx.a[j]]);
        for (uint32_t j = h.exr.ptr[a]; j < h.exr.ptr[a + 1]; ++j) {
          const uint32_t p = h.exr.a[j];
          add(h.pair_y[p]);
          add_role(h.pair_role[p]);
          for (uint32_t k = h.psup.ptr[p]; k < h.psup.ptr[p + 1]; ++k) add_role(h.pair_role[h.psup.a[k]]);
        }
        for (uint32_t j = h.exl.ptr[a]; j < h.exl.ptr[a + 1]; ++j) add(h.exl.b[j]);
        // range (DistEL, H1): a link into a — made on any rank — puts rng(r) into every S(X)
        // holding a
        for (uint32_t q = h.fp_ptr[a]; q < h.fp_ptr[a + 1]; ++q) {
          const uint32_t r = h.pair_role[q];
          for (uint32_t j = h.rng.ptr[r]; j < h.rng.ptr[r + 1]; ++j) add(h.rng.a[j]);
        }
        continue;
      }
      const uint32_t r = rst.back();
      rst.pop_back();
      for (uint32_t j = h.chf.ptr[r]; j < h.chf.ptr[r + 1]; ++j) add_role(h.chf.b[j]);
      for (uint32_t j = h.chs.ptr[r]; j < h.chs.ptr[r + 1]; ++j) add_role(h.chs.b[j]);
      for (uint32_t j = h.dom.ptr[r]; j < h.dom.ptr[r + 1]; ++j) add(h.dom.a[j]);
      for (uint32_t j = h.rng.ptr[r]; j < h.rng.ptr[r + 1]; ++j) add(h.rng.a[j]);
    }
    c_lo = h.N, c_hi = 2;
    for (uint32_t a = 2; a < h.N; ++a)
      if (seen[a]) c_lo = std::min(c_lo, a), c_hi = a + 1;
    if (c_hi <= c_lo) c_lo = c_hi = 2;
  }
  ix.c_lo = c_lo;
  ix.c_hi = c_hi;
  // words per bit row, padded to 16 B (the S-row read-out streams rows with 16-B loads).  Not
  // to whole 64-B lines: a row stride with a large power-of-two factor maps one column of
  // every row onto a few L2 channels, and the CR4 fan-out walks columns (G3 with 64-B rows:
  // +10 % saturation time)
  ix.W = (((uint64_t)2 + (c_hi - c_lo) + 31) / 32 + 3) & ~3ull;
}

void el_ctx::free_index() {
  for (void* p : index_bufs) (void)hipFree(p);
  index_bufs.clear();
}

void el_ctx::free_state() {
  if (rstream) (void)hipStreamSynchronize(rstream);  // a reset behind a releasing copy-back
  pre_reset = false;
  free_closure();
  dfree(bits);
  dfree(summ);
  dfree(slog_x);
  dfree(slog_a);
  dfree(slog_f);
  dfree(ct_x);
  dfree(ct_a);
  dfree(lhash);
  dfree(llog_x);
  dfree(llog_p);
  dfree(ahash);
  dfree(alog_y);
  dfree(alog_c);
  dfree(has_act);
  dfree(phash);
  dfree(plog_p);
  dfree(plog_b);
  dfree(cp_p);
  dfree(cp_b);
  for (uint32_t** p : {&rt_x, &rt_a, &rt_lx, &rt_lp}) dfree(*p);
  dfree(rt_f);
  rt_ns = rt_nl = rt_scap = rt_lcap = 0;
  inc_pending = false;
  pend_dA.clear();
  pend_dX.clear();
  pend_dP.clear();
  rs.release();
  rl.release();
  if (dstream) (void)hipStreamSynchronize(dstream);
  for (uint32_t*& p : stage) dfree(p);
  stage_cap = 0;
  rsc.release();
  rsc_l.release();
  asc.release();
  dfree(act_ptr);
  dfree(act_k);
  act_k_cap = 0;
  act_n = ~0ull;
  PR.release();
  SC.release();
  PP.release();
  dfree(cs_x);
  dfree(cs_a);
  dfree(cl_x);
  dfree(cl_p);
  dfree(ca_y);
  dfree(ca_c);
  dfree(jobs);
  dfree(ctr);
  if (hc_pinned) (void)hipHostFree(hc_pinned);
  hc_pinned = nullptr;
  dfree(ev_sum);
  dfree(lines_dbg);
  if (ev_host) (void)hipHostFree(ev_host);
  ev_host = nullptr;
  events_queued = false;
  dfree(ev);
  dfree(scan_flags);
  dfree(commit_done);
  dfree(xlog_x);
  dfree(xlog_p);
  dfree(xs_x);
  dfree(xs_p);
  dfree(xp_p);
  dfree(xp_b);
  dfree(xa_y);
  dfree(xa_c);
  xs_cap = xp_cap = xa_cap = 0;
  dfree(sc_own);
  dfree(xsend);
  dfree(xrecv);
  if (pin_word) (void)hipHostFree(pin_word);
  pin_word = nullptr;
}

void el_ctx::alloc_state() {
  const uint64_t N = hx.N, P = hx.P;
  W = ix.W;  // bit-row words: ⊥, ⊤ and the column window
  bits = dalloc<uint32_t>((uint64_t)(hi - lo) * W);  // owned rows only
  SB = summ_stride(W);
  summ = no_summary ? nullptr : dalloc<uint8_t>((uint64_t)(hi - lo) * SB);
  bits_logged = false;
  // Capacities follow the owned rows (a partition of a ×8 ontology holds one copy's rows: its
  // queues and logs are sized for those, not for the whole index it loads).  What the first
  // superstep needs depends on the told closure, which only el_init derives: closure_state
  // grows the logs and queues to it (grow-only, so later classifications allocate nothing).
  const uint64_t Nown = hi - lo;
  slog_cap = std::max<uint64_t>(1u << 20, 8 * Nown);
  slog_x = dalloc<uint32_t>(slog_cap);
  slog_a = dalloc<uint32_t>(slog_cap);
  slog_f = dalloc<uint8_t>(slog_cap);
  llog_cap = std::max<uint64_t>(1u << 20, 4 * Nown);
  llog_x = dalloc<uint32_t>(llog_cap);
  llog_p = dalloc<uint32_t>(llog_cap);
  lhash_cap = next_pow2(2 * llog_cap);
  lhash = dalloc<unsigned long long>(lhash_cap);
  alog_cap = 1u << 12;
  alog_y = dalloc<uint32_t>(alog_cap);
  alog_c = dalloc<uint32_t>(alog_cap);
  ahash_cap = next_pow2(2 * alog_cap);
  ahash = dalloc<unsigned long long>(ahash_cap);
  has_act = dalloc<uint8_t>(N);
  plog_cap = std::max<uint64_t>(1u << 16, P);
  plog_p = dalloc<uint32_t>(plog_cap);
  plog_b = dalloc<uint32_t>(plog_cap);
  phash_cap = next_pow2(2 * plog_cap);
  phash = dalloc<unsigned long long>(phash_cap);
  cp_cap = plog_cap;
  cp_p = dalloc<uint32_t>(cp_cap);
  cp_b = dalloc<uint32_t>(cp_cap);
  cs_cap = std::max<uint64_t>(1u << 20, 4 * Nown);
  cl_cap = std::max<uint64_t>(1u << 20, 4 * Nown);
  if (const char* e = getenv("EL_QUEUE_CAP")) {  // tests: small queues force overflowing steps
    cs_cap = cl_cap = std::max<uint64_t>(256, next_pow2(strtoull(e, nullptr, 10)));
  }
  if (part()) {
    // records per rank per all-gather; grows on demand (EL_XCHG_CAP: a smaller start, tests)
    xcap = 1u << 12;
    if (const char* e = getenv("EL_XCHG_CAP")) xcap = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
  }
  // gapped CSRs, only where the rules read them; overflow queues hold a step's appends.  Their
  // initial layouts are laid per classification (closure_state): rows sized for the first
  // supersteps' links (the base links and their CR5 lifts, the base propagations), as the oracle
  // sizes its rows (el_oracle.c, elo_create), so no early re-layout is needed
  if (P && need_pred) PR.alloc((uint32_t)P, cl_cap);
  if (need_succ) SC.alloc((uint32_t)N, cl_cap + (part() ? (uint64_t)part_count * xcap : 0));
  if (use_props) PP.alloc((uint32_t)P, cp_cap + remote_bound());
  HIPCHK(hipHostMalloc((void**)&pin_word, sizeof(uint32_t), hipHostMallocDefault));
  // range activation candidates: a new link (X, r, Y) emits one (Y, C) per C ∈ rng(r), so a
  // step's links bound them; an undersized queue would re-run a whole generation
  ca_cap = 1u << 12;
  max_rng = 0;
  for (uint32_t r = 0; r < hx.R && !hx.rng.a.empty(); ++r) max_rng = std::max(max_rng, hx.rng.ptr[r + 1] - hx.rng.ptr[r]);
  ca_cap = std::max<uint64_t>(ca_cap, next_pow2(cl_cap * max_rng));
  cs_x = dalloc<uint32_t>(cs_cap);
  cs_a = dalloc<uint32_t>(cs_cap);
  ct_cap = cs_cap;
  ct_x = dalloc<uint32_t>(ct_cap);
  ct_a = dalloc<uint32_t>(ct_cap);
  cl_x = dalloc<uint32_t>(cl_cap);
  cl_p = dalloc<uint32_t>(cl_cap);
  ca_y = dalloc<uint32_t>(ca_cap);
  ca_c = dalloc<uint32_t>(ca_cap);
  job_cap = std::max<uint64_t>(1u << 20, 2 * Nown);
  jobs = dalloc<uint4>(job_cap);
  ctr = dalloc<DCounters>(1);
  // coherent: k_commit's stores reach the host while later kernels of the step still run
  HIPCHK(hipHostMalloc((void**)&hc_pinned, sizeof(HCounters), hipHostMallocCoherent | hipHostMallocMapped));
  memset(hc_pinned, 0, sizeof(HCounters));
  commit_seq = 0;
  ev = dalloc<unsigned long long>(EV_WORDS);
  ev_sum = dalloc<unsigned long long>(EV_TOTAL);
  if (trace_cands) {
    lines_dbg = dalloc<unsigned long long>(3);
    HIPCHK(hipMemset(lines_dbg, 0, 3 * sizeof(unsigned long long)));
  }
  HIPCHK(hipHostMalloc((void**)&ev_host, EV_TOTAL * sizeof(unsigned long long), hipHostMallocDefault));
  HIPCHK(hipHostGetDevicePointer((void**)&hc_dev, hc_pinned, 0));
  scan_tiles = 0;
  scan_tiles = (std::max(N, P) + 1 + SCAN_TILE - 1) / SCAN_TILE;  // a gapped CSR re-layout
  scan_flags = dalloc<unsigned long long>(scan_tiles);
  commit_done = dalloc<uint32_t>((DONE_SHARDS + 1) * CTR_STRIDE);
  HIPCHK(hipMemset(scan_flags, 0, scan_tiles * sizeof(unsigned long long)));
  scan_epoch = 0;
  if (part()) {
    xlog_cap = std::max<uint64_t>(1u << 16, (uint64_t)part_count * xcap);
    xlog_x = dalloc<uint32_t>(xlog_cap);
    xlog_p = dalloc<uint32_t>(xlog_cap);
    fit_xqueues(cl_cap, cp_cap, ca_cap);
    xsend = dalloc<uint32_t>(XH + 2 * xcap);
    xrecv = dalloc<uint32_t>((uint64_t)part_count * (XH + 2 * xcap));
  }
  alloc_closure();
}

// The device part of reset_state on stream s: clear the bit matrix (by the fact log), the
// sets and counters.  Reads only the logs and counts of the finished state.  (The gapped rows
// get this classification's layout from el_init's closure_state.)
void el_ctx::reset_device(hipStream_t stream, uint32_t clear_from, uint32_t summ_from) {
  FillArgs f{};
  auto add = [&](void* p, uint64_t bytes, uint32_t pattern) { f.seg[f.n++] = FillSeg{p, bytes, pattern}; };
  auto flush = [&]() {
    if (!f.n) return;
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(BLOCK), 0, stream, f);
    HIPCHK(hipGetLastError());
    f.n = 0;
  };
  // The matrix first, then the sets and counters (A/B on G3, the told closure beside the reset:
  // the sets first 23.91 / 23.79 vs 23.81 / 23.68 ms, `EL_RESET_SETS_FIRST=1`)
  static const bool clear_first = getenv("EL_RESET_SETS_FIRST") == nullptr;
  auto sets = [&]() {
    // the link set is by far the largest (G3: 2 GB): the runtime's fill reaches a higher write
    // rate than k_fill's grid-stride loop for it (k_fill: 2.0 ms per G3 classification); the
    // activation and propagation sets go with the counters in one k_fill (A/B with the runtime
    // fill for them too: 23.73–23.97 vs 23.95–24.10 ms, `profiles/r04_clear_kernel_ab.txt`)
    if (lhash_cap * sizeof(unsigned long long) >= (64ull << 20))
      HIPCHK(hipMemsetAsync(lhash, 0xff, lhash_cap * sizeof(unsigned long long), stream));
    else
      add(lhash, lhash_cap * sizeof(unsigned long long), ~0u);
    add(ahash, ahash_cap * sizeof(unsigned long long), ~0u);
    add(phash, phash_cap * sizeof(unsigned long long), ~0u);
    add(has_act, hx.N, 0u);
    add(ctr, sizeof(DCounters), 0u);
    add(commit_done, (DONE_SHARDS + 1) * CTR_STRIDE * sizeof(uint32_t), 0u);
    add(ev, EV_WORDS * sizeof(unsigned long long), 0u);
    flush();
  };
  if (!clear_first) sets();
  const uint64_t matrix_bytes = (uint64_t)(hi - lo) * W * sizeof(uint32_t);
  if (clear_from >= hi) {
    // the releasing copy-back zeroed the matrix as it read the rows
  } else if (bits_logged && summ && summ_from == clear_from && !getenv("EL_CLEAR_LOGGED")) {
    // by the block summary (it marks every block holding a bit, whoever set it, once the matrix
    // was cleared whole: bits_logged); clears the summary of those rows too
    const uint64_t r0 = clear_from - lo;
    hipLaunchKernelGGL(k_clear_summ, dim3(clear_grid), dim3(BLOCK), 0, stream, bits + r0 * W, (uint64_t)W, summ + r0 * SB,
                       SB, (uint64_t)(hi - clear_from));
    HIPCHK(hipGetLastError());
    summ_from = hi;
  } else if (bits_logged && (clear_from > lo || s_count * 64 < matrix_bytes)) {
    // one 64-B line per logged fact (of the rows still set) vs. the whole matrix
    hipLaunchKernelGGL(k_clear_logged, dim3(grid_for(s_count)), dim3(BLOCK), 0, stream, ix, dstate().bits, slog_x,
                       slog_a, (uint32_t)s_count, clear_from);
    HIPCHK(hipGetLastError());
  } else {
    add(bits, matrix_bytes, 0u);
  }
  if (summ && summ_from < hi)  // (whichever way the bits were cleared)
    add(summ + (uint64_t)(summ_from - lo) * SB, (uint64_t)(hi - summ_from) * SB, 0u);
  flush();
  if (clear_first) sets();
}

void el_ctx::reset_state() {
  if (pre_reset) {  // done behind the copy-back that released the state (el_copy_result)
    // the told closure (el_init's first part) touches none of what the reset clears: the
    // engine stream waits for the reset only before the init facts (closure_state), so the
    // reset's matrix clear runs beside the closure build
    reset_wait = true;
    pre_reset = false;
  } else {
    reset_device(stream);
  }
  bits_logged = true;  // from here on every set bit is in the fact log (the init facts and k_commit append)
  // an increment carried over into the state this reset discards re-triggers nothing: the next
  // el_saturate starts from the fresh init facts (round-5 advisor: a stale re-trigger step ran here)
  inc_pending = false;
  rt_ns = rt_nl = 0;
  pend_dA.clear();
  pend_dX.clear();
  pend_dP.clear();
  uc_s_n = uc_l_n = ~0ull;
  s_count = l_count = a_count = p_count = s_init = x_count = 0;
  part_fixpoint = false;
  if (base_filling) HIPCHK(hipStreamWaitEvent(stream, ev_base[1], 0));  // (an interrupted saturation)
  base_filling = false;
  l_base = p_base = 0;
  ix.base = 0;
  rs.n = rl.n = ~0ull;  // result rows are stale
  act_n = ~0ull;
  for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) wm_s[r] = wm_l[r] = wm_a[r] = wm_p[r] = 0;
  wm_x = 0;
  xrounds_bytes = 0;
  xspec = 0;
  p_import = 0;
  memset(launches, 0, sizeof launches);
  memset(host_ev, 0, sizeof host_ev);
  memset(kms, 0, sizeof kms);
  tr_s.clear();
  tr_l.clear();
  tr_a.clear();
}

void el_ctx::rehash_links(uint64_t cap) {
  if (base_filling) HIPCHK(hipEventSynchronize(ev_base[1]));  // (not while the set fill writes it)
  dfree(lhash);
  lhash_cap = cap;
  lhash = dalloc<unsigned long long>(cap);
  HIPCHK(hipMemsetAsync(lhash, 0xff, cap * sizeof(unsigned long long), stream));
  if (l_count > l_base)  // the base links stay out of the set
    launch(EL_K_REHASH, [&] {
      hipLaunchKernelGGL(k_rehash, dim3(grid_for(l_count - l_base)), dim3(BLOCK), 0, stream, lhash, cap - 1,
                         llog_x + l_base, llog_p + l_base, (uint32_t)(l_count - l_base));
    });
}

void el_ctx::rehash_acts(uint64_t cap) {
  dfree(ahash);
  ahash_cap = cap;
  ahash = dalloc<unsigned long long>(cap);
  HIPCHK(hipMemsetAsync(ahash, 0xff, cap * sizeof(unsigned long long), stream));
  if (a_count)
    launch(EL_K_REHASH, [&] {
      hipLaunchKernelGGL(k_rehash, dim3(grid_for(a_count)), dim3(BLOCK), 0, stream, ahash, cap - 1,
                         alog_y, alog_c, (uint32_t)a_count);
    });
}

void el_ctx::rehash_props(uint64_t cap) {
  if (base_filling) HIPCHK(hipEventSynchronize(ev_base[1]));  // (not while the set fill writes it)
  dfree(phash);
  phash_cap = cap;
  phash = dalloc<unsigned long long>(cap);
  HIPCHK(hipMemsetAsync(phash, 0xff, cap * sizeof(unsigned long long), stream));
  if (p_count > p_base)  // the base propagations stay out of the set
    launch(EL_K_REHASH, [&] {
      hipLaunchKernelGGL(k_rehash, dim3(grid_for(p_count - p_base)), dim3(BLOCK), 0, stream, phash, cap - 1,
                         plog_b + p_base, plog_p + p_base, (uint32_t)(p_count - p_base));
    });
}

// The activation index (expand_s / expand_a read it): the activation log's entries by Y.
// Rebuilt before a generation whenever activations were added (a few supersteps at most).
void el_ctx::refresh_acts() {
  if (hx.rng.a.empty() || act_n == a_count) return;
  if (!act_ptr) act_ptr = dalloc<uint64_t>((uint64_t)hx.N + 1);
  if (a_count > act_k_cap || !act_k) {
    dfree(act_k);
    act_k_cap = std::max<uint64_t>(alog_cap, a_count);
    act_k = dalloc<uint32_t>(act_k_cap);
  }
  elrows::build(stream, asc, alog_y, nullptr, a_count, 0, hx.N, nullptr, act_ptr, act_k, elrows::Clear{});
  act_n = a_count;
}

// entries of a log whose row is below `limit` (the caller's rows when ELK range fillers exist)
__global__ void k_count_below(const uint32_t* __restrict__ rows, uint64_t n, uint32_t limit,
                              unsigned long long* __restrict__ out) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += rows[i] < limit;
  c = wave_sum_u64(c);
  if (__lane_id() == 0 && c) atomicAdd(out, c);
}

uint64_t el_ctx::user_count(bool facts) {
  const uint64_t n = facts ? s_count : l_count;
  if (uhi() == hi) return n;
  uint64_t& key = facts ? uc_s_n : uc_l_n;
  uint64_t& val = facts ? uc_s : uc_l;
  if (key == n) return val;
  unsigned long long* d = dalloc<unsigned long long>(1);
  HIPCHK(hipMemsetAsync(d, 0, sizeof *d, stream));
  if (n)
    hipLaunchKernelGGL(k_count_below, dim3(grid_for(n)), dim3(BLOCK), 0, stream, facts ? slog_x : llog_x, n, uhi(), d);
  HIPCHK(hipGetLastError());
  unsigned long long h = 0;
  HIPCHK(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  dfree(d);
  key = n;
  val = h;
  return h;
}

// Result rows from the logs (el_rows.hip): S rows X -> {B} ascending (long rows read off the
// bit matrix), link rows X -> {q} ascending, q = the link's pair rank in (role, filler) order.
// dst: device memory or mapped page-locked host memory (the copy-back writes the sorted rows
// straight over PCIe).  Enqueued on s.
void el_ctx::build_rows(bool facts, hipStream_t s, uint64_t* ptr, uint32_t* dst, int half, bool clear) {
  const uint32_t R = uhi() - lo;
  elrows::Scratch& sc = facts ? rsc : rsc_l;
  clear = clear && facts;
  if (half != 2) {
    if (facts)
      elrows::build_prep(s, sc, slog_x, slog_a, s_count, lo, R, nullptr, ptr, dst,
                         colperm() ? elrows::Clear{} : elrows::Clear{dstate().bits, W, lo, ix.c_lo, ix.c_hi}, clear);
    else
      elrows::build_prep(s, sc, llog_x, llog_p, l_count, lo, R, pid_rank, ptr, dst, elrows::Clear{}, false);
  }
  if (half != 1)
    elrows::build_sort(s, sc, ptr, dst, clear ? elrows::Clear{dstate().bits, W, lo, ix.c_lo, ix.c_hi} : elrows::Clear{});
}

// S rows to the caller's page-locked buffers by read-out (el_copy_result): row counts from the
// fact log, the offsets to the host (the caller's s_ptr or a scratch copy; one sync), then
// chunks of rows read off the bit matrix into four device staging buffers in turn, each
// shipped by DMA on dstream while the next is read.  clear: the read-out zeroes the matrix.
void el_ctx::readout_rows(uint64_t* dptr, uint64_t* ptr_out, uint32_t* val_out, bool clear, hipEvent_t counted) {
  const uint32_t R = uhi() - lo;
  elrows::build_counts(stream, rsc, slog_x, s_count, lo, R, dptr);
  if (counted) HIPCHK(hipEventRecord(counted, stream));
  std::vector<uint64_t> tmp;
  uint64_t* hp = ptr_out;
  if (!hp) {
    tmp.resize((size_t)R + 1);
    hp = tmp.data();
  }
  HIPCHK(hipMemcpyAsync(hp, dptr, ((uint64_t)R + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  const uint64_t CHUNK = readout_chunk;  // entries per DMA (32 MB)
  uint64_t longest = 0;
  for (uint32_t r = 0; r < R; ++r) longest = std::max(longest, hp[r + 1] - hp[r]);
  const uint64_t need = std::max(CHUNK, longest);
  if (need > stage_cap) {
    HIPCHK(hipStreamSynchronize(dstream));
    for (uint32_t*& p : stage) {
      dfree(p);
      p = dalloc<uint32_t>(need);
    }
    stage_cap = need;
  }
  elrows::Clear m{dstate().bits, W, lo, ix.c_lo, ix.c_hi};
  if (summ) {
    m.summ = dstate().summ;
    m.SB = SB;
  }
  hipStream_t os = ostream ? ostream : stream;  // (the counts above are done: the host waited)
  uint32_t k = 0;
  for (uint32_t ra = 0; ra < R; ++k) {
    uint32_t rb = ra + 1;  // rows while the chunk fits (at least one)
    {
      uint32_t lo_r = rb, hi_r = R;
      // chunks grow from 1 MB: the first DMA starts after a short read-out (PCIe idles until then)
      const uint64_t lim = std::max<uint64_t>(std::min<uint64_t>(stage_cap, (uint64_t)(1u << 18) << std::min(k, 8u)),
                                              longest);
      while (lo_r < hi_r) {  // the last rb with hp[rb] - hp[ra] <= lim
        const uint32_t mid = lo_r + (hi_r - lo_r + 1) / 2;
        if (hp[mid] - hp[ra] <= lim)
          lo_r = mid;
        else
          hi_r = mid - 1;
      }
      rb = lo_r;
    }
    const uint32_t slot = k % NSTAGE;
    if (k >= NSTAGE) HIPCHK(hipStreamWaitEvent(os, ev_dma[slot], 0));  // the staging buffer is free
    elrows::readout(os, dptr, ra, rb, hp[ra], stage[slot], m, clear);
    HIPCHK(hipEventRecord(ev_stage[slot], os));
    HIPCHK(hipStreamWaitEvent(dstream, ev_stage[slot], 0));
    if (hp[rb] > hp[ra])
      HIPCHK(hipMemcpyAsync(val_out + hp[ra], stage[slot], (hp[rb] - hp[ra]) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            dstream));
    HIPCHK(hipEventRecord(ev_dma[slot], dstream));
    ra = rb;
  }
  if (ostream) {  // the engine stream's next work (the next classification) runs behind the read-out
    HIPCHK(hipEventRecord(ev_out, ostream));
    HIPCHK(hipStreamWaitEvent(stream, ev_out, 0));
  }
}

// Device-resident result rows (el_get_subsumers, el_copy_facts / links, el_export_result),
// kept until the logs change.
void el_ctx::ensure_rows(bool facts, bool links) {
  const uint32_t R = uhi() - lo;
  auto fit = [&](Rows& r, uint64_t n) {
    if (!r.ptr) r.ptr = dalloc<uint64_t>((uint64_t)R + 1);
    if (n > r.cap || !r.val) {
      dfree(r.val);
      r.cap = n + n / 8 + 1024;
      r.val = dalloc<uint32_t>(r.cap);
    }
  };
  if (facts && rs.n != s_count) {
    fit(rs, s_count);
    build_rows(true, stream, rs.ptr, rs.val);
    rs.n = s_count;
  }
  if (links && rl.n != l_count) {
    fit(rl, l_count);
    build_rows(false, stream, rl.ptr, rl.val);
    rl.n = l_count;
  }
}

// One Jacobi superstep over the given trigger ranges; one host sync.  Returns true if
// anything new.  Generation, commit and CSR merges are enqueued back to back: commits
// and merges read their counts on the device.  Capacities are kept ahead of demand
// (logs ≥ count + candidate capacity); if a candidate or job buffer still overflowed,
// the step is completed by re-running generation over the same triggers with larger
// buffers (already committed facts are filtered out, so the result is exact).
bool el_ctx::superstep(uint32_t mask, uint64_t sb, uint64_t se, uint64_t lb, uint64_t le,
                       uint64_t ab, uint64_t ae, uint64_t pb, uint64_t pe) {
  const bool do_a = (mask & M_RRNG) && ae > ab;
  const bool do_p = (mask & M_R4P) && pe > pb;
  if (!(se > sb || le > lb || do_a || do_p)) return false;
  const uint64_t s0 = s_count, l0 = l_count, a0 = a_count, p0 = p_count;
  for (int attempt = 0;; ++attempt) {
    check_u32_room();
    // ---- capacities: every candidate could be new.  Growth copies device arrays outside
    // the stream, so the previous step's kernels must have finished first.
    const bool grow = s_count + cs_cap + ct_cap > slog_cap || l_count + cl_cap > llog_cap ||
                      2 * (l_count - l_base + cl_cap) > lhash_cap || a_count + ca_cap > alog_cap ||
                      2 * (a_count + ca_cap) > ahash_cap || p_count + cp_cap > plog_cap ||
                      2 * (p_count - p_base + cp_cap) > phash_cap;
    if (grow) {
      sync();
      if (strm) HIPCHK(hipStreamSynchronize(dstream));  // (a streamed result may still read the logs)
      static const bool trace = getenv("EL_TRACE_GROW") != nullptr;
      if (trace)
        fprintf(stderr, "grow: s %d l %d lhash %d a %d ahash %d p %d phash %d\n", s_count + cs_cap + ct_cap > slog_cap,
                l_count + cl_cap > llog_cap, 2 * (l_count - l_base + cl_cap) > lhash_cap, a_count + ca_cap > alog_cap,
                2 * (a_count + ca_cap) > ahash_cap, p_count + cp_cap > plog_cap, 2 * (p_count - p_base + cp_cap) > phash_cap);
    }
    auto grow_log = [&](uint64_t used, uint64_t add, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
      if (used + add <= cap) return;
      uint64_t c = &cap == &slog_cap || &cap == &llog_cap ? stream_log_cap(used + add) : log_cap(used + add);
      dgrow(a, used, c);
      dgrow(b, used, c);
      cap = c;
    };
    {
      const uint64_t old_cap = slog_cap;
      grow_log(s_count, cs_cap + ct_cap, slog_cap, slog_x, slog_a);
      if (slog_cap != old_cap) dgrow(slog_f, s_count, slog_cap);
    }
    grow_log(l_count, cl_cap, llog_cap, llog_x, llog_p);
    if (2 * (l_count - l_base + cl_cap) > lhash_cap) rehash_links(next_pow2(2 * (l_count - l_base + cl_cap)));
    grow_log(a_count, ca_cap, alog_cap, alog_y, alog_c);
    if (2 * (a_count + ca_cap) > ahash_cap) rehash_acts(next_pow2(2 * (a_count + ca_cap)));
    grow_log(p_count, cp_cap, plog_cap, plog_p, plog_b);
    if (2 * (p_count - p_base + cp_cap) > phash_cap) rehash_props(next_pow2(2 * (p_count - p_base + cp_cap)));

    // ---- generation (reads only the state of step t-1; candidate counters are zero here)
    static const bool trace_inc = getenv("EL_TRACE_INC") != nullptr;
    if (trace_inc && trig_override)
      fprintf(stderr, "re-trigger step: capacities checked at %.3f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - inc_t0).count());
    refresh_acts();
    DState st = dstate();
    ExpandArgs ea{};
    if (se > sb) wave_triggers(se - sb, tune_expand, ea.gs, ea.ts);
    if (le > lb) wave_triggers(le - lb, tune_expand, ea.gl, ea.tl);
    ea.ga = do_a ? grid_for(se) : 0u;  // the facts known at t-1 meet the new activations
    ea.gp = do_p ? grid_for(pe - pb) : 0u;
    ea.sb = (uint32_t)sb, ea.se = (uint32_t)se, ea.lb = (uint32_t)lb, ea.le = (uint32_t)le;
    ea.ab = (uint32_t)ab, ea.ae = (uint32_t)ae, ea.pb = (uint32_t)pb, ea.pe = (uint32_t)pe;
    // an empty link / propagation set (the first superstep): their probes cannot hit
    ea.mask = mask | (!part() && l_count == l_base ? (uint32_t)M_LEMPTY : 0u) |
              (!part() && p_count == p_base ? (uint32_t)M_PEMPTY : 0u);
    ea.a_end = (uint32_t)a0;
    // S-queue reservations for a big step, if the queue holds the holes too: at most one
    // reservation's worth per wave of the expand and jobs launches (wq_publish_s)
    if (!part() && !small_queues && (se - sb) + (le - lb) >= (1u << 18)) {
      const uint64_t waves = (uint64_t)(ea.gs + ea.gl + ea.ga + ea.gp + tune_jobs) * (BLOCK / 64);
      for (uint32_t c = 4096; c >= 1024 && !st.cs_chunk; c >>= 1)
        if (4 * waves * c <= cs_cap) st.cs_chunk = c;
    }
    // k_expand's view of the state (taken here: st is final for this launch): after an increment,
    // the triggers come from the re-trigger lists
    DState sx = st;
    if (trig_override) {
      sx.slog_x = rt_x;
      sx.slog_a = rt_a;
      sx.slog_f = rt_f;
      sx.llog_x = rt_lx;
      sx.llog_p = rt_lp;
    }
    if (split_expand) {  // the roles are independent: run them one launch each (rocprof sees each)
      const uint32_t g[4] = {ea.gs, ea.gl, ea.ga, ea.gp};
      // EL_SPLIT_EXPAND=2: the S role once more per rule group (CR1, CR2, CR3, CR4, the rest)
      const bool by_rule = getenv("EL_SPLIT_EXPAND")[0] == '2';
      const uint32_t keep = M_LEMPTY | M_PEMPTY;
      const uint32_t groups[5] = {M_R1, M_R2, M_R3, M_R4Y | M_R4D, ~(M_R1 | M_R2 | M_R3 | M_R4Y | M_R4D)};
      // (and the link role per rule group: CR4 half-2, CR5, CR6, the rest)
      const uint32_t lgroups[4] = {M_R4L | M_R4D, M_R5, M_R6, ~(M_R4L | M_R5 | M_R6)};
      for (int r = 0; r < 4; ++r) {
        if (!g[r]) continue;
        for (int k = 0; k < (by_rule && r < 2 ? 5 - r : 1); ++k) {
          ExpandArgs e1 = ea;
          e1.gs = r == 0 ? ea.gs : 0u;
          e1.gl = r == 1 ? ea.gl : 0u;
          e1.ga = r == 2 ? ea.ga : 0u;
          e1.gp = r == 3 ? ea.gp : 0u;
          if (r == 0 && by_rule) e1.mask = (ea.mask & groups[k]) | (ea.mask & keep);
          if (r == 1 && by_rule) e1.mask = (ea.mask & lgroups[k]) | (ea.mask & keep);
          hipLaunchKernelGGL(k_expand, dim3(g[r]), dim3(BLOCK), 0, stream, ix, sx, e1);
        }
      }
    } else {
      launch(EL_K_EXPAND_S, [&] {
        hipLaunchKernelGGL(k_expand, dim3(ea.gs + ea.gl + ea.ga + ea.gp), dim3(BLOCK), 0, stream, ix, sx, ea);
      });
    }
    launch(EL_K_JOBS, [&] {
      hipLaunchKernelGGL(k_jobs, dim3(tune_jobs), dim3(BLOCK), 0, stream, ix, st, ea.mask);
    });
    // ---- commit (counts read on the device); its last block publishes the counters to
    // pinned host memory and zeroes the candidate counters, so the step ends with ONE sync
    CommitArgs ca{};
    // commit grids sized from the step's triggers (the candidate counts are only known on the
    // device; the roles loop grid-stride, so any size is correct): a small step gets a small
    // launch, whose dispatch and completion protocol cost less than 1024 idle workgroups
    const uint64_t est = std::max<uint64_t>(2 * ((se - sb) + (le - lb)), 16384);
    ca.gs = grid_for(std::min<uint64_t>(cs_cap, est), tune_commit);
    ca.gl = grid_for(std::min<uint64_t>(cl_cap, est), tune_commit);
    ca.ga = hx.rng.a.size() ? grid_for(ca_cap, 64) : 0u;
    ca.gp = hx.exl.a.size() ? grid_for(cp_cap, 256) : 0u;
    ca.cs_cap = (uint32_t)cs_cap, ca.cl_cap = (uint32_t)cl_cap;
    ca.ca_cap = (uint32_t)ca_cap, ca.cp_cap = (uint32_t)cp_cap;
    ca.pub = PubArgs{hc_dev, commit_done, ++commit_seq};
    ca.publish = 1;
    launch(EL_K_COMMIT_T, [&] {  // CR1 told-closure candidates first (see k_commit_told)
      hipLaunchKernelGGL(k_commit_told, dim3(grid_for(std::min<uint64_t>(ct_cap, 8 * est), tune_commit)), dim3(BLOCK),
                         0, stream, ix, st, (uint32_t)ct_cap);
    });
    if (split_commit) {  // diagnostic: S role alone, then the other roles (rocprof sees both)
      CommitArgs c1 = ca;
      c1.gl = c1.ga = c1.gp = 0;
      c1.publish = 0;
      hipLaunchKernelGGL(k_commit, dim3(c1.gs), dim3(BLOCK), 0, stream, ix, st, c1);
      ca.gs = 0;
    }
    launch(EL_K_COMMIT_S, [&] {
      hipLaunchKernelGGL(k_commit, dim3(ca.gs + ca.gl + ca.ga + ca.gp), dim3(BLOCK), 0, stream, ix, st, ca);
    });
    if (strm) {  // the last step's segment goes now, beside this step's kernels; this step's
                 // entries are final behind the event recorded here (stream_mark picks it up)
      stream_flush(false);
      HIPCHK(hipEventRecord(ev_strm, stream));
      strm_marked = true;
    }
    // the new links / propagations are already in their (gapped) CSR rows; S rows are
    // built lazily, for export only
    auto inc_lap = [&](const char* what) {
      if (trace_inc && trig_override)
        fprintf(stderr, "re-trigger step: %s at %.3f ms\n", what,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - inc_t0).count());
    };
    inc_lap("launched");
    wait_commit(ca.pub.seq);
    inc_lap("committed");
    if (trace_cands)  // diagnostic (EL_TRACE_CANDS): candidates vs. new facts per step
    {
      unsigned long long ln[3] = {0, 0, 0};
      if (lines_dbg) {
        HIPCHK(hipMemcpy(ln, lines_dbg, sizeof(ln), hipMemcpyDeviceToHost));
        HIPCHK(hipMemset(lines_dbg, 0, sizeof(ln)));
      }
      fprintf(stderr,
              "step cand_t %u cand_s %u new_s %llu cand_l %u new_l %llu cand_p %u jobs %u | S atomics %llu lines %llu "
              "instr %llu\n",
              hc.cand_t, hc.cand_s, (unsigned long long)(hc.s_log - s_count), hc.cand_l,
              (unsigned long long)(hc.l_log - l_count), hc.cand_p, hc.jobs, ln[0], ln[1], ln[2]);
    }
    const uint64_t next_trig = (hc.s_log - s_count) + (hc.l_log - l_count);  // the next step's triggers
    s_count = hc.s_log;
    l_count = hc.l_log;
    a_count = hc.a_log;
    p_count = hc.p_log;
    gap_relocate_all();  // rows that outgrew their slack move to new slots before anyone reads them
    inc_lap("relocated");
    // ---- keep the buffers ahead of demand; complete the step if one overflowed
    bool overflow = false;
    // Each trigger of the next step fans out to a few S conclusions (G3 step 1: 25 M new links
    // -> 88 M candidates, 3.5 per link): a queue sized ahead for that spares re-running a whole
    // generation after an overflow (capped: an outlier step still overflows and re-runs).
    if (const uint64_t want = std::min<uint64_t>(4 * next_trig, 1ull << 28); want > cs_cap && !small_queues) {
      sync();
      cs_cap = next_pow2(want);
      dfree(cs_x);
      dfree(cs_a);
      cs_x = dalloc<uint32_t>(cs_cap);
      cs_a = dalloc<uint32_t>(cs_cap);
    }
    auto regrow2 = [&](uint32_t need, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
      if (2ull * need <= cap) return;
      sync();  // the step's kernels are still queued: free nothing under them
      overflow |= need > cap;
      cap = next_pow2(2ull * need + 1024);
      dfree(a);
      dfree(b);
      a = dalloc<uint32_t>(cap);
      b = dalloc<uint32_t>(cap);
    };
    regrow2(hc.cand_s, cs_cap, cs_x, cs_a);
    regrow2(hc.cand_t, ct_cap, ct_x, ct_a);
    regrow2(hc.cand_l, cl_cap, cl_x, cl_p);
    regrow2(hc.cand_a, ca_cap, ca_y, ca_c);
    regrow2(hc.cand_p, cp_cap, cp_p, cp_b);
    if (max_rng && cl_cap * max_rng > ca_cap)  // activation candidates follow the link queue
      regrow2((uint32_t)std::min<uint64_t>(cl_cap * max_rng / 2, 0xffffffffu), ca_cap, ca_y, ca_c);
    PR.set_ovq(cl_cap);  // overflow queues hold one step's appends
    SC.set_ovq(sc_ovq());
    PP.set_ovq(cp_cap + remote_bound());
    // fan-out jobs: about one per trigger at most (G5 step 1: 4.4 M new links -> 1.7 M jobs)
    if (const uint64_t want = std::min<uint64_t>(next_trig, 1ull << 26); want > job_cap && !small_queues) {
      sync();
      job_cap = next_pow2(want);
      dfree(jobs);
      jobs = dalloc<uint4>(job_cap);
    }
    if (2ull * hc.jobs > job_cap) {
      sync();
      overflow |= hc.jobs > job_cap;
      job_cap = next_pow2(2ull * hc.jobs + 1024);
      dfree(jobs);
      jobs = dalloc<uint4>(job_cap);
    }
    inc_lap("capacities kept");
    if (!overflow) break;
    if (trace_cands) fprintf(stderr, "step re-run after a queue overflow (attempt %d)\n", attempt + 1);
  }
  return s_count > s0 || l_count > l0 || a_count > a0 || p_count > p0;
}

// Exchange capacity: records per rank per all-gather (xcap) and every structure the import
// appends to (replicated propagations / activations / chain links and their CSRs).
void el_ctx::grow_part(uint64_t new_xcap) {
  sync();
  if (new_xcap > xcap) {
    xcap = new_xcap;
    dfree(xsend);
    dfree(xrecv);
    xsend = dalloc<uint32_t>(XH + 2 * xcap);
    xrecv = dalloc<uint32_t>((uint64_t)part_count * (XH + 2 * xcap));
    if (SC.live) SC.set_ovq(sc_ovq());
    if (PP.live) PP.set_ovq(cp_cap + remote_bound());
  }
  const uint64_t rb = remote_bound(), xb = (uint64_t)part_count * xcap;
  auto grow_log = [&](uint64_t used, uint64_t need, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
    if (need <= cap) return;
    const uint64_t c = log_cap(need);
    dgrow(a, used, c);
    dgrow(b, used, c);
    cap = c;
  };
  grow_log(p_count, p_count + cp_cap + rb, plog_cap, plog_p, plog_b);
  if (2 * (p_count + cp_cap + rb) > phash_cap) rehash_props(next_pow2(2 * (p_count + cp_cap + rb)));
  grow_log(a_count, a_count + ca_cap + rb, alog_cap, alog_y, alog_c);
  if (2 * (a_count + ca_cap + rb) > ahash_cap) rehash_acts(next_pow2(2 * (a_count + ca_cap + rb)));
  grow_log(x_count, x_count + cl_cap + xb, xlog_cap, xlog_x, xlog_p);
}

// Pack this rank's new records, all-gather every rank's, import them, merge the CSRs.
// Two rounds: the headers first (XH words per rank), whose record counts size the second
// round to the largest rank's records this superstep (not the capacity: late supersteps send
// almost nothing), then the records.  Returns the largest rank's record count after the import
// published; hc then holds the global g_* words (g_max > xcap: nothing was imported).
uint32_t el_ctx::exchange_round(uint32_t s0, uint32_t l0, uint32_t a0, uint32_t p0, uint32_t x0) {
  DState st = dstate();
  XchgArgs xa{};
  xa.send = xsend;
  xa.recv = xrecv;
  xa.cap = (uint32_t)xcap;
  xa.nranks = part_count;
  xa.me = part_rank;
  xa.s0 = s0, xa.l0 = l0, xa.a0 = a0, xa.p0 = p0, xa.x0 = x0;
  xa.cs_cap = (uint32_t)cs_cap, xa.cl_cap = (uint32_t)cl_cap, xa.ca_cap = (uint32_t)ca_cap;
  xa.cp_cap = (uint32_t)cp_cap, xa.job_cap = (uint32_t)job_cap, xa.ct_cap = (uint32_t)ct_cap;
  hipLaunchKernelGGL(k_xpack, dim3(grid_for(xcap, 64)), dim3(BLOCK), 0, stream, st, xa);
  HIPCHK(hipGetLastError());
  // One round in the common case: the headers and up to xspec records per rank (the size the
  // previous superstep's largest rank suggests, agreed by every rank from gathered words) go in
  // one all-gather, and the import — which reads every rank's header — publishes the step's
  // global words with the one host wait of the superstep.  A rank with more records than the
  // round carried makes every rank import nothing (g_max > round); the record round is then redone
  // at the size g_max asks for (round 4 always ran a header round, a stream sync and the record
  // round: two host round trips per superstep).
  auto round = [&](uint32_t cap) {
    xa.cap = cap;
    xa.recv = xrecv;
    xchg->allgather(xsend, xrecv, (XH + 2 * (uint64_t)cap) * sizeof(uint32_t), stream);
    xrounds_bytes += (uint64_t)part_count * (XH + 2 * (uint64_t)cap) * sizeof(uint32_t);
    const uint32_t seq = ++commit_seq;
    hipLaunchKernelGGL(k_ximport, dim3(grid_for(std::max<uint64_t>((uint64_t)part_count * cap, 1), 256)), dim3(BLOCK),
                       0, stream, ix, st, xa, PubArgs{hc_dev, commit_done, seq});
    HIPCHK(hipGetLastError());
    wait_commit(seq);
    if (hc.g_ovf >> 16) throw ElError{EL_EHIP, "exchange: a send queue overflowed"};
  };
  const uint32_t spec = (uint32_t)std::min<uint64_t>(xspec, xcap);
  round(spec);
  const bool redo = hc.g_max > spec && hc.g_max <= xcap;
  if (redo) round(std::min<uint32_t>((uint32_t)xcap, (hc.g_max + 63) & ~63u));
  // (g_max > xcap: nothing imported; the caller grows the slots and redoes the whole exchange)
  if (trace_xchg)
    fprintf(stderr, "xchg rank %u: round %u records, largest rank %u%s\n", part_rank, spec, hc.g_max,
            redo ? " (redone)" : "");
  // the next round: this one's largest rank + 1/8 (the late supersteps shrink; a growing one redoes)
  xspec = std::min<uint64_t>(xcap, ((uint64_t)hc.g_max + hc.g_max / 8 + 63) & ~63ull);
  s_count = hc.s_log;
  l_count = hc.l_log;
  a_count = hc.a_log;
  p_count = hc.p_log;
  x_count = hc.x_log;
  p_import = p0 + hc.g_pown;  // [p0, p_import): this rank's own new propagations; then the imported
  gap_relocate_all();
  return hc.g_max;
}

// One Jacobi superstep of a row partition (protocol: oracle/partition_model.py).  Every
// rank runs it in lock-step, including ranks without local triggers: the exchange is
// collective.  Redo decisions (exchange cap, candidate overflow) use all-gathered words,
// so every rank takes the same branch.
uint64_t el_ctx::superstep_part(uint32_t mask, uint64_t sb, uint64_t se, uint64_t lb, uint64_t le, uint64_t ab,
                                uint64_t ae, uint64_t pb, uint64_t pe, uint64_t xb, uint64_t xe) {
  uint64_t gdelta = 0;
  for (int attempt = 0;; ++attempt) {
    // ---- capacities for the local candidates (as in superstep) and the remote imports
    const uint64_t rb = remote_bound();
    const bool grow = s_count + cs_cap + ct_cap > slog_cap || l_count + cl_cap > llog_cap ||
                      2 * (l_count - l_base + cl_cap) > lhash_cap || a_count + ca_cap + rb > alog_cap ||
                      2 * (a_count + ca_cap + rb) > ahash_cap || p_count + cp_cap + rb > plog_cap ||
                      2 * (p_count - p_base + cp_cap + rb) > phash_cap ||
                      x_count + cl_cap + part_count * xcap > xlog_cap;
    if (grow) {
      sync();
      if (strm) HIPCHK(hipStreamSynchronize(dstream));
      auto grow_log = [&](uint64_t used, uint64_t add, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
        if (used + add <= cap) return;
        uint64_t c = &cap == &slog_cap || &cap == &llog_cap ? stream_log_cap(used + add) : log_cap(used + add);
        dgrow(a, used, c);
        dgrow(b, used, c);
        cap = c;
      };
      {
        const uint64_t old_cap = slog_cap;
        grow_log(s_count, cs_cap + ct_cap, slog_cap, slog_x, slog_a);
        if (slog_cap != old_cap) dgrow(slog_f, s_count, slog_cap);
      }
        grow_log(l_count, cl_cap, llog_cap, llog_x, llog_p);
      if (2 * (l_count - l_base + cl_cap) > lhash_cap) rehash_links(next_pow2(2 * (l_count - l_base + cl_cap)));
      grow_part(xcap);
    }
    const uint32_t s0 = (uint32_t)s_count, l0 = (uint32_t)l_count, a0 = (uint32_t)a_count, p0 = (uint32_t)p_count,
                   x0 = (uint32_t)x_count;

    // ---- generation + local commit (no publish: the import publishes for the step)
    refresh_acts();
    DState st = dstate();
    ExpandArgs ea{};
    const bool do_a = (mask & M_RRNG) && ae > ab;
    const bool do_p = (mask & M_R4P) && pe > pb;
    if (se > sb) wave_triggers(se - sb, 1024, ea.gs, ea.ts);
    if (le > lb) wave_triggers(le - lb, 1024, ea.gl, ea.tl);
    ea.ga = do_a ? grid_for(se) : 0u;
    ea.gp = do_p ? grid_for(pe - pb) : 0u;
    ea.gx = ((mask & M_R6) && xe > xb) ? grid_for(xe - xb) : 0u;
    ea.sb = (uint32_t)sb, ea.se = (uint32_t)se, ea.lb = (uint32_t)lb, ea.le = (uint32_t)le;
    ea.ab = (uint32_t)ab, ea.ae = (uint32_t)ae, ea.pb = (uint32_t)pb, ea.pe = (uint32_t)pe;
    ea.xb = (uint32_t)xb, ea.xe = (uint32_t)xe;
    // an empty link / propagation set (the first superstep over the base links): probes cannot
    // hit (the imports of a superstep come after its generation)
    ea.mask = mask | (l_count == l_base ? (uint32_t)M_LEMPTY : 0u) | (p_count == p_base ? (uint32_t)M_PEMPTY : 0u);
    ea.a_end = (uint32_t)ab;  // activations known at t-1 (the exchange appended this step's)
    // S-queue reservations for a big step (wq_publish_s), as in superstep()
    if (!small_queues && (se - sb) + (le - lb) >= (1u << 18)) {
      const uint64_t waves = (uint64_t)(ea.gs + ea.gl + ea.ga + ea.gp + ea.gx + tune_jobs) * (BLOCK / 64);
      for (uint32_t c = 4096; c >= 1024 && !st.cs_chunk; c >>= 1)
        if (4 * waves * c <= cs_cap) st.cs_chunk = c;
    }
    const uint32_t eg = ea.gs + ea.gl + ea.ga + ea.gp + ea.gx;
    if (eg) {
      launch(EL_K_EXPAND_S, [&] { hipLaunchKernelGGL(k_expand, dim3(eg), dim3(BLOCK), 0, stream, ix, st, ea); });
      launch(EL_K_JOBS, [&] { hipLaunchKernelGGL(k_jobs, dim3(tune_jobs), dim3(BLOCK), 0, stream, ix, st, ea.mask); });
    }
    CommitArgs ca{};
    // grids from the step's triggers, as in superstep() (the roles loop grid-stride)
    const uint64_t est = std::max<uint64_t>(2 * ((se - sb) + (le - lb) + (xe - xb) + (pe - pb)), 16384);
    ca.gs = grid_for(std::min<uint64_t>(cs_cap, est), tune_commit);
    ca.gl = grid_for(std::min<uint64_t>(cl_cap, est), tune_commit);
    ca.ga = hx.rng.a.size() ? grid_for(ca_cap, 64) : 0u;
    ca.gp = use_props ? grid_for(cp_cap, 256) : 0u;
    ca.cs_cap = (uint32_t)cs_cap, ca.cl_cap = (uint32_t)cl_cap;
    ca.ca_cap = (uint32_t)ca_cap, ca.cp_cap = (uint32_t)cp_cap;
    ca.publish = 0;
    launch(EL_K_COMMIT_T, [&] {
      hipLaunchKernelGGL(k_commit_told, dim3(grid_for(std::min<uint64_t>(ct_cap, 8 * est), tune_commit)), dim3(BLOCK),
                         0, stream, ix, st, (uint32_t)ct_cap);
    });
    launch(EL_K_COMMIT_S, [&] {
      hipLaunchKernelGGL(k_commit, dim3(ca.gs + ca.gl + ca.ga + ca.gp), dim3(BLOCK), 0, stream, ix, st, ca);
    });

    // ---- delta exchange; a too-small exchange imports nothing and is redone larger
    uint32_t gmax = exchange_round(s0, l0, a0, p0, x0);
    if (gmax > xcap) {
      grow_part(next_pow2(gmax));
      gmax = exchange_round(s0, l0, a0, p0, x0);
      if (gmax > xcap) throw std::runtime_error("exchange overflow after growth");
    }
    gdelta += hc.g_delta;

    // ---- candidate queues: grow ahead of demand; a global overflow re-runs generation
    auto regrow2 = [&](uint32_t need, uint64_t& cap, uint32_t*& a, uint32_t*& b) {
      if (2ull * need <= cap) return false;
      sync();
      cap = next_pow2(2ull * need + 1024);
      dfree(a);
      dfree(b);
      a = dalloc<uint32_t>(cap);
      b = dalloc<uint32_t>(cap);
      return true;
    };
    regrow2(hc.cand_s, cs_cap, cs_x, cs_a);
    regrow2(hc.cand_t, ct_cap, ct_x, ct_a);
    if (regrow2(hc.cand_l, cl_cap, cl_x, cl_p)) {
      PR.set_ovq(cl_cap);
      SC.set_ovq(sc_ovq());
    }
    regrow2(hc.cand_a, ca_cap, ca_y, ca_c);
    if (regrow2(hc.cand_p, cp_cap, cp_p, cp_b)) PP.set_ovq(cp_cap + remote_bound());
    fit_xqueues(cl_cap, cp_cap, ca_cap);  // (sent: the queues are empty)
    if (2ull * hc.jobs > job_cap) {
      sync();
      job_cap = next_pow2(2ull * hc.jobs + 1024);
      dfree(jobs);
      jobs = dalloc<uint4>(job_cap);
    }
    if (hc.g_ovf == 0) break;
  }
  return gdelta;
}

// new row starts = exclusive scan of gap_cap(len[r]) (k_gap_scan)
void el_ctx::launch_gap_scan(const uint32_t* len, uint32_t R, uint32_t* start_out) {
  ScanArgs sa{};
  sa.len = len;
  sa.start_out = start_out;
  sa.n1 = R + 1;
  sa.tiles = (R + 1 + SCAN_TILE - 1) / SCAN_TILE;
  if (sa.tiles > scan_tiles) throw std::runtime_error("scan tile overflow");
  if (++scan_epoch >= (1u << 30)) {
    HIPCHK(hipMemsetAsync(scan_flags, 0, scan_tiles * sizeof(unsigned long long), stream));
    scan_epoch = 1;
  }
  sa.epoch = scan_epoch;
  sa.flags = scan_flags;
  sa.ticket = &ctr->ticket;
  launch(EL_K_SCAN, [&] { hipLaunchKernelGGL(k_gap_scan, dim3(sa.tiles), dim3(256), 0, stream, sa); });
}

// A gapped CSR laid out for, and filled with, the n logged entries (rows[i], vals[i]).
void el_ctx::gap_build_from_log(GapCsr& g, const uint32_t* rows, const uint32_t* vals, uint64_t n,
                                const uint8_t* keep) {
  const GapKeep gk{keep, keep ? ix.pair_role : nullptr};
  const uint32_t R = g.rows;
  HIPCHK(hipMemsetAsync(g.len, 0, (uint64_t)R * sizeof(uint32_t), stream));
  if (n) {
    hipLaunchKernelGGL(k_gap_count, dim3(grid_for(n)), dim3(BLOCK), 0, stream, g.len, rows, vals, n, gk);
    HIPCHK(hipGetLastError());
  }
  launch_gap_scan(g.len, R, g.start);
  hipLaunchKernelGGL(k_gap_ends, dim3(grid_for(R)), dim3(BLOCK), 0, stream, g.start, g.end, R);
  HIPCHK(hipGetLastError());
  const uint64_t total = (uint64_t)GAP_MUL * n + (uint64_t)gap_cap(0) * R;
  if (total > 0xffffffffull) throw ElError{EL_ENOMEM, "gapped CSR beyond 2^32 slots"};
  if (total > g.val_cap) {
    sync();
    dfree(g.val);
    g.val_cap = total + total / 2;
    g.val = dalloc<uint32_t>(g.val_cap);
  }
  g.used = total;
  HIPCHK(hipMemsetAsync(g.len, 0, (uint64_t)R * sizeof(uint32_t), stream));
  if (n) {
    hipLaunchKernelGGL(k_gap_fill, dim3(grid_for(n)), dim3(BLOCK), 0, stream, g.view(&ctr->ov_pr), rows, vals, n, gk);
    HIPCHK(hipGetLastError());
  }
}

// The same layout and contents by a radix sort of the entries by row instead of a counter atomic
// per entry: the predecessor rows of G3's 33 M links by pid took 5.9 ms to count and 5.2 ms to
// fill with atomics (a hub pid's entries serialise on its counter), the sort and the grouped
// fill well under one.  bits: bits of a row index.
void el_ctx::gap_build_sorted(GapCsr& g, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t bits) {
  const uint32_t R = g.rows;
  if (n > 0xffffffffull) throw ElError{EL_ENOMEM, "gapped CSR beyond 2^32 entries"};
  if (n > sk_cap) {
    sk_cap = n + n / 8;
    dfree(sk);
    dfree(sv);
    sk = dalloc<uint32_t>(sk_cap);
    sv = dalloc<uint32_t>(sk_cap);
  }
  const size_t need = elcl::sort_temp_bytes((uint32_t)std::max<uint64_t>(n, 1));
  if (need > csort_bytes) {
    dfree(csort_tmp);
    csort_bytes = need;
    csort_tmp = dalloc<uint8_t>(need);
  }
  // first / last of each row's run: the relocation scratch (nstart) and the row ends (rewritten
  // by k_gap_ends below)
  HIPCHK(hipMemsetAsync(g.nstart, 0, (uint64_t)R * sizeof(uint32_t), stream));
  HIPCHK(hipMemsetAsync(g.end, 0, (uint64_t)R * sizeof(uint32_t), stream));
  if (n) {
    elcl::sort_pairs(stream, csort_tmp, csort_bytes, rows, sk, vals, sv, (uint32_t)n, bits);
    elcl::runs(stream, sk, (uint32_t)n, g.nstart, g.end);
  }
  elcl::caps(stream, g.nstart, g.end, R, nullptr, nullptr, nullptr, g.len);
  launch_gap_scan(g.len, R, g.start);
  hipLaunchKernelGGL(k_gap_ends, dim3(grid_for(R)), dim3(BLOCK), 0, stream, g.start, g.end, R);
  HIPCHK(hipGetLastError());
  const uint64_t total = (uint64_t)GAP_MUL * n + (uint64_t)gap_cap(0) * R;
  if (total > 0xffffffffull) throw ElError{EL_ENOMEM, "gapped CSR beyond 2^32 slots"};
  if (total > g.val_cap) {
    sync();
    dfree(g.val);
    g.val_cap = total + total / 2;
    g.val = dalloc<uint32_t>(g.val_cap);
  }
  g.used = total;
  if (n) elcl::group_fill(stream, sk, sv, (uint32_t)n, g.nstart, g.start, g.val);
}

// ---- the told closure on the device (el_closure.h), rebuilt inside every el_init: nothing
// derived from the axioms survives from one classification to the next except buffer sizes

void el_ctx::alloc_closure() {
  const uint64_t N = hx.N, P = std::max<uint32_t>(hx.P, 1u);
  auto cap32 = [](uint64_t v) { return (uint32_t)std::min<uint64_t>(v, 0x7fffffffull); };
  cl.meta = dalloc<uint4>(2 * N);
  cl.meta2 = dalloc<uint4>(2 * N);
  // first guesses (G3: 24 M / 25 M / 36 M entries) for the concepts the build covers — a
  // partition's column window (×8 of G3: one copy's, not 8 copies' worth: 4 GB less per rank);
  // an overflowing build grows and runs again
  const uint64_t Nc = part() && ix.c_hi > ix.c_lo ? std::min<uint64_t>(N, (uint64_t)ix.c_hi - ix.c_lo) : N;
  const uint64_t waste = std::min<uint64_t>(Nc, elcl::SLOTS) * elcl::CHUNK;  // partly used chunks
  cl.t_cap = cap32(64 * Nc + waste + (1u << 16));
  cl.e_cap = cap32(64 * Nc + waste + (1u << 16));
  cl.l_cap = cap32(96 * Nc + waste + (1u << 16));
  cl.t_val = dalloc<uint32_t>(cl.t_cap);
  cl.e_val = dalloc<uint32_t>(cl.e_cap);
  cl.l_r = dalloc<uint32_t>(cl.l_cap);
  cl.l_b = dalloc<uint32_t>(cl.l_cap);
  cl.level = dalloc<uint32_t>(N);
  cl.indeg = dalloc<uint32_t>(N);
  cl.lvl_flag = dalloc<uint32_t>(N + 2);
  cl.dirty = dalloc<uint8_t>(N);
  cl.dirty2 = dalloc<uint8_t>(N);
  cl.changed = dalloc<uint32_t>(N);
  cl.nd = dalloc<uint32_t>(elcl::ND_NUM * (N + 1));
  HIPCHK(hipMemset(cl.nd, 0, elcl::ND_NUM * (N + 1) * sizeof(uint32_t)));  // (entry N of a column stays 0)
  cl.rsv = dalloc<uint32_t>(elcl::RSV_WORDS);
  cl.scratch_cap = 1u << 20;
  cl.scratch = dalloc<uint32_t>(cl.scratch_cap);
  cl.ctr = dalloc<elcl::Ctr>(1);
  HIPCHK(hipHostMalloc((void**)&clh, sizeof(ClHost), hipHostMallocDefault));
  memset(clh, 0, sizeof(ClHost));
  for (uint32_t*& p : cpos) p = dalloc<uint32_t>(N + 1);
  cscan_bytes = std::max<size_t>(elcl::scan_temp_bytes((uint32_t)N + 1), 16);
  cscan_tmp = dalloc<uint8_t>(cscan_bytes);
  for (uint32_t** p : {&pr_first, &pr_last, &bpp_s, &bpp_e, &cap_pr, &cap_pp}) {
    *p = dalloc<uint32_t>(P);
    HIPCHK(hipMemset(*p, 0, P * sizeof(uint32_t)));
  }
  cl_alloc_n = N;
  cl_alloc_p = P;
  level_hint = 32;
  set_closure_ix();
}

void el_ctx::free_closure() {
  dfree(cl.meta);
  dfree(cl.meta2);
  dfree(cl.t_val);
  dfree(cl.e_val);
  dfree(cl.l_r);
  dfree(cl.l_b);
  dfree(cl.level);
  dfree(cl.indeg);
  dfree(cl.lvl_flag);
  dfree(cl.dirty);
  dfree(cl.dirty2);
  dfree(cl.changed);
  dfree(cl.nd);
  dfree(cl.rsv);
  dfree(cl.scratch);
  dfree(cl.ctr);
  cl = elcl::Out{};
  if (clh) (void)hipHostFree(clh);
  clh = nullptr;
  for (uint32_t*& p : cpos) dfree(p);
  dfree(cscan_tmp);
  dfree(csort_tmp);
  cscan_bytes = csort_bytes = 0;
  dfree(sk);
  dfree(sv);
  sk_cap = 0;
  for (uint32_t** p : {&pr_first, &pr_last, &bpp_s, &bpp_e, &cap_pr, &cap_pp}) dfree(*p);
  nb = nbp = nc = 0;
}

// the kernels' view of this classification's rows
void el_ctx::set_closure_ix() {
  ix.told_b = cl.t_val;
  ix.exr_pid = cl.e_val;
  ix.exl_r = cl.l_r;
  ix.exl_b = cl.l_b;
  ix.meta = cl.meta;
  ix.bpp_s = bpp_s;
  ix.bpp_e = bpp_e;
}

// a build overflowed a row array or the big-row scratch: grow what overflowed (to what it asked
// for, at least double) and build again
void el_ctx::closure_grow() {
  const elcl::Ctr& c = clh->ctr;
  auto grow = [&](std::initializer_list<uint32_t**> ps, uint32_t& cap, uint64_t tail) {
    if (tail <= cap) return;
    uint64_t n = std::max<uint64_t>(2ull * cap, tail + tail / 2);
    if (tail >= 0x7fffffffull) throw ElError{EL_ENOMEM, "told closure rows beyond 2^31 entries"};
    n = std::min<uint64_t>(n, 0x7fffffffull);
    for (uint32_t** p : ps) {
      dfree(*p);
      *p = dalloc<uint32_t>(n);
    }
    cap = (uint32_t)n;
  };
  sync();
  grow({&cl.t_val}, cl.t_cap, c.t_tail);
  grow({&cl.e_val}, cl.e_cap, c.e_tail);
  grow({&cl.l_r, &cl.l_b}, cl.l_cap, c.l_tail);
  if (2 * c.s_tail > cl.scratch_cap) {
    dfree(cl.scratch);
    cl.scratch_cap = std::max<unsigned long long>(2 * cl.scratch_cap, 3 * c.s_tail);
    cl.scratch = dalloc<uint32_t>(cl.scratch_cap);
  }
  set_closure_ix();
}

// After the Kahn levels launched so far: stuck concepts, totals over [a, b), the scans of the
// rows' counts, and one readback (counters, the flag of level L, the rows of ⊤).
void el_ctx::closure_tail(uint32_t a, uint32_t b, uint32_t L, bool all) {
  HIPCHK(hipMemsetAsync(&cl.ctr->tot[elcl::T_STUCK], 0, sizeof(unsigned long long), stream));
  // (told cycles' followers whose representative is final; each once per build)
  if (caxk.nfol) launch(EL_K_CLOSURE, [&] { elcl::follow(stream, caxk, cl, L, all); });
  elcl::check(stream, caxk, cl);
  elcl::stats(stream, cax, cl, 0, hx.N, use_props);  // (every row: the SC layout spans them)
  HIPCHK(hipMemsetAsync(cl.ctr->tot, 0, elcl::T_STUCK * sizeof(unsigned long long), stream));
  HIPCHK(hipMemsetAsync(cl.ctr->ev, 0, sizeof(cl.ctr->ev), stream));
  elcl::totals(stream, cax, cl, a, b);
  const uint64_t N1 = (uint64_t)hx.N + 1;
  const uint32_t cols[3] = {elcl::ND_INIT, elcl::ND_EXR, elcl::ND_PROPS};
  for (int i = 0; i < 3; ++i) elcl::scan(stream, cscan_tmp, cscan_bytes, cl.nd + cols[i] * N1 + a, cpos[i], b - a + 1);
  HIPCHK(hipMemcpyAsync(&clh->ctr, cl.ctr, sizeof(elcl::Ctr), hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&clh->flag, cl.lvl_flag + std::min<uint32_t>(L, hx.N + 1), sizeof(uint32_t),
                        hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(clh->top, cl.meta + 2 * EL_TOP, 2 * sizeof(uint4), hipMemcpyDeviceToHost, stream));
  sync();
}

// The rows told*, exr*, exl* of every concept (Kahn levels; relaxation rounds for told cycles)
// and the totals / scans over the rows [a, b) (el_init: the owned rows; an increment: the new
// ones).  Readbacks: one after the levels (two when the graph is deeper than the levels launched
// up front), one per relaxation round.
void el_ctx::closure_rows(uint32_t a, uint32_t b) {
  const uint32_t N = hx.N;
  // a partitioned context builds the rows of its column window only (×N of G3 on N ranks: each
  // builds its own copy's closure, not the N copies')
  cax.w_lo = caxk.w_lo = part() ? ix.c_lo : 2u;
  cax.w_hi = caxk.w_hi = part() ? ix.c_hi : 0xffffffffu;
  for (int attempt = 0;; ++attempt) {
    if (attempt > 32) throw ElError{EL_EHIP, "told closure: the build did not fit its buffers"};
    launch(EL_K_CLOSURE, [&] { elcl::start(stream, caxk, cl); });
    uint32_t L = 0;
    bool redo = false;
    if (caxk.slevel) {  // static levels: exactly the levels there are, each a list of its concepts
      launch(EL_K_CLOSURE, [&] { elcl::level(stream, caxk, cl, 0); });
      const uint32_t depth = (uint32_t)lvl_ptr.size() - 2;
      for (L = 1; L <= depth; ++L)
        launch(EL_K_CLOSURE, [&] { elcl::level_list(stream, caxk, cl, L, lvl_ptr[L], lvl_ptr[L + 1] - lvl_ptr[L]); });
      init_lap("levels enqueued");
      closure_tail(a, b, L, false);
      init_lap("closure tail read");
      if (clh->ctr.bad) throw ElError{EL_EHIP, "told closure: a told cycle's representative row lacks its follower"};
      redo = clh->ctr.ovf != 0;
    }
    for (; !caxk.slevel;) {
      const uint32_t end = (uint32_t)std::min<uint64_t>((uint64_t)N + 1, (uint64_t)L + level_hint);
      for (; L < end; ++L) launch(EL_K_CLOSURE, [&] { elcl::level(stream, caxk, cl, L); });
      init_lap("levels enqueued");
      closure_tail(a, b, L, false);
      init_lap("closure tail read");
      if (clh->ctr.bad) throw ElError{EL_EHIP, "told closure: a told cycle's representative row lacks its follower"};
      if (clh->ctr.ovf) {
        redo = true;
        break;
      }
      if (L <= N && clh->flag) {  // deeper than the levels launched: more of them
        level_hint = std::min<uint32_t>(2 * level_hint, N + 1);
        continue;
      }
      break;
    }
    if (!redo && clh->ctr.tot[elcl::T_STUCK]) {  // told cycles: relaxation rounds until no row grows
      for (uint64_t round = 0;; ++round) {
        launch(EL_K_CLOSURE, [&] { elcl::relax(stream, caxk, cl); });
        HIPCHK(hipMemcpyAsync(&clh->ctr, cl.ctr, sizeof(elcl::Ctr), hipMemcpyDeviceToHost, stream));
        sync();
        if (clh->ctr.ovf) {
          redo = true;
          break;
        }
        if (!clh->ctr.dirty) break;
        if (round > (uint64_t)N + 1) throw ElError{EL_EHIP, "told closure: relaxation did not converge"};
      }
      if (!redo) {
        closure_tail(a, b, L, true);
        if (clh->ctr.bad) throw ElError{EL_EHIP, "told closure: a told cycle's representative row lacks its follower"};
        redo = clh->ctr.ovf != 0;
      }
    }
    if (!redo) break;
    closure_grow();
  }
  clt = clh->ctr;
  host_ev[EL_K_CLOSURE][EL_EV_TRIG] += clt.ev[elcl::E_TRIG];
  host_ev[EL_K_CLOSURE][EL_EV_ROW] += clt.ev[elcl::E_ROW];
  host_ev[EL_K_CLOSURE][EL_EV_ENT] += clt.ev[elcl::E_ENT];
  host_ev[EL_K_CLOSURE][EL_EV_RMW] += clt.ev[elcl::E_RMW];
}

// The owned rows' init facts S(X) = {X, ⊤} ∪ told*(X) (fact log + bits), the base links /
// propagations of the owned rows in the heads of their logs (installed by el_saturate), the base
// links by pid (radix sort) and this classification's gapped-row layouts.  Buffers grow first to
// what the closure asks for (grow-only).  A row partition does the same for its own rows (its
// base links are local; el_saturate routes the chain-second ones and the propagations that other
// ranks' rows can reach into the first exchange).
void el_ctx::closure_state() {
  if (reset_wait) {
    HIPCHK(hipStreamWaitEvent(stream, ev_reset, 0));
    reset_wait = false;
  }
  const unsigned long long* T = clt.tot;
  const uint64_t N = hx.N, P = hx.P;
  const uint64_t n_init = T[elcl::T_INIT], two = T[elcl::T_TWO];
  const uint4 tb = clh->top[0], te = clh->top[1];
  // the first superstep re-triggers every init fact: CR3 over exr*, CR2 over the closures'
  // conjunctions, CR4 half-1 over exl* (per own row X: X, ⊤ and the told closure)
  const uint64_t b_link = T[elcl::T_EXR] + two * (te.z - tb.z);
  const uint64_t b_conj = T[elcl::T_CIDX] + two * (te.y - tb.y) + T[elcl::T_CZ];
  const uint64_t b_prop = T[elcl::T_EXL] + two * (te.w - tb.w);
  nb = T[elcl::T_EXR];
  nbp = use_props ? T[elcl::T_PROPS] : 0;
  nc = SC.live ? T[elcl::T_SC0] : 0;
  if (n_init > 0xffffffffull || nb > 0xffffffffull || nbp > 0xffffffffull)
    throw ElError{EL_ENOMEM, "init facts or base links beyond 2^32 (uint32 device counters)"};
  auto realloc2 = [](uint64_t cap, uint32_t*& a, uint32_t*& b) {
    dfree(a);
    dfree(b);
    a = dalloc<uint32_t>(cap);
    b = dalloc<uint32_t>(cap);
  };
  if (!small_queues) {
    if (const uint64_t w = next_pow2(b_conj + b_conj / 4); w > cs_cap) realloc2(cs_cap = w, cs_x, cs_a);
    if (const uint64_t w = next_pow2(b_link + b_link / 4); w > cl_cap) realloc2(cl_cap = w, cl_x, cl_p);
  }
  if (const uint64_t w = next_pow2(b_prop + b_prop / 4); w > cp_cap) realloc2(cp_cap = w, cp_p, cp_b);
  if (const uint64_t w = std::max<uint64_t>(cs_cap, next_pow2(2 * T[elcl::T_TOLD] + 1024)); w > ct_cap)
    realloc2(ct_cap = w, ct_x, ct_a);
  if (max_rng && next_pow2(cl_cap * max_rng) > ca_cap) realloc2(ca_cap = next_pow2(cl_cap * max_rng), ca_y, ca_c);
  PR.set_ovq(cl_cap);
  SC.set_ovq(sc_ovq());
  PP.set_ovq(cp_cap + remote_bound());
  if (part()) {  // (the queues and the chain-link log are empty at el_init)
    fit_xqueues(cl_cap + nc, cp_cap + nbp, ca_cap);
    if (const uint64_t w = nc + cl_cap + (uint64_t)part_count * xcap; w > xlog_cap) {
      xlog_cap = log_cap(w);
      realloc2(xlog_cap, xlog_x, xlog_p);
    }
  }
  if (n_init + cs_cap + ct_cap > slog_cap) {  // (s_count is 0: nothing to keep)
    slog_cap = next_pow2(n_init + cs_cap + ct_cap);
    realloc2(slog_cap, slog_x, slog_a);
    dfree(slog_f);
    slog_f = dalloc<uint8_t>(slog_cap);
  }
  if (nb + cl_cap > llog_cap) realloc2(llog_cap = stream_log_cap(nb + cl_cap), llog_x, llog_p);
  if (2 * (nb + cl_cap) > lhash_cap) rehash_links(next_pow2(2 * (nb + cl_cap)));
  if (nbp + cp_cap > plog_cap) realloc2(plog_cap = log_cap(nbp + cp_cap), plog_p, plog_b);
  if (2 * (nbp + cp_cap) > phash_cap) rehash_props(next_pow2(2 * (nbp + cp_cap)));
  // initial gapped layouts: row capacities gap_cap(c) for the first supersteps' entries c
  auto fit_gap = [&](GapCsr& g, uint64_t entries) {
    if (!g.live) return;
    g.total0 = (uint64_t)GAP_MUL * entries + (uint64_t)gap_cap(0) * g.rows;
    if (g.total0 > 0xffffffffull) throw ElError{EL_ENOMEM, "gapped CSR beyond 2^32 slots"};
    if (g.val_cap < g.total0) {
      dfree(g.val);
      g.val_cap = g.total0;
      g.val = dalloc<uint32_t>(g.val_cap);
    }
    g.laid = false;
  };
  fit_gap(PR, nb + T[elcl::T_LIFT]);
  fit_gap(SC, T[elcl::T_SC]);
  fit_gap(PP, nbp);
  if (PR.live && nb) {
    if (nb > sk_cap) {
      sk_cap = nb + nb / 8;
      realloc2(sk_cap, sk, sv);
    }
    const size_t need = elcl::sort_temp_bytes((uint32_t)nb);
    if (need > csort_bytes) {
      dfree(csort_tmp);
      csort_bytes = need;
      csort_tmp = dalloc<uint8_t>(need);
    }
  }
  set_closure_ix();
  init_lap("state sized");
  // ---- the init facts: a random-access kernel (a bit per fact) beside the base links and the
  // layouts below (streaming work), on rstream unless profiled; they touch disjoint buffers and the
  // engine stream joins at the end of closure_state
  DState st = dstate();
  const bool init_side = !profile && !getenv("EL_INIT_INLINE");
  if (init_side) {
    HIPCHK(hipEventRecord(ev_init[0], stream));  // (the engine stream waited for the reset above)
    HIPCHK(hipStreamWaitEvent(rstream, ev_init[0], 0));
    launches[EL_K_INIT]++;
    elcl::init_facts(rstream, cax, cl, lo, hi, cpos[0], 0, slog_x, slog_a, slog_f, st.bits, W, ix.c_lo, ix.c_hi,
                     st.summ, SB);
    HIPCHK(hipEventRecord(ev_init[1], rstream));
  } else {
    launch(EL_K_INIT, [&] {
      elcl::init_facts(stream, cax, cl, lo, hi, cpos[0], 0, slog_x, slog_a, slog_f, st.bits, W, ix.c_lo, ix.c_hi,
                       st.summ, SB);
    });
  }
  hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, stream, &ctr->s_log, (uint32_t)n_init);
  HIPCHK(hipGetLastError());
  s_count = n_init;
  s_init = T[elcl::T_OWN] + two;
  // (per row X: its slots, the row's entries read)
  host_ev[EL_K_INIT][EL_EV_ENT] += T[elcl::T_OWN] + T[elcl::T_TOLD];
  host_ev[EL_K_INIT][EL_EV_RMW] += n_init;
  host_ev[EL_K_INIT][EL_EV_EMIT] += n_init;
  // ---- base links / propagations and the layouts they ask for
  {
    const uint32_t n32 = (uint32_t)N, p32 = (uint32_t)P;
    if (nb) elcl::base_links(stream, cax, cl, lo, hi, cpos[1], llog_x, llog_p);
    if (P) {
      HIPCHK(hipMemsetAsync(bpp_s, 0, P * sizeof(uint32_t), stream));
      HIPCHK(hipMemsetAsync(bpp_e, 0, P * sizeof(uint32_t), stream));
    }
    if (nbp) {
      elcl::base_props(stream, cax, cl, lo, hi, cpos[2], plog_p, plog_b);
      elcl::runs(stream, plog_p, (uint32_t)nbp, bpp_s, bpp_e);
    }
    if (PR.live) {
      for (uint32_t* p : {pr_first, pr_last, cap_pr}) HIPCHK(hipMemsetAsync(p, 0, P * sizeof(uint32_t), stream));
      if (nb) {
        elcl::sort_pairs(stream, csort_tmp, csort_bytes, llog_p, sk, llog_x, sv, (uint32_t)nb, key_bits);
        elcl::runs(stream, sk, (uint32_t)nb, pr_first, pr_last);
      }
      elcl::caps(stream, pr_first, pr_last, p32, ix.psup_ptr, ix.psup_pid, cap_pr, nullptr);
      launch_gap_scan(cap_pr, p32, PR.start0);
      PR.laid = true;
    }
    if (SC.live) {
      const uint32_t* sc_cap = cl.nd + elcl::ND_SC * (N + 1);
      if (part()) {  // the own rows' capacities only (T_SC sized the slots): other rows grow on demand
        if (!sc_own) sc_own = dalloc<uint32_t>(N + 1);
        HIPCHK(hipMemsetAsync(sc_own, 0, (N + 1) * sizeof(uint32_t), stream));
        if (hi > lo)
          HIPCHK(hipMemcpyAsync(sc_own + lo, sc_cap + lo, (uint64_t)(hi - lo) * sizeof(uint32_t),
                                hipMemcpyDeviceToDevice, stream));
        sc_cap = sc_own;
      }
      launch_gap_scan(sc_cap, n32, SC.start0);
      SC.laid = true;
    }
    if (PP.live) {
      HIPCHK(hipMemsetAsync(cap_pp, 0, P * sizeof(uint32_t), stream));
      elcl::caps(stream, bpp_s, bpp_e, p32, nullptr, nullptr, cap_pp, nullptr);
      launch_gap_scan(cap_pp, p32, PP.start0);
      PP.laid = true;
    }
  }
  for (GapCsr* g : {&PR, &SC, &PP}) {
    if (!g->live) continue;
    g->used = g->laid ? g->total0 : (uint64_t)gap_cap(0) * g->rows;
    hipLaunchKernelGGL(k_gap_init, dim3(grid_for(g->rows + 1)), dim3(BLOCK), 0, stream, g->start, g->end, g->len, g->rows,
                       g->laid ? g->start0 : nullptr);
    HIPCHK(hipGetLastError());
  }
  if (init_side) HIPCHK(hipStreamWaitEvent(stream, ev_init[1], 0));  // (everything after sees the init facts)
}

// The base links {(X, p) : p ∈ exr*(X)} — what CR3 derives from the init facts X ∈ S(X) in the
// first superstep — installed before it (el_saturate of a fresh state): el_init left them in the
// head of the link log (X order) and sorted by pid; here the predecessor rows take them
// (pid-major), the successor rows their chain-second ones, and the link set gets them beside
// the first superstep, which finds them by a binary search of exr*(X) meanwhile (link_known).
// The base propagations likewise (the CR4 half-1 records of the init facts, pulled by the
// base links in the first superstep).  The first superstep then expands the base links, which
// the second did before; its queues start at what the second got.  The CPU oracle installs the
// same links (el_oracle.c, base_links).
void el_ctx::install_base() {
  if (nb == 0 || l_count != 0) return;
  const uint64_t trig = s_count + nb;
  if (!small_queues) {
    if (const uint64_t want = std::min<uint64_t>(4 * trig, 1ull << 28); want > cs_cap) {
      sync();
      cs_cap = next_pow2(want);
      dfree(cs_x);
      dfree(cs_a);
      cs_x = dalloc<uint32_t>(cs_cap);
      cs_a = dalloc<uint32_t>(cs_cap);
    }
    if (const uint64_t want = std::min<uint64_t>(trig, 1ull << 26); want > job_cap) {
      sync();
      job_cap = next_pow2(want);
      dfree(jobs);
      jobs = dalloc<uint4>(job_cap);
    }
  }
  const uint32_t P = hx.P;
  hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, stream, &ctr->l_log, (uint32_t)nb);
  HIPCHK(hipGetLastError());
  if (PR.live)
    launch(EL_K_INIT, [&] {
      elcl::group_fill(stream, sk, sv, (uint32_t)nb, pr_first, PR.start, PR.val);
      elcl::caps(stream, pr_first, pr_last, P, nullptr, nullptr, nullptr, PR.len);
    });
  if (SC.live && nc) launch(EL_K_INIT, [&] { elcl::succ_fill(stream, cax, cl, lo, hi, SC.start, SC.len, SC.val); });
  const bool props = nbp && use_props && PP.live;
  if (props) {
    launch(EL_K_INIT, [&] {
      elcl::group_fill(stream, plog_p, plog_b, (uint32_t)nbp, bpp_s, PP.start, PP.val);
      elcl::caps(stream, bpp_s, bpp_e, P, nullptr, nullptr, nullptr, PP.len);
    });
    hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, stream, &ctr->p_log, (uint32_t)nbp);
    HIPCHK(hipGetLastError());
    p_count = p_base = nbp;
    for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) wm_p[r] = nbp;  // (nothing left to fan out)
    host_ev[EL_K_INIT][EL_EV_ENT] += 2 * nbp;
    host_ev[EL_K_INIT][EL_EV_EMIT] += nbp;
  }
  // The base links and propagations stay out of the hash sets for the whole saturation: a
  // membership test is a binary search of the sorted row exr*(X) (bpp(pid) for a propagation,
  // a few lines of L2) before the set probe (link_known / prop_known).  Filling the sets with
  // them instead costs 25 M + 2.6 M random CAS on G3 (k_rehash, ≈2.3 ms each beside the first
  // superstep).  EL_BASE_JOIN=1 restores that fill (A/B only: the CPU oracle counts the
  // binary searches, so the event parity holds without it).
  if (getenv("EL_BASE_JOIN") && !part()) {
    HIPCHK(hipEventRecord(ev_base[0], stream));
    HIPCHK(hipStreamWaitEvent(rstream, ev_base[0], 0));
    hipLaunchKernelGGL(k_rehash, dim3(grid_for(nb, 2048)), dim3(BLOCK), 0, rstream, lhash, lhash_cap - 1, llog_x,
                       llog_p, (uint32_t)nb);
    if (props)
      hipLaunchKernelGGL(k_rehash, dim3(grid_for(nbp, 2048)), dim3(BLOCK), 0, rstream, phash, phash_cap - 1, plog_b,
                         plog_p, (uint32_t)nbp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_base[1], rstream));
    base_filling = true;
  }
  l_count = l_base = nb;
  ix.base = 1;
  // the log entries read and written, the rows' entries
  host_ev[EL_K_INIT][EL_EV_ENT] += nb + (PR.live ? nb : 0) + (SC.live ? nc : 0);
  host_ev[EL_K_INIT][EL_EV_EMIT] += nb;
  if (part()) {
    // the chain-second base links join the replicated chain-link log (the triggers of CR6 with
    // their role second, expand_x); those and the base propagations that other ranks' rows can
    // reach go into the send queues of the first exchange (the commit routes every later one)
    DState st = dstate();
    hipLaunchKernelGGL(k_base_route, dim3(grid_for(std::max(nb, nbp))), dim3(BLOCK), 0, stream, ix, st, (uint32_t)nb,
                       props ? (uint32_t)nbp : 0u);
    HIPCHK(hipGetLastError());
    x_count = nc;
  }
}

// Streamed result, in two halves so that no copy work sits between two supersteps:
// stream_mark() (after a superstep) notes the log entries committed so far, behind ev_strm (the
// event the superstep recorded right after its commit, or one recorded now behind everything);
// stream_flush() enqueues their copies and run encoding — called by the NEXT superstep once its
// own kernels are enqueued (the host's enqueue work then overlaps them), or at the fixpoint.
void el_ctx::stream_mark() {
  if (!strm) return;
  const uint64_t s1 = s_count, l1 = l_count;
  if (s1 == (mark_pending ? mark_s : strm_s) && l1 == (mark_pending ? mark_l : strm_l)) return;
  if (!strm_marked) HIPCHK(hipEventRecord(ev_strm, stream));  // (no commit of this step marked it)
  strm_marked = false;
  mark_s = s1;
  mark_l = l1;
  mark_pending = true;
}

void el_ctx::stream_flush(bool force) {
  if (!strm || !mark_pending) return;
  if (!force && (mark_s - strm_s) + (mark_l - strm_l) < stream_min) return;
  mark_pending = false;
  const uint64_t s1 = mark_s, l1 = mark_l;
  HIPCHK(hipStreamWaitEvent(dstream, ev_strm, 0));
  HIPCHK(hipStreamWaitEvent(nstream, ev_strm, 0));
  // the values by hipMemcpyAsync on dstream (NoCU: the copy-engine request for page-locked
  // buffers the device has mapped)
  auto dma = [&](uint32_t* dst, uint32_t* dst_dev, const uint32_t* src, uint64_t a, uint64_t b, uint64_t cap) {
    b = std::min(b, cap);
    if (!dst || b <= a) return;
    if (dst_dev && !dma_hostptr)
      HIPCHK(hipMemcpyAsync(dst_dev + a, src + a, (b - a) * sizeof(uint32_t), hipMemcpyDeviceToDeviceNoCU, dstream));
    else
      HIPCHK(hipMemcpyAsync(dst + a, src + a, (b - a) * sizeof(uint32_t), hipMemcpyDeviceToHost, dstream));
  };
  if (!packed) dma(strm->s_b, s_b_dev, slog_a, strm_s, s1, strm->s_cap);
  dma(strm->l_p, l_p_dev, llog_p, strm_l, l1, strm->l_cap);
  if (((strm->s_b || packed) && s1 > strm->s_cap) || (strm->l_p && l1 > strm->l_cap)) strm_ovf = true;
  runs_out(false);  // (the runs of the earlier segments whose encoding is done)
  if (s_run_dev) stream_runs(slog_x, strm_s, s1, srun, strm->s_run_cap, 0);
  if (l_run_dev) stream_runs(llog_x, strm_l, l1, lrun, strm->l_run_cap, 1);
  HIPCHK(hipEventRecord(ev_run, nstream));
  run_pending = true;
  strm_s = s1;
  strm_l = l1;
}

void el_ctx::stream_out() {
  stream_mark();
  stream_flush();
}

// DMA the runs encoded so far (wait: block until the encodings enqueued are done; else only if
// they are).  rtot_h was written by the last encoding before ev_run, so it is read only after it.
void el_ctx::runs_out(bool wait) {
  if (!run_pending) return;
  if (wait) {
    HIPCHK(hipEventSynchronize(ev_run));
  } else {
    const hipError_t q = hipEventQuery(ev_run);
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      return;
    }
    HIPCHK(q);
  }
  run_pending = false;
  const uint64_t caps[2] = {strm->s_run_cap, strm->l_run_cap};
  uint2* devs[2] = {s_run_dev, l_run_dev};
  const uint2* srcs[2] = {srun, lrun};
  for (int w = 0; w < 2; ++w) {
    const uint64_t n = std::min<uint64_t>(rtot_h[w], caps[w]);
    if (!devs[w] || n <= run_sent[w]) continue;
    if (dma_hostptr)
      HIPCHK(hipMemcpyAsync(reinterpret_cast<uint2*>(w ? strm->l_run : strm->s_run) + run_sent[w], srcs[w] + run_sent[w],
                            (n - run_sent[w]) * sizeof(uint2), hipMemcpyDeviceToHost, dstream));
    else
      HIPCHK(hipMemcpyAsync(devs[w] + run_sent[w], srcs[w] + run_sent[w], (n - run_sent[w]) * sizeof(uint2),
                            hipMemcpyDeviceToDeviceNoCU, dstream));
    run_sent[w] = n;
  }
  if (packed) {  // the codes of the segments encoded, and the escapes written so far
    auto to_host = [&](void* host, void* host_dev, const void* src, uint64_t bytes) {
      if (dma_hostptr || !host_dev)
        HIPCHK(hipMemcpyAsync(host, src, bytes, hipMemcpyDeviceToHost, dstream));
      else
        HIPCHK(hipMemcpyAsync(host_dev, src, bytes, hipMemcpyDeviceToDeviceNoCU, dstream));
    };
    const uint64_t ce = std::min<uint64_t>(code_enc, strm->s_cap);
    if (ce > code_sent)
      to_host(strm->s_code + code_sent, s_code_dev ? s_code_dev + code_sent : nullptr, scode + code_sent,
              (ce - code_sent) * sizeof(uint16_t));
    code_sent = std::max(code_sent, ce);
    const uint64_t ee = std::min<uint64_t>(etot_h[0], strm->s_esc_cap);
    if (ee > esc_sent)
      to_host(strm->s_esc + esc_sent, s_esc_dev ? s_esc_dev + esc_sent : nullptr, sesc + esc_sent,
              (ee - esc_sent) * sizeof(uint32_t));
    esc_sent = std::max(esc_sent, ee);
  }
}

// The runs of x over keys[a, b) (a log segment) into the caller's run buffer, numbered on from
// the runs of the earlier segments (rbase[which]); on nstream, which waited for the commit.
// Packed, the fact log's pass (which = 0) also writes the segment's codes and escapes.
void el_ctx::stream_runs(const uint32_t* keys, uint64_t a, uint64_t b, uint2* out, uint64_t cap, int which) {
  if (b <= a) return;
  const uint64_t nt = elst::tiles(b - a);
  stream_tiles(nt);
  elst::Codes pk;
  const bool pack = packed && which == 0;
  if (pack) {
    pk.vals = slog_a, pk.cperm = ix.cperm, pk.c_lo = ix.c_lo, pk.c_hi = ix.c_hi;
    pk.cnt = rcnt + rtiles_cap, pk.off = roff + rtiles_cap;
    pk.codes = scode, pk.code_cap = scode_cap, pk.esc = sesc, pk.esc_cap = sesc_cap;
    pk.base = ebase, pk.total = etot_d;
  }
  elst::count(nstream, keys, a, b, rcnt, pack ? &pk : nullptr);
  elcl::scan(nstream, rscan_tmp, rscan_bytes, rcnt, roff, (uint32_t)nt);
  if (pack) elcl::scan(nstream, rscan_tmp, rscan_bytes, rcnt + rtiles_cap, roff + rtiles_cap, (uint32_t)nt);
  elst::emit(nstream, keys, a, b, roff, rcnt, out, cap, rbase + which, rtot_d + which, pack ? &pk : nullptr);
  if (pack) code_enc = b;
}

void el_ctx::stream_tiles(uint64_t nt) {
  if (nt > rtiles_cap) {
    HIPCHK(hipStreamSynchronize(nstream));  // (the scratch of the last segment is free)
    dfree(rcnt);
    dfree(roff);
    dfree(rscan_tmp);
    rtiles_cap = std::max<uint64_t>(2 * nt, 4096);
    if (rtiles_cap > 0x7fffffffull) throw ElError{EL_ENOMEM, "streamed result: log segment too long"};
    rcnt = dalloc<uint32_t>(2 * rtiles_cap);
    roff = dalloc<uint32_t>(2 * rtiles_cap);
    rscan_bytes = elcl::scan_temp_bytes((uint32_t)rtiles_cap);
    rscan_tmp = dalloc<uint8_t>(rscan_bytes);
  }
}

// The fixpoint: the last segments, the counts, and (release) the next classification's reset on
// the third stream beside the DMA tail (it reads the logs, as the DMA does; el_init waits for both).
// A buffer that was too small keeps the state, so the caller can stream it again, fitted.
void el_ctx::stream_end(bool release) {
  if (!strm) return;
  stream_out();
  strm->n_facts = s_count;
  strm->n_links = l_count;
  // the last runs (the encoding is short work on its own stream: a short run buffer is known
  // here, before the release decision)
  runs_out(true);
  strm->n_s_runs = s_run_dev ? rtot_h[0] : 0;
  strm->n_l_runs = l_run_dev ? rtot_h[1] : 0;
  if (strm->n_s_runs > strm->s_run_cap || strm->n_l_runs > strm->l_run_cap) strm_ovf = true;
  strm->n_s_esc = packed ? etot_h[0] : 0;
  if (packed && strm->n_s_esc > strm->s_esc_cap) strm_ovf = true;
  strm = nullptr;
  HIPCHK(hipEventRecord(ev_copied[0], cstream));
  HIPCHK(hipEventRecord(ev_copied[1], stream));
  HIPCHK(hipEventRecord(ev_copied[2], dstream));
  copy_pending = true;
  if (release && !strm_ovf) {
    HIPCHK(hipEventRecord(ev_rows[0], stream));
    HIPCHK(hipStreamWaitEvent(rstream, ev_rows[0], 0));
    reset_device(rstream, lo, lo);
    HIPCHK(hipEventRecord(ev_reset, rstream));
    pre_reset = true;
    inited = false;
    rs.n = rl.n = ~0ull;
  }
}

// After the first superstep: the link set holds the base links (k_rehash on rstream), so
// later supersteps probe the set alone (ix.base off).  The oracle's base_join mirrors it.
void el_ctx::join_base() {
  if (!base_filling) return;
  HIPCHK(hipStreamWaitEvent(stream, ev_base[1], 0));
  base_filling = false;
  host_ev[EL_K_REHASH][EL_EV_HASH] += l_base + p_base;
  l_base = p_base = 0;
  ix.base = 0;
}

// Carry a saturated state over to indexes rebuilt for old ∪ increment (el_add_axioms).
void el_ctx::migrate_state(uint32_t N0, const std::vector<uint32_t>& pmap, const std::vector<uint8_t>& dA,
                           const std::vector<uint8_t>& dX, const std::vector<uint8_t>& dP) {
  const uint64_t N = hx.N, P = hx.P, W0 = W, W1 = ix.W;  // (column_window of the new index)
  sync();
  // (EL_TRACE_INC: per-phase wall times on stderr)
  static const bool trace = getenv("EL_TRACE_INC") != nullptr;
  auto lap_t = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!trace) return;
    sync();
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "migrate %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - lap_t).count());
    lap_t = t;
  };
  if (N != N0) {  // wider bit rows, more rows: pitched copy of the old matrix
    uint32_t* nb = dalloc<uint32_t>(N * W1);
    HIPCHK(hipMemsetAsync(nb, 0, N * W1 * sizeof(uint32_t), stream));
    HIPCHK(hipMemcpy2DAsync(nb, W1 * 4, bits, W0 * 4, W0 * 4, N0, hipMemcpyDeviceToDevice, stream));
    uint8_t* ha = dalloc<uint8_t>(N);
    HIPCHK(hipMemsetAsync(ha, 0, N, stream));
    HIPCHK(hipMemcpyAsync(ha, has_act, N0, hipMemcpyDeviceToDevice, stream));
    sync();
    dfree(bits);
    dfree(has_act);
    bits = nb;
    has_act = ha;
    W = W1;
  }
  if (summ && N != N0) {  // the summary of the re-laid-out matrix (unchanged rows keep theirs)
    dfree(summ);
    SB = summ_stride(W);
    summ = dalloc<uint8_t>((uint64_t)(hi - lo) * SB);
    HIPCHK(hipMemsetAsync(summ, 0, (uint64_t)(hi - lo) * SB, stream));
    hipLaunchKernelGGL(k_summ_build, dim3(2048), dim3(BLOCK), 0, stream, bits, W, (uint64_t)(hi - lo) * W, summ, SB);
    HIPCHK(hipGetLastError());
  }
  lap("matrix");
  rs.release();  // result rows: more rows, remapped pair ids — rebuilt on demand
  rl.release();
  dfree(act_ptr);  // the activation index covers the grown concept space
  act_n = ~0ull;
  dfree(scan_flags);
  scan_tiles = (std::max(N, P) + 1 + SCAN_TILE - 1) / SCAN_TILE;
  scan_flags = dalloc<unsigned long long>(scan_tiles);
  HIPCHK(hipMemsetAsync(scan_flags, 0, scan_tiles * sizeof(unsigned long long), stream));
  scan_epoch = 0;
  // pair ids in the logs, then the sets keyed by them
  if (!pmap.empty() && (l_count || p_count)) {
    uint32_t* dmap = dupload(pmap);
    if (l_count) hipLaunchKernelGGL(k_remap, dim3(grid_for(l_count)), dim3(BLOCK), 0, stream, llog_p, l_count, dmap);
    if (p_count) hipLaunchKernelGGL(k_remap, dim3(grid_for(p_count)), dim3(BLOCK), 0, stream, plog_p, p_count, dmap);
    HIPCHK(hipGetLastError());
    sync();
    dfree(dmap);
  }
  lap("remap");
  join_base();
  l_base = p_base = 0;  // every link goes into the set: the base links of the old index are plain links now
  ix.base = 0;
  fresh = false;
  // (sized as the next superstep's capacity check will ask, now that the base links and
  // propagations are in the sets: a second rehash there cost milliseconds)
  rehash_links(std::max<uint64_t>(lhash_cap, next_pow2(2 * (l_count + cl_cap))));
  rehash_props(std::max<uint64_t>(phash_cap, next_pow2(2 * (p_count + cp_cap))));
  lap("rehash");
  // predecessor / successor / propagation rows for the new pair and concept spaces
  if (P && need_pred) {
    PR.reshape((uint32_t)P, cl_cap);
    gap_build_sorted(PR, llog_p, llog_x, l_count, key_bits);
  } else {
    PR.release();
  }
  if (need_succ) {
    SC.reshape((uint32_t)N, cl_cap);
    gap_build_from_log(SC, llog_x, llog_p, l_count, ix.role_chs);
  } else {
    SC.release();
  }
  if (use_props) {
    PP.reshape((uint32_t)P, cp_cap + remote_bound());
    gap_build_from_log(PP, plog_p, plog_b, p_count);
  } else {
    PP.release();
  }
  lap("csrs");
  // the told closure of the new index (every concept's: old closures may have grown), with the
  // counts of the new concepts' init facts
  if (cl_alloc_n == N) {  // same concept space: only the pair-keyed buffers follow P (closure_state zeroes them)
    const uint64_t P1 = std::max<uint64_t>(P, 1);
    if (P1 > cl_alloc_p) {
      for (uint32_t** p : {&pr_first, &pr_last, &bpp_s, &bpp_e, &cap_pr, &cap_pp}) {
        dfree(*p);
        *p = dalloc<uint32_t>(P1);
      }
      cl_alloc_p = P1;
    }
    set_closure_ix();
  } else {
    free_closure();
    alloc_closure();
  }
  lap("cl-alloc");
  closure_rows(N0, (uint32_t)N);
  set_closure_ix();
  lap("closure");
  const uint64_t s_old = s_count;
  // S(X) = {X, ⊤} ∪ told*(X) for the new concepts, appended to the fact log
  if (N > N0) {
    const unsigned long long* T = clt.tot;
    const uint64_t n = T[elcl::T_INIT];
    if (s_count + n + cs_cap + ct_cap > slog_cap) {
      const uint64_t c = next_pow2(s_count + n + cs_cap + ct_cap);
      dgrow(slog_x, s_count, c);
      dgrow(slog_a, s_count, c);
      dgrow(slog_f, s_count, c);
      slog_cap = c;
    }
    check_u32_room();
    DState st = dstate();
    launch(EL_K_INIT, [&] {
      elcl::init_facts(stream, cax, cl, N0, (uint32_t)N, cpos[0], (uint32_t)s_count, slog_x, slog_a, slog_f, st.bits, W,
                       ix.c_lo, ix.c_hi, st.summ, SB);
    });
    s_count += n;
    s_init += T[elcl::T_OWN] + T[elcl::T_TWO];
    hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(1), 0, stream, &ctr->s_log, (uint32_t)s_count);
    HIPCHK(hipGetLastError());
    host_ev[EL_K_INIT][EL_EV_ENT] += T[elcl::T_OWN] + T[elcl::T_TOLD];
    host_ev[EL_K_INIT][EL_EV_RMW] += n;
    host_ev[EL_K_INIT][EL_EV_EMIT] += n;
  }
  lap("init");
  // The delta (the reference's first iteration after an increment reads
  // only the keys scored at currInc, Type1_1AxiomProcessor.java:138-141, AxiomLoader.java:119-131):
  // the state was closed under the old axioms, so a rule instance that can conclude something new
  // involves a new axiom, i.e. an index row that changed.  The first superstep therefore
  // re-triggers only the logged facts (X, A) whose A is a source of a new told / existential axiom
  // or an operand of a new conjunction (dA above), or whose X became a new link target (a new pair
  // (r, X): X's CR4 half-1 pair range grew), the logged links whose role has new role axioms (or is
  // below one), and the new concepts' init facts; from then on the saturation is semi-naive as
  // usual (retrigger_step).
  {
    uint8_t* da = dupload(dA);
    uint8_t* dx = dupload(dX);
    uint8_t* dp = dupload(dP);
    // (the lists keep their capacity across increments: a re-allocation of ~1 GB per increment
    // cost milliseconds)
    if (s_count > rt_scap) {
      dfree(rt_x);
      dfree(rt_a);
      dfree(rt_f);
      rt_scap = next_pow2(s_count);
      rt_x = dalloc<uint32_t>(rt_scap);
      rt_a = dalloc<uint32_t>(rt_scap);
      rt_f = dalloc<uint8_t>(rt_scap);
    }
    if (std::max<uint64_t>(l_count, 1) > rt_lcap) {
      dfree(rt_lx);
      dfree(rt_lp);
      rt_lcap = next_pow2(std::max<uint64_t>(l_count, 1));
      rt_lx = dalloc<uint32_t>(rt_lcap);
      rt_lp = dalloc<uint32_t>(rt_lcap);
    }
    unsigned long long* cnt = dalloc<unsigned long long>(3);
    HIPCHK(hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), stream));
    const uint64_t rn = std::max<uint64_t>(s_count, l_count);
    hipLaunchKernelGGL(k_retrigger, dim3((uint32_t)std::max<uint64_t>((rn + RT_TILE - 1) / RT_TILE, 1)), dim3(256), 0, stream,
                       slog_x, slog_a, slog_f, (uint32_t)s_old, (uint32_t)s_count, llog_x, llog_p, (uint32_t)l_count, da,
                       dx, dp, rt_x, rt_a, rt_f, rt_lx, rt_lp, cl.meta, cnt);
    HIPCHK(hipGetLastError());
    unsigned long long h[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, stream));
    sync();
    rt_ns = h[0];
    rt_nl = h[1];
    // the re-trigger step's told candidates: the rows its told sources re-walk (a longer bound
    // grew the fact log in that step — a copy of every logged fact)
    const uint64_t ct_need = next_pow2(h[2] + 1024);
    if (ct_need > ct_cap) {
      dfree(ct_x);
      dfree(ct_a);
      ct_cap = ct_need;
      ct_x = dalloc<uint32_t>(ct_cap);
      ct_a = dalloc<uint32_t>(ct_cap);
    }
    dfree(cnt);
    dfree(da);
    dfree(dx);
    dfree(dp);
    host_ev[EL_K_REHASH][EL_EV_TRIG] += s_count + l_count;  // (the selection's reads of the logs)
  }
  // The watermarks stay: what lies above them (a state that was not saturated — e.g. el_init
  // then el_add_axioms — and the new concepts' init facts) is expanded by the next supersteps
  // with the new index as usual; what lies below was closed under the old axioms, and the
  // re-trigger lists cover the part of it the new axioms reach.
  wm_x = 0;
  inc_pending = true;
  lap("retrigger");
  sync();
  stats_stale = true;
}

// Device bytes per structure (EL_TRACE_MEM, after el_saturate): what a context holds, for the
// multi-GPU memory budget.  "other" = the device's used bytes minus the listed ones
// (index buffers, scan / sort scratch, stream buffers, other contexts).
void el_ctx::mem_report() const {
  const double G = 1e9;
  const uint64_t N = hx.N, rows = hi - lo;
  auto gap = [](const GapCsr& g) { return g.live ? (double)g.val_cap * 4 + (double)g.rows * 24 + 12.0 * g.ovq_cap : 0.0; };
  struct {
    const char* what;
    double b;
  } t[] = {
      {"bit rows", (double)rows * W * 4},
      {"block summary", summ ? (double)rows * SB : 0.0},
      {"fact log", (double)slog_cap * 9},
      {"told candidates", (double)ct_cap * 8},
      {"S candidates", (double)cs_cap * 8},
      {"link log", (double)llog_cap * 8},
      {"link set", (double)lhash_cap * 8},
      {"link candidates", (double)cl_cap * 8},
      {"propagations (log, set, candidates)", (double)plog_cap * 8 + (double)phash_cap * 8 + (double)cp_cap * 8},
      {"activations (log, set, candidates)", (double)alog_cap * 8 + (double)ahash_cap * 8 + (double)ca_cap * 8 + N},
      {"jobs", (double)job_cap * 16},
      {"predecessor rows", gap(PR)},
      {"successor rows", gap(SC)},
      {"propagation rows", gap(PP)},
      {"closure rows", (double)cl.t_cap * 4 + (double)cl.e_cap * 4 + (double)cl.l_cap * 8 + 64.0 * N +
                           4.0 * elcl::ND_NUM * (N + 1) + 4.0 * cl.scratch_cap + 16.0 * N},
      {"chain-link log + exchange", (double)xlog_cap * 8 + (double)(xs_cap + xp_cap + xa_cap) * 8 +
                                        (double)(XH + 2 * xcap) * 4 * (1 + part_count)},
      {"re-trigger lists", (double)rt_scap * 9 + (double)rt_lcap * 8},
  };
  double sum = 0;
  for (auto& e : t) sum += e.b;
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  fprintf(stderr, "mem rank %u rows [%u, %u) W %u: listed %.2f GB, device used %.2f GB\n", part_rank, lo, hi, (uint32_t)W,
          sum / G, (double)(tot - fr) / G);
  for (auto& e : t)
    if (e.b > 1e8) fprintf(stderr, "mem   %-38s %7.2f GB\n", e.what, e.b / G);
}

// The first superstep after an increment (migrate_state): k_expand takes its triggers from the
// compacted re-trigger lists; the commit appends to the logs as always, so the next superstep
// continues from the logs' watermarks.
void el_ctx::retrigger_step() {
  if (!inc_pending) return;
  inc_pending = false;
  pend_dA.clear();
  pend_dX.clear();
  pend_dP.clear();
  if (!rt_ns && !rt_nl) return;
  tr_s.push_back(rt_ns);
  tr_l.push_back(rt_nl);
  tr_a.push_back(0);
  trig_override = true;
  try {
    superstep(M_ALL, 0, rt_ns, 0, rt_nl, a_count, a_count, p_count, p_count);
  } catch (...) {
    trig_override = false;
    throw;
  }
  trig_override = false;
  stream_mark();
}

// el_step after an increment: the per-rule schedule re-triggers every logged fact and link once
// (round 4's increment: the closures may have grown, so every fact re-expands its told closure)
void el_ctx::retrigger_all() {
  if (!inc_pending) return;
  inc_pending = false;
  pend_dA.clear();
  pend_dX.clear();
  pend_dP.clear();
  if (s_count) HIPCHK(hipMemsetAsync(slog_f, 0, s_count, stream));
  for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) wm_s[r] = wm_l[r] = wm_a[r] = wm_p[r] = 0;
}

// The rows of the gapped CSRs that overflowed in this step move, each alone, to gap_cap(len)
// fresh slots at the end of its CSR's slot array (the other rows stay where they are): the
// first overflow record of a row claims it and reserves its slots (k_reloc_claim), one readback
// of the slot tails grows an array that would not hold them, then the rows' in-place entries and
// the overflow entries land in the new slots (k_reloc_move) and the rows' bounds switch
// (k_reloc_commit).  Events (the CPU oracle counts the same, el_oracle.c gap_step_end): the
// overflow records read and claimed, the rows relocated, their moved and placed entries.
void el_ctx::gap_relocate_all() {
  const uint32_t ov[3] = {hc.ov_pr, hc.ov_sc, hc.ov_pp};
  if (!(ov[0] | ov[1] | ov[2])) return;
  GapCsr* gs[3] = {&PR, &SC, &PP};
  if (!reloc_rc) {
    reloc_rc = dalloc<unsigned long long>(9);
    HIPCHK(hipHostMalloc((void**)&reloc_h, 10 * sizeof(unsigned long long), hipHostMallocCoherent | hipHostMallocMapped));
    memset(reloc_h, 0, 10 * sizeof(unsigned long long));
    HIPCHK(hipHostGetDevicePointer((void**)&reloc_hd, reloc_h, 0));
  }
  auto args = [&](int i) {
    GapCsr& g = *gs[i];
    return Reloc{g.used, g.start, g.end, g.len, g.val, g.ovq, ov[i], g.nstart, g.rlist, reloc_rc + 3 * i};
  };
  hipLaunchKernelGGL(k_reloc_reset, dim3(1), dim3(64), 0, stream, reloc_rc, &ctr->ov_pr);
  HIPCHK(hipGetLastError());
  for (int i = 0; i < 3; ++i) {
    if (!ov[i]) continue;
    if (ov[i] > gs[i]->ovq_cap) throw std::runtime_error("gapped-CSR overflow queue overrun");
    launch(EL_K_SCAN, [&] { hipLaunchKernelGGL(k_reloc_claim, dim3(grid_for(ov[i])), dim3(BLOCK), 0, stream, args(i)); });
  }
  const unsigned long long seq = ++reloc_seq;
  hipLaunchKernelGGL(k_reloc_publish, dim3(1), dim3(64), 0, stream, reloc_rc, reloc_hd, (uint32_t)seq);
  HIPCHK(hipGetLastError());
  {  // the claims' totals (a spin on the published sequence word, as wait_commit does)
    volatile unsigned long long* p = reloc_h;
    for (uint64_t it = 1; p[9] != seq; ++it) {
      if ((it & 1023) == 0) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess && p[9] != seq) throw std::runtime_error("relocation counters were not published");
        if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  for (int i = 0; i < 3; ++i) {
    if (!ov[i]) continue;
    GapCsr& g = *gs[i];
    const uint64_t tail = g.used + reloc_h[3 * i], nrows = reloc_h[3 * i + 1] & 0xffffffffull,
                   moved = reloc_h[3 * i + 2];
    if (tail > 0xffffffffull) throw ElError{EL_ENOMEM, "gapped CSR beyond 2^32 slots"};
    if (tail > g.val_cap) {  // (rare: the copy needs the stream idle)
      sync();
      const uint64_t c = std::min<uint64_t>(tail + tail / 2, 0xffffffffull);
      dgrow(g.val, g.used, c);
      g.val_cap = c;
    }
    const uint32_t nb = (uint32_t)std::min<uint64_t>(nrows, 2048);
    launch(EL_K_SCATTER_OLD, [&] {
      hipLaunchKernelGGL(k_reloc_move, dim3(nb + grid_for(ov[i])), dim3(BLOCK), 0, stream, args(i), nb);
    });
    launch(EL_K_MERGE_PTR, [&] {
      hipLaunchKernelGGL(k_reloc_commit, dim3(grid_for(nrows)), dim3(BLOCK), 0, stream, args(i));
    });
    g.used = tail;
    host_ev[EL_K_SCAN][EL_EV_TRIG] += ov[i];
    host_ev[EL_K_SCAN][EL_EV_RMW] += ov[i];
    host_ev[EL_K_SCAN][EL_EV_ROW] += nrows;
    host_ev[EL_K_MERGE_PTR][EL_EV_ENT] += 2 * nrows;
    host_ev[EL_K_SCATTER_OLD][EL_EV_TRIG] += moved;
    host_ev[EL_K_SCATTER_OLD][EL_EV_ENT] += moved;
    host_ev[EL_K_SCATTER_OLD][EL_EV_EMIT] += moved;
    host_ev[EL_K_SCATTER_NEW][EL_EV_TRIG] += ov[i];
    host_ev[EL_K_SCATTER_NEW][EL_EV_ENT] += 3ull * ov[i];
    host_ev[EL_K_SCATTER_NEW][EL_EV_EMIT] += ov[i];
  }
  hc.ov_pr = hc.ov_sc = hc.ov_pp = 0;  // (zeroed on the device by k_reloc_reset)
}

void el_ctx::fill_stats(el_stats* out, double ms) {
  read_events();
  el_stats st{};
  st.supersteps = (uint32_t)tr_s.size();
  st.s_facts = s_count;
  st.s_init = s_init;
  st.links = l_count;
  st.derived = s_count - s_init + l_count;
  st.activations = a_count;
  st.propagations = p_count;
  uint64_t bytes = 0;
  static const uint64_t width[EL_NUM_EVENTS] = {8, 8, 4, 4, 8, 8, 16, 8};
  for (int k = 0; k < EL_NUM_KERNELS; ++k)
    for (int e = 0; e < EL_NUM_EVENTS; ++e) bytes += (hev[k][e] + host_ev[k][e]) * width[e];
  st.bytes = bytes;
  st.ms = ms;
  st.exchange_bytes = xrounds_bytes;
  last = st;
  stats_stale = false;
  if (out) *out = st;
}

// ---------------------------------------------------------------- C ABI

namespace {

int fail(el_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}

template <class F>
int guarded(el_ctx* c, F&& f) {
  if (!c) return EL_EINVAL;
  try {
    HIPCHK(hipSetDevice(c->device));
    c->wait_copy();  // (an EL_RESULT_ASYNC copy-back still in flight: every call sees it landed)
    return f();
  } catch (const ElError& e) {
    return fail(c, e.code, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(c, EL_ENOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(c, EL_EHIP, e.what());
  }
}

}  // namespace

extern "C" {

int el_abi_version(void) { return EL_ABI_VERSION; }

int el_device_count(int* n) {
  if (!n) return EL_EINVAL;
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return EL_EHIP;
  }
  return EL_OK;
}

int el_create(el_ctx** out, const el_config* cfg) {
  if (!out) return EL_EINVAL;
  *out = nullptr;
  el_ctx* c = new (std::nothrow) el_ctx();
  if (!c) return EL_ENOMEM;
  if (cfg) {
    if (cfg->flags & ~EL_FLAGS_KNOWN) {
      delete c;
      return EL_EINVAL;
    }
    c->flags = cfg->flags;
    c->device = cfg->device;
    c->profile = cfg->profile;
    c->xmode = cfg->exchange;
    if (c->xmode != EL_XCHG_NONE) {
      const bool bad = (c->xmode != EL_XCHG_LOCAL && c->xmode != EL_XCHG_RCCL && c->xmode != EL_XCHG_HOST) ||
                       cfg->part_count < 1 || (c->xmode == EL_XCHG_HOST && !cfg->host_allgather) ||
                       cfg->part_rank >= cfg->part_count || cfg->row_hi < cfg->row_lo ||
                       (c->xmode == EL_XCHG_LOCAL && (!cfg->group || cfg->group->n != (int)cfg->part_count));
      if (bad) {
        delete c;
        return EL_EINVAL;
      }
      c->part_rank = cfg->part_rank;
      c->part_count = cfg->part_count;
      c->cfg_lo = cfg->row_lo;
      c->cfg_hi = cfg->row_hi;
    }
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    delete c;
    return EL_EHIP;
  }
  if (c->device < 0 || c->device >= n) {
    delete c;
    return EL_EINVAL;
  }
  int rc = guarded(c, [&] {
    if (getenv("EL_STREAM_PRIO")) {
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
      HIPCHK(hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, least));
      HIPCHK(hipStreamCreateWithPriority(&c->rstream, hipStreamNonBlocking, least));
      HIPCHK(hipStreamCreateWithPriority(&c->dstream, hipStreamNonBlocking, least));
      HIPCHK(hipStreamCreateWithPriority(&c->nstream, hipStreamNonBlocking, least));
      HIPCHK(hipStreamCreateWithPriority(&c->ostream, hipStreamNonBlocking, least));
      HIPCHK(hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));
    } else {
      HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&c->rstream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&c->nstream, hipStreamNonBlocking));
    }
    for (hipEvent_t& e : c->ev_stage) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_dma) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_rows) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_reset, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_copied) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_base) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : c->ev_init) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_strm, hipEventDisableTiming | hipEventReleaseToSystem));
    if (c->xmode == EL_XCHG_LOCAL) c->xchg.reset(new LocalExchange(cfg->group, (int)c->part_rank));
    if (c->xmode == EL_XCHG_RCCL)  // collective: every rank of the group calls el_create
      c->xchg.reset(new RcclExchange((int)c->part_rank, (int)c->part_count, cfg->rccl_id));
    if (c->xmode == EL_XCHG_HOST)
      c->xchg.reset(new HostExchange((int)c->part_rank, (int)c->part_count, cfg->host_allgather, cfg->host_user));
    return EL_OK;
  });
  if (rc != EL_OK) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->rstream) (void)hipStreamDestroy(c->rstream);
    if (c->dstream) (void)hipStreamDestroy(c->dstream);
    if (c->nstream) (void)hipStreamDestroy(c->nstream);
    if (c->ostream) (void)hipStreamDestroy(c->ostream);
    if (c->ev_out) (void)hipEventDestroy(c->ev_out);
    for (hipEvent_t e : c->ev_rows)
      if (e) (void)hipEventDestroy(e);
    if (c->ev_reset) (void)hipEventDestroy(c->ev_reset);
    for (hipEvent_t e : c->ev_copied)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_base)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_init)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_stage)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_dma)
      if (e) (void)hipEventDestroy(e);
    if (c->ev_strm) (void)hipEventDestroy(c->ev_strm);
    delete c;
    return rc;
  }
  *out = c;
  return EL_OK;
}

int el_group_create(el_group** g, int n) {
  if (!g || n < 1) return EL_EINVAL;
  el_group* p = new (std::nothrow) el_group();
  if (!p) return EL_ENOMEM;
  p->n = n;
  p->src.assign(n, nullptr);
  *g = p;
  return EL_OK;
}

void el_group_destroy(el_group* g) { delete g; }

int el_rccl_unique_id(uint8_t out[128]) {
  if (!out) return EL_EINVAL;
  try {
    ncclUniqueId id;
    RCCLCHK(rccl_api().get_id(&id));
    memcpy(out, &id, 128);
    return EL_OK;
  } catch (...) {
    return EL_EHIP;
  }
}

int el_load(el_ctx* c, const el_axioms* ax) {
  if (!c || !ax) return EL_EINVAL;
  return guarded(c, [&] {
    el::AxiomStore store, eff;
    std::vector<uint32_t> fb, fr;
    std::string e = store.append(*ax);
    el::HostIndex hx;
    if (e.empty()) {
      if (c->flags & EL_FLAG_COMPAT_DISTEL_RANGE)
        eff = store;
      else
        el::elk_ranges(store, eff, fb, fr);  // H1: ELK's reading of ranges (the default)
      e = el::build_index(eff.view(), hx, c->flags);
    }
    if (!e.empty()) return fail(c, EL_EINVAL, e);
    HIPCHK(hipStreamSynchronize(c->stream));
    c->free_state();
    c->free_index();
    c->n_user = store.N;
    c->fresh_b = std::move(fb);
    c->fresh_r = std::move(fr);
    c->store = std::move(store);
    e = c->install_index(std::move(hx));
    if (!e.empty()) return fail(c, EL_EINVAL, e);
    c->alloc_state();
    c->loaded = true;
    c->inited = false;
    return EL_OK;
  });
}

// Incremental classification (AxiomLoader's isIncrementalData,
// AxiomLoader.java:119-131, 149-186): the context's ontology becomes old ∪ increment, the
// saturated state is carried over to the new indexes (pair ids remapped, bit rows widened,
// CSRs rebuilt from the logs), and every watermark is reset so the next el_saturate /
// el_step re-triggers all facts once against the new axioms and then continues semi-naively.
int el_add_axioms(el_ctx* c, const el_axioms* inc) {
  if (!c || !inc) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "el_add_axioms before el_load");
  if (c->part()) return fail(c, EL_ESTATE, "increments need a whole-ontology context");
  if (!(c->flags & EL_FLAG_COMPAT_DISTEL_RANGE) && (!c->store.rng_r.empty() || inc->n_range))
    return fail(c, EL_EINVAL, "increments with range axioms need EL_FLAG_COMPAT_DISTEL_RANGE "
                              "(ELK range fillers are numbered after the concepts)");
  return guarded(c, [&] {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    el::AxiomStore store = c->store;
    std::string e = store.append(*inc);
    el::HostIndex hx;
    if (e.empty()) e = el::build_index(store.view(), hx, c->flags);
    if (!e.empty()) return fail(c, EL_EINVAL, e);
    c->inc_ms[0] = ms_since(t0);
    c->inc_ms[1] = c->inc_ms[2] = 0;
    c->sync();
    if (!c->inited) {  // nothing saturated yet: a plain reload
      c->free_state();
      c->free_index();
      c->n_user = store.N;
      c->store = std::move(store);
      e = c->install_index(std::move(hx));
      if (!e.empty()) return fail(c, EL_EINVAL, e);
      c->alloc_state();
      return EL_OK;
    }
    // old pair id -> new pair id (the pair universe only grows)
    std::vector<uint32_t> pmap(c->hx.P);
    for (uint32_t p = 0; p < c->hx.P; ++p) {
      const uint32_t r = c->hx.pair_role[p], y = c->hx.pair_y[p];
      uint32_t q = hx.fp_ptr[y];
      while (q < hx.fp_ptr[y + 1] && hx.pair_role[q] != r) ++q;
      if (q == hx.fp_ptr[y + 1]) return fail(c, EL_EHIP, "pair universe lost a pair");
      pmap[p] = q;
    }
    const uint32_t N0 = c->hx.N;
    // the carried-over matrix keeps its columns: the old order, the new concepts after it
    if (c->hx.cperm.size() == N0) {
      hx.cperm.resize(hx.N);
      std::copy(c->hx.cperm.begin(), c->hx.cperm.end(), hx.cperm.begin());
      for (uint32_t a = N0; a < hx.N; ++a) hx.cperm[a] = a;
    }
    const auto t1 = clk::now();
    c->free_index();
    c->n_user = store.N;
    c->store = std::move(store);
    e = c->install_index(std::move(hx));
    if (!e.empty()) return fail(c, EL_EINVAL, e);
    c->sync();
    c->inc_ms[1] = ms_since(t1);
    const auto t2 = clk::now();
    // What the increment's axioms reach (migrate_state re-triggers only that):
    //  dA  the sources of new told / existential axioms and the operands of new conjunctions.
    //      told*, exr* and exl* are closed downward over told subs, so every concept below a
    //      source A has a changed row too — but each fact (X, C) with C below A has (X, A) in
    //      S(X) (the state is closed under CR1), and re-triggering (X, A) over the new rows
    //      concludes what (X, C) could: the sources alone suffice (bit 1: a new told super,
    //      the re-triggered fact re-walks its told closure)
    //  dX  concepts that became new link targets (a new pair (r, X): X's pair range grew)
    //  dP  pairs whose role has new role axioms (r ⊑ s, chains, domain, range) or is below one
    const el::HostIndex& h = c->hx;
    std::vector<uint8_t> dA(std::max<uint32_t>(h.N, 1), 0), dX(std::max<uint32_t>(h.N, 1), 0),
        dP(std::max<uint32_t>(h.P, 1), 0), dR(h.R + 1, 0);
    std::vector<uint32_t> stk;
    auto markA = [&](uint32_t a, uint8_t m) {
      if (a < h.N) dA[a] |= m;
    };
    for (uint32_t i = 0; i < inc->n_sub; ++i) markA(inc->sub_a[i], 3);
    for (uint32_t i = 0; i < inc->n_ex_rhs; ++i) markA(inc->exr_a[i], 1);
    for (uint32_t i = 0; i < inc->n_ex_lhs; ++i) markA(inc->exl_a[i], 1);
    for (uint32_t i = 0; i < inc->n_conj; ++i)
      for (uint32_t k = inc->conj_ptr[i]; k < inc->conj_ptr[i + 1]; ++k) markA(inc->conj_ops[k], 1);
    std::vector<std::vector<uint32_t>> rsub(h.R);  // role -> told sub-roles (of old ∪ increment)
    for (size_t i = 0; i < c->store.sr_r.size(); ++i)
      if (c->store.sr_s[i] < h.R) rsub[c->store.sr_s[i]].push_back(c->store.sr_r[i]);
    auto markR = [&](uint32_t r) {
      if (r < h.R && !dR[r]) dR[r] = 1, stk.push_back(r);
    };
    for (uint32_t i = 0; i < inc->n_subrole; ++i) markR(inc->sr_r[i]);
    for (uint32_t i = 0; i < inc->n_chain; ++i) markR(inc->ch_r[i]), markR(inc->ch_s[i]);
    for (uint32_t i = 0; i < inc->n_domain; ++i) markR(inc->dom_r[i]);
    for (uint32_t i = 0; i < inc->n_range; ++i) markR(inc->rng_r[i]);
    while (!stk.empty()) {
      const uint32_t r = stk.back();
      stk.pop_back();
      for (uint32_t q : rsub[r]) markR(q);
    }
    std::vector<uint8_t> had(std::max<uint32_t>(h.P, 1), 0);
    for (uint32_t q : pmap) had[q] = 1;
    for (uint32_t q = 0; q < h.P; ++q) {
      dP[q] = dR[h.pair_role[q]];
      if (!had[q]) dX[h.pair_y[q]] = 1;
    }
    // an earlier increment not saturated yet (round-5 advisor): its re-trigger lists are rebuilt
    // from the logs below, so its masks join this one's (concept ids are stable, its pair ids move
    // by pmap) — otherwise what only its axioms reach would sit below the watermarks unexpanded
    if (c->inc_pending) {
      for (size_t a = 0; a < c->pend_dA.size() && a < dA.size(); ++a) dA[a] |= c->pend_dA[a];
      for (size_t a = 0; a < c->pend_dX.size() && a < dX.size(); ++a) dX[a] |= c->pend_dX[a];
      for (size_t p = 0; p < c->pend_dP.size() && p < pmap.size(); ++p) dP[pmap[p]] |= c->pend_dP[p];
    }
    c->migrate_state(N0, pmap, dA, dX, dP);
    c->pend_dA = std::move(dA);
    c->pend_dX = std::move(dX);
    c->pend_dP = std::move(dP);
    c->inc_ms[2] = ms_since(t2);
    return EL_OK;
  });
}

int el_increment_info(el_ctx* c, double* ms, uint64_t* retrigger) {
  if (!c || !ms || !retrigger) return EL_EINVAL;
  for (int i = 0; i < 3; ++i) ms[i] = c->inc_ms[i];
  retrigger[0] = c->rt_ns;
  retrigger[1] = c->rt_nl;
  return EL_OK;
}

int el_init(el_ctx* c) {
  if (!c) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "el_init before el_load");
  return guarded(c, [&] {
    // (EL_TRACE_INIT: host wall time at each phase's end, no syncs added: where el_init's host
    // side spends its time)
    init_t0 = std::chrono::steady_clock::now();
    auto lap = init_lap;
    c->reset_state();
    lap("reset");
    c->closure_rows(c->lo, c->hi);  // told*, exr*, exl* of every concept (el_closure.h)
    lap("closure rows");
    c->closure_state();             // the init facts; base links / propagations, row layouts
    lap("state enqueued");
    c->fresh = true;
    c->inited = true;
    c->stats_stale = true;
    return EL_OK;
  });
}

int el_step(el_ctx* c, el_rule rule, int* changed) {
  if (!c || !changed || (int)rule < 0 || (int)rule >= EL_NUM_RULE_TYPES) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "el_step before el_init");
  if (c->part()) return fail(c, EL_ESTATE, "el_step needs a whole-ontology context (use el_saturate)");
  return guarded(c, [&] {
    const int r = (int)rule;
    c->retrigger_all();  // (after an increment: every logged fact once, per rule)
    c->fresh = false;  // per-rule stepping derives every link (DistEL's granularity)
    const uint64_t se = c->s_count, le = c->l_count, ae = c->a_count, pe = c->p_count;
    bool ch = c->superstep(kRuleMask[r], c->wm_s[r], se, c->wm_l[r], le, c->wm_a[r], ae, c->wm_p[r], pe);
    c->wm_s[r] = se;
    c->wm_l[r] = le;
    c->wm_a[r] = ae;
    c->wm_p[r] = pe;
    *changed = ch ? 1 : 0;
    c->fill_stats(nullptr, 0.0);
    return EL_OK;
  });
}

int el_saturate(el_ctx* c, el_stats* stats) {
  if (!c) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "el_saturate before el_init");
  return guarded(c, [&] {
    auto t0 = std::chrono::steady_clock::now();
    if (c->part() && !c->part_fixpoint) c->exchange_windows();  // (collective, once per el_load)
    if (c->fresh) c->install_base();
    c->fresh = false;
    c->stream_mark();  // (a streamed result: the init facts and base links go beside the first superstep)
    // all rule types share one frontier: start at the oldest watermark
    uint64_t sb = c->s_count, lb = c->l_count, ab = c->a_count, pb = c->p_count;
    for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) {
      sb = std::min(sb, c->wm_s[r]);
      lb = std::min(lb, c->wm_l[r]);
      ab = std::min(ab, c->wm_a[r]);
    }
    // propagations left by per-rule stepping that CR_TYPE3_2 has not fanned out yet; every
    // propagation generated by a fused superstep fans out immediately (M_R4D)
    pb = std::min(pb, c->wm_p[EL_CR_TYPE3_2]);
    uint64_t pe = c->p_count;
    c->tr_s.clear();
    c->tr_l.clear();
    c->tr_a.clear();
    const bool inc = c->inc_pending;
    c->inc_t0 = t0;
    if (!c->part()) c->retrigger_step();  // (the first superstep after an increment)
    const auto t_rt = std::chrono::steady_clock::now();
    // A partitioned context at its global fixpoint (an el_saturate that returned since the last
    // el_init: a re-stream into fitted buffers after EL_ERANGE, which one rank may do alone) runs
    // no collective superstep: its peers have left the exchange.
    if (c->part() && !c->part_fixpoint) {  // collective: every rank runs the same supersteps (global delta)
      // The whole-ontology schedule: a propagation this rank generates fans out over its own
      // predecessors at generation (M_R4D); the ones the import brought from other ranks fan out
      // over this rank's predecessors in the next superstep (M_R4P over [p_import, p_count)).
      uint64_t xb = 0;
      for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) pb = std::min(pb, c->wm_p[r]);
      xb = std::min<uint64_t>(c->x_count, c->wm_x);
      uint64_t pe2 = c->p_count;
      for (;;) {
        const uint64_t se = c->s_count, le = c->l_count, ae = c->a_count, xe = c->x_count;
        c->tr_s.push_back(se - sb);
        c->tr_l.push_back(le - lb);
        c->tr_a.push_back(ae - ab);
        const uint32_t mask = pb < pe2 ? (M_ALL | M_R4P) : M_ALL;
        const uint64_t g = c->superstep_part(mask, sb, se, lb, le, ab, ae, pb, pe2, xb, xe);
        c->stream_mark();
        c->stream_flush(false);
        sb = se, lb = le, ab = ae, xb = xe;
        pb = c->p_import, pe2 = c->p_count;
        if (g == 0) break;
      }
      c->wm_x = c->x_count;
      c->part_fixpoint = true;
    }
    for (;;) {
      if (c->part()) break;
      const uint64_t se = c->s_count, le = c->l_count, ae = c->a_count;
      if (se == sb && le == lb && ae == ab && pb == pe) break;
      c->tr_s.push_back(se - sb);
      c->tr_l.push_back(le - lb);
      c->tr_a.push_back(ae - ab);
      c->superstep(pb < pe ? (M_ALL | M_R4P) : M_ALL, sb, se, lb, le, ab, ae, pb, pe);
      c->join_base();
      c->stream_mark();
      sb = se;
      lb = le;
      ab = ae;
      pb = pe = c->p_count;
    }
    for (int r = 0; r < EL_NUM_RULE_TYPES; ++r) {
      c->wm_s[r] = c->s_count;
      c->wm_l[r] = c->l_count;
      c->wm_a[r] = c->a_count;
      c->wm_p[r] = c->p_count;
    }
    c->enqueue_events();  // hc is current (published by the last k_commit); events ride along
    const bool rel = c->strm && (c->strm->flags & EL_RESULT_RELEASE);
    c->stream_end(rel);
    c->sync();
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    static const bool trace_inc = getenv("EL_TRACE_INC") != nullptr;
    if (trace_inc && inc)
      fprintf(stderr, "increment saturate: re-trigger step %.3f ms (host clock), all %.3f ms\n",
              std::chrono::duration<double, std::milli>(t_rt - t0).count(), ms);
    c->fill_stats(stats, ms);
    static const bool trace_mem = getenv("EL_TRACE_MEM") != nullptr;
    if (trace_mem) c->mem_report();
    return EL_OK;
  });
}

int el_get_stats(el_ctx* c, el_stats* stats) {
  if (!c || !stats) return EL_EINVAL;
  if (c->stats_stale)
    return guarded(c, [&] {
      c->sync();
      c->fill_stats(stats, 0.0);
      c->stats_stale = false;
      return EL_OK;
    });
  *stats = c->last;
  return EL_OK;
}

int el_kernel_stats(el_ctx* c, el_kernel_stat* out, int n) {
  if (!c || !out || n < EL_NUM_KERNELS) return EL_EINVAL;
  return guarded(c, [&] {
    c->sync();
    c->read_counters();
    c->read_events();
    static const uint64_t width[EL_NUM_EVENTS] = {8, 8, 4, 4, 8, 8, 16, 8};
    for (int k = 0; k < EL_NUM_KERNELS; ++k) {
      el_kernel_stat s{};
      s.launches = c->launches[k];
      for (int e = 0; e < EL_NUM_EVENTS; ++e) {
        s.events[e] = c->hev[k][e] + c->host_ev[k][e];
        s.bytes += s.events[e] * width[e];
      }
      s.ms = c->kms[k];
      s.group = kernel_group(k);
      out[k] = s;
    }
    return EL_OK;
  });
}

int el_set_profile(el_ctx* c, int on) {
  if (!c) return EL_EINVAL;
  return guarded(c, [&] {
    c->sync();  // (events of launches already bracketed are read into kms first)
    c->profile = on ? 1 : 0;
    return EL_OK;
  });
}

int el_superstep_trace(el_ctx* c, uint64_t* ds, uint64_t* dl, uint64_t* da, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  *n = c->tr_s.size();
  if (cap < *n) return EL_ERANGE;
  for (size_t i = 0; i < *n; ++i) {
    if (ds) ds[i] = c->tr_s[i];
    if (dl) dl[i] = c->tr_l[i];
    if (da) da[i] = c->tr_a[i];
  }
  return EL_OK;
}

int el_get_subsumers(el_ctx* c, uint32_t x, uint32_t* out, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  if (x >= c->n_user) return fail(c, EL_EINVAL, "concept id out of range");
  if (x < c->lo || x >= c->uhi()) return fail(c, EL_EINVAL, "row not owned by this partition");
  return guarded(c, [&] {
    c->ensure_rows(true, false);
    c->sync();
    uint64_t p[2];
    HIPCHK(hipMemcpy(p, c->rs.ptr + (x - c->lo), sizeof p, hipMemcpyDeviceToHost));
    *n = p[1] - p[0];
    if (cap < *n) return EL_ERANGE;
    if (*n) HIPCHK(hipMemcpy(out, c->rs.val + p[0], *n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return EL_OK;
  });
}

namespace {
// host copy of result rows: ptr (rows + 1) and, when vals is given, the values
void read_rows(el_ctx* c, const el_ctx::Rows& r, std::vector<uint64_t>& ptr, uint32_t* vals, uint64_t n) {
  ptr.resize((size_t)(c->uhi() - c->lo) + 1);
  HIPCHK(hipMemcpy(ptr.data(), r.ptr, ptr.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (vals && n) HIPCHK(hipMemcpy(vals, r.val, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
}
}  // namespace

int el_copy_facts(el_ctx* c, uint32_t* x, uint32_t* a, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  return guarded(c, [&] {
    c->sync();
    *n = c->user_count(true);
    if (cap < *n) return EL_ERANGE;
    if (!*n) return EL_OK;
    c->ensure_rows(true, false);
    c->sync();
    std::vector<uint64_t> ptr;
    read_rows(c, c->rs, ptr, a, *n);
    for (uint32_t r = 0; r + 1 < ptr.size(); ++r)
      for (uint64_t j = ptr[r]; j < ptr[r + 1]; ++j) x[j] = c->lo + r;
    return EL_OK;
  });
}

// Links sorted by (x, r, y): each link row holds pair ranks in (role, filler) order.
int el_copy_links(el_ctx* c, uint32_t* x, uint32_t* r, uint32_t* y, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  return guarded(c, [&] {
    c->sync();
    *n = c->user_count(false);
    if (cap < *n) return EL_ERANGE;
    if (!*n) return EL_OK;
    c->ensure_rows(false, true);
    c->sync();
    std::vector<uint64_t> ptr;
    std::vector<uint32_t> q(*n);
    read_rows(c, c->rl, ptr, q.data(), *n);
    for (uint32_t row = 0; row + 1 < ptr.size(); ++row)
      for (uint64_t j = ptr[row]; j < ptr[row + 1]; ++j) {
        x[j] = c->lo + row;
        r[j] = c->rank_role[q[j]];
        y[j] = c->rank_y[q[j]];
      }
    return EL_OK;
  });
}

int el_result_info(el_ctx* c, el_result* res) {
  if (!c || !res) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  return guarded(c, [&] {
    c->sync();
    res->row_lo = c->lo;
    res->row_hi = c->uhi();
    res->n_facts = c->user_count(true);
    res->n_links = c->user_count(false);
    res->n_pairs = c->hx.P;
    return EL_OK;
  });
}

namespace {
// device address of page-locked host memory (el_host_alloc / hipHostMalloc / registered), or null
uint32_t* mapped_for_device(void* h) {
  hipPointerAttribute_t a{};
  if (!h || hipPointerGetAttributes(&a, h) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error of ours
    return nullptr;
  }
  return a.type == hipMemoryTypeHost && a.devicePointer ? (uint32_t*)a.devicePointer : nullptr;
}
}  // namespace

// Result copy-back.  Into page-locked buffers the row sorts write the sorted rows straight over
// PCIe: the S rows on the engine stream and the link rows on the copy stream at the same time,
// each row offset array by DMA behind its rows.  Rows already resident on the device (an earlier
// export) and pageable buffers go by DMA from the device rows.  EL_RESULT_RELEASE: once the
// row builds have read the state (their prep halves), the next el_init's reset runs on a third
// stream while the sorted rows still stream over PCIe; the context then has no state until
// that el_init.
int el_copy_result(el_ctx* c, el_result* res) {
  if (!c || !res) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  if (res->flags & ~EL_RESULT_FLAGS_KNOWN) return fail(c, EL_EINVAL, "unknown el_result flags");
  return guarded(c, [&] {
    c->sync();  // counts of the last superstep
    const uint64_t R1 = (uint64_t)(c->uhi() - c->lo) + 1;
    const uint64_t nf = c->user_count(true), nl = c->user_count(false);
    res->row_lo = c->lo;
    res->row_hi = c->uhi();
    res->n_facts = nf;
    res->n_links = nl;
    res->n_pairs = c->hx.P;
    if ((res->s_val && res->s_cap < nf) || (res->l_pair && res->l_cap < nl))
      return fail(c, EL_ERANGE, "result buffer too small (el_result_info gives the sizes)");
    const bool release = (res->flags & EL_RESULT_RELEASE) != 0;
    const bool async = (res->flags & EL_RESULT_ASYNC) != 0;
    if (async && !release) return fail(c, EL_EINVAL, "EL_RESULT_ASYNC needs EL_RESULT_RELEASE");
    // the S-row sorts clear the bit matrix only when they write every row (no ELK range fillers)
    const bool fuse_clear = release && c->uhi() == c->hi && !c->colperm();
    struct Part {
      bool facts;
      uint64_t* ptr_out;
      uint32_t* val_out;
      el_ctx::Rows* rows;
      uint64_t n;
      hipStream_t s;
      uint32_t* direct;
      bool readout;  // S rows read off the bit matrix in chunks, each DMA'd behind its read-out
      bool queued;   // the rows' transfers are already enqueued (read-out, or device sort + DMA)
    };
    Part parts[2] = {{false, res->l_ptr, res->l_pair, &c->rl, nl, c->cstream, nullptr, false, false},
                     {true, res->s_ptr, res->s_val, &c->rs, nf, c->stream, nullptr, false, false}};
    // the copy stream starts behind the saturation
    HIPCHK(hipEventRecord(c->ev_rows[1], c->stream));
    HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_rows[1], 0));
    // 1. everything that reads the state
    for (Part& p : parts) {
      if (!p.ptr_out && !p.val_out) continue;
      el_ctx::Rows& r = *p.rows;
      const uint64_t logged = p.facts ? c->s_count : c->l_count;  // Rows::n counts log entries
      p.direct = r.n == logged || !p.n ? nullptr : mapped_for_device(p.val_out);
      // The S rows of a page-locked buffer come off the bit matrix when reading it (its row
      // words up to each row's last entry) costs less than the log's count-scatter-sort: the
      // read-out streams at HBM rate in chunks that the DMA engine ships at PCIe rate behind it,
      // so the transfer starts after the row counts instead of after the whole build (G3:
      // matrix 19 GB vs. 415 MB of rows; PCIe at ~57 GB/s is the bound either way).
      // (measured: G3, matrix / rows = 46, read-out 0.6 ms faster; G5, 61, 0.17 ms slower)
      // With the block summary the read-out loads only marked blocks, so the matrix-to-rows ratio
      // no longer decides (the dense read-out keeps it).
      p.readout = p.direct && p.facts && !c->readout_off && !c->colperm() && p.val_out && p.n >= c->readout_min &&
                  (c->summ || (uint64_t)(c->uhi() - c->lo) * c->W * 4 <= 48 * 4 * p.n);
      if (p.readout) {
        if (!r.ptr) r.ptr = dalloc<uint64_t>(R1);
        r.n = ~0ull;
        c->readout_rows(r.ptr, p.ptr_out, p.val_out, release, release ? c->ev_rows[0] : nullptr);
        p.queued = true;
      } else if (p.direct && (p.facts ? c->s_dma : !c->links_direct)) {
        // rows sorted into device memory on the part's stream, then one DMA each for the
        // offsets and the rows (the DMA engine keeps PCIe busier than the sorts' own writes
        // to host memory, which share it with the S read-out's DMAs: G3 copy-back 13.8 -> 12.7 ms)
        const uint64_t logged = p.facts ? c->s_count : c->l_count;
        if (!r.ptr) r.ptr = dalloc<uint64_t>(R1);
        if (p.n > r.cap || !r.val) {
          dfree(r.val);
          r.cap = p.n + p.n / 8 + 1024;
          r.val = dalloc<uint32_t>(r.cap);
        }
        c->build_rows(p.facts, p.s, r.ptr, r.val);
        r.n = logged;
        if (p.ptr_out) HIPCHK(hipMemcpyAsync(p.ptr_out, r.ptr, R1 * sizeof(uint64_t), hipMemcpyDeviceToHost, p.s));
        HIPCHK(hipMemcpyAsync(p.val_out, r.val, p.n * sizeof(uint32_t), hipMemcpyDeviceToHost, p.s));
        p.queued = true;  // (phase 2 skips it)
        p.direct = nullptr;
      } else if (p.direct) {  // sorted rows straight into the caller's page-locked buffer
        if (!r.ptr) r.ptr = dalloc<uint64_t>(R1);
        r.n = ~0ull;  // r.ptr is reused; the device rows are not built
        c->build_rows(p.facts, p.s, r.ptr, p.direct, 1, fuse_clear);
      } else {
        p.direct = nullptr;
        c->ensure_rows(p.facts, !p.facts);  // engine stream
      }
    }
    if (release) {  // the next classification's reset, beside the rest of the copy-back
      // (the read-out recorded ev_rows[0] once it had counted the rows: the reset touches no
      // row it reads)
      if (!parts[1].readout) HIPCHK(hipEventRecord(c->ev_rows[0], c->stream));
      HIPCHK(hipEventRecord(c->ev_rows[1], c->cstream));
      HIPCHK(hipStreamWaitEvent(c->rstream, c->ev_rows[0], 0));
      HIPCHK(hipStreamWaitEvent(c->rstream, c->ev_rows[1], 0));
      // rows the S-row sorts (all rows) or the read-out (the caller's rows) cleared as they went
      const uint32_t clear_from = parts[1].readout ? c->uhi() : fuse_clear && parts[1].direct ? c->hi : c->lo;
      c->reset_device(c->rstream, clear_from, parts[1].readout ? c->uhi() : c->lo);
      HIPCHK(hipEventRecord(c->ev_reset, c->rstream));
    }
    // 2. the sorts into the caller's buffers, the device rows by DMA
    for (Part& p : parts) {
      if (!p.ptr_out && !p.val_out) continue;
      el_ctx::Rows& r = *p.rows;
      if (p.queued) continue;  // (its transfers are enqueued)
      if (p.direct) {
        c->build_rows(p.facts, p.s, r.ptr, p.direct, 2, fuse_clear);
        if (p.ptr_out) HIPCHK(hipMemcpyAsync(p.ptr_out, r.ptr, R1 * sizeof(uint64_t), hipMemcpyDeviceToHost, p.s));
        continue;
      }
      HIPCHK(hipEventRecord(c->ev_rows[0], c->stream));
      HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_rows[0], 0));
      if (p.ptr_out) HIPCHK(hipMemcpyAsync(p.ptr_out, r.ptr, R1 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->cstream));
      if (p.val_out && p.n)
        HIPCHK(hipMemcpyAsync(p.val_out, r.val, p.n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->cstream));
    }
    if (async) {  // the host returns now; el_result_wait (or the next call) waits for these
      HIPCHK(hipEventRecord(c->ev_copied[0], c->cstream));
      HIPCHK(hipEventRecord(c->ev_copied[1], c->stream));
      HIPCHK(hipEventRecord(c->ev_copied[2], c->dstream));
      c->copy_pending = true;
    } else {
      HIPCHK(hipStreamSynchronize(c->cstream));
      HIPCHK(hipStreamSynchronize(c->stream));
      HIPCHK(hipStreamSynchronize(c->dstream));
    }
    if (release) {  // the reset may still run: el_init waits for it, free_state too
      c->pre_reset = true;
      c->inited = false;  // no state until el_init
      c->rs.n = c->rl.n = ~0ull;
    }
    return EL_OK;
  });
}

int el_result_wait(el_ctx* c) {
  return guarded(c, [&] {  // (guarded waits for an async copy-back or a streamed result)
    if (c->strm_ovf) return fail(c, EL_ERANGE, "streamed result: a buffer was smaller than its part");
    return EL_OK;
  });
}

int el_stream_result(el_ctx* c, el_stream* s) {
  if (!c || !s) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "el_stream_result before el_init");
  if (s->flags & ~(EL_RESULT_RELEASE | EL_STREAM_PACKED)) return fail(c, EL_EINVAL, "unknown el_stream flags");
  return guarded(c, [&] {
    // the run buffers are written by the device: page-locked and mapped (el_host_alloc)
    c->s_run_dev = reinterpret_cast<uint2*>(mapped_for_device(s->s_run));
    c->l_run_dev = reinterpret_cast<uint2*>(mapped_for_device(s->l_run));
    c->s_b_dev = mapped_for_device(s->s_b);
    c->l_p_dev = mapped_for_device(s->l_p);
    if ((s->s_run && !c->s_run_dev) || (s->l_run && !c->l_run_dev))
      return fail(c, EL_EINVAL, "el_stream run buffers must be page-locked host memory (el_host_alloc)");
    c->packed = (s->flags & EL_STREAM_PACKED) != 0;
    if (c->packed) {
      c->s_code_dev = reinterpret_cast<uint16_t*>(mapped_for_device(s->s_code));
      c->s_esc_dev = mapped_for_device(s->s_esc);
      if (!s->s_code || !s->s_esc || !s->s_run)
        return fail(c, EL_EINVAL, "EL_STREAM_PACKED needs s_code, s_esc and s_run buffers");
      if (!c->ebase) {
        c->ebase = dalloc<unsigned long long>(1);
        HIPCHK(hipHostMalloc((void**)&c->etot_h, sizeof(unsigned long long), hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void**)&c->etot_d, c->etot_h, 0));
      }
      auto fitv = [&](auto*& d, uint64_t& cap, uint64_t want) {
        if (want <= cap) return;
        HIPCHK(hipStreamSynchronize(c->nstream));
        HIPCHK(hipStreamSynchronize(c->dstream));
        dfree(d);
        d = dalloc<std::remove_reference_t<decltype(*d)>>(want);
        cap = want;
      };
      fitv(c->scode, c->scode_cap, s->s_cap);
      fitv(c->sesc, c->sesc_cap, s->s_esc_cap);
      HIPCHK(hipMemsetAsync(c->ebase, 0, sizeof(unsigned long long), c->nstream));
      c->etot_h[0] = 0;
      c->code_enc = c->code_sent = c->esc_sent = 0;
    }
    if (!c->rbase) {
      c->rbase = dalloc<unsigned long long>(2);
      HIPCHK(hipHostMalloc((void**)&c->rtot_h, 2 * sizeof(unsigned long long), hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer((void**)&c->rtot_d, c->rtot_h, 0));
      HIPCHK(hipEventCreateWithFlags(&c->ev_run, hipEventDisableTiming | hipEventReleaseToSystem));
    }
    // device run buffers of the caller's capacities (grow-only; nothing of a last stream reads them)
    auto fit = [&](uint2*& d, uint64_t& cap, uint64_t want) {
      if (want <= cap) return;
      HIPCHK(hipStreamSynchronize(c->nstream));
      HIPCHK(hipStreamSynchronize(c->dstream));
      dfree(d);
      d = dalloc<uint2>(want);
      cap = want;
    };
    if (c->s_run_dev) fit(c->srun, c->srun_cap, s->s_run_cap);
    if (c->l_run_dev) fit(c->lrun, c->lrun_cap, s->l_run_cap);
    HIPCHK(hipMemsetAsync(c->rbase, 0, 2 * sizeof(unsigned long long), c->nstream));
    c->rtot_h[0] = c->rtot_h[1] = 0;
    c->run_sent[0] = c->run_sent[1] = 0;
    c->run_pending = false;
    c->strm = s;
    c->strm_ovf = false;
    // everything already logged is streamed too (from the first entry)
    c->strm_s = c->strm_l = 0;
    c->mark_pending = c->strm_marked = false;
    s->n_facts = s->n_links = s->n_s_runs = s->n_l_runs = 0;
    if (c->packed) s->n_s_esc = 0;
    return EL_OK;
  });
}

int el_stream_codes(el_ctx* c, uint32_t* concept, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "no ontology loaded");
  *n = c->code_table.size();
  if (cap < *n) return EL_ERANGE;
  if (concept) std::copy(c->code_table.begin(), c->code_table.end(), concept);
  return EL_OK;
}

int el_pid_table(el_ctx* c, uint32_t* role, uint32_t* filler, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "no ontology loaded");
  *n = c->hx.P;
  if (cap < *n) return EL_ERANGE;
  if (role) std::copy(c->hx.pair_role.begin(), c->hx.pair_role.end(), role);
  if (filler) std::copy(c->hx.pair_y.begin(), c->hx.pair_y.end(), filler);
  return EL_OK;
}

int el_pair_table(el_ctx* c, uint32_t* role, uint32_t* filler, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "no ontology loaded");
  *n = c->rank_role.size();
  if (cap < *n) return EL_ERANGE;
  if (role) std::copy(c->rank_role.begin(), c->rank_role.end(), role);
  if (filler) std::copy(c->rank_y.begin(), c->rank_y.end(), filler);
  return EL_OK;
}

int el_fresh_fillers(el_ctx* c, uint32_t* filler, uint32_t* role, size_t cap, size_t* n) {
  if (!c || !n) return EL_EINVAL;
  if (!c->loaded) return fail(c, EL_ESTATE, "no ontology loaded");
  *n = c->fresh_b.size();
  if (cap < *n) return EL_ERANGE;
  if (filler) std::copy(c->fresh_b.begin(), c->fresh_b.end(), filler);
  if (role) std::copy(c->fresh_r.begin(), c->fresh_r.end(), role);
  return EL_OK;
}

// Page-locked result buffers.  From 2 MB on: anonymous memory on 2-MB boundaries with
// MADV_HUGEPAGE, touched by the calling thread (its NUMA node), then registered mapped and
// portable — the SDMA engines' D2H copies into it ran at 56-57 GB/s in every buffer measured,
// hipHostMalloc's 4-KB pages at 50-57 and 46-55 with huge pages refused
// (scripts/micro/d2h_pages.hip, profiles/r05_d2h_pages.txt).  Smaller ones: hipHostMalloc.
namespace {
constexpr size_t HUGE_PAGE = 2ull << 20;
std::mutex host_mu;
std::unordered_map<void*, std::pair<void*, size_t>> host_maps;  // registered pointer -> mapping
}  // namespace

void* el_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (bytes >= HUGE_PAGE) {
    const size_t len = (bytes + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE + HUGE_PAGE;
    void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m != MAP_FAILED) {
      p = (void*)(((uintptr_t)m + HUGE_PAGE - 1) & ~(uintptr_t)(HUGE_PAGE - 1));
      const size_t n = len - ((char*)p - (char*)m);
      (void)madvise(p, n, MADV_HUGEPAGE);
      memset(p, 0, n);
      if (hipHostRegister(p, n, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess) {
        std::lock_guard<std::mutex> g(host_mu);
        host_maps[p] = {m, len};
        return p;
      }
      munmap(m, len);
    }
  }
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return nullptr;
  return p;
}

void el_host_free(void* p) {
  if (!p) return;
  std::pair<void*, size_t> m{nullptr, 0};
  {
    std::lock_guard<std::mutex> g(host_mu);
    auto it = host_maps.find(p);
    if (it != host_maps.end()) m = it->second, host_maps.erase(it);
  }
  if (m.first) {
    (void)hipHostUnregister(p);
    munmap(m.first, m.second);
  } else {
    (void)hipHostFree(p);
  }
}

int el_export_result(el_ctx* c, int layout, el_sink sink, void* user) {
  if (!c || !sink || (layout != EL_LAYOUT_X_TO_B && layout != EL_LAYOUT_B_TO_X)) return EL_EINVAL;
  if (!c->inited) return fail(c, EL_ESTATE, "no state");
  return guarded(c, [&] {
    c->ensure_rows(true, false);
    c->sync();
    const uint32_t N = c->n_user, lo = c->lo, hi = c->uhi();
    std::vector<uint64_t> ptr;
    std::vector<uint32_t> val(c->user_count(true));
    read_rows(c, c->rs, ptr, val.data(), val.size());
    // result node rows: classes and individuals only (⊥ and datatypes have no key)
    auto exported = [&](uint32_t x) {
      return x != EL_BOTTOM && c->hx.kind[x] != EL_KIND_DATATYPE;
    };
    std::vector<uint32_t> ks, vs;
    const size_t batch = 1 << 16;
    auto flush = [&]() -> int {
      if (ks.empty()) return 0;
      int rc = sink(user, ks.data(), vs.data(), ks.size());
      ks.clear();
      vs.clear();
      return rc;
    };
    if (layout == EL_LAYOUT_X_TO_B) {
      for (uint32_t x = lo; x < hi; ++x) {
        if (!exported(x)) continue;
        for (uint64_t j = ptr[x - lo]; j < ptr[x - lo + 1]; ++j) {
          ks.push_back(x);
          vs.push_back(val[j]);
          if (ks.size() >= batch && flush()) return fail(c, EL_EINVAL, "sink aborted");
        }
      }
    } else {
      std::vector<uint64_t> cnt(N + 1, 0);
      for (uint32_t x = lo; x < hi; ++x)
        if (exported(x))
          for (uint64_t j = ptr[x - lo]; j < ptr[x - lo + 1]; ++j) cnt[val[j] + 1]++;
      for (uint32_t b = 0; b < N; ++b) cnt[b + 1] += cnt[b];
      std::vector<uint32_t> mem(cnt[N]);
      std::vector<uint64_t> cur(cnt.begin(), cnt.end() - 1);
      for (uint32_t x = lo; x < hi; ++x)
        if (exported(x))
          for (uint64_t j = ptr[x - lo]; j < ptr[x - lo + 1]; ++j) mem[cur[val[j]]++] = x;
      for (uint32_t b = 0; b < N; ++b)
        for (uint64_t j = cnt[b]; j < cnt[b + 1]; ++j) {
          ks.push_back(b);
          vs.push_back(mem[j]);
          if (ks.size() >= batch && flush()) return fail(c, EL_EINVAL, "sink aborted");
        }
    }
    if (flush()) return fail(c, EL_EINVAL, "sink aborted");
    return EL_OK;
  });
}

const char* el_last_error(el_ctx* c) { return c ? c->err.c_str() : "null context"; }

void el_destroy(el_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& pe : c->pending) {
    (void)hipEventDestroy(pe.a);
    (void)hipEventDestroy(pe.b);
  }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  if (c->rstream) (void)hipStreamSynchronize(c->rstream);
  if (c->dstream) (void)hipStreamSynchronize(c->dstream);  // (an async copy-back's last DMAs)
  if (c->nstream) (void)hipStreamSynchronize(c->nstream);
  if (c->ostream) (void)hipStreamSynchronize(c->ostream);
  c->copy_pending = false;
  c->free_state();
  c->free_index();
  dfree(c->reloc_rc);
  if (c->reloc_h) (void)hipHostFree(c->reloc_h);
  dfree(c->rcnt);
  dfree(c->roff);
  dfree(c->rscan_tmp);
  dfree(c->rbase);
  dfree(c->srun);
  dfree(c->scode);
  dfree(c->sesc);
  dfree(c->ebase);
  if (c->etot_h) (void)hipHostFree(c->etot_h);
  dfree(c->lrun);
  if (c->rtot_h) (void)hipHostFree(c->rtot_h);
  if (c->ev_run) (void)hipEventDestroy(c->ev_run);
  if (c->nstream) (void)hipStreamDestroy(c->nstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->rstream) (void)hipStreamDestroy(c->rstream);
  if (c->dstream) (void)hipStreamDestroy(c->dstream);
  if (c->ostream) (void)hipStreamDestroy(c->ostream);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  for (hipEvent_t e : c->ev_rows)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_reset) (void)hipEventDestroy(c->ev_reset);
  for (hipEvent_t e : c->ev_copied)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_base)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_init)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_stage)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_dma)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_strm) (void)hipEventDestroy(c->ev_strm);
  delete c;
}

}  // extern "C"
