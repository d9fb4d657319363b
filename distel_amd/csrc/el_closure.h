// el_closure.h — the told closure and everything derived from it, built on the device inside
// every classification (el_init).
//
// The reference loader stores told supers only (insertType11Axioms, AxiomLoader.java:959-1049:
// one ZADD of B under A); every closure is classification work (Type1_1AxiomProcessorBase.java:
// 22-43 climbs one told edge per iteration).  This engine fires a fact's whole told closure at
// once (CR1), and CR3 / CR4 half-1 over it, so it needs per concept A
//
//   told*(A)  every B reachable from A over told A ⊑ B axioms (B != A), sorted
//   exr*(A)   the pair ids of A' ⊑ ∃r.Y over A' ∈ {A} ∪ told*(A), sorted, unique
//   exl*(A)   the (r, B) of ∃r.A' ⊑ B over the same A', sorted by (r, B), unique
//
// all of which are derived facts, so they are computed here, on the device, per classification
// — never at load.  Algorithm: Kahn levels over the told DAG, top down.  A concept is ready when
// all its told supers are done; its rows are the union of its supers' rows (plus the supers
// themselves, plus its own axioms), gathered into the wave's LDS, bitonic-sorted and made unique
// (rows beyond the LDS capacity sort in global scratch).  A level is one launch; a concept's
// children whose last super it was become the next level.  Told cycles (A ⊑ B ⊑ A) never get
// ready: those concepts (and everything below them) are closed afterwards by Jacobi relaxation
// rounds over the same row merge (rows only grow; the least fixpoint is the closure).
//
// The state pass then writes, for the context's own rows, the init facts S(X) = {X, ⊤} ∪ told*(X)
// (fact log + bit rows), the base links {(X, p) : p ∈ exr*(X)} and the base propagations
// {((r, X), B) : (r, B) ∈ exl*(X), (r, X) a pair} into the heads of their logs, at offsets from
// device scans, so the logs come out in X order, exactly as the CPU oracle writes them.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace elcl {

// The raw axiom CSRs the closure is derived from (el_load uploads them; read-only).
struct Axioms {
  uint32_t N = 0, P = 0;
  const uint32_t* cperm = nullptr;  // concept -> bit-matrix column (whole ontology; null: window order)
  const uint32_t *par_ptr = nullptr, *par = nullptr;    // A -> told supers B (A ⊑ B), sorted, B != A
  const uint32_t *chi_ptr = nullptr, *chi = nullptr;    // B -> told subs A (the transpose)
  const uint32_t *xr_ptr = nullptr, *xr = nullptr;      // A -> pids of A ⊑ ∃r.Y, sorted unique
  const uint32_t *xl_ptr = nullptr, *xl_r = nullptr, *xl_b = nullptr;  // A -> (r, B) of ∃r.A ⊑ B
  const uint32_t* cidx_ptr = nullptr;                   // A -> conjunctions A is an operand of
  const uint32_t* psup_ptr = nullptr;                   // pid -> super-role pairs (CR5 lifts)
  const uint8_t* sc_self = nullptr;                     // pid -> its role is second in a chain
  const uint32_t* sc_w = nullptr;                       // pid -> sc_self + Σ sc_self of its lifts
  // k_stats' per-entry lookups packed (one load per row entry instead of two or three lines):
  const uint2* pstat = nullptr;    // pid -> {sc_w, |psup(pid)| << 1 | sc_self}
  const uint32_t* cz = nullptr;    // A -> |cidx(A)|
  const uint32_t *fp_ptr = nullptr, *pair_role = nullptr;  // Y -> pairs (r, Y), sorted by r
  const uint8_t* kind = nullptr;
  // the concepts whose rows are built: ⊥, ⊤ and [w_lo, w_hi) (a partitioned context: its column
  // window, which holds every concept its rows can reach and is closed under told supers); the
  // others keep empty rows and cost nothing
  uint32_t w_lo = 2, w_hi = 0xffffffffu;
  // told cycles (el_index.h, HostIndex::scc_rep): the Kahn levels run over the condensed told
  // graph (par / chi / xr / xl above are then the condensed rows); null when acyclic
  const uint32_t* rep = nullptr;                        // concept -> its component's representative
  const uint32_t *tx_ptr = nullptr, *tx = nullptr;      // representative -> the other members
  const uint32_t* fol = nullptr;                        // the followers (non-representative members)
  uint32_t nfol = 0;
  // Static Kahn levels (round 6): a concept's level is a property of the told axioms (and of the
  // built window), computed once at el_load (el_ctx::static_levels): level(A) = 0 without told
  // supers, 1 for a cycle's representative without outside supers, else 1 + the largest level
  // of its supers; SKIP / FOLLOW / NONE (never ready) as k_start marks them.  With them the
  // level launches read their concepts off a list (no scan of 3N tasks per level, no pending-count
  // atomics) and get grids sized to the level.  Null: the dynamic levels.
  const uint32_t* slevel = nullptr;                     // concept -> static level
  const uint32_t* lvl_ids = nullptr;                    // the concepts of levels >= 1, by level
};

// per-node statistics (Out::nd + k * N)
enum : uint32_t {
  ND_INIT = 0,   // init facts of X: X, ⊤ (classes, individuals), told*(X) without a second ⊤
  ND_EXR = 1,    // |exr*(X)| (its base links)
  ND_PROPS = 2,  // base propagations of X (as the filler Y)
  ND_CZ = 3,     // Σ_{A ∈ told*(X)} |cidx(A)|   (CR2 candidates of the first superstep)
  ND_SC = 4,     // successor-row capacity of X: chain-second base links and their lifts
  ND_SC0 = 5,    // chain-second base links of X
  ND_LIFT = 6,   // Σ_{p ∈ exr*(X)} |psup(p)|   (CR5 lifts of the base links)
  ND_NUM = 7
};

// totals (Ctr::tot), over the own rows [lo, hi) unless noted
enum : uint32_t {
  T_INIT = 0, T_TOLD, T_EXR, T_EXL, T_PROPS, T_CZ, T_CIDX, T_TWO, T_SC, T_SC0, T_LIFT, T_OWN,
  T_STUCK,   // concepts (all rows) not closed by the Kahn levels (told cycles and below)
  T_NUM
};

// closure events (EL_K_CLOSURE), summed over all concepts
enum : uint32_t { E_TRIG = 0, E_ROW, E_ENT, E_RMW, E_NUM };

struct Ctr {
  uint32_t t_tail, e_tail, l_tail;  // row arrays: next free entry
  uint32_t ovf;                     // a row or the scratch did not fit: the build is redone larger
  unsigned long long s_tail;        // big-row scratch: next free 64-bit word
  uint32_t dirty;                   // relaxation: some row changed in this round
  uint32_t bad;                     // k_follow met a representative's row without its follower
  uint32_t pad[2];
  unsigned long long tot[T_NUM];
  unsigned long long ev[E_NUM];
};

// Per-classification outputs and working storage (device; sized by the host, grown on overflow).
struct Out {
  uint4* meta = nullptr;       // 2N: begin {told, cidx, exr, exl}, end {told, cidx, exr, exl}
  uint4* meta2 = nullptr;      // 2N: relaxation rounds write here first
  uint32_t *t_val = nullptr, *e_val = nullptr, *l_r = nullptr, *l_b = nullptr;
  uint32_t t_cap = 0, e_cap = 0, l_cap = 0;
  uint32_t* level = nullptr;   // N: Kahn level of a concept (NONE: not ready)
  uint32_t* indeg = nullptr;   // N: told supers not yet closed
  uint32_t* lvl_flag = nullptr;  // N + 2: level L has at least one concept
  uint8_t *dirty = nullptr, *dirty2 = nullptr;  // N each (relaxation)
  uint32_t* changed = nullptr;  // N: relaxation: bit T = row type T grew this round
  uint32_t* nd = nullptr;      // ND_NUM × (N + 1)
  uint32_t* rsv = nullptr;     // per wave slot: 3 × (next, end) row reservations
  uint32_t* scratch = nullptr;  // big rows
  unsigned long long scratch_cap = 0;  // 32-bit words
  Ctr* ctr = nullptr;
};

// Launch geometry shared by every level launch (the per-wave row reservations persist across them).
#ifndef EL_CLOSURE_GRID
#define EL_CLOSURE_GRID 1024
#endif
constexpr uint32_t GRID = EL_CLOSURE_GRID;  // 4 blocks per CU (k_level: 121 VGPRs, 4 waves per SIMD)
constexpr uint32_t BLOCK = 256;
constexpr uint32_t SLOTS = GRID * (BLOCK / 64);
// level marks (Out::level, Axioms::slevel)
constexpr uint32_t LVL_NONE = 0xffffffffu, LVL_SKIP = LVL_NONE - 1u, LVL_FOLLOW = LVL_NONE - 2u;
constexpr uint32_t RSV_WORDS = 6 * SLOTS;
// per-wave row reservation (entries): a row array holds its rows plus at most one partly used
// chunk per wave slot
constexpr uint32_t CHUNK = 4096;

// Everything is enqueued on s; nothing is read back (the caller reads Ctr).  Throws
// std::runtime_error on a HIP error.
// Kahn levels.  start: counters cleared, every concept's pending supers, level 0 = no told
// supers, meta = empty rows (with the static cidx ranges), per-wave reservations cleared.
void start(hipStream_t s, const Axioms& ax, const Out& o);
// one level (reads its concepts off level[]; sets the next level's flag): the three row types
// of each of its concepts are independent tasks spread over all waves
void level(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L);
// one static level L >= 1: its n concepts at ax.lvl_ids[first, first + n)
void level_list(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L, uint32_t first, uint32_t n);
// after the levels: T_STUCK, and every stuck concept marked dirty for the relaxation
void check(hipStream_t s, const Axioms& ax, const Out& o);
// after the levels: the rows of the told cycles' followers from their representatives' rows
// followers of told cycles whose representative's row is final (level < L: built by the levels
// launched so far; all: every representative, after the relaxation rounds)
void follow(hipStream_t s, const Axioms& ax, const Out& o, uint32_t L, bool all);
// one relaxation round over the dirty concepts (told cycles), its grown rows committed;
// Ctr::dirty = some row grew
void relax(hipStream_t s, const Axioms& ax, const Out& o);
// per-concept statistics (Out::nd) of the final rows of [a, b); props: count the base
// propagations (ND_PROPS)
void stats(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, bool props);
// totals over the own rows [lo, hi) and the closure events over all rows (adds to Ctr::tot / ev)
void totals(hipStream_t s, const Axioms& ax, const Out& o, uint32_t lo, uint32_t hi);

// device-wide exclusive scan (n entries) and stable key/value radix sort (hipcub); *_temp_bytes
// sizes their scratch
size_t scan_temp_bytes(uint32_t n);
void scan(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n);
size_t sort_temp_bytes(uint32_t n);
void sort_pairs(hipStream_t s, void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                uint32_t* vout, uint32_t n, uint32_t key_bits);

// ---- state pass over the rows [a, b); pos = exclusive scan of the rows' counts (b - a + 1)
// init facts at slog[base + pos[x - a] ...] and their bits (row x at bits + x·W, columns ⊥, ⊤,
// then [c_lo, c_hi); block summary summ + x·SB, or null)
void init_facts(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t base, uint32_t* slog_x, uint32_t* slog_a, uint8_t* slog_f, uint32_t* bits, uint64_t W,
                uint32_t c_lo, uint32_t c_hi, uint8_t* summ, uint32_t SB);
// base links (X, p), p ∈ exr*(X), at llog[pos[x - a] ...]
void base_links(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t* llog_x, uint32_t* llog_p);
// base propagations (pid, B) of every Y at plog[pos[y - a] ...]
void base_props(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* pos,
                uint32_t* plog_p, uint32_t* plog_b);
// first[k] / last[k] + 1: the run of key k in keys[0, n) (keys grouped; absent keys untouched)
void runs(hipStream_t s, const uint32_t* keys, uint32_t n, uint32_t* first, uint32_t* last);
// per key p < n: c = last[p] - first[p]; len[p] = c (if len); cap[p] += c and, with psup_ptr,
// cap[u] += c for every u in psup(p) (if cap)
void caps(hipStream_t s, const uint32_t* first, const uint32_t* last, uint32_t n, const uint32_t* psup_ptr,
          const uint32_t* psup, uint32_t* cap, uint32_t* len);
// val[start[keys[i]] + i - first[keys[i]]] = vals[i]
void group_fill(hipStream_t s, const uint32_t* keys, const uint32_t* vals, uint32_t n, const uint32_t* first,
                const uint32_t* start, uint32_t* val);
// successor rows of the base links of rows [a, b): chain-second pids of exr*(X)
void succ_fill(hipStream_t s, const Axioms& ax, const Out& o, uint32_t a, uint32_t b, const uint32_t* start,
               uint32_t* len, uint32_t* val);

}  // namespace elcl
