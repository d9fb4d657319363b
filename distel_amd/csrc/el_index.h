// el_index.h — host-side construction of the device-resident axiom indexes.
//
// The reference keeps every axiom type in its own Redis shard keyed by the
// packed-ID string of the premise (AxiomLoader.java:654-1132).  Here the same
// information becomes read-only CSR arrays in HBM, one per rule family, in a
// canonical order (every row sorted ascending, duplicates dropped) so the GPU
// kernels and the CPU oracle count identical algorithmic events.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "el_gpu.h"

namespace el {

struct Csr {
  std::vector<uint32_t> ptr;   // rows + 1
  std::vector<uint32_t> a;     // first value column
  std::vector<uint32_t> b;     // optional second value column (empty if unused)
};

struct HostIndex {
  uint32_t N = 0;   // concepts
  uint32_t R = 0;   // roles
  uint32_t P = 0;   // (role, filler) pairs = link targets
  std::vector<uint8_t> kind;          // EntityType digit per concept

  Csr told;       // A -> B of told A ⊑ B (B != A), sorted    CR1 (the closure is built on the device)
  Csr toldT;      // B -> A of told A ⊑ B: the transpose (the device closure's Kahn levels)
  Csr cidx;       // A -> conj id c              CR2  conjunct index (AxiomLoader.java:931-941, DB3)
  Csr conj;       // c -> operands (sorted)      CR2
  std::vector<uint32_t> conj_b;     // c -> B
  Csr exr;        // A -> pid of A ⊑ ∃r.B, sorted unique                 CR3 (told axioms only)
  Csr exl;        // A -> (r, B) of ∃r.A ⊑ B, sorted by (r, B), unique   CR4 half-1 (idem)
  std::vector<uint32_t> fp_ptr;     // Y -> pid range (pairs sorted by (Y, r))
  std::vector<uint32_t> pair_role;  // pid -> r
  std::vector<uint32_t> pair_y;     // pid -> Y
  Csr psup;       // pid -> pids of (s, Y), s ∈ supers+(r)       CR5
  Csr chf;        // r -> (s, t) for r ∘ s ⊑ t                    CR6 (r first)
  Csr chs;        // s -> (p, t) for p ∘ s ⊑ t                    CR6 (s second)
  Csr dom;        // r -> D
  Csr rng;        // r -> C
  std::vector<uint8_t> role_has_exl;  // r -> any ∃r.A ⊑ B
  // per pid: its role is second in a chain (its links feed the successor rows), and that count
  // plus the same for its CR5 lifts (the successor-row capacity one base link asks for)
  std::vector<uint8_t> sc_self;
  std::vector<uint32_t> sc_w;
  // Told cycles (A ⊑ B ⊑ A, e.g. a named equivalence: Normalizer.java:277-279 turns
  // EquivalentClasses(A B) into two SubClassOf axioms): the strongly connected components of the
  // told graph, condensed for the device closure's Kahn levels.  Every member of a component C has
  // the same told*(A) ∪ {A} = C ∪ the supers' closures and the same exr* / exl* rows, so the
  // closure builds them once, for C's representative (its smallest member), over C's outside
  // supers and all members' own axioms; the other members (followers) copy the told row (with
  // the representative in and themselves out) and share the other two.  Empty when acyclic.
  // (A property of the told axioms, like the transpose and the role closure: the closure over it
  // is still built on the device in every el_init.)
  std::vector<uint32_t> scc_rep;      // concept -> its component's representative (itself if none)
  std::vector<uint32_t> followers;    // members that are not representatives, ascending
  Csr told_c, toldT_c, exr_c, exl_c;  // the condensed told rows / transpose / own-axiom rows
  Csr told_x;                         // representative -> the other members (its told row's extras)
  // concept -> bit-matrix column of a whole-ontology context (column_order): ⊥ and ⊤ at 0 and 1,
  // the concepts expected to be the most frequent CR4 conclusions next, then the rest in id order.
  // (A layout of the axioms' statistics, like the transposes: no concept closure is used.)
  std::vector<uint32_t> cperm;
  std::vector<double> cscore;  // the order's score per concept (a partition orders its window by it)
  std::vector<double> cdesc;   // told-DAG descendants per concept (paths counted): the init facts' weight
};

// Owned copy of the typed axioms (el_load copies its input; el_add_axioms appends an
// increment: the concept and role id spaces may grow, existing ids keep their kind).
struct AxiomStore {
  uint32_t N = 0, R = 0;
  std::vector<uint8_t> kind;
  std::vector<uint32_t> sub_a, sub_b, conj_ptr{0}, conj_ops, conj_b, exr_a, exr_r, exr_b, exl_r, exl_a, exl_b,
      sr_r, sr_s, ch_r, ch_s, ch_t, dom_r, dom_c, rng_r, rng_c;
  std::string append(const el_axioms& ax);  // "" or an error (nothing appended then)
  el_axioms view() const;
};

// Validates ids and builds the canonical indexes of the axioms as told: rows of the typed
// axioms the way AxiomLoader.java:959-1132 keys them, plus the role tables (role hierarchy
// closure, pair universe, chains).  Nothing here depends on a concept closure: told*(A) and
// the rows over it are classification work (el_closure.h).  Returns "" on success or an error
// message (the reference throws on unknown concepts, AxiomLoader.java:1343-1354).
// flags: el_config.flags (EL_FLAG_COMPAT_DISTEL_CHAIN indexes the DistEL chain set).
std::string build_index(const el_axioms& ax, HostIndex& out, uint32_t flags = 0);
void column_order(const el_axioms& ax, HostIndex& o);
// concept -> column for the window [lo, hi): ⊥, ⊤, the window's HOT highest scores, the rest of
// the window in id order (entries outside the window: NONE)
std::vector<uint32_t> column_perm(const HostIndex& o, uint32_t lo, uint32_t hi);

// H1, the default: ranges read the ELK way, as the normalizer eliminates
// them (Normalizer.java:122-137, 455-497).  Every CR3 axiom A ⊑ ∃r.B whose role has ranges
// ranges*(r) (the ranges of r and of its super-roles) and whose filler is a class gets the
// fresh filler F = n_concepts + i standing for B ⊓ ranges*(r) — one per (B, r), numbered in
// first-occurrence order — with told F ⊑ B and F ⊑ C for C ∈ ranges*(r); an individual filler
// b gets b ⊑ C (it is an r-successor); a datatype filler is left alone.  The range axioms are
// consumed.  fresh_b / fresh_r describe the fresh fillers.  (Exact for ontologies within
// EL++'s restriction that a role inclusion r1∘…∘rk ⊑ s implies ranges(s) ⊆ ranges(rk).)
void elk_ranges(const AxiomStore& in, AxiomStore& out, std::vector<uint32_t>& fresh_b,
                std::vector<uint32_t>& fresh_r);

// H2 (EL_FLAG_COMPAT_DISTEL_CHAIN): the chain set DistEL's CR6 effectively applies,
// {r∘s⊑t : some r∘s⊑t' and some r∘s'⊑t told}, sorted and deduplicated.
void distel_chain_set(const el_axioms& ax, std::vector<uint32_t>& r, std::vector<uint32_t>& s,
                      std::vector<uint32_t>& t);

}  // namespace el
