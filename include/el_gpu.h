/*
 * el_gpu.h — C-ABI of the MI355X-native EL+ saturation engine (distel_amd).
 *
 * Drop-in boundary for DistEL's hot path:
 *
 *   reference interface                                  replaced by
 *   ---------------------------------------------------  ---------------------------
 *   AxiomLoader typed KV layout (AxiomLoader.java:597-   el_load()   (typed uint32 arrays,
 *     1132, ids from mapConceptToID :1155-1341)                       one per rule crosswalk row)
 *   S(X)={X,T} init (AxiomLoader.java:1237-1245,         el_init()
 *     individuals :1281-1289)
 *   AxiomProcessor.processOneWorkChunk(...) -> boolean   el_step(ctx, rule, &changed)
 *     (base/AxiomProcessor.java:14-21), dispatched by
 *     ELClassifier.classify() switch (ELClassifier.java:74-111)
 *   whole classify-all.sh run + CommunicationHandler     el_saturate()
 *     termination (CommunicationHandler.java:49-84)
 *   result node DB0 B->{X} / ResultRearranger DB1         el_copy_result() (copy-back, CSR),
 *     X->{B} (ResultRearranger.java:57-105)                el_export_result(), el_get_subsumers()
 *   AxiomCounter totals (AxiomCounter.java:168-216)      el_stats
 *
 * Conventions
 *   - Concept ids are dense uint32 in [0, n_concepts).  0 = owl:Nothing (BOTTOM_ID,
 *     Constants.java:30), 1 = owl:Thing (TOP_ID, Constants.java:31).  Classes,
 *     individuals and datatypes share this space; concept_kind[] carries the
 *     EntityType digit (EntityType.java:9-12: 0 class, 1 individual, 3 datatype).
 *   - Role ids are dense uint32 in [0, n_roles) (their own space).
 *   - Every function returns 0 (EL_OK) or a negative EL_E* code; no C++ exception
 *     crosses the ABI.  el_last_error() gives the message for the last failure.
 *   - Input arrays are COPIED; the caller keeps ownership.
 *   - A context is single-threaded (like one DistEL rule process); independent
 *     contexts are thread-safe.  Multi-GPU = one context per rank (config.device).
 *   - There is no CPU fallback: every compute entry point runs HIP kernels on
 *     gfx950 and fails with EL_EHIP when no device is present.
 */
#ifndef EL_GPU_H
#define EL_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EL_ABI_VERSION 8

/* return codes */
#define EL_OK        0
#define EL_EINVAL   -1   /* bad argument / malformed axioms (AxiomLoader.java:1343-1354 throws) */
#define EL_ENOMEM   -2   /* device or host allocation failed */
#define EL_EHIP     -3   /* HIP runtime error (no device, launch failure, ...) */
#define EL_ESTATE   -4   /* call out of order (e.g. el_step before el_init) */
#define EL_ERANGE   -5   /* caller buffer too small; *n holds the size needed */

/* concept kinds = EntityType digits (EntityType.java:9-12) */
#define EL_KIND_CLASS      0
#define EL_KIND_INDIVIDUAL 1
#define EL_KIND_DATATYPE   3

#define EL_BOTTOM 0u
#define EL_TOP    1u

/* Per-rule-type entry points = AxiomDistributionType (init/AxiomDistributionType.java:9-31).
 * Each maps to the completion rules it owns in this engine:
 *   CR_TYPE1_1  CR1  A ⊑ B
 *   CR_TYPE1_2  CR2  A1 ⊓ … ⊓ An ⊑ B
 *   CR_TYPE2    CR3  A ⊑ ∃r.B, plus domain/range class assertions
 *               (RolePairHandler.insertClassAssertions :456-491 runs in the T2 process)
 *   CR_TYPE3_1  CR4 half-1: new A ∈ S(Y), ∃r.A ⊑ B, (X,Y) ∈ R(r)  => B ∈ S(X)
 *   CR_TYPE3_2  CR4 half-2: new (X,Y) ∈ R(r), A ∈ S(Y), ∃r.A ⊑ B  => B ∈ S(X)
 *   CR_TYPE4    CR5  r ⊑ s
 *   CR_TYPE5    CR6  r ∘ s ⊑ t
 *   CR_TYPE_BOTTOM  ⊥ ∈ S(Y), (X,Y) ∈ R(r) => ⊥ ∈ S(X)               */
typedef enum el_rule {
  EL_CR_TYPE1_1 = 0,
  EL_CR_TYPE1_2 = 1,
  EL_CR_TYPE2 = 2,
  EL_CR_TYPE3_1 = 3,
  EL_CR_TYPE3_2 = 4,
  EL_CR_TYPE4 = 5,
  EL_CR_TYPE5 = 6,
  EL_CR_TYPE_BOTTOM = 7,
  EL_NUM_RULE_TYPES = 8
} el_rule;

/* Normalized axioms, one typed array group per rule crosswalk row.
 * All pointers may be NULL when the matching count is 0. */
typedef struct el_axioms {
  uint32_t n_concepts;            /* >= 2 (⊥, ⊤) */
  uint32_t n_roles;
  const uint8_t* concept_kind;    /* n_concepts entries, or NULL = all classes */

  /* CR1  A ⊑ B                                   (insertType11Axioms :959-1049) */
  uint32_t n_sub;
  const uint32_t* sub_a;
  const uint32_t* sub_b;

  /* CR2  A1 ⊓ … ⊓ An ⊑ B, operands as CSR      (insertType12Axioms :900-957) */
  uint32_t n_conj;
  const uint32_t* conj_ptr;       /* n_conj + 1 offsets into conj_ops */
  const uint32_t* conj_ops;
  const uint32_t* conj_b;

  /* CR3  A ⊑ ∃r.B (incl. property assertions)   (insertType2Axioms :747-841) */
  uint32_t n_ex_rhs;
  const uint32_t* exr_a;
  const uint32_t* exr_r;
  const uint32_t* exr_b;

  /* CR4  ∃r.A ⊑ B                                (insertType31Axioms :654-729) */
  uint32_t n_ex_lhs;
  const uint32_t* exl_r;
  const uint32_t* exl_a;
  const uint32_t* exl_b;

  /* CR5  r ⊑ s                                   (insertType4Axioms :1051-1082) */
  uint32_t n_subrole;
  const uint32_t* sr_r;
  const uint32_t* sr_s;

  /* CR6  r ∘ s ⊑ t  (binary chains only, :1109) (insertType5Axioms :1084-1132) */
  uint32_t n_chain;
  const uint32_t* ch_r;
  const uint32_t* ch_s;
  const uint32_t* ch_t;

  /* domain(r) = D, range(r) = C                (insertPropertyDomainRangeAxioms :843-898) */
  uint32_t n_domain;
  const uint32_t* dom_r;
  const uint32_t* dom_c;
  uint32_t n_range;
  const uint32_t* rng_r;
  const uint32_t* rng_c;
} el_axioms;

/* Row partition of the concept space.  A partitioned context owns the
 * rows S(X), X in [row_lo, row_hi), and the links (X, r, Y) of those X; CR4 propagations,
 * range activations and the links of chain-second roles are replicated where they can matter.
 * Every superstep all-gathers the per-rank delta counts, whose sum is the termination test
 * (replaces the "anything new?" broadcast, CommunicationHandler.java:49-84), and each rank's
 * new propagations / activations / chain links that some OTHER rank's rows can reach (the
 * delta exchange; every rank's column window is all-gathered once, at the first el_saturate
 * after el_load).  All ranks of a group must call el_saturate together (it is collective),
 * except a re-stream at the fixpoint after EL_ERANGE, which runs no superstep. */
#define EL_XCHG_NONE  0   /* whole ontology, no partition (the default) */
#define EL_XCHG_LOCAL 1   /* in-process group: one context per thread (el_group_create) */
#define EL_XCHG_RCCL  2   /* one context per process/GPU, RCCL all-gather over xGMI */
#define EL_XCHG_HOST  3   /* one context per process, all-gather by the caller's transport */

typedef struct el_group el_group;

/* EL_XCHG_HOST transport: the caller's all-gather over host memory (MPI, gloo, the JNI host's
 * own sockets — what CommunicationHandler.java:49-84 does over Redis).  send holds this rank's
 * `bytes`; recv (size × bytes) gets every rank's block in rank order.  Both are page-locked host
 * buffers of the context, valid for the call only.  Return 0, or nonzero to fail the superstep
 * (el_saturate returns EL_ESTATE).  Called on the thread that calls el_init / el_saturate. */
typedef int (*el_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);

/* el_config.flags.  EL_FLAG_COMPAT_DISTEL_CHAIN reproduces parity hazard H2 (SURVEY.md
 * §8.H) deterministically: DistEL's CR6 joins DB1["Yr"] (X with (X,Y) ∈ R(r)) with DB4["Yr"]
 * (Z with (Y,Z) ∈ R(s) for ANY s second in a chain whose first role is r) and adds (X,Z) to
 * the t of EVERY chain whose first role is r (Type5AxiomProcessorBase.java:115-154;
 * RolePairHandler.java:395-443).  That is the complete join over the chain set
 * {r∘s⊑t : s ∈ second(r), t ∈ third(r)}, which el_load builds in place of the told chains.
 * Default (0): the correct EL+ join on s. */
#define EL_FLAG_COMPAT_DISTEL_CHAIN 0x1u
/* Range axioms (parity hazard H1).  Default: ELK's reading, by the range
 * elimination of the normalizer (Normalizer.java:122-137, 455-497): a CR3 axiom A ⊑ ∃r.B whose
 * role has ranges points its links at a fresh internal filler F = B ⊓ ranges*(r) (ids
 * n_concepts, n_concepts + 1, …; see el_fresh_fillers); an individual filler b gets b ⊑ C;
 * datatype fillers are untouched.  ranges*(r) holds the ranges of r AND of its super-roles: an
 * r-successor is an s-successor for r ⊑ s, so ELK (the reference's diff oracle) puts it under
 * range(s) too.  Deliberate deviation: the reference Normalizer looks up the existential's own
 * property only (objPropRangeMap.get(ope), Normalizer.java:462-489), which misses those
 * subsumptions (KAT tests/golden/kat_range.elax pins the complete reading).  The result rows
 * cover the caller's concepts only; link fillers may be fresh ids.
 * EL_FLAG_COMPAT_DISTEL_RANGE: DistEL's reading instead (RolePairHandler.java:471-479, K10
 * ScriptsCollection.java:45-62): a link into Y activates Y ⊑ C, and C joins every S(X)
 * holding Y. */
#define EL_FLAG_COMPAT_DISTEL_RANGE 0x2u
#define EL_FLAGS_KNOWN (EL_FLAG_COMPAT_DISTEL_CHAIN | EL_FLAG_COMPAT_DISTEL_RANGE)

typedef struct el_config {
  int device;            /* HIP device ordinal (one context per GPU / rank) */
  int profile;           /* 1 = record per-kernel HIP-event times (el_kernel_stats) */
  uint32_t flags;        /* EL_FLAG_* bits; an unknown bit is EL_EINVAL */
  int exchange;          /* EL_XCHG_*; NONE ignores every field below */
  uint32_t part_rank;    /* this context's rank in [0, part_count) */
  uint32_t part_count;   /* ranks in the group */
  uint32_t row_lo, row_hi;  /* owned rows; row_lo = row_hi = 0: the equal split of [0, N) */
  el_group* group;       /* EL_XCHG_LOCAL: shared by the group's contexts */
  uint8_t rccl_id[128];  /* EL_XCHG_RCCL: ncclUniqueId made by el_rccl_unique_id on rank 0 */
  el_allgather_fn host_allgather;  /* EL_XCHG_HOST: the transport */
  void* host_user;                 /* EL_XCHG_HOST: its first argument */
} el_config;

/* Work-phase ids for el_kernel_stats.  Several phases share one launch: the
 * generation roles run in k_expand, the commit roles in k_commit, the scan and the
 * new row offsets in k_scan_merge (names as in the rocprofv3 kernel trace).  A
 * phase's events are its own; launches and ms are reported on the phase that
 * names the launch (el_kernel_stat.group). */
typedef enum el_kernel {
  EL_K_EXPAND_S = 0,     /* k_expand, ΔS role:   CR1, CR2, CR3, CR4 half-1, ⊥ (Y side), range */
  EL_K_EXPAND_L = 1,     /* k_expand, Δlink role: CR4 half-2, CR5, CR6, ⊥, domain/range */
  EL_K_JOBS = 2,         /* k_jobs:      fan-out over predecessor / successor lists */
  EL_K_EXPAND_A = 3,     /* k_expand, activation role: column sweep of S */
  EL_K_COMMIT_S = 4,     /* k_commit, S role:    bit-row atomicOr dedup + ΔS append */
  EL_K_COMMIT_L = 5,     /* k_commit, link role: link hash-set dedup + Δlink append */
  EL_K_COMMIT_A = 6,     /* k_commit, activation role: activation set dedup */
  EL_K_SCAN = 7,         /* k_reloc_claim: gapped-CSR rows that overflowed claim fresh slots */
  EL_K_MERGE_PTR = 8,    /* k_reloc_commit: the relocated rows' new bounds */
  EL_K_SCATTER_OLD = 9,  /* k_reloc_move: a relocated row's in-place entries to its new slots */
  EL_K_SCATTER_NEW = 10, /*   … and the overflow entries placed at their rank (same launch) */
  EL_K_INIT = 11,        /* k_init_facts: S(X) = {X, ⊤} ∪ told*(X); the base links / propagations */
  EL_K_REHASH = 12,      /* k_rehash:    link / activation / propagation set growth */
  EL_K_EXPAND_P = 13,    /* k_expand, propagation role: new CR4 propagations × predecessors */
  EL_K_COMMIT_P = 14,    /* k_commit, propagation role: CR4 propagation set dedup ("Yr" -> B) */
  EL_K_COMMIT_T = 15,    /* k_commit_told: CR1 told-closure candidates, committed first */
  EL_K_CLOSURE = 16,     /* k_level / k_relax: the told closure rows told*, exr*, exl* (el_init) */
  EL_NUM_KERNELS = 17
} el_kernel;

/* Algorithmic event counters; identical in the CPU oracle. */
typedef enum el_event {
  EL_EV_TRIG = 0,   /* trigger facts read             8 B */
  EL_EV_ROW = 1,    /* index / CSR row lookups        8 B (ptr pair) */
  EL_EV_ENT = 2,    /* 4-byte index entries read      4 B */
  EL_EV_TEST = 3,   /* bit-word tests                 4 B */
  EL_EV_HASH = 4,   /* link / activation set probes   8 B (nominal, one per lookup) */
  EL_EV_EMIT = 5,   /* candidates / facts written     8 B */
  EL_EV_JOB = 6,    /* fan-out job records written or read 16 B */
  EL_EV_RMW = 7,    /* bit-word read-modify-writes    8 B */
  EL_NUM_EVENTS = 8
} el_event;

typedef struct el_kernel_stat {
  uint64_t launches;
  uint64_t events[EL_NUM_EVENTS];
  uint64_t bytes;        /* algorithmic bytes = Σ events × width above */
  double ms;             /* Σ HIP-event time (only with config.profile = 1) */
  uint32_t group;        /* phase whose launches / ms include this phase's work */
} el_kernel_stat;

typedef struct el_stats {
  uint32_t supersteps;         /* Jacobi supersteps until the delta was empty */
  uint64_t s_facts;            /* Σ_X |S(X)| over all concepts (incl. init) */
  uint64_t s_init;             /* init facts (S(X) = {X, ⊤}) */
  uint64_t links;              /* Σ_r |R(r)| */
  uint64_t derived;            /* s_facts - s_init + links   */
  uint64_t activations;        /* range activations (Y, C) */
  uint64_t propagations;       /* CR4 propagations ((r, Y), B): B for every X with (X, Y) ∈ R(r) */
  uint64_t bytes;              /* Σ algorithmic bytes over all kernels */
  double ms;                   /* wall ms of the call (device synchronised) */
  uint64_t exchange_bytes;     /* partitioned: bytes this rank received from the delta all-gathers */
} el_stats;

typedef struct el_ctx el_ctx;

/* batch sink for el_export_result: n (key, value) pairs */
typedef int (*el_sink)(void* user, const uint32_t* keys, const uint32_t* vals, size_t n);

#define EL_LAYOUT_X_TO_B 0   /* rearranged view X -> {B}   (ResultRearranger DB1) */
#define EL_LAYOUT_B_TO_X 1   /* result node DB0 B -> {X}   (AxiomLoader.java:1237-1245) */

int el_abi_version(void);
int el_device_count(int* n);

int el_create(el_ctx** ctx, const el_config* cfg);
/* in-process exchange group for EL_XCHG_LOCAL (n contexts on n threads) */
int el_group_create(el_group** g, int n);
void el_group_destroy(el_group* g);
/* RCCL unique id for EL_XCHG_RCCL (rank 0 makes it, the launcher broadcasts it) */
int el_rccl_unique_id(uint8_t out[128]);
int el_load(el_ctx* ctx, const el_axioms* ax);
int el_init(el_ctx* ctx);
/* Incremental classification (AxiomLoader isIncrementalData, AxiomLoader.java:119-131):
 * the ontology becomes old ∪ inc.  inc uses the same id spaces, possibly extended
 * (n_concepts / n_roles >= the loaded ones; existing concepts keep their kind; NULL
 * concept_kind = new concepts are classes).  A saturated state is kept and the next
 * el_saturate / el_step continues from it.  Whole-ontology contexts only. */
int el_add_axioms(el_ctx* ctx, const el_axioms* inc);

/* The last el_add_axioms, for measurement: ms[0] the host index build of old ∪ increment
   (AxiomLoader's part), ms[1] its upload, ms[2] the device state carried over (told closure of
   the new index, CSRs, sets, re-trigger lists: classification work); retrigger[0] / [1] the logged
   facts / links the increment's axioms reach, which the next el_saturate's first superstep
   re-triggers (Type1_1AxiomProcessor.java:138-141 reads only the keys scored at currInc). */
int el_increment_info(el_ctx* ctx, double ms[3], uint64_t retrigger[2]);
int el_step(el_ctx* ctx, el_rule rule, int* changed);
int el_saturate(el_ctx* ctx, el_stats* stats);
int el_get_stats(el_ctx* ctx, el_stats* stats);
int el_kernel_stats(el_ctx* ctx, el_kernel_stat* out, int n);
/* Per-kernel HIP-event timing on or off between calls (config.profile at el_create sets the
   start): a partitioned context whose ranks time their steps unprofiled can profile one more
   classification, all ranks together, without a new communicator. */
int el_set_profile(el_ctx* ctx, int on);
/* per-superstep delta sizes of the last el_saturate (|ΔS|, |Δlink|, |Δact|) */
int el_superstep_trace(el_ctx* ctx, uint64_t* ds, uint64_t* dl, uint64_t* da, size_t cap, size_t* n);

/* ---- results --------------------------------------------------------------------------
 * Result copy-back (the metric runs from IR-in-HBM to fixpoint PLUS this
 * copy).  The result node in its rearranged form X -> {B} (ResultRearranger DB1,
 * ResultRearranger.java:57-105) and the role links X -> {(r, Y)} (the T3_2 DB1 "Yr" -> {X}
 * keys, RolePairHandler.java:374-376, counted by AxiomCounter.java:193-215), as CSR rows over
 * this context's rows [row_lo, row_hi):
 *   S(X)   = s_val[s_ptr[X - row_lo] .. s_ptr[X - row_lo + 1]), ascending
 *   links  = l_pair[l_ptr[X - row_lo] .. l_ptr[X - row_lo + 1]), ascending pair ids q; pair q is
 *            (role, filler) = el_pair_table()[q], so each row is in (role, filler) order.
 * Every row is present (S(X) includes X itself and ⊤; ⊥ / datatype rows are the caller's to
 * skip, as ResultRearranger does).  Buffers are caller-owned; a NULL pointer skips that array.
 * Buffers from el_host_alloc are page-locked: the row sorts write the sorted rows into them
 * straight over PCIe (no device staging copy).
 * flags: EL_RESULT_RELEASE = the caller is done with this classification: once the state has
 * been read, the next el_init's reset runs beside the rest of the copy-back, and the context
 * has no state (EL_ESTATE) until el_init.
 * EL_RESULT_ASYNC (with EL_RESULT_RELEASE) = return once the copy-back is enqueued: the
 * buffers are complete when el_result_wait(ctx) returns (every other call on the context waits
 * for them first).  The caller may classify on ANOTHER context meanwhile, so one context's
 * copy-back rides over PCIe under the other's saturation (stream overlap, no extra work). */
#define EL_RESULT_RELEASE 0x1u
#define EL_RESULT_ASYNC 0x2u
#define EL_RESULT_FLAGS_KNOWN (EL_RESULT_RELEASE | EL_RESULT_ASYNC)
typedef struct el_result {
  uint32_t row_lo, row_hi;  /* out: rows of this context (whole ontology: 0, n_concepts) */
  uint64_t n_facts;         /* out: Σ_X |S(X)| over the rows */
  uint64_t n_links;         /* out: links (X, r, Y) with X in the rows */
  uint32_t n_pairs;         /* out: entries of el_pair_table */
  uint32_t flags;           /* in: EL_RESULT_* */
  uint64_t* s_ptr;          /* in: row_hi - row_lo + 1 entries, or NULL */
  uint32_t* s_val;          /* in: s_cap entries (>= n_facts), or NULL */
  uint64_t s_cap;
  uint64_t* l_ptr;          /* in: row_hi - row_lo + 1 entries, or NULL */
  uint32_t* l_pair;         /* in: l_cap entries (>= n_links), or NULL */
  uint64_t l_cap;
} el_result;

/* Streamed result: the result node's writes as the supersteps commit them (the reference's
 * classification output is result-node DB0, sets filled by ZADD as facts are derived; the
 * X -> {B} flip is ResultRearranger's post-pass, ResultRearranger.java:57-105).  Armed after
 * el_init, before el_saturate: while the saturation runs, every committed segment of the fact
 * log and of the link log crosses PCIe into the caller's page-locked buffers (beside the next
 * supersteps; a fact once derived never changes), so little is left to copy at the fixpoint.
 * Commit order, row-run encoded (the log's x comes in long runs: init facts and base links in
 * x order, the commit's staged batches):
 *   S facts  s_b[i], i < n_facts: the B of every fact, in commit order (no duplicates);
 *            s_run[2k], s_run[2k + 1] = (x, end), k < n_s_runs: s_b[i] ∈ S(x) for
 *            i in [end of run k - 1 (0 for k = 0), end)
 *   links    l_p[i], i < n_links: pair ids ((r, y) = el_pid_table()[l_p[i]]); l_run likewise
 *            gives their x: (x, y) ∈ R(r)
 * 4 B per entry plus 8 B per run instead of 8 B per entry.  The run buffers are written by the
 * device and must be page-locked host memory (el_host_alloc): EL_EINVAL otherwise.
 * Rows x ≥ n_concepts are the ELK range fillers (el_fresh_fillers), internal concepts.
 * The n_* counts are set when el_saturate returns; the buffers are complete when
 * el_result_wait returns (every other call on the context waits for them first).  A buffer
 * smaller than its part: what fits arrives, el_result_wait returns EL_ERANGE and the state is
 * kept (not released): arm again with buffers of the n_* counts and call el_saturate, which at
 * the fixpoint runs no superstep and streams the whole logs (a row partition too: that call is
 * not collective, so one rank may re-stream alone).  flags EL_RESULT_RELEASE: the state
 * is released behind the saturation (no state until el_init), as for el_copy_result. */
typedef struct el_stream {
  uint32_t flags;           /* in: EL_RESULT_* (RELEASE) */
  uint32_t* s_b;            /* in: s_cap entries, or NULL */
  uint64_t s_cap;
  uint32_t* s_run;          /* in: 2 × s_run_cap words (page-locked), or NULL */
  uint64_t s_run_cap;
  uint32_t* l_p;            /* in: l_cap entries, or NULL */
  uint64_t l_cap;
  uint32_t* l_run;          /* in: 2 × l_run_cap words (page-locked), or NULL */
  uint64_t l_run_cap;
  uint64_t n_facts;         /* out */
  uint64_t n_links;         /* out */
  uint64_t n_s_runs;        /* out */
  uint64_t n_l_runs;        /* out */
  /* EL_STREAM_PACKED (ABI 8): the facts' values cross as 16-bit codes instead of s_b — code c
     < 0xFFFF is the concept el_stream_codes()[c] (its bit column: the column order puts the
     frequent subsumers first), 0xFFFF takes the next value of s_esc (fact order).  2 B per
     fact plus 4 B per escape instead of 4 B per fact (G3: 96.6 % of the facts coded). */
  uint16_t* s_code;         /* in: s_cap codes (page-locked), with EL_STREAM_PACKED */
  uint32_t* s_esc;          /* in: s_esc_cap escape values (page-locked) */
  uint64_t s_esc_cap;
  uint64_t n_s_esc;         /* out */
} el_stream;
#define EL_STREAM_PACKED 0x4u
int el_stream_result(el_ctx* ctx, el_stream* s);  /* arms the next el_saturate; s stays valid until then */
/* the code table of EL_STREAM_PACKED: concept[c] for every code c < *n (= 65535); codes of
   columns no concept occupies hold 0xFFFFFFFF and are never emitted */
int el_stream_codes(el_ctx* ctx, uint32_t* concept, size_t cap, size_t* n);
/* pair id -> (role, filler) in pid order (the ids the streamed links carry) */
int el_pid_table(el_ctx* ctx, uint32_t* role, uint32_t* filler, size_t cap, size_t* n);

int el_result_info(el_ctx* ctx, el_result* res);   /* the out fields only */
int el_copy_result(el_ctx* ctx, el_result* res);   /* EL_ERANGE if a buffer is too small */
int el_result_wait(el_ctx* ctx);                    /* an EL_RESULT_ASYNC copy-back has landed */
/* pair q -> (role, filler), q ascending = (role, filler) ascending */
int el_pair_table(el_ctx* ctx, uint32_t* role, uint32_t* filler, size_t cap, size_t* n);
/* ELK range fillers (default range reading): fresh concept n_concepts + i stands for
 * filler[i] ⊓ ranges*(role[i]); *n = their number (0 without range axioms) */
int el_fresh_fillers(el_ctx* ctx, uint32_t* filler, uint32_t* role, size_t cap, size_t* n);
/* page-locked host memory for result buffers (NULL on failure); a JNI host wraps it in a
 * direct ByteBuffer (NewDirectByteBuffer) */
void* el_host_alloc(size_t bytes);
void el_host_free(void* p);

int el_get_subsumers(el_ctx* ctx, uint32_t x, uint32_t* out, size_t cap, size_t* n);
/* all S facts (x[i], a[i]) meaning a ∈ S(x), grouped by x (rows in id order) */
int el_copy_facts(el_ctx* ctx, uint32_t* x, uint32_t* a, size_t cap, size_t* n);
/* all links (x[i], r[i], y[i]) meaning (x, y) ∈ R(r) */
int el_copy_links(el_ctx* ctx, uint32_t* x, uint32_t* r, uint32_t* y, size_t cap, size_t* n);
int el_export_result(el_ctx* ctx, int layout, el_sink sink, void* user);

const char* el_last_error(el_ctx* ctx);
void el_destroy(el_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* EL_GPU_H */
