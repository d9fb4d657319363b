/*
 * el_oracle.h — CPU oracle for the EL+ saturation hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code, and only as the checker / the timed CPU baseline.  The product
 * (distel_amd, libel_gpu.so) never links or calls it.
 *
 * Parity status: the reference (Java + Redis/Lua, ELK 0.4.3 as its diff oracle)
 * cannot run in this image (no JVM, no redis-server: SURVEY.md §8(c)) and ships no
 * fixtures, golden vectors or ontologies.  The oracle is a restatement of the
 * reference's completion rules (file:line cited per rule in el_oracle.c) pinned by
 * hand-derived known-answer tests (tests/golden/) and by agreement of two
 * independent algorithms (semi-naive Jacobi vs naive fixpoint).  With respect to
 * the reference's own outputs it is "parity unpinned".
 */
#ifndef EL_ORACLE_H
#define EL_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#include "el_gpu.h" /* el_axioms, el_rule, el_kernel, el_event: the boundary types */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct elo_ctx elo_ctx;

/* mode 0: semi-naive Jacobi supersteps (same deltas and event counts as the GPU);
 * mode 1: naive fixpoint over the full sets (independent check, small inputs only) */
int elo_create(elo_ctx** out, const el_axioms* ax, int mode);
int elo_init(elo_ctx* c);
int elo_step(elo_ctx* c, int rule, int* changed); /* mode 0 only */
int elo_saturate(elo_ctx* c);
uint64_t elo_num_facts(const elo_ctx* c);
uint64_t elo_num_links(const elo_ctx* c);
uint64_t elo_num_init(const elo_ctx* c);
uint64_t elo_num_acts(const elo_ctx* c);
uint32_t elo_supersteps(const elo_ctx* c);
/* facts sorted by (x, a) */
int elo_copy_facts(const elo_ctx* c, uint32_t* x, uint32_t* a, size_t cap);
int elo_copy_log(const elo_ctx* c, uint32_t* x, uint32_t* a, size_t cap);
/* links sorted by (x, r, y) */
int elo_copy_links(const elo_ctx* c, uint32_t* x, uint32_t* r, uint32_t* y, size_t cap);
/* per-superstep |ΔS|, |Δlink|, |Δact| of the last elo_saturate */
int elo_trace(const elo_ctx* c, uint64_t* ds, uint64_t* dl, uint64_t* da, size_t cap);
/* events[k * EL_NUM_EVENTS + e] */
int elo_events(const elo_ctx* c, uint64_t* events, size_t cap);
const char* elo_error(const elo_ctx* c);
void elo_destroy(elo_ctx* c);

#ifdef __cplusplus
}
#endif
#endif
