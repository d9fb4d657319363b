/*
 * el_oracle.c — CPU oracle for EL+ saturation.  TEST INFRASTRUCTURE ONLY (see el_oracle.h):
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by
 * the product library.  Parity: "parity unpinned" w.r.t. the reference's own outputs
 * (none exist and the Java/Redis reference cannot run here); pinned by hand-derived
 * KATs in tests/golden/ and by naive-vs-semi-naive agreement.
 *
 * The completion rules restated here (reference file:line):
 *   init  S(X) = {X, ⊤}                          AxiomLoader.java:1237-1245 (classes),
 *         individuals {a, ⊤}                     AxiomLoader.java:1281-1289
 *   CR1   A ∈ S(X), A ⊑ B        => B ∈ S(X)     Type1_1AxiomProcessorBase.java:22-43, 118-162
 *   CR2   A1..An ∈ S(X), ⊓Ai ⊑ B => B ∈ S(X)     Type1_2AxiomProcessorBase.java:45-66, 191-230
 *   CR3   A ∈ S(X), A ⊑ ∃r.B     => (X,B) ∈ R(r) Type2AxiomProcessorBase.java:45-75;
 *                                                RolePairHandler.java:353-446
 *   CR4   (X,Y) ∈ R(r), A ∈ S(Y), ∃r.A ⊑ B => B ∈ S(X)
 *                                                Type3_1AxiomProcessorBase.java:194-239 (half 1),
 *                                                Type3_2AxiomProcessorBase.java:67-96, 182-224
 *   CR5   (X,Y) ∈ R(r), r ⊑ s    => (X,Y) ∈ R(s) Type4AxiomProcessorBase.java:38-76
 *   CR6   (X,Y) ∈ R(r), (Y,Z) ∈ R(s), r∘s ⊑ t => (X,Z) ∈ R(t)
 *                                                Type5AxiomProcessorBase.java:115-154 (complete
 *                                                join; the reference's missing s-check is H2)
 *   ⊥     ⊥ ∈ S(Y), (X,Y) ∈ R(r) => ⊥ ∈ S(X)     TypeBottomAxiomProcessorBase.java:62-123;
 *                                                RolePairHandler.java:358-372, 611-634
 *   dom   (X,Y) ∈ R(r), domain(r)=D, X ≠ ⊤, X not a datatype => D ∈ S(X)
 *                                                RolePairHandler.java:480-490
 *   range (X,Y) ∈ R(r), range(r)=C, Y ≠ ⊤, Y not a datatype, Y ∈ S(X') => C ∈ S(X')
 *                                                RolePairHandler.java:471-479 + K10
 *                                                ScriptsCollection.java:45-62 (H1, closed
 *                                                under later additions: H3)
 *
 * Mode 0 runs the same Jacobi supersteps as the GPU engine (generation reads only
 * the state of step t-1, then commit) and counts the same algorithmic events per
 * kernel, so tests can compare deltas and event counters exactly.  Mode 1 is an
 * independent naive fixpoint straight over the axiom arrays (small inputs only).
 */
#include "el_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NONE 0xffffffffu
#define EMPTY_KEY (~0ull)

enum {
  M_R1 = 1u << 0, M_R2 = 1u << 1, M_R3 = 1u << 2, M_R4Y = 1u << 3, M_R4L = 1u << 4,
  M_R5 = 1u << 5, M_R6 = 1u << 6, M_RBOT = 1u << 7, M_RDOM = 1u << 8, M_RRNG = 1u << 9,
  M_R4P = 1u << 10, /* new propagations × existing predecessors (per-rule stepping) */
  M_R4D = 1u << 11, /* fused mode: a new propagation fans out to predecessors at once */
  M_LEMPTY = 1u << 12, /* no link committed before this step: link probes would all miss */
  M_PEMPTY = 1u << 13, /* no propagation committed before this step: idem */
  M_ALL = M_R1 | M_R2 | M_R3 | M_R4Y | M_R4L | M_R5 | M_R6 | M_RBOT | M_RDOM | M_RRNG | M_R4D
};
/* el_rule -> sub-rules; CR4 is factored through propagations ((r, Y), B) exactly as the
 * reference splits it: T3_1 writes "Yr" -> B (Type3_1AxiomProcessorBase.java:208-234),
 * T3_2 joins them with R(r) (Type3_2AxiomProcessorBase.java:67-96, parts 1 and 2). */
static const uint32_t rule_mask[EL_NUM_RULE_TYPES] = {
    M_R1, M_R2, M_R3 | M_RDOM | M_RRNG, M_R4Y, M_R4L | M_R4P, M_R5, M_R6, M_RBOT};

/* ------------------------------------------------------------------ small containers */

typedef struct {
  uint32_t* v;
  size_t n, cap;
} vec;

static void vpush(vec* a, uint32_t x) {
  if (a->n == a->cap) {
    a->cap = a->cap ? 2 * a->cap : 4;
    a->v = (uint32_t*)realloc(a->v, a->cap * sizeof(uint32_t));
    if (!a->v) {
      fprintf(stderr, "el_oracle: out of memory\n");
      abort();
    }
  }
  a->v[a->n++] = x;
}

typedef struct {
  uint32_t k, a, b;
} trip;

static int u32_cmp(const void* x, const void* y) {
  const uint32_t p = *(const uint32_t*)x, q = *(const uint32_t*)y;
  return p < q ? -1 : p > q;
}

static int trip_cmp(const void* x, const void* y) {
  const trip *p = (const trip*)x, *q = (const trip*)y;
  if (p->k != q->k) return p->k < q->k ? -1 : 1;
  if (p->a != q->a) return p->a < q->a ? -1 : 1;
  if (p->b != q->b) return p->b < q->b ? -1 : 1;
  return 0;
}

typedef struct {
  uint32_t* ptr; /* rows + 1 */
  uint32_t* a;
  uint32_t* b;
} csr;

static csr csr_build(uint32_t rows, trip* t, size_t n);

/* rows of src for {A} ∪ toldc(A) per A, as one CSR (src is freed) */
static csr csr_star(csr* src, const csr* toldc, uint32_t N) {
  size_t n = 0, m = 0;
  uint32_t A, j, q;
  trip* t;
  csr out;
  for (A = 0; A < N; ++A) {
    n += src->ptr[A + 1] - src->ptr[A];
    for (j = toldc->ptr[A]; j < toldc->ptr[A + 1]; ++j) n += src->ptr[toldc->a[j] + 1] - src->ptr[toldc->a[j]];
  }
  t = (trip*)malloc((n + 1) * sizeof(trip));
  for (A = 0; A < N; ++A) {
    for (q = src->ptr[A]; q < src->ptr[A + 1]; ++q) t[m++] = (trip){A, src->a[q], src->b[q]};
    for (j = toldc->ptr[A]; j < toldc->ptr[A + 1]; ++j) {
      uint32_t B = toldc->a[j];
      for (q = src->ptr[B]; q < src->ptr[B + 1]; ++q) t[m++] = (trip){A, src->a[q], src->b[q]};
    }
  }
  out = csr_build(N, t, m);
  free(t);
  free(src->ptr), free(src->a), free(src->b);
  return out;
}

/* rows sorted by (a, b), duplicates removed */
static csr csr_build(uint32_t rows, trip* t, size_t n) {
  csr c;
  size_t m = 0, i;
  qsort(t, n, sizeof(trip), trip_cmp);
  for (i = 0; i < n; ++i)
    if (m == 0 || trip_cmp(&t[m - 1], &t[i]) != 0) t[m++] = t[i];
  c.ptr = (uint32_t*)calloc(rows + 1, sizeof(uint32_t));
  c.a = (uint32_t*)malloc((m ? m : 1) * sizeof(uint32_t));
  c.b = (uint32_t*)malloc((m ? m : 1) * sizeof(uint32_t));
  for (i = 0; i < m; ++i) c.ptr[t[i].k + 1]++;
  for (i = 0; i < rows; ++i) c.ptr[i + 1] += c.ptr[i];
  for (i = 0; i < m; ++i) {
    c.a[i] = t[i].a;
    c.b[i] = t[i].b;
  }
  return c;
}

static void csr_free(csr* c) {
  free(c->ptr);
  free(c->a);
  free(c->b);
}

/* open-addressing set of 64-bit keys */
typedef struct {
  uint64_t* t;
  uint64_t cap, n;
} hset;

static uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

static void hs_init(hset* h, uint64_t cap) {
  h->cap = cap;
  h->n = 0;
  h->t = (uint64_t*)malloc(cap * sizeof(uint64_t));
  memset(h->t, 0xff, cap * sizeof(uint64_t));
}

static int hs_has(const hset* h, uint64_t key) {
  uint64_t i = mix64(key) & (h->cap - 1);
  for (;;) {
    if (h->t[i] == key) return 1;
    if (h->t[i] == EMPTY_KEY) return 0;
    i = (i + 1) & (h->cap - 1);
  }
}

static int hs_add(hset* h, uint64_t key);

static void hs_grow(hset* h) {
  hset g;
  uint64_t i;
  hs_init(&g, h->cap * 2);
  for (i = 0; i < h->cap; ++i)
    if (h->t[i] != EMPTY_KEY) hs_add(&g, h->t[i]);
  free(h->t);
  *h = g;
}

static int hs_add(hset* h, uint64_t key) {
  uint64_t i;
  if (2 * (h->n + 1) > h->cap) hs_grow(h);
  i = mix64(key) & (h->cap - 1);
  for (;;) {
    if (h->t[i] == key) return 0;
    if (h->t[i] == EMPTY_KEY) {
      h->t[i] = key;
      h->n++;
      return 1;
    }
    i = (i + 1) & (h->cap - 1);
  }
}

static uint64_t lkey(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }

/* ------------------------------------------------------------------ context */

struct elo_ctx {
  int mode;
  char err[256];
  uint32_t N, R, P;
  uint64_t W;
  uint8_t* kind;
  /* raw axioms (naive mode reads them directly) */
  el_axioms ax;
  uint32_t *cp_ptr, *cp_ops, *cp_b;
  /* indexes */
  csr told, cidx, conj, exr, exl, psup, chf, chs, dom, rng;
  csr toldc;        /* told closure: A -> every B reachable over A ⊑ B axioms (B != A) */
  uint32_t *xr_n, *xl_n; /* per A: its own A ⊑ ∃r.B pairs / ∃r.A ⊑ B entries (before the closure) */
  uint32_t* nsub;        /* per B: told subs A ⊑ B */
  uint32_t* conj_b;
  uint32_t *fp_ptr, *pair_role, *pair_y;
  uint8_t* role_has_exl;
  uint32_t* supers_ptr; /* naive mode: strict supers+ */
  uint32_t* supers;
  /* state */
  uint32_t* bits;
  vec slog_x, slog_a;
  vec slog_f; /* 1: the fact came from a CR1 told closure, so its own closure, links and
               * propagations are already out; 2: init X ∈ S(X), closure written; 0: neither */
  vec* srow;
  hset links;
  vec llog_x, llog_p;
  vec *pred, *succ;
  hset acts;
  vec alog_y, alog_c;
  uint8_t* has_act;
  vec* actrow; /* activation log indices by Y, ascending (the GPU's activation index) */
  hset props; /* CR4 propagations (pid, B) */
  vec plog_p, plog_b;
  vec* prow; /* propagations per pid */
  uint64_t s_init;
  /* base links {(X, p) : p ∈ exr(X)} installed by elo_saturate before its first superstep
   * (el_ctx::install_base): the head of the link log, not in the link set */
  int base, fresh;
  uint64_t l_base, p_base;
  uint32_t* bpn; /* base propagations per pid: the head of prow[pid], B ascending */
  int need_pred, need_succ; /* the GPU maintains these CSRs only when they have readers */
  int has_bot;              /* some axiom concludes ⊥: else the ⊥ rule cannot fire (skipped, as on the GPU) */
  /* slack capacities of the GPU's gapped CSR rows (predecessors, successors, propagations)
   * and this step's entries past them: the GPU re-lays out a CSR after a step with any */
  uint32_t *cap_pr, *cap_sc, *cap_pp;
  uint64_t ov_pr, ov_sc, ov_pp;
  uint64_t wm_s[EL_NUM_RULE_TYPES], wm_l[EL_NUM_RULE_TYPES], wm_a[EL_NUM_RULE_TYPES], wm_p[EL_NUM_RULE_TYPES];
  uint64_t ev[EL_NUM_KERNELS][EL_NUM_EVENTS];
  vec tr_s, tr_l, tr_a; /* low 32 bits suffice for tests */
  uint32_t supersteps;
  /* naive mode links: dense byte cube R × N × N */
  uint8_t* cube;
};

static int bit(const elo_ctx* c, uint32_t x, uint32_t b) {
  return (c->bits[(uint64_t)x * c->W + (b >> 5)] >> (b & 31)) & 1u;
}
static int setbit(elo_ctx* c, uint32_t x, uint32_t b) { /* returns 1 if newly set */
  uint32_t* w = &c->bits[(uint64_t)x * c->W + (b >> 5)];
  uint32_t m = 1u << (b & 31);
  if (*w & m) return 0;
  *w |= m;
  return 1;
}

/* gapped-CSR row capacity after a re-layout: gap_cap() in distel_amd/csrc/el_gpu.hip */
#define GAP_CAP(n) (8u * (uint32_t)(n) + 64u)

#define EV(k, e) (c->ev[(k)][(e)]++)
#define EVN(k, e, n) (c->ev[(k)][(e)] += (n))

static int build_index(elo_ctx* c, const el_axioms* ax) {
  uint32_t N = ax->n_concepts, R = ax->n_roles, i, j, r;
  trip* t;
  size_t n, cap;
  uint32_t **reach, *reach_n, **sup, *sup_n;
  uint8_t* seen;
  uint32_t* stack;
  vec *re_edges, *su_edges;

  if (N < 2) return snprintf(c->err, sizeof c->err, "n_concepts < 2"), -1;
  c->N = N;
  c->R = R;
  c->W = (N + 31) / 32;
  c->kind = (uint8_t*)calloc(N, 1);
  if (ax->concept_kind) memcpy(c->kind, ax->concept_kind, N);
  c->kind[0] = c->kind[1] = EL_KIND_CLASS;

#define BADC(v) ((v) >= N)
#define BADR(v) ((v) >= R)
  for (i = 0; i < ax->n_sub; ++i)
    if (BADC(ax->sub_a[i]) || BADC(ax->sub_b[i])) return snprintf(c->err, 256, "sub"), -1;
  for (i = 0; i < ax->n_ex_rhs; ++i)
    if (BADC(ax->exr_a[i]) || BADR(ax->exr_r[i]) || BADC(ax->exr_b[i]))
      return snprintf(c->err, 256, "ex_rhs"), -1;
  for (i = 0; i < ax->n_ex_lhs; ++i)
    if (BADR(ax->exl_r[i]) || BADC(ax->exl_a[i]) || BADC(ax->exl_b[i]))
      return snprintf(c->err, 256, "ex_lhs"), -1;
  for (i = 0; i < ax->n_subrole; ++i)
    if (BADR(ax->sr_r[i]) || BADR(ax->sr_s[i])) return snprintf(c->err, 256, "subrole"), -1;
  for (i = 0; i < ax->n_chain; ++i)
    if (BADR(ax->ch_r[i]) || BADR(ax->ch_s[i]) || BADR(ax->ch_t[i]))
      return snprintf(c->err, 256, "chain"), -1;
  for (i = 0; i < ax->n_domain; ++i)
    if (BADR(ax->dom_r[i]) || BADC(ax->dom_c[i])) return snprintf(c->err, 256, "domain"), -1;
  for (i = 0; i < ax->n_range; ++i)
    if (BADR(ax->rng_r[i]) || BADC(ax->rng_c[i])) return snprintf(c->err, 256, "range"), -1;

  cap = 16 + ax->n_sub + ax->n_ex_rhs + ax->n_ex_lhs + ax->n_chain + ax->n_domain + ax->n_range;
  if (ax->n_conj) cap += ax->conj_ptr[ax->n_conj];

  /* CR1 */
  t = (trip*)malloc(cap * sizeof(trip));
  for (n = 0, i = 0; i < ax->n_sub; ++i)
    if (ax->sub_a[i] != ax->sub_b[i]) t[n++] = (trip){ax->sub_a[i], ax->sub_b[i], 0};
  c->told = csr_build(N, t, n);
  {
    /* told closure by a BFS from every concept (stamped visits) */
    uint32_t* stamp = (uint32_t*)calloc(N, sizeof(uint32_t));
    uint32_t* q = (uint32_t*)malloc(N * sizeof(uint32_t));
    vec out = {0, 0, 0};
    uint32_t A;
    c->toldc.ptr = (uint32_t*)calloc(N + 1, sizeof(uint32_t));
    for (A = 0; A < N; ++A) {
      uint32_t h = 0, tl = 0, st = A + 1, base = (uint32_t)out.n, z;
      stamp[A] = st;
      q[tl++] = A;
      while (h < tl) {
        uint32_t u = q[h++], jj;
        for (jj = c->told.ptr[u]; jj < c->told.ptr[u + 1]; ++jj) {
          uint32_t v = c->told.a[jj];
          if (stamp[v] == st) continue;
          stamp[v] = st;
          q[tl++] = v;
          vpush(&out, v);
        }
      }
      (void)z;
      qsort(out.v + base, out.n - base, sizeof(uint32_t), u32_cmp);  /* sorted, as every index row */
      c->toldc.ptr[A + 1] = (uint32_t)out.n;
    }
    c->toldc.a = out.v ? out.v : (uint32_t*)malloc(4);
    c->toldc.b = NULL;
    free(stamp);
    free(q);
  }

  /* CR2: sorted unique operands per conjunction, conj ids in input order */
  c->conj.ptr = (uint32_t*)calloc(ax->n_conj + 1, sizeof(uint32_t));
  c->conj.a = (uint32_t*)malloc((cap + 1) * sizeof(uint32_t));
  c->conj.b = NULL;
  c->conj_b = (uint32_t*)malloc((ax->n_conj + 1) * sizeof(uint32_t));
  n = 0;
  for (i = 0; i < ax->n_conj; ++i) {
    uint32_t b0 = ax->conj_ptr[i], b1 = ax->conj_ptr[i + 1], k, m0 = c->conj.ptr[i], m;
    if (b1 <= b0) return snprintf(c->err, 256, "conj %u empty", i), -1;
    if (BADC(ax->conj_b[i])) return snprintf(c->err, 256, "conj rhs"), -1;
    for (k = b0; k < b1; ++k) {
      uint32_t v = ax->conj_ops[k], q, dup = 0;
      if (BADC(v)) return snprintf(c->err, 256, "conj op"), -1;
      /* insertion into the sorted run [m0, end) */
      m = m0 + (uint32_t)(n - m0);
      for (q = m0; q < m; ++q)
        if (c->conj.a[q] == v) dup = 1;
      if (dup) continue;
      q = m;
      while (q > m0 && c->conj.a[q - 1] > v) {
        c->conj.a[q] = c->conj.a[q - 1];
        --q;
      }
      c->conj.a[q] = v;
      ++n;
    }
    c->conj.ptr[i + 1] = (uint32_t)n;
    c->conj_b[i] = ax->conj_b[i];
  }
  {
    size_t m = 0;
    trip* u = (trip*)malloc((n + 1) * sizeof(trip));
    for (i = 0; i < ax->n_conj; ++i)
      for (j = c->conj.ptr[i]; j < c->conj.ptr[i + 1]; ++j) u[m++] = (trip){c->conj.a[j], i, 0};
    c->cidx = csr_build(N, u, m);
    free(u);
  }

  /* role closures: supers+(r) over r ⊑ s; reach*(r) over r ⊑ s and s → t (p ∘ s ⊑ t) */
  re_edges = (vec*)calloc(R ? R : 1, sizeof(vec));
  su_edges = (vec*)calloc(R ? R : 1, sizeof(vec));
  for (i = 0; i < ax->n_subrole; ++i) {
    vpush(&su_edges[ax->sr_r[i]], ax->sr_s[i]);
    vpush(&re_edges[ax->sr_r[i]], ax->sr_s[i]);
  }
  for (i = 0; i < ax->n_chain; ++i) vpush(&re_edges[ax->ch_s[i]], ax->ch_t[i]);
  reach = (uint32_t**)calloc(R ? R : 1, sizeof(uint32_t*));
  reach_n = (uint32_t*)calloc(R ? R : 1, sizeof(uint32_t));
  sup = (uint32_t**)calloc(R ? R : 1, sizeof(uint32_t*));
  sup_n = (uint32_t*)calloc(R ? R : 1, sizeof(uint32_t));
  seen = (uint8_t*)malloc(R ? R : 1);
  stack = (uint32_t*)malloc((R ? R : 1) * sizeof(uint32_t));
  for (r = 0; r < R; ++r) {
    int pass;
    for (pass = 0; pass < 2; ++pass) {
      vec* g = pass == 0 ? su_edges : re_edges;
      uint32_t sp = 0, q, cnt = 0;
      memset(seen, 0, R);
      seen[r] = 1;
      stack[sp++] = r;
      while (sp) {
        uint32_t u = stack[--sp];
        size_t e;
        for (e = 0; e < g[u].n; ++e)
          if (!seen[g[u].v[e]]) {
            seen[g[u].v[e]] = 1;
            stack[sp++] = g[u].v[e];
          }
      }
      for (q = 0; q < R; ++q)
        if (seen[q] && (pass == 1 || q != r)) cnt++;
      if (pass == 0) {
        sup[r] = (uint32_t*)malloc((cnt + 1) * sizeof(uint32_t));
        sup_n[r] = 0;
        for (q = 0; q < R; ++q)
          if (seen[q] && q != r) sup[r][sup_n[r]++] = q;
      } else {
        reach[r] = (uint32_t*)malloc((cnt + 1) * sizeof(uint32_t));
        reach_n[r] = 0;
        for (q = 0; q < R; ++q)
          if (seen[q]) reach[r][reach_n[r]++] = q;
      }
    }
  }
  /* naive mode uses supers+ too */
  c->supers_ptr = (uint32_t*)calloc(R + 1, sizeof(uint32_t));
  for (r = 0; r < R; ++r) c->supers_ptr[r + 1] = c->supers_ptr[r] + sup_n[r];
  c->supers = (uint32_t*)malloc((c->supers_ptr[R] + 1) * sizeof(uint32_t));
  for (r = 0; r < R; ++r) memcpy(c->supers + c->supers_ptr[r], sup[r], sup_n[r] * sizeof(uint32_t));

  /* pair universe: (Y, t) for A ⊑ ∃r.Y and t ∈ reach*(r); pid order = sorted (Y, t) */
  {
    size_t m = 0, pc = 0, k;
    trip* u;
    for (i = 0; i < ax->n_ex_rhs; ++i) pc += reach_n[ax->exr_r[i]];
    u = (trip*)malloc((pc + 1) * sizeof(trip));
    for (i = 0; i < ax->n_ex_rhs; ++i)
      for (k = 0; k < reach_n[ax->exr_r[i]]; ++k) u[m++] = (trip){ax->exr_b[i], reach[ax->exr_r[i]][k], 0};
    qsort(u, m, sizeof(trip), trip_cmp);
    pc = 0;
    for (k = 0; k < m; ++k)
      if (pc == 0 || trip_cmp(&u[pc - 1], &u[k]) != 0) u[pc++] = u[k];
    c->P = (uint32_t)pc;
    c->pair_y = (uint32_t*)malloc((pc + 1) * sizeof(uint32_t));
    c->pair_role = (uint32_t*)malloc((pc + 1) * sizeof(uint32_t));
    c->fp_ptr = (uint32_t*)calloc(N + 1, sizeof(uint32_t));
    for (k = 0; k < pc; ++k) {
      c->pair_y[k] = u[k].k;
      c->pair_role[k] = u[k].a;
      c->fp_ptr[u[k].k + 1]++;
    }
    for (i = 0; i < N; ++i) c->fp_ptr[i + 1] += c->fp_ptr[i];
    free(u);
  }
#define PID_OF(rr, yy, out)                                                \
  do {                                                                     \
    uint32_t p_;                                                           \
    (out) = NONE;                                                          \
    for (p_ = c->fp_ptr[(yy)]; p_ < c->fp_ptr[(yy) + 1]; ++p_)             \
      if (c->pair_role[p_] == (rr)) {                                      \
        (out) = p_;                                                        \
        break;                                                             \
      }                                                                    \
  } while (0)
  for (n = 0, i = 0; i < ax->n_ex_rhs; ++i) {
    uint32_t p;
    PID_OF(ax->exr_r[i], ax->exr_b[i], p);
    t[n++] = (trip){ax->exr_a[i], p, 0};
  }
  c->exr = csr_build(N, t, n);
  c->role_has_exl = (uint8_t*)calloc(R ? R : 1, 1);
  for (n = 0, i = 0; i < ax->n_ex_lhs; ++i) {
    t[n++] = (trip){ax->exl_a[i], ax->exl_r[i], ax->exl_b[i]};
    c->role_has_exl[ax->exl_r[i]] = 1;
  }
  c->exl = csr_build(N, t, n);
  c->xr_n = (uint32_t*)calloc(N, sizeof(uint32_t));
  c->xl_n = (uint32_t*)calloc(N, sizeof(uint32_t));
  c->nsub = (uint32_t*)calloc(N, sizeof(uint32_t));
  for (i = 0; i < N; ++i) {
    c->xr_n[i] = c->exr.ptr[i + 1] - c->exr.ptr[i];
    c->xl_n[i] = c->exl.ptr[i + 1] - c->exl.ptr[i];
    for (j = c->told.ptr[i]; j < c->told.ptr[i + 1]; ++j) c->nsub[c->told.a[j]]++;
  }
  /* CR3 / CR4 half-1 over the told closure (el_index.cpp): row A gathers the rows of every
   * B ∈ {A} ∪ told*(A), sorted and unique, so a fact emits its closure's links and
   * propagations in the superstep that emits the closure; closure facts skip both rules */
  c->exr = csr_star(&c->exr, &c->toldc, N);
  c->exl = csr_star(&c->exl, &c->toldc, N);
  {
    size_t m = 0, pc = 0;
    trip* u;
    uint32_t p, k;
    for (p = 0; p < c->P; ++p) pc += sup_n[c->pair_role[p]];
    u = (trip*)malloc((pc + 1) * sizeof(trip));
    for (p = 0; p < c->P; ++p)
      for (k = 0; k < sup_n[c->pair_role[p]]; ++k) {
        uint32_t q;
        PID_OF(sup[c->pair_role[p]][k], c->pair_y[p], q);
        if (q == NONE) return snprintf(c->err, 256, "pair universe not closed"), -1;
        u[m++] = (trip){p, q, 0};
      }
    c->psup = csr_build(c->P, u, m);
    free(u);
  }
  for (n = 0, i = 0; i < ax->n_chain; ++i) t[n++] = (trip){ax->ch_r[i], ax->ch_s[i], ax->ch_t[i]};
  c->chf = csr_build(R, t, n);
  for (n = 0, i = 0; i < ax->n_chain; ++i) t[n++] = (trip){ax->ch_s[i], ax->ch_r[i], ax->ch_t[i]};
  c->chs = csr_build(R, t, n);
  for (n = 0, i = 0; i < ax->n_domain; ++i) t[n++] = (trip){ax->dom_r[i], ax->dom_c[i], 0};
  c->dom = csr_build(R, t, n);
  for (n = 0, i = 0; i < ax->n_range; ++i) t[n++] = (trip){ax->rng_r[i], ax->rng_c[i], 0};
  c->rng = csr_build(R, t, n);

  for (r = 0; r < R; ++r) {
    free(reach[r]);
    free(sup[r]);
    free(re_edges[r].v);
    free(su_edges[r].v);
  }
  free(reach);
  free(reach_n);
  free(sup);
  free(sup_n);
  free(seen);
  free(stack);
  free(re_edges);
  free(su_edges);
  free(t);
  return 0;
}

static void copy_axioms(elo_ctx* c, const el_axioms* ax) {
  /* naive mode reads the raw axioms; keep private copies */
  c->ax = *ax;
#define DUP(f, cnt)                                                          \
  do {                                                                       \
    if ((cnt) && ax->f) {                                                    \
      uint32_t* p_ = (uint32_t*)malloc((cnt) * sizeof(uint32_t));            \
      memcpy(p_, ax->f, (cnt) * sizeof(uint32_t));                           \
      c->ax.f = p_;                                                          \
    } else                                                                   \
      c->ax.f = NULL;                                                        \
  } while (0)
  DUP(sub_a, ax->n_sub);
  DUP(sub_b, ax->n_sub);
  DUP(conj_ptr, ax->n_conj ? ax->n_conj + 1 : 0);
  DUP(conj_ops, ax->n_conj ? ax->conj_ptr[ax->n_conj] : 0);
  DUP(conj_b, ax->n_conj);
  DUP(exr_a, ax->n_ex_rhs);
  DUP(exr_r, ax->n_ex_rhs);
  DUP(exr_b, ax->n_ex_rhs);
  DUP(exl_r, ax->n_ex_lhs);
  DUP(exl_a, ax->n_ex_lhs);
  DUP(exl_b, ax->n_ex_lhs);
  DUP(sr_r, ax->n_subrole);
  DUP(sr_s, ax->n_subrole);
  DUP(ch_r, ax->n_chain);
  DUP(ch_s, ax->n_chain);
  DUP(ch_t, ax->n_chain);
  DUP(dom_r, ax->n_domain);
  DUP(dom_c, ax->n_domain);
  DUP(rng_r, ax->n_range);
  DUP(rng_c, ax->n_range);
  c->ax.concept_kind = NULL;
#undef DUP
}

int elo_create(elo_ctx** out, const el_axioms* ax, int mode) {
  elo_ctx* c;
  if (!out || !ax || (mode != 0 && mode != 1)) return EL_EINVAL;
  c = (elo_ctx*)calloc(1, sizeof(elo_ctx));
  c->mode = mode;
  if (build_index(c, ax) != 0) {
    *out = c;
    return EL_EINVAL;
  }
  copy_axioms(c, ax);
  {
    uint32_t i;
    int bot = 0;
    for (i = 0; i < ax->n_sub; ++i) bot |= ax->sub_b[i] == EL_BOTTOM;
    for (i = 0; i < ax->n_conj; ++i) bot |= ax->conj_b[i] == EL_BOTTOM;
    for (i = 0; i < ax->n_ex_rhs; ++i) bot |= ax->exr_b[i] == EL_BOTTOM;
    for (i = 0; i < ax->n_ex_lhs; ++i) bot |= ax->exl_b[i] == EL_BOTTOM;
    for (i = 0; i < ax->n_domain; ++i) bot |= ax->dom_c[i] == EL_BOTTOM;
    for (i = 0; i < ax->n_range; ++i) bot |= ax->rng_c[i] == EL_BOTTOM;
    c->need_succ = ax->n_chain > 0;
    c->need_pred = ax->n_ex_lhs > 0 || ax->n_chain > 0 || bot;
    c->has_bot = bot;
  }
  c->bits = (uint32_t*)calloc((size_t)c->N * c->W + 1, sizeof(uint32_t));
  if (!c->bits) {
    *out = c;
    snprintf(c->err, 256, "bit matrix allocation failed");
    return EL_ENOMEM;
  }
  c->srow = (vec*)calloc(c->N, sizeof(vec));
  c->pred = (vec*)calloc(c->P ? c->P : 1, sizeof(vec));
  c->succ = (vec*)calloc(c->N, sizeof(vec));
  c->has_act = (uint8_t*)calloc(c->N, 1);
  c->actrow = (vec*)calloc(c->N, sizeof(vec));
  c->prow = (vec*)calloc(c->P ? c->P : 1, sizeof(vec));
  c->bpn = (uint32_t*)calloc(c->P ? c->P : 1, sizeof(uint32_t));
  c->cap_pr = (uint32_t*)malloc((c->P ? c->P : 1) * sizeof(uint32_t));
  c->cap_pp = (uint32_t*)malloc((c->P ? c->P : 1) * sizeof(uint32_t));
  c->cap_sc = (uint32_t*)malloc((c->N ? c->N : 1) * sizeof(uint32_t));
  {
    uint32_t q;
    uint32_t j;
    for (q = 0; q < (c->P ? c->P : 1); ++q) c->cap_pr[q] = c->cap_pp[q] = 0;
    for (q = 0; q < c->N; ++q) c->cap_sc[q] = 0;
    /* initial row capacities sized for the first supersteps' links (as el_ctx::alloc_state
     * sizes the GPU's): every init fact X ∈ S(X) emits the pairs of exr(X) and CR5 lifts them
     * to their super-role pairs psup, so pid p's predecessor row receives its count of both and
     * X's successor row its chain-second ones; slack as after a re-layout */
    for (q = 0; q < c->N; ++q)
      for (j = c->exr.ptr[q]; j < c->exr.ptr[q + 1]; ++j) {
        uint32_t p = c->exr.a[j], r = c->pair_role[p], k;
        ++c->cap_pr[p];
        if (c->chs.ptr[r + 1] > c->chs.ptr[r]) ++c->cap_sc[q];
        for (k = c->psup.ptr[p]; k < c->psup.ptr[p + 1]; ++k) { /* CR5 lifts them in the next step */
          uint32_t u = c->psup.a[k], ru = c->pair_role[u];
          ++c->cap_pr[u];
          if (c->chs.ptr[ru + 1] > c->chs.ptr[ru]) ++c->cap_sc[q];
        }
      }
    /* propagation rows: init fact X (as Y) records ((r, X), B) for every (r, B) of exl(X) */
    for (q = 0; q < c->N; ++q)
      for (j = c->exl.ptr[q]; j < c->exl.ptr[q + 1]; ++j) {
        uint32_t p;
        PID_OF(c->exl.a[j], q, p);
        if (p != NONE) ++c->cap_pp[p];
      }
    for (q = 0; q < (c->P ? c->P : 1); ++q) c->cap_pr[q] = GAP_CAP(c->cap_pr[q]), c->cap_pp[q] = GAP_CAP(c->cap_pp[q]);
    for (q = 0; q < c->N; ++q) c->cap_sc[q] = GAP_CAP(c->cap_sc[q]);
  }
  hs_init(&c->props, 1024);
  hs_init(&c->links, 1024);
  hs_init(&c->acts, 64);
  if (mode == 1) {
    uint64_t cube = (uint64_t)(c->R ? c->R : 1) * c->N * c->N;
    if (cube > (1ull << 28)) {
      *out = c;
      snprintf(c->err, 256, "naive mode: R*N*N too large");
      return EL_EINVAL;
    }
    c->cube = (uint8_t*)calloc(cube, 1);
  }
  *out = c;
  return EL_OK;
}

/* ------------------------------------------------------------------ semi-naive engine */

typedef struct {
  vec sx, sa, lx, lp, ay, ac, pp, pb;
  vec s1x, s1a; /* CR1 told-closure candidates: committed after every other S candidate */
  vec jt, jb, jo, jl, ja, jbb; /* job records: type, list owner, offset, length, a, b */
} cands;

static void cands_free(cands* k) {
  free(k->sx.v), free(k->sa.v), free(k->lx.v), free(k->lp.v), free(k->ay.v), free(k->ac.v);
  free(k->pp.v), free(k->pb.v), free(k->s1x.v), free(k->s1a.v);
  free(k->jt.v), free(k->jb.v), free(k->jo.v), free(k->jl.v), free(k->ja.v), free(k->jbb.v);
}

static void emit_s(elo_ctx* c, cands* k, int kern, uint32_t x, uint32_t a) {
  EV(kern, EL_EV_EMIT);
  vpush(&k->sx, x);
  vpush(&k->sa, a);
}
static void emit_l(elo_ctx* c, cands* k, int kern, uint32_t x, uint32_t p) {
  EV(kern, EL_EV_EMIT);
  vpush(&k->lx, x);
  vpush(&k->lp, p);
}
/* a fan-out list of len items becomes ceil(len / JOB_CHUNK) job records (as on the GPU) */
#define JOB_CHUNK 256u
static void emit_job(elo_ctx* c, cands* k, int kern, uint32_t type, uint32_t b, uint32_t len, uint32_t a,
                     uint32_t bb) {
  uint32_t off;
  for (off = 0; off < len; off += JOB_CHUNK) {
    EV(kern, EL_EV_JOB);
    vpush(&k->jt, type);
    vpush(&k->jb, b);
    vpush(&k->jo, off);
    vpush(&k->jl, len - off < JOB_CHUNK ? len - off : JOB_CHUNK);
    vpush(&k->ja, a);
    vpush(&k->jbb, bb);
  }
}

enum { JOB_PRED_S = 0, JOB_PRED_L = 1, JOB_PRED_U = 2, JOB_R6A = 3 }; /* U: unprobed (first superstep) */

/* scan of the filler's pair range (sorted by role): one row lookup + entries read */
static uint32_t pair_lookup(elo_ctx* c, int kern, uint32_t r, uint32_t y) {
  uint32_t p;
  EV(kern, EL_EV_ROW);
  for (p = c->fp_ptr[y]; p < c->fp_ptr[y + 1]; ++p) {
    EV(kern, EL_EV_ENT);
    if (c->pair_role[p] == r) return p;
    if (c->pair_role[p] > r) return NONE;
  }
  return NONE;
}

/* (x, pid) is a base link: binary search of exr(x) (base_has on the GPU, same probe sequence) */
static int base_has(elo_ctx* c, int kern, uint32_t x, uint32_t pid) {
  uint32_t lo = c->exr.ptr[x], hi = c->exr.ptr[x + 1];
  EV(kern, EL_EV_ROW);
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1, v;
    EV(kern, EL_EV_ENT);
    v = c->exr.a[mid];
    if (v == pid) return 1;
    if (v < pid)
      lo = mid + 1;
    else
      hi = mid;
  }
  return 0;
}

/* (x, pid) known at t-1: a base link, or in the link set (lempty: the set is empty, no probe) */
static int link_known(elo_ctx* c, int kern, uint32_t x, uint32_t pid, int lempty) {
  if (c->base && base_has(c, kern, x, pid)) return 1;
  if (lempty) return 0;
  EV(kern, EL_EV_HASH);
  return hs_has(&c->links, lkey(pid, x));
}

/* ((r, Y), B) known at t-1: a base propagation (binary search of the head of prow[pid], as
 * prop_known searches bpp on the GPU), or in the set (pempty: the set is empty, no probe) */
static int prop_known(elo_ctx* c, int kern, uint32_t pid, uint32_t b, int pempty) {
  if (c->base) {
    uint32_t lo = 0, hi = c->bpn[pid];
    EV(kern, EL_EV_ROW);
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1, v;
      EV(kern, EL_EV_ENT);
      v = c->prow[pid].v[mid];
      if (v == b) return 1;
      if (v < b)
        lo = mid + 1;
      else
        hi = mid;
    }
  }
  if (pempty) return 0;
  EV(kern, EL_EV_HASH);
  return hs_has(&c->props, lkey(pid, b));
}

/* predecessor / succ / S-row "CSR" views: begin offset is irrelevant on the CPU, the
 * job carries the list identity (kind + owner) instead */
/* diagnostic (ELO_CR1STAT): per superstep, the CR1 told-closure walk — facts walked, entries
 * tested, entries already in S(X), distinct (X, B) among the tested entries */
static int cr1_stat = -1;
static uint64_t cr1_facts, cr1_tests, cr1_hit, cr1_n, cr1_cap;
static uint64_t* cr1_keys;
static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}
static void cr1_report(uint32_t step) {
  uint64_t i, u = 0;
  if (cr1_stat <= 0) return;
  qsort(cr1_keys, cr1_n, sizeof(uint64_t), cmp_u64);
  for (i = 0; i < cr1_n; ++i) u += i == 0 || cr1_keys[i] != cr1_keys[i - 1];
  fprintf(stderr, "cr1 step %u facts %llu tests %llu already %llu distinct %llu%s\n", step,
          (unsigned long long)cr1_facts, (unsigned long long)cr1_tests, (unsigned long long)cr1_hit,
          (unsigned long long)u, cr1_n < cr1_tests ? " (distinct over a prefix)" : "");
  cr1_facts = cr1_tests = cr1_hit = cr1_n = 0;
}

static void expand_s(elo_ctx* c, cands* k, uint32_t mask, uint64_t b, uint64_t e, uint64_t a_end) {
  const int K = EL_K_EXPAND_S;
  uint64_t i;
  uint32_t j;
  if (cr1_stat < 0) {
    cr1_stat = getenv("ELO_CR1STAT") != NULL;
    if (cr1_stat) {
      cr1_cap = 1ull << 28;
      cr1_keys = (uint64_t*)malloc(cr1_cap * sizeof(uint64_t));
    }
  }
  for (i = b; i < e; ++i) {
    uint32_t X = c->slog_x.v[i], A = c->slog_a.v[i];
    EV(K, EL_EV_TRIG);
    /* CR1 over the told closure (Type1_1AxiomProcessorBase.java:22-43 applied transitively at
     * once, as the GPU index does): a fact that came out of a closure is not re-expanded */
    if (mask & M_R1) {
      if (!c->slog_f.v[i]) {
        EV(K, EL_EV_ROW);
        if (cr1_stat) cr1_facts++;
        for (j = c->toldc.ptr[A]; j < c->toldc.ptr[A + 1]; ++j) {
          uint32_t B = c->toldc.a[j];
          EV(K, EL_EV_ENT);
          EV(K, EL_EV_TEST);
          if (cr1_stat) {
            cr1_tests++;
            cr1_hit += bit(c, X, B) ? 1 : 0;
            if (cr1_n < cr1_cap) cr1_keys[cr1_n++] = ((uint64_t)X << 32) | B;
          }
          if (!bit(c, X, B)) {
            EV(K, EL_EV_EMIT);
            vpush(&k->s1x, X);
            vpush(&k->s1a, B);
          }
        }
      }
    }
    if (mask & M_R2) {
      EV(K, EL_EV_ROW);
      for (j = c->cidx.ptr[A]; j < c->cidx.ptr[A + 1]; ++j) {
        uint32_t cc = c->cidx.a[j], q;
        int ok = 1;
        EV(K, EL_EV_ENT);
        EV(K, EL_EV_ROW);
        for (q = c->conj.ptr[cc]; q < c->conj.ptr[cc + 1]; ++q) {
          uint32_t op = c->conj.a[q];
          EV(K, EL_EV_ENT);
          if (op == A) continue;
          EV(K, EL_EV_TEST);
          if (!bit(c, X, op)) {
            ok = 0;
            break;
          }
        }
        if (ok) {
          uint32_t B = c->conj_b[cc];
          EV(K, EL_EV_ENT);
          EV(K, EL_EV_TEST);
          if (!bit(c, X, B)) emit_s(c, k, K, X, B);
        }
      }
    }
    /* CR3 / CR4 half-1 over the told closure: a fact that came out of a closure (flag 1) was
     * covered by the fact that emitted the closure (the exr / exl rows span {A} ∪ told*(A)) */
    /* (an init fact's own links are the base links, already in place) */
    if ((mask & M_R3) && c->slog_f.v[i] != 1 && !(c->base && c->slog_f.v[i] == 2)) {
      EV(K, EL_EV_ROW);
      for (j = c->exr.ptr[A]; j < c->exr.ptr[A + 1]; ++j) {
        uint32_t pid = c->exr.a[j];
        EV(K, EL_EV_ENT);
        if (!link_known(c, K, X, pid, (mask & M_LEMPTY) != 0)) emit_l(c, k, K, X, pid);
      }
    }
    /* A ∈ S(Y=X) new, ∃r.A ⊑ B => propagation ((r, Y), B); an init fact's own propagations are
     * the base propagations, already in place */
    if ((mask & M_R4Y) && c->slog_f.v[i] != 1 && !(c->base && c->slog_f.v[i] == 2)) {
      EV(K, EL_EV_ROW);
      for (j = c->exl.ptr[A]; j < c->exl.ptr[A + 1]; ++j) {
        uint32_t r = c->exl.a[j], B = c->exl.b[j], pid;
        EVN(K, EL_EV_ENT, 2);
        pid = pair_lookup(c, K, r, X);
        if (pid != NONE) {
          if (!prop_known(c, K, pid, B, (mask & M_PEMPTY) != 0)) {
            EV(K, EL_EV_EMIT);
            vpush(&k->pp, pid);
            vpush(&k->pb, B);
            if (mask & M_R4D) {
              EV(K, EL_EV_ROW);
              if (c->pred[pid].n)
                emit_job(c, k, K, (mask & M_LEMPTY) ? JOB_PRED_U : JOB_PRED_S, pid, (uint32_t)c->pred[pid].n, 0, B);
            }
          }
        }
      }
    }
    if ((mask & M_RBOT) && c->has_bot && A == EL_BOTTOM) {
      uint32_t p;
      EV(K, EL_EV_ROW);
      for (p = c->fp_ptr[X]; p < c->fp_ptr[X + 1]; ++p) {
        EV(K, EL_EV_ROW);
        if (c->pred[p].n)
          emit_job(c, k, K, (mask & M_LEMPTY) ? JOB_PRED_U : JOB_PRED_S, p, (uint32_t)c->pred[p].n, 0, EL_BOTTOM);
      }
    }
    if ((mask & M_RRNG) && c->rng.ptr[c->R] > 0) {
      EV(K, EL_EV_ENT);
      if (c->has_act[A]) { /* A's row of the activation index */
        uint64_t j;
        EV(K, EL_EV_ROW);
        for (j = 0; j < c->actrow[A].n; ++j) {
          uint32_t q = c->actrow[A].v[j], C;
          if (q >= a_end) break;
          EVN(K, EL_EV_ENT, 2);
          C = c->alog_c.v[q];
          EV(K, EL_EV_TEST);
          if (!bit(c, X, C)) emit_s(c, k, K, X, C);
        }
      }
    }
  }
}

static void expand_l(elo_ctx* c, cands* k, uint32_t mask, uint64_t b, uint64_t e) {
  const int K = EL_K_EXPAND_L;
  uint64_t i;
  uint32_t j;
  for (i = b; i < e; ++i) {
    uint32_t X = c->llog_x.v[i], pid = c->llog_p.v[i];
    uint32_t r = c->pair_role[pid], Y = c->pair_y[pid];
    EV(K, EL_EV_TRIG);
    EVN(K, EL_EV_ENT, 2);
    if (mask & M_R4L) { /* (X, Y) ∈ R(r) new, propagation ((r, Y), B) => B ∈ S(X) */
      size_t q;
      EV(K, EL_EV_ROW);
      for (q = 0; q < c->prow[pid].n; ++q) {
        uint32_t B = c->prow[pid].v[q];
        EV(K, EL_EV_ENT);
        emit_s(c, k, K, X, B); /* unprobed (as on the GPU): the commit drops facts already present */
      }
    }
    if ((mask & M_RBOT) && c->has_bot) {
      EV(K, EL_EV_TEST);
      if (bit(c, Y, EL_BOTTOM)) {
        EV(K, EL_EV_TEST);
        if (!bit(c, X, EL_BOTTOM)) emit_s(c, k, K, X, EL_BOTTOM);
      }
    }
    if (mask & M_R5) {
      EV(K, EL_EV_ROW);
      for (j = c->psup.ptr[pid]; j < c->psup.ptr[pid + 1]; ++j) {
        uint32_t q = c->psup.a[j];
        EV(K, EL_EV_ENT);
        if (!link_known(c, K, X, q, (mask & M_LEMPTY) != 0)) emit_l(c, k, K, X, q);
      }
    }
    if (mask & M_R6) {
      EV(K, EL_EV_ROW);
      if (c->chf.ptr[r + 1] > c->chf.ptr[r]) {
        EV(K, EL_EV_ROW);
        if (c->succ[Y].n) emit_job(c, k, K, JOB_R6A, Y, (uint32_t)c->succ[Y].n, X, r);
      }
      EV(K, EL_EV_ROW);
      for (j = c->chs.ptr[r]; j < c->chs.ptr[r + 1]; ++j) {
        uint32_t p = c->chs.a[j], t = c->chs.b[j], pq;
        EVN(K, EL_EV_ENT, 2);
        pq = pair_lookup(c, K, p, X);
        if (pq != NONE) {
          EV(K, EL_EV_ROW);
          if (c->pred[pq].n) {
            uint32_t pt = pair_lookup(c, K, t, Y);
            emit_job(c, k, K, JOB_PRED_L, pq, (uint32_t)c->pred[pq].n, pt, 0);
          }
        }
      }
    }
    if (mask & M_RDOM) {
      int ok = 0;
      EV(K, EL_EV_ROW);
      if (c->dom.ptr[r + 1] > c->dom.ptr[r]) {
        EV(K, EL_EV_ENT);
        ok = X != EL_TOP && c->kind[X] != EL_KIND_DATATYPE;
      }
      for (j = c->dom.ptr[r]; j < c->dom.ptr[r + 1]; ++j) {
        uint32_t D = c->dom.a[j];
        EV(K, EL_EV_ENT);
        if (ok) {
          EV(K, EL_EV_TEST);
          if (!bit(c, X, D)) emit_s(c, k, K, X, D);
        }
      }
    }
    if (mask & M_RRNG) {
      int ok = 0;
      EV(K, EL_EV_ROW);
      if (c->rng.ptr[r + 1] > c->rng.ptr[r]) {
        EV(K, EL_EV_ENT);
        ok = Y != EL_TOP && c->kind[Y] != EL_KIND_DATATYPE;
      }
      for (j = c->rng.ptr[r]; j < c->rng.ptr[r + 1]; ++j) {
        uint32_t C = c->rng.a[j];
        EV(K, EL_EV_ENT);
        if (ok) {
          EV(K, EL_EV_HASH);
          if (!hs_has(&c->acts, lkey(C, Y))) {
            EV(K, EL_EV_EMIT);
            vpush(&k->ay, Y);
            vpush(&k->ac, C);
          }
        }
      }
    }
  }
}

static void run_jobs(elo_ctx* c, cands* k, int lempty) {
  const int K = EL_K_JOBS;
  size_t j;
  uint32_t q, e;
  for (j = 0; j < k->jt.n; ++j) {
    uint32_t type = k->jt.v[j], owner = k->jb.v[j], o0 = k->jo.v[j], len = k->jl.v[j], a = k->ja.v[j],
             b = k->jbb.v[j];
    EV(K, EL_EV_JOB);
    if (type == JOB_PRED_S || type == JOB_PRED_U) {
      for (q = 0; q < len; ++q) {
        uint32_t xp = c->pred[owner].v[o0 + q];
        EV(K, EL_EV_ENT);
        if (type == JOB_PRED_U) {
          emit_s(c, k, K, xp, b);
          continue;
        }
        EV(K, EL_EV_TEST);
        if (!bit(c, xp, b)) emit_s(c, k, K, xp, b);
      }
    } else if (type == JOB_PRED_L) {
      for (q = 0; q < len; ++q) {
        uint32_t xp = c->pred[owner].v[o0 + q];
        EV(K, EL_EV_ENT);
        if (!link_known(c, K, xp, a, lempty)) emit_l(c, k, K, xp, a);
      }
    } else { /* JOB_R6A */
      uint32_t X = a, r = b;
      for (q = 0; q < len; ++q) {
        uint32_t qq = c->succ[owner].v[o0 + q], s2 = c->pair_role[qq], Z = c->pair_y[qq];
        EV(K, EL_EV_ENT);
        EVN(K, EL_EV_ENT, 2);
        EV(K, EL_EV_ROW);
        for (e = c->chf.ptr[r]; e < c->chf.ptr[r + 1]; ++e) {
          uint32_t s = c->chf.a[e], t = c->chf.b[e];
          EVN(K, EL_EV_ENT, 2);
          if (s == s2) {
            uint32_t pt = pair_lookup(c, K, t, Z);
            if (!link_known(c, K, X, pt, lempty)) emit_l(c, k, K, X, pt);
          }
        }
      }
    }
  }
}

/* New activations (Y, C) = act log[ab, ae) meet every fact (X, Y) known at t-1 (the fact log
 * [0, s_end)) through Y's row of the activation index (newest last) */
static void expand_a(elo_ctx* c, cands* k, uint64_t s_end, uint64_t ab, uint64_t ae) {
  const int K = EL_K_EXPAND_A;
  uint64_t i;
  for (i = 0; i < s_end; ++i) {
    uint32_t x = c->slog_x.v[i], Y = c->slog_a.v[i];
    EV(K, EL_EV_TRIG);
    EV(K, EL_EV_ENT);
    if (c->has_act[Y]) {
      uint64_t j;
      EV(K, EL_EV_ROW);
      for (j = c->actrow[Y].n; j > 0; --j) {
        uint32_t q = c->actrow[Y].v[j - 1], C;
        if (q < ab) break;
        if (q >= ae) continue;
        EVN(K, EL_EV_ENT, 2);
        C = c->alog_c.v[q];
        EV(K, EL_EV_TEST);
        if (!bit(c, x, C)) emit_s(c, k, K, x, C);
      }
    }
  }
}

static void expand_p(elo_ctx* c, cands* k, uint64_t pb, uint64_t pe) {
  const int K = EL_K_EXPAND_P;
  uint64_t i;
  for (i = pb; i < pe; ++i) {
    uint32_t pid = c->plog_p.v[i], B = c->plog_b.v[i];
    EV(K, EL_EV_TRIG);
    EV(K, EL_EV_ROW);
    if (c->pred[pid].n) emit_job(c, k, K, JOB_PRED_S, pid, (uint32_t)c->pred[pid].n, 0, B);
  }
}

/* append of one entry to a gapped CSR row holding n entries with capacity cap (gap_append
 * on the GPU): the len atomic, the row bounds, the value; past the capacity a 3-word
 * overflow record */
static void gap_append_ev(elo_ctx* c, int K, uint64_t n, uint32_t cap, uint64_t* ov) {
  EV(K, EL_EV_RMW);
  EV(K, EL_EV_ROW);
  EV(K, EL_EV_ENT);
  if (n >= cap) {
    EVN(K, EL_EV_ENT, 2);
    ++*ov;
  }
}

/* A step's overflowing rows are relocated, each alone, to GAP_CAP(n) fresh slots (the GPU's
 * gap_relocate_all; every other row keeps its capacity).  Events: the overflow records read
 * and claimed, the rows relocated (their bounds read and written), their in-place entries
 * moved (a full row: its old capacity) and the overflow entries placed by rank. */
static void gap_step_end(elo_ctx* c, const vec* rows, uint32_t R, uint32_t* cap, uint64_t* ov, uint64_t entries) {
  uint32_t r;
  uint64_t nrows = 0, moved = 0, n = *ov;
  if (!n) return;
  if (getenv("ELO_GAPTRACE")) /* diagnostic: which gapped CSR relocates rows after which step */
    fprintf(stderr, "step %u relocate rows %u ovf %llu entries %llu\n", c->supersteps, R, (unsigned long long)n,
            (unsigned long long)entries);
  for (r = 0; r < R; ++r)
    if (rows[r].n > cap[r]) {
      ++nrows;
      moved += cap[r];
      cap[r] = GAP_CAP(rows[r].n);
    }
  EVN(EL_K_SCAN, EL_EV_TRIG, n);
  EVN(EL_K_SCAN, EL_EV_RMW, n);
  EVN(EL_K_SCAN, EL_EV_ROW, nrows);
  EVN(EL_K_MERGE_PTR, EL_EV_ENT, 2 * nrows);
  EVN(EL_K_SCATTER_OLD, EL_EV_TRIG, moved);
  EVN(EL_K_SCATTER_OLD, EL_EV_ENT, moved);
  EVN(EL_K_SCATTER_OLD, EL_EV_EMIT, moved);
  EVN(EL_K_SCATTER_NEW, EL_EV_TRIG, n);
  EVN(EL_K_SCATTER_NEW, EL_EV_ENT, 3 * n);
  EVN(EL_K_SCATTER_NEW, EL_EV_EMIT, n);
  *ov = 0;
}

static int superstep(elo_ctx* c, uint32_t mask, uint64_t sb, uint64_t se, uint64_t lb, uint64_t le,
                     uint64_t ab, uint64_t ae, uint64_t pb, uint64_t pe) {
  cands k;
  size_t i;
  uint64_t s0 = c->slog_x.n, l0 = c->llog_x.n, a0 = c->alog_y.n, p0 = c->plog_p.n;
  int do_a = (mask & M_RRNG) && ae > ab, do_p = (mask & M_R4P) && pe > pb;
  uint64_t ev0[EL_NUM_KERNELS][EL_NUM_EVENTS];
  if (!(se > sb || le > lb || do_a || do_p)) return 0;
  memcpy(ev0, c->ev, sizeof ev0);
  if (c->llog_x.n == c->l_base) mask |= M_LEMPTY; /* empty sets: their probes are skipped (as on the GPU) */
  if (c->plog_p.n == c->p_base) mask |= M_PEMPTY;
  memset(&k, 0, sizeof k);
  /* generation: reads only the state of the previous step */
  expand_s(c, &k, mask, sb, se, a0);
  cr1_report(c->supersteps);
  expand_l(c, &k, mask, lb, le);
  if (do_a) expand_a(c, &k, se, ab, ae);
  if (do_p) expand_p(c, &k, pb, pe);
  run_jobs(c, &k, (mask & M_LEMPTY) != 0);
  if (k.sx.n + k.s1x.n + k.lx.n + k.ay.n + k.pp.n == 0) {
    cands_free(&k);
    return 0;
  }
  /* commit: the CR1 closure candidates first (k_commit_told on the GPU), so a fact that is
   * also a closure candidate is marked closed whatever else derived it */
  for (i = 0; i < k.s1x.n; ++i) {
    uint32_t x = k.s1x.v[i], a = k.s1a.v[i];
    EV(EL_K_COMMIT_T, EL_EV_TRIG);
    EV(EL_K_COMMIT_T, EL_EV_RMW);
    if (setbit(c, x, a)) {
      EV(EL_K_COMMIT_T, EL_EV_EMIT);
      vpush(&c->slog_x, x);
      vpush(&c->slog_a, a);
      vpush(&c->slog_f, 1);
      vpush(&c->srow[x], a);
    }
  }
  if (getenv("ELO_WINSTAT") && k.sx.n) { /* diagnostic: distinct (x, word) / (x, a) per window of W candidates */
    size_t w, W, q, r;
    for (W = 64; W <= 4096; W *= 8) {
      uint64_t dw = 0, da = 0;
      uint64_t* key = (uint64_t*)malloc(W * sizeof(uint64_t));
      for (w = 0; w < k.sx.n; w += W) {
        size_t m = k.sx.n - w < W ? k.sx.n - w : W;
        for (q = 0; q < m; ++q) key[q] = ((uint64_t)k.sx.v[w + q] << 32) | k.sa.v[w + q];
        qsort(key, m, sizeof(uint64_t), cmp_u64);
        for (q = 0; q < m; ++q) {
          da += q == 0 || key[q] != key[q - 1];
          r = q == 0 || (key[q] >> 5) != (key[q - 1] >> 5);
          dw += r;
        }
      }
      free(key);
      fprintf(stderr, "winstat step %u cands %zu window %zu distinct_fact %llu distinct_word %llu\n", c->supersteps,
              k.sx.n, W, (unsigned long long)da, (unsigned long long)dw);
    }
  }
  for (i = 0; i < k.sx.n; ++i) {
    uint32_t x = k.sx.v[i], a = k.sa.v[i];
    EV(EL_K_COMMIT_S, EL_EV_TRIG);
    EV(EL_K_COMMIT_S, EL_EV_RMW);
    if (setbit(c, x, a)) {
      EV(EL_K_COMMIT_S, EL_EV_EMIT);
      vpush(&c->slog_x, x);
      vpush(&c->slog_a, a);
      vpush(&c->slog_f, 0);
      vpush(&c->srow[x], a);
    }
  }
  for (i = 0; i < k.lx.n; ++i) {
    uint32_t x = k.lx.v[i], p = k.lp.v[i];
    EV(EL_K_COMMIT_L, EL_EV_TRIG);
    EV(EL_K_COMMIT_L, EL_EV_HASH);
    if (hs_add(&c->links, lkey(p, x))) {
      EV(EL_K_COMMIT_L, EL_EV_EMIT);
      if (c->need_pred) gap_append_ev(c, EL_K_COMMIT_L, c->pred[p].n, c->cap_pr[p], &c->ov_pr);
      /* successor rows are read only by CR6 with the row's role second: other links stay out */
      if (c->need_succ && c->chs.ptr[c->pair_role[p] + 1] > c->chs.ptr[c->pair_role[p]]) {
        gap_append_ev(c, EL_K_COMMIT_L, c->succ[x].n, c->cap_sc[x], &c->ov_sc);
        vpush(&c->succ[x], p);
      }
      vpush(&c->llog_x, x);
      vpush(&c->llog_p, p);
      vpush(&c->pred[p], x);
    }
  }
  for (i = 0; i < k.ay.n; ++i) {
    uint32_t y = k.ay.v[i], cc = k.ac.v[i];
    EV(EL_K_COMMIT_A, EL_EV_TRIG);
    EV(EL_K_COMMIT_A, EL_EV_HASH);
    if (hs_add(&c->acts, lkey(cc, y))) {
      EV(EL_K_COMMIT_A, EL_EV_EMIT);
      vpush(&c->actrow[y], (uint32_t)c->alog_y.n);
      vpush(&c->alog_y, y);
      vpush(&c->alog_c, cc);
      c->has_act[y] = 1;
    }
  }
  for (i = 0; i < k.pp.n; ++i) {
    uint32_t pid = k.pp.v[i], b = k.pb.v[i];
    EV(EL_K_COMMIT_P, EL_EV_TRIG);
    EV(EL_K_COMMIT_P, EL_EV_HASH);
    if (hs_add(&c->props, lkey(pid, b))) {
      EV(EL_K_COMMIT_P, EL_EV_EMIT);
      gap_append_ev(c, EL_K_COMMIT_P, c->prow[pid].n, c->cap_pp[pid], &c->ov_pp);
      vpush(&c->plog_p, pid);
      vpush(&c->plog_b, b);
      vpush(&c->prow[pid], b);
    }
  }
  cands_free(&k);
  /* the S-row CSR is not read during saturation (built lazily for export); a gapped CSR
   * with overflowing rows is re-laid out */
  gap_step_end(c, c->pred, c->P, c->cap_pr, &c->ov_pr, c->llog_x.n);
  gap_step_end(c, c->succ, c->N, c->cap_sc, &c->ov_sc, c->llog_x.n);
  gap_step_end(c, c->prow, c->P, c->cap_pp, &c->ov_pp, c->plog_p.n);
  if (getenv("ELO_STEPEV")) { /* diagnostic: this superstep's events per kernel (nonzero rows) */
    int kk, ee;
    for (kk = 0; kk < EL_NUM_KERNELS; ++kk) {
      uint64_t tot = 0;
      for (ee = 0; ee < EL_NUM_EVENTS; ++ee) tot += c->ev[kk][ee] - ev0[kk][ee];
      if (!tot) continue;
      fprintf(stderr, "stepev %u k%d", c->supersteps, kk);
      for (ee = 0; ee < EL_NUM_EVENTS; ++ee) fprintf(stderr, " %llu", (unsigned long long)(c->ev[kk][ee] - ev0[kk][ee]));
      fprintf(stderr, "\n");
    }
  }
  return c->slog_x.n > s0 || c->llog_x.n > l0 || c->alog_y.n > a0 || c->plog_p.n > p0;
}

/* ------------------------------------------------------------------ naive engine */

static uint8_t* cube_at(elo_ctx* c, uint32_t r, uint32_t x, uint32_t y) {
  return &c->cube[((uint64_t)r * c->N + x) * c->N + y];
}

static int naive_saturate(elo_ctx* c) {
  const el_axioms* ax = &c->ax;
  uint32_t N = c->N, i, x, y, z, q;
  int changed = 1;
  c->supersteps = 0;
  while (changed) {
    changed = 0;
    c->supersteps++;
    for (i = 0; i < ax->n_sub; ++i)
      for (x = 0; x < N; ++x)
        if (bit(c, x, ax->sub_a[i])) changed |= setbit(c, x, ax->sub_b[i]);
    for (i = 0; i < ax->n_conj; ++i)
      for (x = 0; x < N; ++x) {
        int all = 1;
        for (q = ax->conj_ptr[i]; q < ax->conj_ptr[i + 1]; ++q)
          if (!bit(c, x, ax->conj_ops[q])) all = 0;
        if (all) changed |= setbit(c, x, ax->conj_b[i]);
      }
    for (i = 0; i < ax->n_ex_rhs; ++i)
      for (x = 0; x < N; ++x)
        if (bit(c, x, ax->exr_a[i])) {
          uint8_t* l = cube_at(c, ax->exr_r[i], x, ax->exr_b[i]);
          if (!*l) *l = 1, changed = 1;
        }
    for (i = 0; i < ax->n_ex_lhs; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, ax->exl_r[i], x, y) && bit(c, y, ax->exl_a[i]))
            changed |= setbit(c, x, ax->exl_b[i]);
    for (i = 0; i < ax->n_subrole; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, ax->sr_r[i], x, y)) {
            uint8_t* l = cube_at(c, ax->sr_s[i], x, y);
            if (!*l) *l = 1, changed = 1;
          }
    for (i = 0; i < ax->n_chain; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, ax->ch_r[i], x, y))
            for (z = 0; z < N; ++z)
              if (*cube_at(c, ax->ch_s[i], y, z)) {
                uint8_t* l = cube_at(c, ax->ch_t[i], x, z);
                if (!*l) *l = 1, changed = 1;
              }
    for (i = 0; i < c->R; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, i, x, y) && bit(c, y, EL_BOTTOM)) changed |= setbit(c, x, EL_BOTTOM);
    for (i = 0; i < ax->n_domain; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, ax->dom_r[i], x, y) && x != EL_TOP && c->kind[x] != EL_KIND_DATATYPE)
            changed |= setbit(c, x, ax->dom_c[i]);
    for (i = 0; i < ax->n_range; ++i)
      for (x = 0; x < N; ++x)
        for (y = 0; y < N; ++y)
          if (*cube_at(c, ax->rng_r[i], x, y) && y != EL_TOP && c->kind[y] != EL_KIND_DATATYPE)
            for (z = 0; z < N; ++z)
              if (bit(c, z, y)) changed |= setbit(c, z, ax->rng_c[i]);
  }
  return 0;
}

/* ------------------------------------------------------------------ API */

/* The device builds told*, exr*, exl* per classification (el_closure.hip, Kahn levels: each
 * concept merges its told supers' rows); its events by the algorithm's definition, per concept
 * A: one trigger; rows: its supers, its subs, its own exr / exl rows, the three rows of every
 * super; entries: the supers, the subs, the rows gathered (the supers' rows, its own axioms)
 * and the rows written; one pending-count decrement per sub. */
static void closure_events(elo_ctx* c) {
  uint32_t A, j;
#define RL(cs, x) ((uint64_t)((cs).ptr[(x) + 1] - (cs).ptr[(x)]))
  for (A = 0; A < c->N; ++A) {
    uint64_t np = RL(c->told, A), g = 0;
    for (j = c->told.ptr[A]; j < c->told.ptr[A + 1]; ++j) {
      uint32_t p = c->told.a[j];
      g += RL(c->toldc, p) + RL(c->exr, p) + 2 * RL(c->exl, p);
    }
    EV(EL_K_CLOSURE, EL_EV_TRIG);
    EVN(EL_K_CLOSURE, EL_EV_ROW, 4 + 3 * np);
    EVN(EL_K_CLOSURE, EL_EV_ENT, np + c->nsub[A] + g + c->xr_n[A] + 2ull * c->xl_n[A] + RL(c->toldc, A) + RL(c->exr, A) +
                                     2 * RL(c->exl, A));
    EVN(EL_K_CLOSURE, EL_EV_RMW, c->nsub[A]);
  }
#undef RL
}

int elo_init(elo_ctx* c) {
  uint32_t x;
  if (!c) return EL_EINVAL;
  uint64_t init = 0;
  closure_events(c);
  /* S(X) = {X, ⊤} (classes, individuals) and the told closure of X, flagged — what CR1 would
   * derive from the init fact in the first superstep (k_init on the GPU) */
  for (x = 0; x < c->N; ++x) {
    int two = x != EL_TOP && x != EL_BOTTOM && c->kind[x] != EL_KIND_DATATYPE;
    uint32_t j;
    EV(EL_K_INIT, EL_EV_ENT);
    EV(EL_K_INIT, EL_EV_RMW);
    EV(EL_K_INIT, EL_EV_EMIT);
    setbit(c, x, x);
    vpush(&c->slog_x, x);
    vpush(&c->slog_a, x);
    vpush(&c->slog_f, 2); /* its closure is written right here; its links / propagations are not */
    vpush(&c->srow[x], x);
    ++init;
    if (two) {
      EV(EL_K_INIT, EL_EV_RMW);
      EV(EL_K_INIT, EL_EV_EMIT);
      setbit(c, x, EL_TOP);
      vpush(&c->slog_x, x);
      vpush(&c->slog_a, EL_TOP);
      vpush(&c->slog_f, 0);
      vpush(&c->srow[x], EL_TOP);
      ++init;
    }
    for (j = c->toldc.ptr[x]; j < c->toldc.ptr[x + 1]; ++j) {
      uint32_t b = c->toldc.a[j];
      EV(EL_K_INIT, EL_EV_ENT);
      if (two && b == EL_TOP) continue;
      EV(EL_K_INIT, EL_EV_RMW);
      EV(EL_K_INIT, EL_EV_EMIT);
      setbit(c, x, b);
      vpush(&c->slog_x, x);
      vpush(&c->slog_a, b);
      vpush(&c->slog_f, 1);
      vpush(&c->srow[x], b);
    }
  }
  c->s_init = init;
  c->base = 0;
  c->l_base = 0;
  c->fresh = 1;
  return EL_OK;
}

/* the base links (el_ctx::install_base): exr in X order into the link log, each X into the
 * predecessor row of its pids (so rows hold ascending X, as exrT), chain-second pids into the
 * successor row of X (exrC); events of the coalesced writes as the GPU host counts them */
static void base_links(elo_ctx* c) {
  uint32_t x, j;
  uint64_t nb = c->exr.ptr[c->N], nc = 0;
  if (nb == 0 || c->llog_x.n != 0) return;
  for (x = 0; x < c->N; ++x)
    for (j = c->exr.ptr[x]; j < c->exr.ptr[x + 1]; ++j) {
      uint32_t p = c->exr.a[j], r = c->pair_role[p];
      vpush(&c->llog_x, x);
      vpush(&c->llog_p, p);
      vpush(&c->pred[p], x);
      if (c->need_succ && c->chs.ptr[r + 1] > c->chs.ptr[r]) {
        vpush(&c->succ[x], p);
        ++nc;
      }
    }
  EVN(EL_K_INIT, EL_EV_ENT, nb + (c->need_pred ? nb : 0) + nc);
  EVN(EL_K_INIT, EL_EV_EMIT, nb);
  c->l_base = nb;
  c->base = 1;
  /* base propagations: the CR4 half-1 records of every init fact Y ∈ S(Y), ((r, Y), B) for
   * (r, B) ∈ exl(Y) over its told closure — pid-major, B ascending (pids sort by (Y, r)) */
  {
    uint64_t nbp = 0;
    uint32_t y, p;
    for (y = 0; y < c->N; ++y)
      for (j = c->exl.ptr[y]; j < c->exl.ptr[y + 1]; ++j) {
        PID_OF(c->exl.a[j], y, p);
        if (p == NONE) continue;
        vpush(&c->plog_p, p);
        vpush(&c->plog_b, c->exl.b[j]);
        vpush(&c->prow[p], c->exl.b[j]);
        c->bpn[p]++;
        ++nbp;
      }
    if (nbp) {
      int r;
      EVN(EL_K_INIT, EL_EV_ENT, 2 * nbp);
      EVN(EL_K_INIT, EL_EV_EMIT, nbp);
      for (r = 0; r < EL_NUM_RULE_TYPES; ++r) c->wm_p[r] = nbp; /* nothing left to fan out */
    }
    c->p_base = nbp;
  }
}

/* The base links / propagations stay out of the sets for the whole saturation (as on the GPU,
 * el_ctx::install_base): a membership test is base_has / the bpp binary search, then the set
 * probe.  (Round 2 filled the sets after the first superstep, EL_K_REHASH.) */
static void base_join(elo_ctx* c) { (void)c; }

int elo_step(elo_ctx* c, int rule, int* changed) {
  uint64_t se, le, ae, pe;
  if (!c || !changed || rule < 0 || rule >= EL_NUM_RULE_TYPES || c->mode != 0) return EL_EINVAL;
  c->fresh = 0; /* per-rule stepping derives every link */
  se = c->slog_x.n, le = c->llog_x.n, ae = c->alog_y.n, pe = c->plog_p.n;
  *changed = superstep(c, rule_mask[rule], c->wm_s[rule], se, c->wm_l[rule], le, c->wm_a[rule], ae,
                       c->wm_p[rule], pe);
  c->wm_s[rule] = se;
  c->wm_l[rule] = le;
  c->wm_a[rule] = ae;
  c->wm_p[rule] = pe;
  return EL_OK;
}

int elo_saturate(elo_ctx* c) {
  uint64_t sb, lb, ab, pb, pe;
  int r;
  if (!c) return EL_EINVAL;
  if (c->mode == 1) return naive_saturate(c);
  if (c->fresh) base_links(c);
  c->fresh = 0;
  sb = c->slog_x.n, lb = c->llog_x.n, ab = c->alog_y.n;
  for (r = 0; r < EL_NUM_RULE_TYPES; ++r) {
    if (c->wm_s[r] < sb) sb = c->wm_s[r];
    if (c->wm_l[r] < lb) lb = c->wm_l[r];
    if (c->wm_a[r] < ab) ab = c->wm_a[r];
  }
  /* propagations from per-rule stepping not yet fanned out by CR_TYPE3_2 */
  pb = c->wm_p[EL_CR_TYPE3_2] < c->plog_p.n ? c->wm_p[EL_CR_TYPE3_2] : c->plog_p.n;
  pe = c->plog_p.n;
  c->tr_s.n = c->tr_l.n = c->tr_a.n = 0;
  c->supersteps = 0;
  for (;;) {
    uint64_t se = c->slog_x.n, le = c->llog_x.n, ae = c->alog_y.n;
    if (se == sb && le == lb && ae == ab && pb == pe) break;
    vpush(&c->tr_s, (uint32_t)(se - sb));
    vpush(&c->tr_l, (uint32_t)(le - lb));
    vpush(&c->tr_a, (uint32_t)(ae - ab));
    c->supersteps++;
    superstep(c, pb < pe ? (M_ALL | M_R4P) : M_ALL, sb, se, lb, le, ab, ae, pb, pe);
    base_join(c);
    sb = se, lb = le, ab = ae;
    pb = pe = c->plog_p.n;
  }
  for (r = 0; r < EL_NUM_RULE_TYPES; ++r) {
    c->wm_s[r] = c->slog_x.n;
    c->wm_l[r] = c->llog_x.n;
    c->wm_a[r] = c->alog_y.n;
    c->wm_p[r] = c->plog_p.n;
  }
  return EL_OK;
}

static uint64_t naive_count_facts(const elo_ctx* c) {
  uint64_t n = 0, i, words = (uint64_t)c->N * c->W;
  for (i = 0; i < words; ++i) n += (uint64_t)__builtin_popcount(c->bits[i]);
  return n;
}

uint64_t elo_num_facts(const elo_ctx* c) { return c->mode == 1 ? naive_count_facts(c) : c->slog_x.n; }
uint64_t elo_num_init(const elo_ctx* c) { return c->s_init; }
uint64_t elo_num_acts(const elo_ctx* c) { return c->alog_y.n; }
uint32_t elo_supersteps(const elo_ctx* c) { return c->supersteps; }

uint64_t elo_num_links(const elo_ctx* c) {
  if (c->mode == 1) {
    uint64_t n = 0, i, tot = (uint64_t)(c->R ? c->R : 1) * c->N * c->N;
    for (i = 0; i < tot; ++i) n += c->cube[i];
    return n;
  }
  return c->llog_x.n;
}

int elo_copy_facts(const elo_ctx* c, uint32_t* x, uint32_t* a, size_t cap) {
  uint64_t n = 0;
  uint32_t r, b;
  if (cap < elo_num_facts(c)) return EL_ERANGE;
  for (r = 0; r < c->N; ++r)
    for (b = 0; b < c->N; ++b)
      if (bit(c, r, b)) {
        x[n] = r;
        a[n] = b;
        ++n;
      }
  return EL_OK;
}

static int u64cmp(const void* p, const void* q) {
  uint64_t a = *(const uint64_t*)p, b = *(const uint64_t*)q;
  return a < b ? -1 : a > b;
}

int elo_copy_links(const elo_ctx* c, uint32_t* x, uint32_t* r, uint32_t* y, size_t cap) {
  uint64_t n = elo_num_links(c), i = 0;
  if (cap < n) return EL_ERANGE;
  if (c->mode == 1) {
    uint32_t xx, rr, yy;
    for (xx = 0; xx < c->N; ++xx)
      for (rr = 0; rr < c->R; ++rr)
        for (yy = 0; yy < c->N; ++yy)
          if (c->cube[((uint64_t)rr * c->N + xx) * c->N + yy]) {
            x[i] = xx, r[i] = rr, y[i] = yy;
            ++i;
          }
    return EL_OK;
  }
  {
    /* (x, r, y) order: sort by x then pid (pids are sorted by (y, r)), then re-sort */
    uint64_t* k = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    for (i = 0; i < n; ++i) {
      uint32_t p = c->llog_p.v[i];
      /* key: x (22+ bits) | r | y packed as x<<40 would overflow for big ids; use two passes */
      k[i] = ((uint64_t)c->llog_x.v[i] << 32) | p;
    }
    qsort(k, n, sizeof(uint64_t), u64cmp);
    for (i = 0; i < n; ++i) {
      uint32_t p = (uint32_t)k[i];
      x[i] = (uint32_t)(k[i] >> 32);
      r[i] = c->pair_role[p];
      y[i] = c->pair_y[p];
    }
    /* within one x, order by (r, y): insertion sort of the small runs */
    {
      uint64_t s = 0;
      while (s < n) {
        uint64_t e = s, a2, b2;
        while (e < n && x[e] == x[s]) ++e;
        for (a2 = s + 1; a2 < e; ++a2) {
          uint32_t rr = r[a2], yy = y[a2];
          b2 = a2;
          while (b2 > s && (r[b2 - 1] > rr || (r[b2 - 1] == rr && y[b2 - 1] > yy))) {
            r[b2] = r[b2 - 1];
            y[b2] = y[b2 - 1];
            --b2;
          }
          r[b2] = rr;
          y[b2] = yy;
        }
        s = e;
      }
    }
    free(k);
  }
  return EL_OK;
}

/* The fact log in append order (init facts, then superstep by superstep): diagnostics
 * (scripts/commit_floor.py splits it by superstep with elo_trace). */
int elo_copy_log(const elo_ctx* c, uint32_t* x, uint32_t* a, size_t cap) {
  if (cap < c->slog_x.n) return EL_ERANGE;
  memcpy(x, c->slog_x.v, c->slog_x.n * sizeof(uint32_t));
  memcpy(a, c->slog_a.v, c->slog_a.n * sizeof(uint32_t));
  return EL_OK;
}

int elo_trace(const elo_ctx* c, uint64_t* ds, uint64_t* dl, uint64_t* da, size_t cap) {
  size_t i;
  if (cap < c->tr_s.n) return EL_ERANGE;
  for (i = 0; i < c->tr_s.n; ++i) {
    if (ds) ds[i] = c->tr_s.v[i];
    if (dl) dl[i] = c->tr_l.v[i];
    if (da) da[i] = c->tr_a.v[i];
  }
  return EL_OK;
}

int elo_events(const elo_ctx* c, uint64_t* events, size_t cap) {
  if (cap < (size_t)EL_NUM_KERNELS * EL_NUM_EVENTS) return EL_ERANGE;
  memcpy(events, c->ev, sizeof c->ev);
  return EL_OK;
}

const char* elo_error(const elo_ctx* c) { return c ? c->err : "null"; }

void elo_destroy(elo_ctx* c) {
  uint32_t i;
  if (!c) return;
  csr_free(&c->told), csr_free(&c->toldc), csr_free(&c->cidx), csr_free(&c->exr), csr_free(&c->exl);
  csr_free(&c->psup), csr_free(&c->chf), csr_free(&c->chs), csr_free(&c->dom), csr_free(&c->rng);
  free(c->conj.ptr), free(c->conj.a), free(c->conj_b);
  free(c->fp_ptr), free(c->pair_role), free(c->pair_y), free(c->role_has_exl);
  free(c->supers_ptr), free(c->supers), free(c->kind), free(c->bits);
  free(c->xr_n), free(c->xl_n), free(c->nsub);
  if (c->srow)
    for (i = 0; i < c->N; ++i) free(c->srow[i].v);
  if (c->succ)
    for (i = 0; i < c->N; ++i) free(c->succ[i].v);
  if (c->pred)
    for (i = 0; i < c->P; ++i) free(c->pred[i].v);
  if (c->prow)
    for (i = 0; i < c->P; ++i) free(c->prow[i].v);
  free(c->prow), free(c->bpn), free(c->props.t), free(c->plog_p.v), free(c->plog_b.v);
  if (c->actrow)
    for (uint32_t y = 0; y < c->N; ++y) free(c->actrow[y].v);
  free(c->actrow);
  free(c->srow), free(c->succ), free(c->pred), free(c->has_act);
  free(c->cap_pr), free(c->cap_sc), free(c->cap_pp);
  free(c->slog_x.v), free(c->slog_a.v), free(c->slog_f.v), free(c->llog_x.v), free(c->llog_p.v);
  free(c->alog_y.v), free(c->alog_c.v), free(c->tr_s.v), free(c->tr_l.v), free(c->tr_a.v);
  free(c->links.t), free(c->acts.t), free(c->cube);
  free((void*)c->ax.sub_a), free((void*)c->ax.sub_b), free((void*)c->ax.conj_ptr);
  free((void*)c->ax.conj_ops), free((void*)c->ax.conj_b), free((void*)c->ax.exr_a);
  free((void*)c->ax.exr_r), free((void*)c->ax.exr_b), free((void*)c->ax.exl_r);
  free((void*)c->ax.exl_a), free((void*)c->ax.exl_b), free((void*)c->ax.sr_r);
  free((void*)c->ax.sr_s), free((void*)c->ax.ch_r), free((void*)c->ax.ch_s);
  free((void*)c->ax.ch_t), free((void*)c->ax.dom_r), free((void*)c->ax.dom_c);
  free((void*)c->ax.rng_r), free((void*)c->ax.rng_c);
  free(c);
}
