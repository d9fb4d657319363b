/*
 * worklist.c — an independent EL+ saturator (TEST INFRASTRUCTURE ONLY: the checker that pins
 * the semi-naive oracle el_oracle.c, never the product).
 *
 * A textbook worklist completion (the "context" algorithm of CEL / ELK): every derived fact
 * A ∈ S(X) or link (X, r, Y) ∈ R(r) is inserted into a hash set once and queued once; taking
 * it off the queue applies every completion rule in which it is a premise, joined with the
 * current sets.  It shares no code and no data structure with el_oracle.c: no bit matrix, no
 * supersteps, no told closure, no pair universe, no fact flags, no event accounting.  The
 * rules are the ones the reference's rule kernels implement:
 *   CR1  A ⊑ B                     Type1_1AxiomProcessorBase.java:22-43
 *   CR2  A1 ⊓ … ⊓ An ⊑ B           Type1_2AxiomProcessorBase.java:45-66
 *   CR3  A ⊑ ∃r.B                  Type2AxiomProcessorBase.java:45-75, RolePairHandler.java:353-446
 *   CR4  ∃r.A ⊑ B                  Type3_1AxiomProcessorBase.java:194-239, Type3_2AxiomProcessorBase.java:67-96
 *   CR5  r ⊑ s                     Type4AxiomProcessorBase.java:38-76
 *   CR6  r ∘ s ⊑ t (s checked)     Type5AxiomProcessorBase.java:115-154
 *   ⊥    ⊥ ∈ S(Y), (X,Y) ∈ R(r)    TypeBottomAxiomProcessorBase.java:62-123
 *   domain(r) = D                  RolePairHandler.java:480-490 (X ≠ ⊤, X not a datatype)
 *   range(r) = C                   distel_range = 1: DistEL's K10 (RolePairHandler.java:471-479,
 *                                  ScriptsCollection.java:45-62): C ∈ S(Z) for every Z with
 *                                  Y ∈ S(Z) (Y ≠ ⊤, Y not a datatype);
 *                                  distel_range = 0: ELK-style — the link (X, r, Y) made by CR3
 *                                  from A ⊑ ∃r.B goes to the filler B ⊓ ranges(r) instead, i.e.
 *                                  the link target is the normalizer's fresh X_{B,r} with
 *                                  X ⊑ B, X ⊑ C for C ∈ ranges*(r) (Normalizer.java:122-137,
 *                                  455-497); an individual filler b is an instance of each C;
 *                                  see wl_saturate.
 *   init S(X) = {X, ⊤}             AxiomLoader.java:1237-1245, 1281-1289
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "el_gpu.h"

typedef struct {
  uint32_t* a;
  uint64_t n, cap;
} vec;

static int vpush(vec* v, uint32_t x) {
  if (v->n == v->cap) {
    uint64_t c = v->cap ? 2 * v->cap : 4;
    uint32_t* p = (uint32_t*)realloc(v->a, c * sizeof(uint32_t));
    if (!p) return -1;
    v->a = p;
    v->cap = c;
  }
  v->a[v->n++] = x;
  return 0;
}

/* open-addressing set of 64-bit keys (~0 = empty), grown at load 1/2 */
typedef struct {
  uint64_t* k;
  uint64_t cap, n;
} hset;

static uint64_t mix(uint64_t k) {
  k ^= k >> 31;
  k *= 0x7fb5d329728ea185ull;
  k ^= k >> 27;
  k *= 0x81dadef4bc2dd44dull;
  return k ^ (k >> 33);
}

static int hs_insert(hset* h, uint64_t key);

static int hs_grow(hset* h) {
  hset g = {NULL, h->cap ? 2 * h->cap : 1024, 0};
  g.k = (uint64_t*)malloc(g.cap * sizeof(uint64_t));
  if (!g.k) return -1;
  memset(g.k, 0xff, g.cap * sizeof(uint64_t));
  for (uint64_t i = 0; i < h->cap; ++i)
    if (h->k[i] != ~0ull) hs_insert(&g, h->k[i]);
  free(h->k);
  *h = g;
  return 0;
}

/* 1 = inserted, 0 = present, -1 = out of memory */
static int hs_insert(hset* h, uint64_t key) {
  if (2 * (h->n + 1) > h->cap && hs_grow(h)) return -1;
  uint64_t i = mix(key) & (h->cap - 1);
  while (h->k[i] != ~0ull) {
    if (h->k[i] == key) return 0;
    i = (i + 1) & (h->cap - 1);
  }
  h->k[i] = key;
  h->n++;
  return 1;
}

static int hs_has(const hset* h, uint64_t key) {
  if (!h->cap) return 0;
  uint64_t i = mix(key) & (h->cap - 1);
  while (h->k[i] != ~0ull) {
    if (h->k[i] == key) return 1;
    i = (i + 1) & (h->cap - 1);
  }
  return 0;
}

/* key -> list of values (pairs stored as two consecutive entries), a CSR built once */
typedef struct {
  uint32_t* ptr; /* nkeys + 1 */
  uint32_t* val;
  uint32_t width;
} multimap;

static int mm_build(multimap* m, uint32_t nkeys, uint32_t n, const uint32_t* key, const uint32_t* v0,
                    const uint32_t* v1) {
  m->width = v1 ? 2 : 1;
  m->ptr = (uint32_t*)calloc((size_t)nkeys + 1, sizeof(uint32_t));
  m->val = (uint32_t*)malloc(((size_t)n * m->width + 1) * sizeof(uint32_t));
  uint32_t* fill = (uint32_t*)calloc((size_t)nkeys + 1, sizeof(uint32_t));
  if (!m->ptr || !m->val || !fill) {
    free(fill);
    return -1;
  }
  for (uint32_t i = 0; i < n; ++i) m->ptr[key[i] + 1]++;
  for (uint32_t k = 0; k < nkeys; ++k) m->ptr[k + 1] += m->ptr[k];
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t at = m->ptr[key[i]] + fill[key[i]]++;
    m->val[(size_t)at * m->width] = v0[i];
    if (v1) m->val[(size_t)at * m->width + 1] = v1[i];
  }
  free(fill);
  return 0;
}

static void mm_free(multimap* m) {
  free(m->ptr);
  free(m->val);
}

enum { EV_FACT = 0, EV_LINK = 1, EV_ACT = 2 };

typedef struct wl_result {
  uint32_t N, R;
  const uint8_t* kind;
  const el_axioms* ax;
  int distel_range;
  hset sset, lset, aset;
  vec *srow, *sinv, *out, *in, *acts;
  vec queue; /* (kind, u, v, w) quads */
  multimap subA, conjOp, exrA, exlA, exlR, subR, chF, chS, domR, rngR;
  uint32_t *rng_ptr, *rng_all; /* ranges*(r): ranges of r and of every super-role of r */
  uint32_t N_out;              /* concepts reported (fresh ELK-range fillers are not) */
  void* owned[4];              /* transformed axiom arrays and kinds this result allocated */
  uint64_t n_facts, n_links;
  int oom;
} wl_result;

static uint64_t lkey(const wl_result* w, uint32_t x, uint32_t r, uint32_t y) {
  return ((uint64_t)x * w->R + r) * w->N + y;
}

static void push_ev(wl_result* w, uint32_t k, uint32_t u, uint32_t v, uint32_t x) {
  if (vpush(&w->queue, k) | vpush(&w->queue, u) | vpush(&w->queue, v) | vpush(&w->queue, x)) w->oom = 1;
}

static void add_fact(wl_result* w, uint32_t x, uint32_t a) {
  const int r = hs_insert(&w->sset, ((uint64_t)x << 32) | a);
  if (r < 0) w->oom = 1;
  if (r != 1) return;
  if (vpush(&w->srow[x], a) | vpush(&w->sinv[a], x)) w->oom = 1;
  push_ev(w, EV_FACT, x, a, 0);
}

static int has_fact(const wl_result* w, uint32_t x, uint32_t a) {
  return hs_has(&w->sset, ((uint64_t)x << 32) | a);
}

static void add_link(wl_result* w, uint32_t x, uint32_t r, uint32_t y) {
  const int k = hs_insert(&w->lset, lkey(w, x, r, y));
  if (k < 0) w->oom = 1;
  if (k != 1) return;
  if (vpush(&w->out[x], r) | vpush(&w->out[x], y) | vpush(&w->in[y], r) | vpush(&w->in[y], x)) w->oom = 1;
  push_ev(w, EV_LINK, x, r, y);
}

static void add_act(wl_result* w, uint32_t y, uint32_t c) {
  const int k = hs_insert(&w->aset, ((uint64_t)y << 32) | c);
  if (k < 0) w->oom = 1;
  if (k != 1) return;
  if (vpush(&w->acts[y], c)) w->oom = 1;
  push_ev(w, EV_ACT, y, c, 0);
}

static void on_fact(wl_result* w, uint32_t x, uint32_t a) {
  const el_axioms* ax = w->ax;
  for (uint32_t i = w->subA.ptr[a]; i < w->subA.ptr[a + 1]; ++i) add_fact(w, x, w->subA.val[i]);  // CR1
  for (uint32_t i = w->conjOp.ptr[a]; i < w->conjOp.ptr[a + 1]; ++i) {                             // CR2
    const uint32_t k = w->conjOp.val[i];
    int all = 1;
    for (uint32_t q = ax->conj_ptr[k]; q < ax->conj_ptr[k + 1] && all; ++q) all = has_fact(w, x, ax->conj_ops[q]);
    if (all) add_fact(w, x, ax->conj_b[k]);
  }
  for (uint32_t i = w->exrA.ptr[a]; i < w->exrA.ptr[a + 1]; ++i)  // CR3
    add_link(w, x, w->exrA.val[2 * i], w->exrA.val[2 * i + 1]);
  for (uint32_t i = w->exlA.ptr[a]; i < w->exlA.ptr[a + 1]; ++i) {  // CR4, new A ∈ S(Y = x)
    const uint32_t r = w->exlA.val[2 * i], b = w->exlA.val[2 * i + 1];
    for (uint64_t j = 0; j < w->in[x].n; j += 2)
      if (w->in[x].a[j] == r) add_fact(w, w->in[x].a[j + 1], b);
  }
  if (a == EL_BOTTOM)  // ⊥ over every link into x
    for (uint64_t j = 0; j < w->in[x].n; j += 2) add_fact(w, w->in[x].a[j + 1], EL_BOTTOM);
  for (uint64_t j = 0; j < w->acts[a].n; ++j) add_fact(w, x, w->acts[a].a[j]);  // range (DistEL)
}

static void on_link(wl_result* w, uint32_t x, uint32_t r, uint32_t y) {
  for (uint32_t i = w->exlR.ptr[r]; i < w->exlR.ptr[r + 1]; ++i)  // CR4, new link
    if (has_fact(w, y, w->exlR.val[2 * i])) add_fact(w, x, w->exlR.val[2 * i + 1]);
  for (uint32_t i = w->subR.ptr[r]; i < w->subR.ptr[r + 1]; ++i) add_link(w, x, w->subR.val[i], y);  // CR5
  for (uint32_t i = w->chF.ptr[r]; i < w->chF.ptr[r + 1]; ++i) {  // CR6, (x,y) ∈ R(r) first
    const uint32_t s = w->chF.val[2 * i], t = w->chF.val[2 * i + 1];
    for (uint64_t j = 0; j < w->out[y].n; j += 2)
      if (w->out[y].a[j] == s) add_link(w, x, t, w->out[y].a[j + 1]);
  }
  for (uint32_t i = w->chS.ptr[r]; i < w->chS.ptr[r + 1]; ++i) {  // CR6, (x,y) ∈ R(r) second
    const uint32_t p = w->chS.val[2 * i], t = w->chS.val[2 * i + 1];
    for (uint64_t j = 0; j < w->in[x].n; j += 2)
      if (w->in[x].a[j] == p) add_link(w, w->in[x].a[j + 1], t, y);
  }
  if (has_fact(w, y, EL_BOTTOM)) add_fact(w, x, EL_BOTTOM);
  if (x != EL_TOP && w->kind[x] != EL_KIND_DATATYPE)  // domain
    for (uint32_t i = w->domR.ptr[r]; i < w->domR.ptr[r + 1]; ++i) add_fact(w, x, w->domR.val[i]);
  if (w->distel_range && y != EL_TOP && w->kind[y] != EL_KIND_DATATYPE)  // range (DistEL K10)
    for (uint32_t i = w->rngR.ptr[r]; i < w->rngR.ptr[r + 1]; ++i) add_act(w, y, w->rngR.val[i]);
}

static void on_act(wl_result* w, uint32_t y, uint32_t c) {
  for (uint64_t j = 0; j < w->sinv[y].n; ++j) add_fact(w, w->sinv[y].a[j], c);
}

static int cmp_u32(const void* p, const void* q) {
  const uint32_t a = *(const uint32_t*)p, b = *(const uint32_t*)q;
  return a < b ? -1 : a > b;
}
static int cmp_pair(const void* p, const void* q) {
  const uint32_t* a = (const uint32_t*)p;
  const uint32_t* b = (const uint32_t*)q;
  if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
  return a[1] < b[1] ? -1 : a[1] > b[1];
}

void wl_free(wl_result* w);

/* Saturate ax.  distel_range = 0 gives ranges the ELK reading: every CR3 axiom A ⊑ ∃r.B whose
 * role r has ranges*(r) ≠ ∅ targets a fresh concept F_{B,r} (one per (B, r)) with told
 * F ⊑ B and F ⊑ C, C ∈ ranges*(r) — the normalizer's range elimination (Normalizer.java:
 * 122-137); fresh concepts are internal and not reported.  Returns 0 or -1 (out of memory). */
int wl_saturate(const el_axioms* ax, int distel_range, wl_result** out) {
  wl_result* w = (wl_result*)calloc(1, sizeof(wl_result));
  *out = w;
  if (!w) return -1;
  el_axioms* own = (el_axioms*)calloc(1, sizeof(el_axioms));
  if (!own) return -1;
  *own = *ax;
  w->ax = own;
  w->distel_range = distel_range;
  w->N_out = ax->n_concepts;
  w->R = ax->n_roles ? ax->n_roles : 1;
  uint32_t N = ax->n_concepts;
  /* ranges*(r): closure of r over told r ⊑ s, ranges of each */
  uint32_t R = ax->n_roles;
  w->rng_ptr = (uint32_t*)calloc((size_t)R + 1, sizeof(uint32_t));
  vec all = {0};
  for (uint32_t r = 0; r < R; ++r) {
    vec seen = {0}, stack = {0};
    vpush(&stack, r);
    while (stack.n) {
      const uint32_t s = stack.a[--stack.n];
      int dup = 0;
      for (uint64_t j = 0; j < seen.n; ++j) dup |= seen.a[j] == s;
      if (dup) continue;
      vpush(&seen, s);
      for (uint32_t i = 0; i < ax->n_subrole; ++i)
        if (ax->sr_r[i] == s) vpush(&stack, ax->sr_s[i]);
    }
    for (uint64_t j = 0; j < seen.n; ++j)
      for (uint32_t i = 0; i < ax->n_range; ++i)
        if (ax->rng_r[i] == seen.a[j]) vpush(&all, ax->rng_c[i]);
    w->rng_ptr[r + 1] = (uint32_t)all.n;
    free(seen.a);
    free(stack.a);
  }
  w->rng_all = all.a;
  /* ELK reading of ranges: redirect CR3 fillers through fresh concepts */
  uint32_t *exr_b2 = NULL, *sub_a2 = NULL, *sub_b2 = NULL;
  uint8_t* kind2 = NULL;
  if (!distel_range && ax->n_range) {
    exr_b2 = (uint32_t*)malloc(((size_t)ax->n_ex_rhs + 1) * sizeof(uint32_t));
    vec sa = {0}, sb = {0};
    for (uint32_t i = 0; i < ax->n_sub; ++i) vpush(&sa, ax->sub_a[i]), vpush(&sb, ax->sub_b[i]);
    hset fresh = {0};  /* (b, r) already given a fresh filler: key -> index via a side vec */
    vec fkey_b = {0}, fkey_r = {0};
    for (uint32_t i = 0; i < ax->n_ex_rhs; ++i) {
      const uint32_t r = ax->exr_r[i], b = ax->exr_b[i];
      const uint8_t kb = ax->concept_kind ? ax->concept_kind[b] : EL_KIND_CLASS;
      exr_b2[i] = b;
      if (w->rng_ptr[r + 1] == w->rng_ptr[r] || kb == EL_KIND_DATATYPE) continue;
      if (kb == EL_KIND_INDIVIDUAL) {  /* an r-successor individual is in every range of r */
        for (uint32_t j = w->rng_ptr[r]; j < w->rng_ptr[r + 1]; ++j) vpush(&sa, b), vpush(&sb, w->rng_all[j]);
        continue;
      }
      uint32_t f = UINT32_MAX;
      if (hs_has(&fresh, ((uint64_t)b << 32) | r))
        for (uint64_t j = 0; j < fkey_b.n; ++j)
          if (fkey_b.a[j] == b && fkey_r.a[j] == r) f = N + (uint32_t)j;
      if (f == UINT32_MAX) {
        hs_insert(&fresh, ((uint64_t)b << 32) | r);
        f = N + (uint32_t)fkey_b.n;
        vpush(&fkey_b, b);
        vpush(&fkey_r, r);
        vpush(&sa, f), vpush(&sb, b);
        for (uint32_t j = w->rng_ptr[r]; j < w->rng_ptr[r + 1]; ++j) vpush(&sa, f), vpush(&sb, w->rng_all[j]);
      }
      exr_b2[i] = f;
    }
    N += (uint32_t)fkey_b.n;
    kind2 = (uint8_t*)calloc(N, 1);
    if (ax->concept_kind) memcpy(kind2, ax->concept_kind, ax->n_concepts);
    sub_a2 = sa.a;
    sub_b2 = sb.a;
    own->n_sub = (uint32_t)sa.n;
    own->sub_a = sub_a2;
    own->sub_b = sub_b2;
    own->exr_b = exr_b2;
    own->n_concepts = N;
    own->concept_kind = kind2;
    w->owned[0] = exr_b2;
    w->owned[1] = sub_a2;
    w->owned[2] = sub_b2;
    w->owned[3] = kind2;
    free(fresh.k);
    free(fkey_b.a);
    free(fkey_r.a);
  }
  w->N = N;
  if (!own->concept_kind) {
    kind2 = (uint8_t*)calloc(N, 1);
    own->concept_kind = kind2;
    w->owned[3] = kind2;
  }
  w->kind = own->concept_kind;
  /* indexes */
  uint32_t nops = own->n_conj ? own->conj_ptr[own->n_conj] : 0;
  uint32_t* conj_id = (uint32_t*)malloc(((size_t)nops + 1) * sizeof(uint32_t));
  for (uint32_t k = 0; k < own->n_conj; ++k)
    for (uint32_t q = own->conj_ptr[k]; q < own->conj_ptr[k + 1]; ++q) conj_id[q] = k;
  int bad = mm_build(&w->subA, N, own->n_sub, own->sub_a, own->sub_b, NULL) |
            mm_build(&w->conjOp, N, nops, own->conj_ops, conj_id, NULL) |
            mm_build(&w->exrA, N, own->n_ex_rhs, own->exr_a, own->exr_r, own->exr_b) |
            mm_build(&w->exlA, N, own->n_ex_lhs, own->exl_a, own->exl_r, own->exl_b) |
            mm_build(&w->exlR, w->R, own->n_ex_lhs, own->exl_r, own->exl_a, own->exl_b) |
            mm_build(&w->subR, w->R, own->n_subrole, own->sr_r, own->sr_s, NULL) |
            mm_build(&w->chF, w->R, own->n_chain, own->ch_r, own->ch_s, own->ch_t) |
            mm_build(&w->chS, w->R, own->n_chain, own->ch_s, own->ch_r, own->ch_t) |
            mm_build(&w->domR, w->R, own->n_domain, own->dom_r, own->dom_c, NULL) |
            mm_build(&w->rngR, w->R, own->n_range, own->rng_r, own->rng_c, NULL);
  free(conj_id);
  w->srow = (vec*)calloc(N, sizeof(vec));
  w->sinv = (vec*)calloc(N, sizeof(vec));
  w->out = (vec*)calloc(N, sizeof(vec));
  w->in = (vec*)calloc(N, sizeof(vec));
  w->acts = (vec*)calloc(N, sizeof(vec));
  if (bad || !w->srow || !w->sinv || !w->out || !w->in || !w->acts) return -1;
  /* init: S(X) = {X, ⊤} (⊤ and ⊥ and datatypes: {X}) */
  for (uint32_t x = 0; x < N; ++x) {
    add_fact(w, x, x);
    if (x != EL_TOP && x != EL_BOTTOM && w->kind[x] != EL_KIND_DATATYPE) add_fact(w, x, EL_TOP);
  }
  /* the worklist, processed in arrival order */
  for (uint64_t h = 0; h < w->queue.n && !w->oom; h += 4) {
    const uint32_t k = w->queue.a[h], u = w->queue.a[h + 1], v = w->queue.a[h + 2], t = w->queue.a[h + 3];
    if (k == EV_FACT)
      on_fact(w, u, v);
    else if (k == EV_LINK)
      on_link(w, u, v, t);
    else
      on_act(w, u, v);
  }
  free(w->queue.a);
  w->queue.a = NULL;
  /* report: the given concepts only (fresh range fillers are internal) */
  for (uint32_t x = 0; x < w->N_out; ++x) {
    uint64_t keep = 0;
    for (uint64_t j = 0; j < w->srow[x].n; ++j)
      if (w->srow[x].a[j] < w->N_out) w->srow[x].a[keep++] = w->srow[x].a[j];
    w->srow[x].n = keep;
    qsort(w->srow[x].a, w->srow[x].n, sizeof(uint32_t), cmp_u32);
    w->n_facts += keep;
    /* links (r, y) of x, sorted (a fresh filler F keeps its id, as the engine reports it) */
    qsort(w->out[x].a, w->out[x].n / 2, 2 * sizeof(uint32_t), cmp_pair);
    w->n_links += w->out[x].n / 2;
  }
  return w->oom ? -1 : 0;
}

uint64_t wl_num_facts(const wl_result* w) { return w->n_facts; }
uint64_t wl_num_links(const wl_result* w) { return w->n_links; }

void wl_copy_facts(const wl_result* w, uint32_t* x, uint32_t* a) {
  uint64_t k = 0;
  for (uint32_t i = 0; i < w->N_out; ++i)
    for (uint64_t j = 0; j < w->srow[i].n; ++j, ++k) {
      x[k] = i;
      a[k] = w->srow[i].a[j];
    }
}

void wl_copy_links(const wl_result* w, uint32_t* x, uint32_t* r, uint32_t* y) {
  uint64_t k = 0;
  for (uint32_t i = 0; i < w->N_out; ++i)
    for (uint64_t j = 0; j < w->out[i].n; j += 2, ++k) {
      x[k] = i;
      r[k] = w->out[i].a[j];
      y[k] = w->out[i].a[j + 1];
    }
}

void wl_free(wl_result* w) {
  if (!w) return;
  for (int i = 0; i < 4; ++i) free(w->owned[i]);
  vec* lists[] = {w->srow, w->sinv, w->out, w->in, w->acts};
  for (int l = 0; l < 5; ++l) {
    if (!lists[l]) continue;
    for (uint32_t i = 0; i < w->N; ++i) free(lists[l][i].a);
    free(lists[l]);
  }
  multimap* mms[] = {&w->subA, &w->conjOp, &w->exrA, &w->exlA, &w->exlR, &w->subR, &w->chF, &w->chS, &w->domR, &w->rngR};
  for (int m = 0; m < 10; ++m) mm_free(mms[m]);
  free(w->sset.k);
  free(w->lset.k);
  free(w->aset.k);
  free(w->queue.a);
  free(w->rng_ptr);
  free(w->rng_all);
  free((void*)w->ax);
  free(w);
}
