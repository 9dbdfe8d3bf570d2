/*
 * cbquery.c -- C restatement of bquery's per-shard groupby -- TEST INFRASTRUCTURE ONLY.
 *
 * Used (a) by tests/ as a fast second oracle that must agree bit-for-bit with the numpy
 * restatement in bquery_oracle.py, and (b) by bench.py's cpu_baseline leg as the timed
 * CPU port of the reference algorithm.  Never linked into, or called by, bqueryd_amd.
 *
 * Structure mirrors what the reference worker runs per shard:
 *   worker.py:303  ct.where_terms(...)      -> materialised uint8 row mask       (pass 1)
 *   worker.py:313  ct.groupby(...):
 *        factorize_groupby_cols             -> khash per key column, int64 labels (pass 2)
 *        create_group_column_factor         -> combine + re-factorize (multi-key)  (pass 3)
 *        '(factor + 1) * bool - 1' + refactorize when filtered (skip_key)          (pass 4)
 *        aggregate_groups: groupby_value per key, one pass per aggregation         (pass 5..)
 * All of that is [ext-bquery, unverified] (bquery is absent); semantics
 * are identical to oracle/bquery_oracle.py, which is the readable statement.
 * Single-threaded, like a bqueryd worker (bcolz.set_nthreads(1), worker.py:40).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { DT_BOOL = 0, DT_I8, DT_I16, DT_I32, DT_I64, DT_U8, DT_U16, DT_U32, DT_U64, DT_F32, DT_F64 };
enum { AG_SUM = 0, AG_COUNT, AG_COUNT_DISTINCT, AG_SORTED_COUNT_DISTINCT, AG_MEAN, AG_STD };
/* term ops after normalisation: 1..8 as bquery, 0 = always true, -1 = always false */
enum { T_FALSE = -1, T_TRUE = 0, T_EQ = 1, T_NE, T_IN, T_NIN, T_GT, T_GE, T_LT, T_LE };

typedef struct {
  int32_t col;
  int32_t op;
  int32_t nvals;
  int32_t is_float; /* compare as double (float columns) else as int64 */
  const int64_t* ivals;
  const double* fvals;
} cbq_term;

static int is_float_dt(int dt) { return dt == DT_F32 || dt == DT_F64; }
static int is_unsigned_dt(int dt) { return dt >= DT_U8 && dt <= DT_U64; }

static inline int64_t get_i(const void* p, int dt, int64_t i) {
  switch (dt) {
    case DT_BOOL: case DT_U8: return ((const uint8_t*)p)[i];
    case DT_I8: return ((const int8_t*)p)[i];
    case DT_I16: return ((const int16_t*)p)[i];
    case DT_U16: return ((const uint16_t*)p)[i];
    case DT_I32: return ((const int32_t*)p)[i];
    case DT_U32: return ((const uint32_t*)p)[i];
    case DT_I64: return ((const int64_t*)p)[i];
    case DT_U64: return (int64_t)((const uint64_t*)p)[i];
    case DT_F32: return (int64_t)((const float*)p)[i];
    default: return (int64_t)((const double*)p)[i];
  }
}
static inline double get_f(const void* p, int dt, int64_t i) {
  switch (dt) {
    case DT_F32: return (double)((const float*)p)[i];
    case DT_F64: return ((const double*)p)[i];
    case DT_U64: return (double)((const uint64_t*)p)[i];
    default: return (double)get_i(p, dt, i);
  }
}
/* canonical 64-bit identity of a value: khash equality (NaN==NaN, -0.0==0.0) */
static inline uint64_t get_bits(const void* p, int dt, int64_t i) {
  if (is_float_dt(dt)) {
    double d = get_f(p, dt, i);
    uint64_t u;
    if (d != d) return 0x7ff8000000000000ull;
    d += 0.0;
    memcpy(&u, &d, 8);
    return u;
  }
  return (uint64_t)get_i(p, dt, i);
}

/* ---------------- open-addressing hash map uint64 -> int64 (khash stand-in) -------------- */
typedef struct {
  uint64_t* keys;
  int64_t* vals;
  uint8_t* used;
  int64_t cap, size;
} hmap;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
static void hm_init(hmap* h, int64_t cap) {
  int64_t c = 16;
  while (c < cap * 2) c <<= 1;
  h->cap = c; h->size = 0;
  h->keys = (uint64_t*)malloc(c * 8); h->vals = (int64_t*)malloc(c * 8); h->used = (uint8_t*)calloc(c, 1);
}
static void hm_free(hmap* h) { free(h->keys); free(h->vals); free(h->used); }
static void hm_grow(hmap* h);
/* returns value; inserts (key -> *next_label) if absent and bumps *next_label */
static inline int64_t hm_get_or_insert(hmap* h, uint64_t key, int64_t* next_label) {
  uint64_t m = (uint64_t)h->cap - 1, pos = mix64(key) & m;
  while (h->used[pos]) {
    if (h->keys[pos] == key) return h->vals[pos];
    pos = (pos + 1) & m;
  }
  h->used[pos] = 1; h->keys[pos] = key; h->vals[pos] = (*next_label)++;
  if (++h->size * 2 > h->cap) hm_grow(h);
  return *next_label - 1;
}
static void hm_grow(hmap* h) {
  hmap n; int64_t i;
  hm_init(&n, h->cap);
  for (i = 0; i < h->cap; i++)
    if (h->used[i]) {
      uint64_t m = (uint64_t)n.cap - 1, pos = mix64(h->keys[i]) & m;
      while (n.used[pos]) pos = (pos + 1) & m;
      n.used[pos] = 1; n.keys[pos] = h->keys[i]; n.vals[pos] = h->vals[i]; n.size++;
    }
  hm_free(h); *h = n;
}

/* ---------------- pass 1: where_terms ---------------- */
static int term_hit(const cbq_term* t, const void* col, int dt, int64_t i) {
  int k;
  if (t->op == T_TRUE) return 1;
  if (t->op == T_FALSE) return 0;
  if (t->is_float) {
    double x = get_f(col, dt, i);
    switch (t->op) {
      case T_EQ: return x == t->fvals[0];
      case T_NE: return x != t->fvals[0];
      case T_GT: return x > t->fvals[0];
      case T_GE: return x >= t->fvals[0];
      case T_LT: return x < t->fvals[0];
      case T_LE: return x <= t->fvals[0];
      case T_IN: case T_NIN:
        for (k = 0; k < t->nvals; k++) if (x == t->fvals[k]) return t->op == T_IN;
        return t->op == T_NIN;
    }
  } else if (dt == DT_U64) {
    uint64_t x = (uint64_t)get_i(col, dt, i);
    const uint64_t* v = (const uint64_t*)t->ivals;
    switch (t->op) {
      case T_EQ: return x == v[0];
      case T_NE: return x != v[0];
      case T_GT: return x > v[0];
      case T_GE: return x >= v[0];
      case T_LT: return x < v[0];
      case T_LE: return x <= v[0];
      case T_IN: case T_NIN:
        for (k = 0; k < t->nvals; k++) if (x == v[k]) return t->op == T_IN;
        return t->op == T_NIN;
    }
  } else {
    int64_t x = get_i(col, dt, i);
    switch (t->op) {
      case T_EQ: return x == t->ivals[0];
      case T_NE: return x != t->ivals[0];
      case T_GT: return x > t->ivals[0];
      case T_GE: return x >= t->ivals[0];
      case T_LT: return x < t->ivals[0];
      case T_LE: return x <= t->ivals[0];
      case T_IN: case T_NIN:
        for (k = 0; k < t->nvals; k++) if (x == t->ivals[k]) return t->op == T_IN;
        return t->op == T_NIN;
    }
  }
  return 0;
}

int64_t cbq_where(int64_t n, const void** cols, const int* dtypes, int nterms,
                  const cbq_term* terms, uint8_t* mask) {
  int64_t i, npass = 0;
  int t;
  for (i = 0; i < n; i++) mask[i] = 1;
  for (t = 0; t < nterms; t++) {
    const cbq_term* tm = &terms[t];
    const void* col = cols[tm->col];
    int dt = dtypes[tm->col];
    if (tm->op == T_GE && !tm->is_float && dt == DT_I32) { /* typed fast loop */
      const int32_t* c = (const int32_t*)col;
      int64_t v = tm->ivals[0];
      for (i = 0; i < n; i++) mask[i] &= (uint8_t)((int64_t)c[i] >= v);
    } else {
      for (i = 0; i < n; i++)
        if (mask[i]) mask[i] = (uint8_t)term_hit(tm, col, dt, i);
    }
  }
  for (i = 0; i < n; i++) npass += mask[i];
  return npass;
}

/* ---------------- pass 2..4: factorisation ---------------- */
/* labels in first-appearance order; returns number of uniques; uniq_rows[k] = first row */
static int64_t factorize_bits(int64_t n, const void* col, int dt, int64_t* labels, int64_t** first_rows) {
  hmap h; int64_t i, next = 0, cap = 1024;
  int64_t* fr = (int64_t*)malloc(sizeof(int64_t) * cap);
  hm_init(&h, 1024);
  if (dt == DT_I32) {
    const int32_t* c = (const int32_t*)col;
    for (i = 0; i < n; i++) {
      int64_t before = next, l = hm_get_or_insert(&h, (uint64_t)(int64_t)c[i], &next);
      if (next != before) { if (l >= cap) { cap *= 2; fr = (int64_t*)realloc(fr, sizeof(int64_t) * cap); } fr[l] = i; }
      labels[i] = l;
    }
  } else {
    for (i = 0; i < n; i++) {
      int64_t before = next, l = hm_get_or_insert(&h, get_bits(col, dt, i), &next);
      if (next != before) { if (l >= cap) { cap *= 2; fr = (int64_t*)realloc(fr, sizeof(int64_t) * cap); } fr[l] = i; }
      labels[i] = l;
    }
  }
  hm_free(&h);
  *first_rows = fr;
  return next;
}
static int64_t refactorize(int64_t n, int64_t* labels, int64_t** first_rows) {
  return factorize_bits(n, labels, DT_I64, labels, first_rows);
}

/* ---------------- result ---------------- */
typedef struct {
  int64_t n_groups;
  int64_t* group_rows;   /* for each output group, one row index holding its keys (last row) */
  void** agg_out;        /* per agg: int64_t[] or double[] or input-dtype array (sum) */
} cbq_result;

static int itemsize(int dt) {
  switch (dt) {
    case DT_BOOL: case DT_I8: case DT_U8: return 1;
    case DT_I16: case DT_U16: return 2;
    case DT_I32: case DT_U32: case DT_F32: return 4;
    default: return 8;
  }
}

static void store_wrapped(void* out, int dt, int64_t g, int64_t v) {
  switch (dt) {
    case DT_I8: ((int8_t*)out)[g] = (int8_t)v; break;
    case DT_U8: case DT_BOOL: ((uint8_t*)out)[g] = (uint8_t)v; break;
    case DT_I16: ((int16_t*)out)[g] = (int16_t)v; break;
    case DT_U16: ((uint16_t*)out)[g] = (uint16_t)v; break;
    case DT_I32: ((int32_t*)out)[g] = (int32_t)v; break;
    case DT_U32: ((uint32_t*)out)[g] = (uint32_t)v; break;
    default: ((int64_t*)out)[g] = v; break;
  }
}

/*
 * Full per-shard groupby.  mask may be NULL (no where terms).  Output arrays are malloc'ed
 * (free with cbq_free_result); groups are in bquery order with the skip slot deleted.
 */
int cbq_groupby(int64_t n, const void** cols, const int* dtypes, int nkeys, const int* keys,
                const uint8_t* mask, int naggs, const int* agg_cols, const int* agg_ops,
                cbq_result* res) {
  int64_t i, g, nr_groups, skip_key, *factor, *fr = NULL;
  int k, a, filtered = 0;
  memset(res, 0, sizeof(*res));
  factor = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  if (nkeys == 0) {
    for (i = 0; i < n; i++) factor[i] = 0;
    nr_groups = 1;
  } else {
    nr_groups = factorize_bits(n, cols[keys[0]], dtypes[keys[0]], factor, &fr);
    free(fr); fr = NULL;
    if (nkeys > 1) {
      int64_t* lab = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
      for (k = 1; k < nkeys; k++) {
        int64_t nu = factorize_bits(n, cols[keys[k]], dtypes[keys[k]], lab, &fr);
        free(fr); fr = NULL;
        for (i = 0; i < n; i++) factor[i] = factor[i] * nu + lab[i]; /* create_group_index */
        nr_groups = refactorize(n, factor, &fr);                       /* re-factorize */
        free(fr); fr = NULL;
      }
      free(lab);
    }
  }
  skip_key = -1;
  if (mask) {
    for (i = 0; i < n; i++) { if (!mask[i]) { filtered = 1; break; } }
    for (i = 0; i < n; i++) factor[i] = (factor[i] + 1) * (int64_t)mask[i] - 1;
    nr_groups = refactorize(n, factor, &fr);
    for (g = 0; g < nr_groups; g++) {
      /* the label whose first row is a filtered row is the skip slot */
      if (!mask[fr[g]]) { skip_key = g; break; }
    }
    free(fr); fr = NULL;
  }
  if (skip_key < 0) skip_key = nr_groups;

  /* groupby_value: one representative (last written) row per slot */
  {
    int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (nr_groups ? nr_groups : 1));
    int64_t o = 0;
    for (g = 0; g < nr_groups; g++) rows[g] = -1;
    for (i = 0; i < n; i++) if (factor[i] != skip_key) rows[factor[i]] = i;
    res->n_groups = filtered ? nr_groups - 1 : nr_groups;
    if (res->n_groups < 0) res->n_groups = 0;
    res->group_rows = (int64_t*)malloc(sizeof(int64_t) * (res->n_groups ? res->n_groups : 1));
    for (g = 0; g < nr_groups; g++) {
      if (filtered && g == skip_key) continue;
      res->group_rows[o++] = rows[g];
    }
    free(rows);
  }

  res->agg_out = (void**)calloc(naggs ? naggs : 1, sizeof(void*));
  for (a = 0; a < naggs; a++) {
    const void* col = cols[agg_cols[a]];
    int dt = dtypes[agg_cols[a]], op = agg_ops[a];
    int64_t ng = nr_groups ? nr_groups : 1;
    void* out = NULL;
    if (op == AG_SUM) {
      if (is_float_dt(dt)) {
        if (dt == DT_F64) {
          const double* c = (const double*)col;
          double* o = (double*)calloc(ng, 8);
          for (i = 0; i < n; i++) if (factor[i] != skip_key) o[factor[i]] += c[i];
          out = o;
        } else {
          const float* c = (const float*)col;
          float* o = (float*)calloc(ng, 4);
          for (i = 0; i < n; i++) if (factor[i] != skip_key) o[factor[i]] += c[i];
          out = o;
        }
      } else {
        int64_t* acc = (int64_t*)calloc(ng, 8);
        out = calloc(ng, itemsize(dt));
        for (i = 0; i < n; i++) if (factor[i] != skip_key) acc[factor[i]] += get_i(col, dt, i);
        for (g = 0; g < nr_groups; g++) store_wrapped(out, dt, g, acc[g]);
        free(acc);
      }
    } else if (op == AG_COUNT) {
      int64_t* o = (int64_t*)calloc(ng, 8);
      for (i = 0; i < n; i++) if (factor[i] != skip_key) o[factor[i]] += 1;
      out = o;
    } else if (op == AG_MEAN) {
      double* o = (double*)calloc(ng, 8);
      int64_t* c = (int64_t*)calloc(ng, 8);
      for (i = 0; i < n; i++) {
        int64_t f = factor[i];
        if (f == skip_key) continue;
        c[f] += 1;
        o[f] += (get_f(col, dt, i) - o[f]) / (double)c[f];
      }
      free(c);
      out = o;
    } else if (op == AG_STD) {
      double* o = (double*)calloc(ng, 8);
      double* m = (double*)calloc(ng, 8);
      int64_t* c = (int64_t*)calloc(ng, 8);
      for (i = 0; i < n; i++) {
        int64_t f = factor[i];
        double x, d;
        if (f == skip_key) continue;
        x = get_f(col, dt, i);
        c[f] += 1;
        d = x - m[f];
        m[f] += d / (double)c[f];
        o[f] += d * (x - m[f]);
      }
      for (g = 0; g < nr_groups; g++) o[g] = c[g] ? sqrt(o[g] / (double)c[g]) : NAN;
      free(m); free(c);
      out = o;
    } else if (op == AG_COUNT_DISTINCT) {
      /* exact (group, value) pair set, open addressing on two 64-bit words */
      int64_t* o = (int64_t*)calloc(ng, 8);
      int64_t cap = 1024, size = 0;
      uint64_t* kg = (uint64_t*)malloc(cap * 8);
      uint64_t* kv = (uint64_t*)malloc(cap * 8);
      uint8_t* used = (uint8_t*)calloc(cap, 1);
      for (i = 0; i < n; i++) {
        int64_t f = factor[i];
        uint64_t v, m, pos;
        if (f == skip_key) continue;
        v = get_bits(col, dt, i);
        m = (uint64_t)cap - 1;
        pos = mix64(v ^ mix64((uint64_t)f)) & m;
        while (used[pos] && !(kg[pos] == (uint64_t)f && kv[pos] == v)) pos = (pos + 1) & m;
        if (used[pos]) continue;
        used[pos] = 1; kg[pos] = (uint64_t)f; kv[pos] = v; o[f] += 1;
        if (++size * 2 > cap) {
          int64_t nc = cap * 2, j;
          uint64_t* ng_ = (uint64_t*)malloc(nc * 8);
          uint64_t* nv = (uint64_t*)malloc(nc * 8);
          uint8_t* nu = (uint8_t*)calloc(nc, 1);
          for (j = 0; j < cap; j++) if (used[j]) {
            uint64_t q = mix64(kv[j] ^ mix64(kg[j])) & (uint64_t)(nc - 1);
            while (nu[q]) q = (q + 1) & (uint64_t)(nc - 1);
            nu[q] = 1; ng_[q] = kg[j]; nv[q] = kv[j];
          }
          free(kg); free(kv); free(used);
          kg = ng_; kv = nv; used = nu; cap = nc;
        }
      }
      free(kg); free(kv); free(used);
      out = o;
    } else if (op == AG_SORTED_COUNT_DISTINCT) {
      int64_t* o = (int64_t*)calloc(ng, 8);
      int first = 1;
      if (is_float_dt(dt)) {
        double* last = (double*)calloc(ng, 8);
        for (i = 0; i < n; i++) {
          int64_t f = factor[i];
          double x;
          if (f == skip_key) continue;
          x = get_f(col, dt, i);
          if (first) { last[0] = x; o[0] = 1; first = 0; }
          else if (x != last[f]) o[f] += 1;
          last[f] = x;
        }
        free(last);
      } else {
        int64_t* last = (int64_t*)calloc(ng, 8);
        for (i = 0; i < n; i++) {
          int64_t f = factor[i], x;
          if (f == skip_key) continue;
          x = get_i(col, dt, i);
          if (first) { last[0] = x; o[0] = 1; first = 0; }
          else if (x != last[f]) o[f] += 1;
          last[f] = x;
        }
        free(last);
      }
      out = o;
    } else {
      free(factor);
      return -1;
    }
    /* delete the skip slot (np.delete) */
    if (filtered && skip_key < nr_groups) {
      int sz = (op == AG_SUM) ? itemsize(dt) : 8;
      char* b = (char*)out;
      memmove(b + skip_key * sz, b + (skip_key + 1) * sz, (size_t)(nr_groups - skip_key - 1) * sz);
    }
    res->agg_out[a] = out;
  }
  free(factor);
  return 0;
}

void cbq_free_result(cbq_result* res, int naggs) {
  int a;
  free(res->group_rows);
  if (res->agg_out) {
    for (a = 0; a < naggs; a++) free(res->agg_out[a]);
    free(res->agg_out);
  }
  memset(res, 0, sizeof(*res));
}
