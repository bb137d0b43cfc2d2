/*
 * gloo_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference (liuxiaotiao/gloo @ /root/reference)
 * semantics for the allreduce hot path.  It is the CHECKER for the HIP path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  Nothing in the product (gloo_amd/) links, loads or calls this file.
 *
 * Parity pin: validated bit-for-bit against (a) oracle/_ref -- the reference's
 * own gloo/math.h + gloo/types.h + AllreduceRingChunked / AllreduceHalvingDoubling
 * compiled from /root/reference sources by oracle/Makefile -- through the
 * committed fixtures in tests/golden/ (generator: tests/golden/make_golden.py),
 * and (b) the reference test KATs (gloo/test/allreduce_test.cc:143-269,
 * gloo/test/math_test.cc:55-143, gloo/test/base_test.h:184-235).
 * bf16 has no reference counterpart: "parity unpinned" (restated as fp32 op +
 * round-to-nearest-even per hop, NaN -> 0x7fff, mirroring the fp16 rule).
 *
 * What is restated (each function cites the reference line it follows):
 *   - element ops sum/product/max/min            gloo/math.h:15-73
 *   - float16 <-> float conversions               gloo/types.h:248-339
 *   - float16 arithmetic (convert, op, round)     gloo/types.h:181-204
 *   - allreduce_ring_chunked data flow            gloo/allreduce_ring_chunked.h:22-236
 *   - allreduce_halving_doubling data flow        gloo/allreduce_halving_doubling.h:37-361
 *
 * The collectives are simulated as per-rank programs of SEND / RECV / REDUCE /
 * COPY steps over FIFO channels (one per ordered rank pair and slot), which is
 * exactly the contract gloo's transport gives the algorithm: a message lands
 * at the start of the receiver's registered buffer before waitRecv() returns.
 * Flow-control notifications carry no data and are not modelled.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { OR_INT8 = 0, OR_UINT8, OR_INT32, OR_INT64, OR_UINT64, OR_FLOAT32,
       OR_FLOAT64, OR_FLOAT16, OR_BFLOAT16, OR_NDTYPES };
enum { OR_SUM = 1, OR_PRODUCT = 2, OR_MAX = 3, OR_MIN = 4 };

static const size_t kSize[OR_NDTYPES] = {1, 1, 4, 8, 8, 4, 8, 2, 2};

size_t oracle_dtype_size(int dtype) {
  return (dtype >= 0 && dtype < OR_NDTYPES) ? kSize[dtype] : 0;
}

/* ------------------------------------------------------------------ */
/* float16 (IEEE binary16) conversions.                                */
/* ------------------------------------------------------------------ */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* float -> half, round to nearest even.  Follows the contract of
 * cpu_float2half_rn (gloo/types.h:248-305): any NaN becomes 0x7fff (sign
 * dropped), overflow becomes +-inf, everything else is IEEE RNE including
 * subnormal results.  Written as "scale the significand into the half grid,
 * then add-half-ulp with ties-to-even" rather than the reference's
 * shift/remainder form. */
uint16_t oracle_f32_to_f16(float f) {
  uint32_t x = f2u(f);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t mag = x & 0x7fffffffu;
  if (mag > 0x7f800000u) return 0x7fffu;              /* NaN */
  if (mag >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520 -> inf */
  int32_t e = (int32_t)(mag >> 23) - 127;             /* unbiased exponent */
  uint32_t sig = (mag & 0x7fffffu) | (mag >= 0x00800000u ? 0x800000u : 0u);
  if (mag < 0x00800000u) e = -126;                    /* f32 subnormal */
  if (sig == 0) return (uint16_t)sign;
  /* value = sig * 2^(e-23).  Half grid unit: 2^-24 for subnormals,
   * 2^(e-10) for normals (e >= -14). */
  int32_t unit_exp = (e >= -14) ? (e - 10) : -24;
  int32_t drop = unit_exp - (e - 23);                 /* bits to drop, >= 13 */
  uint64_t q, rem, half;
  if (drop >= 64) return (uint16_t)sign;
  q = (uint64_t)sig >> drop;
  rem = (uint64_t)sig & (((uint64_t)1 << drop) - 1);
  half = (uint64_t)1 << (drop - 1);
  if (rem > half || (rem == half && (q & 1))) q += 1;
  /* q is the significand in units of 2^unit_exp */
  if (e >= -14) {
    /* normal: q in [1024, 2048]; carry may bump the exponent */
    uint32_t hexp = (uint32_t)(e + 15);
    if (q == 2048) { q = 1024; hexp += 1; }
    if (hexp >= 31) return (uint16_t)(sign | 0x7c00u);
    return (uint16_t)(sign | (hexp << 10) | (uint32_t)(q - 1024));
  }
  /* subnormal half: q in [0, 1024]; q == 1024 is the smallest normal */
  return (uint16_t)(sign | (uint32_t)q);
}

/* half -> float, exact.  Follows cpu_half2float (gloo/types.h:307-339):
 * NaN inputs become 0x7fffffff (positive, all-ones payload). */
float oracle_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu;
  uint32_t m = h & 0x3ffu;
  if (e == 0x1f) return m ? u2f(0x7fffffffu) : u2f(sign | 0x7f800000u);
  if (e == 0) {
    /* subnormal or zero: m * 2^-24 is exact in float */
    float v = (float)m * 5.9604644775390625e-08f;
    return (sign ? -v : v);
  }
  return u2f(sign | ((e + 112u) << 23) | (m << 13));
}

/* bf16: no reference (parity unpinned).  fp32 -> bf16 round-nearest-even,
 * NaN -> 0x7fff (mirrors the float16 NaN rule above). */
uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fffu;
  uint32_t lsb = (u >> 16) & 1u;
  return (uint16_t)((u + 0x7fffu + lsb) >> 16);
}

float oracle_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

void oracle_f32_to_f16_n(const float* in, uint16_t* out, size_t n) {
  size_t i;
  for (i = 0; i < n; i++) out[i] = oracle_f32_to_f16(in[i]);
}

void oracle_f16_to_f32_n(const uint16_t* in, float* out, size_t n) {
  size_t i;
  for (i = 0; i < n; i++) out[i] = oracle_f16_to_f32(in[i]);
}

void oracle_f32_to_bf16_n(const float* in, uint16_t* out, size_t n) {
  size_t i;
  for (i = 0; i < n; i++) out[i] = oracle_f32_to_bf16(in[i]);
}

/* ------------------------------------------------------------------ */
/* Element ops: c = op(a, b).  gloo/math.h:15-73.                      */
/* max(a,b) is std::max: (a < b) ? b : a  -- returns a's bits unless   */
/* a < b, so NaN / signed-zero behaviour is operand-order dependent.   */
/* ------------------------------------------------------------------ */

#define DEF_INT_OPS(NAME, T, UT)                                               \
  static void NAME(int op, T* c, const T* a, const T* b, size_t n) {           \
    size_t i;                                                                  \
    switch (op) {                                                              \
      case OR_SUM:                                                             \
        for (i = 0; i < n; i++) c[i] = (T)((UT)a[i] + (UT)b[i]);               \
        break;                                                                 \
      case OR_PRODUCT:                                                         \
        for (i = 0; i < n; i++) c[i] = (T)((UT)a[i] * (UT)b[i]);               \
        break;                                                                 \
      case OR_MAX:                                                             \
        for (i = 0; i < n; i++) c[i] = (a[i] < b[i]) ? b[i] : a[i];            \
        break;                                                                 \
      case OR_MIN:                                                             \
        for (i = 0; i < n; i++) c[i] = (b[i] < a[i]) ? b[i] : a[i];            \
        break;                                                                 \
    }                                                                          \
  }

DEF_INT_OPS(ops_i8, int8_t, uint32_t)
DEF_INT_OPS(ops_u8, uint8_t, uint32_t)
DEF_INT_OPS(ops_i32, int32_t, uint32_t)
DEF_INT_OPS(ops_i64, int64_t, uint64_t)
DEF_INT_OPS(ops_u64, uint64_t, uint64_t)

#define DEF_FP_OPS(NAME, T)                                                    \
  static void NAME(int op, T* c, const T* a, const T* b, size_t n) {           \
    size_t i;                                                                  \
    switch (op) {                                                              \
      case OR_SUM:                                                             \
        for (i = 0; i < n; i++) c[i] = a[i] + b[i];                            \
        break;                                                                 \
      case OR_PRODUCT:                                                         \
        for (i = 0; i < n; i++) c[i] = a[i] * b[i];                            \
        break;                                                                 \
      case OR_MAX:                                                             \
        for (i = 0; i < n; i++) c[i] = (a[i] < b[i]) ? b[i] : a[i];            \
        break;                                                                 \
      case OR_MIN:                                                             \
        for (i = 0; i < n; i++) c[i] = (b[i] < a[i]) ? b[i] : a[i];            \
        break;                                                                 \
    }                                                                          \
  }

DEF_FP_OPS(ops_f32, float)
DEF_FP_OPS(ops_f64, double)

/* 16-bit floats: widen, op in fp32, round once per call (per hop).
 * gloo/types.h:181-204 (operator+= etc.) and :318-336 (comparisons in fp32,
 * std::max/min return the original 16-bit object untouched).
 *
 * float16 only -- the reference's assignment quirk, restated exactly:
 * float16::operator=(const float16& rhs) (gloo/types.h:129-134) stores only
 * `if (rhs != *this)`, and operator!= (:140-142) compares `*this == rhs.x`,
 * which resolves to operator==(const int&) (:144-147): the bits of the old
 * value are read as an INTEGER and rounded to half.  So an assignment
 * old = v is skipped exactly when v.x == f2h((float)old.x).x.  It fires
 * twice per sum/product (inside operator+= on the copy of the left operand,
 * then for c[i] = ...) and once per max/min (c[i] = std::max(...)).  c's
 * previous contents therefore matter; in place (c == a) it is a's value. */
static inline uint16_t f16_assign(uint16_t old, uint16_t v) {
  return (v == oracle_f32_to_f16((float)old)) ? old : v;
}

static void ops_h16(int op, uint16_t* c, const uint16_t* a, const uint16_t* b,
                    size_t n, int is_bf16) {
  size_t i;
  for (i = 0; i < n; i++) {
    float x = is_bf16 ? oracle_bf16_to_f32(a[i]) : oracle_f16_to_f32(a[i]);
    float y = is_bf16 ? oracle_bf16_to_f32(b[i]) : oracle_f16_to_f32(b[i]);
    uint16_t old = c[i], ai = a[i], bi = b[i], v;
    switch (op) {
      case OR_SUM:
      case OR_PRODUCT: {
        float r = (op == OR_SUM) ? x + y : x * y;
        if (is_bf16) {
          v = oracle_f32_to_bf16(r);
        } else {
          v = f16_assign(ai, oracle_f32_to_f16(r)); /* inside operator+= / *= */
          v = f16_assign(old, v);                   /* c[i] = ... */
        }
        break;
      }
      case OR_MAX:
        v = (x < y) ? bi : ai;
        if (!is_bf16) v = f16_assign(old, v);
        break;
      default: /* OR_MIN */
        v = (y < x) ? bi : ai;
        if (!is_bf16) v = f16_assign(old, v);
        break;
    }
    c[i] = v;
  }
}

/* c = op(a, b) elementwise; c may alias a or b.  Returns 0 or -1. */
int oracle_reduce(int op, int dtype, void* c, const void* a, const void* b,
                  size_t n) {
  if (op < OR_SUM || op > OR_MIN) return -1;
  switch (dtype) {
    case OR_INT8: ops_i8(op, c, a, b, n); break;
    case OR_UINT8: ops_u8(op, c, a, b, n); break;
    case OR_INT32: ops_i32(op, c, a, b, n); break;
    case OR_INT64: ops_i64(op, c, a, b, n); break;
    case OR_UINT64: ops_u64(op, c, a, b, n); break;
    case OR_FLOAT32: ops_f32(op, c, a, b, n); break;
    case OR_FLOAT64: ops_f64(op, c, a, b, n); break;
    case OR_FLOAT16: ops_h16(op, c, a, b, n, 0); break;
    case OR_BFLOAT16: ops_h16(op, c, a, b, n, 1); break;
    default: return -1;
  }
  return 0;
}

/* Scalar fp32 sum exactly as the reference's hot loop is written
 * (gloo/math.h:15-23): the cpu_baseline "port" leg of bench.py times this. */
void oracle_sum_f32(float* c, const float* a, const float* b, size_t n) {
  size_t i;
  for (i = 0; i < n; i++) c[i] = a[i] + b[i];
}

/* ------------------------------------------------------------------ */
/* Synthetic inputs.                            */
/* ------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* kind 0: hashed values  x = ((h >> 40) - 2^23) / 2^23 in [-1, 1)
 *         (ints: h masked to +-2^20; 16-bit floats: the fp32 value rounded)
 * kind 1: reference stride pattern  j*stride + val  (gloo/test/base_test.h:184-191)
 * kind 2: constant val (gloo/test/allreduce_test.cc:156-158: ptr[i] = rank) */
void oracle_fill(int dtype, int kind, uint64_t seed, int rank, int ptr_index,
                 int stride, int val, size_t n, void* out) {
  size_t j;
  for (j = 0; j < n; j++) {
    double v;
    int64_t iv;
    if (kind == 0) {
      uint64_t h = splitmix64(seed ^ ((uint64_t)rank << 40) ^
                              ((uint64_t)ptr_index << 56) ^ (uint64_t)j);
      v = ((double)(int64_t)(h >> 40) - 8388608.0) / 8388608.0;
      iv = (int64_t)((h >> 20) & 0x1fffff) - 0x100000;
    } else if (kind == 1) {
      iv = (int64_t)j * stride + val;
      v = (double)iv;
    } else {
      iv = val;
      v = (double)val;
    }
    switch (dtype) {
      case OR_INT8: ((int8_t*)out)[j] = (int8_t)iv; break;
      case OR_UINT8: ((uint8_t*)out)[j] = (uint8_t)iv; break;
      case OR_INT32: ((int32_t*)out)[j] = (int32_t)iv; break;
      case OR_INT64: ((int64_t*)out)[j] = (int64_t)iv; break;
      case OR_UINT64: ((uint64_t*)out)[j] = (uint64_t)iv; break;
      case OR_FLOAT32: ((float*)out)[j] = (float)v; break;
      case OR_FLOAT64: ((double*)out)[j] = v; break;
      case OR_FLOAT16: ((uint16_t*)out)[j] = oracle_f32_to_f16((float)v); break;
      case OR_BFLOAT16: ((uint16_t*)out)[j] = oracle_f32_to_bf16((float)v); break;
    }
  }
}

/* ------------------------------------------------------------------ */
/* Message-passing simulator for the collectives.                     */
/* ------------------------------------------------------------------ */

enum { ST_SEND = 0, ST_RECV, ST_REDUCE, ST_COPY, ST_LOCAL, ST_BCAST };
/* ST_LOCAL / ST_BCAST (function-style allreduce only): the reference's
 * reduceInputs / broadcastOutputs for [off, off+len) of this rank. */

typedef struct {
  int kind;
  int peer;        /* SEND/RECV */
  int tag;         /* SEND/RECV: slot distinguishing channels of one pair */
  size_t off;      /* SEND: source offset in ptr0; REDUCE/COPY: dst offset in ptr0 */
  size_t len;      /* elements */
  size_t boff;     /* RECV: where the message lands in the rank's scratch;
                      REDUCE/COPY: source offset in scratch */
} step_t;

typedef struct {
  step_t* v;
  size_t n, cap;
} prog_t;

static int prog_push(prog_t* p, step_t s) {
  if (p->n == p->cap) {
    size_t cap = p->cap ? p->cap * 2 : 64;
    step_t* nv = (step_t*)realloc(p->v, cap * sizeof(step_t));
    if (!nv) return -1;
    p->v = nv;
    p->cap = cap;
  }
  p->v[p->n++] = s;
  return 0;
}

typedef struct msg {
  struct msg* next;
  size_t len;
  unsigned char data[];
} msg_t;

typedef struct {
  int src, dst, tag;
  msg_t *head, *tail;
} chan_t;

typedef struct {
  chan_t* v;
  size_t n, cap;
} chans_t;

static chan_t* chan_get(chans_t* cs, int src, int dst, int tag) {
  size_t i;
  for (i = 0; i < cs->n; i++)
    if (cs->v[i].src == src && cs->v[i].dst == dst && cs->v[i].tag == tag)
      return &cs->v[i];
  if (cs->n == cs->cap) {
    size_t cap = cs->cap ? cs->cap * 2 : 32;
    chan_t* nv = (chan_t*)realloc(cs->v, cap * sizeof(chan_t));
    if (!nv) return NULL;
    cs->v = nv;
    cs->cap = cap;
  }
  cs->v[cs->n].src = src;
  cs->v[cs->n].dst = dst;
  cs->v[cs->n].tag = tag;
  cs->v[cs->n].head = cs->v[cs->n].tail = NULL;
  return &cs->v[cs->n++];
}

/* Per-rank input/output buffers of the function-style allreduce. */
typedef struct {
  int nin, nout;
  void** ins;  /* ins[r * nin + i] */
  void** outs; /* outs[r * nout + i] */
} fnbufs_t;

static void fn_local_reduce(const fnbufs_t* fb, int r, int op, int dtype,
                            size_t off, size_t len);
static void fn_local_broadcast(const fnbufs_t* fb, int r, int dtype, size_t off,
                               size_t len);

/* Run P programs to completion.  data[r] = rank r's ptr0; scratch[r] = its
 * receive buffers.  Returns 0, or -2 on deadlock, -3 on length overflow. */
static int simulate_fn(int P, prog_t* progs, int op, int dtype, unsigned char** data,
                       unsigned char** scratch, size_t* scratch_elems,
                       const fnbufs_t* fb) {
  size_t es = kSize[dtype];
  size_t* pc = (size_t*)calloc((size_t)P, sizeof(size_t));
  chans_t cs = {0};
  int rc = 0, r, progress = 1;
  if (!pc) return -1;
  while (progress) {
    int all_done = 1;
    progress = 0;
    for (r = 0; r < P; r++) {
      while (pc[r] < progs[r].n) {
        step_t* s = &progs[r].v[pc[r]];
        if (s->kind == ST_SEND) {
          chan_t* c = chan_get(&cs, r, s->peer, s->tag);
          msg_t* m = (msg_t*)malloc(sizeof(msg_t) + s->len * es + 1);
          if (!c || !m) { rc = -1; goto out; }
          m->next = NULL;
          m->len = s->len;
          memcpy(m->data, data[r] + s->off * es, s->len * es);
          if (c->tail) c->tail->next = m; else c->head = m;
          c->tail = m;
        } else if (s->kind == ST_RECV) {
          chan_t* c = chan_get(&cs, s->peer, r, s->tag);
          msg_t* m;
          if (!c) { rc = -1; goto out; }
          if (!c->head) break; /* blocked */
          m = c->head;
          c->head = m->next;
          if (!c->head) c->tail = NULL;
          if (s->boff + m->len > scratch_elems[r]) { free(m); rc = -3; goto out; }
          memcpy(scratch[r] + s->boff * es, m->data, m->len * es);
          free(m);
        } else if (s->kind == ST_REDUCE) {
          unsigned char* d = data[r] + s->off * es;
          oracle_reduce(op, dtype, d, d, scratch[r] + s->boff * es, s->len);
        } else if (s->kind == ST_LOCAL) {
          fn_local_reduce(fb, r, op, dtype, s->off, s->len);
        } else if (s->kind == ST_BCAST) {
          fn_local_broadcast(fb, r, dtype, s->off, s->len);
        } else { /* ST_COPY */
          memcpy(data[r] + s->off * es, scratch[r] + s->boff * es, s->len * es);
        }
        pc[r]++;
        progress = 1;
      }
      if (pc[r] < progs[r].n) all_done = 0;
    }
    if (all_done) {
      size_t i;
      for (i = 0; i < cs.n; i++)
        if (cs.v[i].head) rc = -4; /* a message nobody received */
      break;
    }
    if (!progress) { rc = -2; break; }
  }
out:
  {
    size_t i;
    for (i = 0; i < cs.n; i++) {
      msg_t* m = cs.v[i].head;
      while (m) { msg_t* nx = m->next; free(m); m = nx; }
    }
    free(cs.v);
  }
  free(pc);
  return rc;
}

static int simulate(int P, prog_t* progs, int op, int dtype, unsigned char** data,
                    unsigned char** scratch, size_t* scratch_elems) {
  return simulate_fn(P, progs, op, dtype, data, scratch, scratch_elems, NULL);
}

static void local_reduce_and(int P, int nptrs, int op, int dtype, size_t count,
                             void** bufs) {
  int r, i;
  for (r = 0; r < P; r++)
    for (i = 1; i < nptrs; i++)
      oracle_reduce(op, dtype, bufs[r * nptrs], bufs[r * nptrs],
                    bufs[r * nptrs + i], count);
}

static void local_broadcast(int P, int nptrs, int dtype, size_t count,
                            void** bufs) {
  int r, i;
  for (r = 0; r < P; r++)
    for (i = 1; i < nptrs; i++)
      memcpy(bufs[r * nptrs + i], bufs[r * nptrs], count * kSize[dtype]);
}

/* ---- allreduce_ring (gloo/allreduce_ring.h) ------------------------ */

/* AllreduceRing<T>::run() (:72-114): local fold into ptrs[0] (:76-79); the
 * outbox starts as that buffer (:82); in round k every rank sends its outbox
 * right, receives its left neighbour's into the inbox, ptrs[0] =
 * fn(ptrs[0], inbox) (:94), and forwards the inbox as its next outbox
 * (:100-102) -- so round k delivers rank r-1-k's locally reduced buffer;
 * finally ptrs[0] is copied to the other pointers (:113-115). */
int oracle_allreduce_ring(int op, int dtype, int P, int nptrs, int count, void** bufs) {
  unsigned char** orig;
  int r, round, rc = 0;
  const size_t bytes = (size_t)(count > 0 ? count : 0) * kSize[dtype >= 0 && dtype < OR_NDTYPES ? dtype : 0];
  if (P < 1 || nptrs < 1 || count < 0 || dtype < 0 || dtype >= OR_NDTYPES) return -1;
  if (count == 0) return 0; /* :72-74 */
  local_reduce_and(P, nptrs, op, dtype, (size_t)count, bufs);
  orig = (unsigned char**)calloc((size_t)P, sizeof(void*));
  if (!orig) return -1;
  for (r = 0; r < P; r++) {
    orig[r] = (unsigned char*)malloc(bytes);
    if (!orig[r]) { rc = -1; goto done; }
    memcpy(orig[r], bufs[r * nptrs], bytes);
  }
  for (round = 0; round < P - 1; round++)
    for (r = 0; r < P; r++)
      oracle_reduce(op, dtype, bufs[r * nptrs], bufs[r * nptrs],
                    orig[(r - 1 - round + 2 * P) % P], (size_t)count);
  local_broadcast(P, nptrs, dtype, (size_t)count, bufs);
done:
  for (r = 0; r < P; r++) free(orig[r]);
  free(orig);
  return rc;
}

/* ---- allreduce_bcube (gloo/allreduce_bcube.h) ---------------------- */

/* setupNodes / updateGroupNodes (:620-695) with Node / Group (:60-240):
 * per rank r and step s its peers (group order, without r), and the count /
 * offset of the range it reduces.  Arrays are [r * steps + s]. */
typedef struct {
  int steps, base;
  int* npeers;  /* [r * steps + s] */
  int* peers;   /* [(r * steps + s) * base + i] */
  long* num;
  long* off;
} bcube_geom_t;

static void bcube_free(bcube_geom_t* g) {
  free(g->npeers);
  free(g->peers);
  free(g->num);
  free(g->off);
}

static int bcube_setup(int nodes, int base, long total, bcube_geom_t* g) {
  /* computeSteps (:514-519): float logs, ceil of their quotient */
  const float lg2n = (float)log2((double)nodes);
  const float lg2p = (float)log2((double)base);
  const float q = lg2n / lg2p;
  int step, first, i;
  long peer_distance = 1;
  g->base = base;
  g->steps = (int)ceil((double)q);
  g->npeers = (int*)calloc((size_t)nodes * (size_t)(g->steps + 1), sizeof(int));
  g->peers = (int*)calloc((size_t)nodes * (size_t)(g->steps + 1) * (size_t)base, sizeof(int));
  g->num = (long*)calloc((size_t)nodes * (size_t)(g->steps + 1), sizeof(long));
  g->off = (long*)calloc((size_t)nodes * (size_t)(g->steps + 1), sizeof(long));
  if (!g->npeers || !g->peers || !g->num || !g->off) return -1;
  for (step = 0; step < g->steps; step++) {
    for (first = 0; first < nodes; first++) {
      int ranks[64], sz = 0;
      long ptr_offset, group_count, num_elems, cnt, rem;
      if (g->npeers[first * g->steps + step] != 0) continue; /* not a first node */
      for (i = 0; i < base && sz < 64; i++) {                 /* Group::getNodeRanks */
        long pr = first + (long)i * peer_distance;
        if (pr < nodes) ranks[sz++] = (int)pr;
      }
      ptr_offset = step == 0 ? 0 : g->off[first * g->steps + step - 1];
      group_count = step == 0 ? total : g->num[first * g->steps + step - 1];
      num_elems = group_count > sz ? group_count : sz;        /* computeNumElems */
      cnt = num_elems / sz;                                   /* updateGroupNodes */
      rem = num_elems % sz;
      if (cnt == 0) cnt = 1;
      for (i = 0; i < sz; i++) {
        const int n = ranks[i];
        const int at = n * g->steps + step;
        const long c = i != sz - 1 ? cnt : cnt + rem;
        int k;
        for (k = 0; k < sz; k++)
          if (ranks[k] != n) g->peers[at * base + g->npeers[at]++] = ranks[k];
        g->num[at] = c;
        g->off[at] = ptr_offset;
        ptr_offset = (ptr_offset + c) % total;
      }
    }
    peer_distance *= base;
  }
  return 0;
}

/* AllreduceBcube<T>::run() (:338-430): reduce-scatter -- every step sends
 * each peer its range, then folds each peer's message into our range in
 * group order (:354-381); all-gather -- the steps in reverse, our range out
 * and theirs copied in (:386-418); local fold / broadcast around it. */
int oracle_allreduce_bcube(int op, int dtype, int P, int nptrs, int count, int base,
                           void** bufs) {
  bcube_geom_t g = {0, 0, NULL, NULL, NULL, NULL};
  prog_t* progs = NULL;
  unsigned char** data = NULL;
  unsigned char** scratch = NULL;
  size_t* scratch_elems = NULL;
  long max_len = 0;
  int r, s, i, rc = 0;
  if (P < 1 || nptrs < 1 || count < 0 || base < 2 || base > 64 || dtype < 0 ||
      dtype >= OR_NDTYPES)
    return -1; /* bcube_setup keeps a group's ranks in a 64-entry array */
  if (count == 0) return 0;                                    /* :339-341 */
  local_reduce_and(P, nptrs, op, dtype, (size_t)count, bufs);  /* :343-345 */
  if (P == 1) {                                                /* :347-353 */
    local_broadcast(P, nptrs, dtype, (size_t)count, bufs);
    return 0;
  }
  if (bcube_setup(P, base, count, &g) != 0) { rc = -1; goto done; }
  for (r = 0; r < P * g.steps; r++)
    if (g.num[r] > max_len) max_len = g.num[r];
  progs = (prog_t*)calloc((size_t)P, sizeof(prog_t));
  data = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch_elems = (size_t*)calloc((size_t)P, sizeof(size_t));
  if (!progs || !data || !scratch || !scratch_elems) { rc = -1; goto done; }
  for (r = 0; r < P; r++) {
    prog_t* p = &progs[r];
    data[r] = (unsigned char*)bufs[r * nptrs];
    scratch_elems[r] = (size_t)max_len * (size_t)P; /* a region per source rank */
    scratch[r] = (unsigned char*)calloc(scratch_elems[r], kSize[dtype]);
    if (!scratch[r]) { rc = -1; goto done; }
    for (s = 0; s < g.steps; s++) {
      const int at = r * g.steps + s;
      for (i = 0; i < g.npeers[at]; i++) {
        const int d = g.peers[at * base + i];
        step_t st = {ST_SEND, d, 0, (size_t)g.off[d * g.steps + s],
                     (size_t)g.num[d * g.steps + s], 0};
        prog_push(p, st);
      }
      for (i = 0; i < g.npeers[at]; i++) {
        const int src = g.peers[at * base + i];
        step_t rv = {ST_RECV, src, 0, 0, 0, (size_t)src * (size_t)max_len};
        step_t red = {ST_REDUCE, 0, 0, (size_t)g.off[at], (size_t)g.num[at],
                      (size_t)src * (size_t)max_len};
        prog_push(p, rv);
        prog_push(p, red);
      }
    }
    for (s = g.steps - 1; s >= 0; s--) {
      const int at = r * g.steps + s;
      for (i = 0; i < g.npeers[at]; i++) {
        step_t st = {ST_SEND, g.peers[at * base + i], 0, (size_t)g.off[at], (size_t)g.num[at], 0};
        prog_push(p, st);
      }
      for (i = 0; i < g.npeers[at]; i++) {
        const int src = g.peers[at * base + i];
        step_t rv = {ST_RECV, src, 0, 0, 0, (size_t)src * (size_t)max_len};
        step_t cp = {ST_COPY, 0, 0, (size_t)g.off[src * g.steps + s],
                     (size_t)g.num[src * g.steps + s], (size_t)src * (size_t)max_len};
        prog_push(p, rv);
        prog_push(p, cp);
      }
    }
  }
  rc = simulate(P, progs, op, dtype, data, scratch, scratch_elems);
  if (rc == 0) local_broadcast(P, nptrs, dtype, (size_t)count, bufs); /* :421-424 */
done:
  if (progs) for (r = 0; r < P; r++) free(progs[r].v);
  if (scratch) for (r = 0; r < P; r++) free(scratch[r]);
  free(progs);
  free(data);
  free(scratch);
  free(scratch_elems);
  bcube_free(&g);
  return rc;
}

/* ---- allreduce_ring_chunked (gloo/allreduce_ring_chunked.h) ------- */

typedef struct { size_t chunks, chunk_size; int count; } ring_geom_t;

/* chunk (offset, length) for a chunk index, as the receiver computes it
 * (gloo/allreduce_ring_chunked.h:128-138). */
static void ring_chunk(const ring_geom_t* g, size_t c, size_t* off, size_t* len) {
  size_t o = c * g->chunk_size, l = g->chunk_size;
  if (o + l <= (size_t)g->count) {
  } else if (o < (size_t)g->count) {
    l = (size_t)g->count - o;
  } else {
    l = 0;
  }
  *off = o;
  *len = l;
}

/* what the sender puts on the wire (copyChunkAtOffset, :215-236): an empty
 * chunk still sends one element from offset 0. */
static void ring_send_step(const ring_geom_t* g, int right, size_t c, prog_t* p) {
  step_t s = {ST_SEND, right, (int)(c & 1), 0, 0, 0};
  size_t off, len;
  ring_chunk(g, c % g->chunks, &off, &len);
  if (len == 0) { off = 0; len = 1; }
  s.off = off;
  s.len = len;
  prog_push(p, s);
}

/* chunkOffset for a round (:125-127) */
static size_t ring_chunk_offset(int rank, int round, size_t chunks) {
  return (size_t)(((long)(2 * rank) - (long)(round & ~1) + (long)(round & 1) +
                   (long)chunks) % (long)chunks);
}

int oracle_allreduce_ring_chunked(int op, int dtype, int P, int nptrs, int count,
                                  void** bufs) {
  ring_geom_t g;
  prog_t* progs;
  unsigned char** data;
  unsigned char** scratch;
  size_t* scratch_elems;
  int r, round, rc = 0;
  const size_t min_size = 256; /* :33 */
  if (P < 1 || nptrs < 1 || count < 0 || dtype < 0 || dtype >= OR_NDTYPES)
    return -1;
  if (count == 0) return 0;                               /* :84-86 */
  local_reduce_and(P, nptrs, op, dtype, (size_t)count, bufs); /* :89-91 */
  if (P == 1) {                                           /* :93-99 */
    local_broadcast(P, nptrs, dtype, (size_t)count, bufs);
    return 0;
  }
  g.count = count;
  g.chunks = (size_t)P * 2;                               /* :34 */
  g.chunk_size = ((size_t)count + g.chunks - 1) / g.chunks; /* :38 */
  if (g.chunk_size < min_size) g.chunk_size = min_size;
  progs = (prog_t*)calloc((size_t)P, sizeof(prog_t));
  data = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch_elems = (size_t*)calloc((size_t)P, sizeof(size_t));
  if (!progs || !data || !scratch || !scratch_elems) { rc = -1; goto done; }
  for (r = 0; r < P; r++) {
    int left = (r + P - 1) % P, right = (r + 1) % P;
    prog_t* p = &progs[r];
    data[r] = (unsigned char*)bufs[r * nptrs];
    scratch_elems[r] = 2 * g.chunk_size; /* inbox_[0], inbox_[1] */
    scratch[r] = (unsigned char*)calloc(scratch_elems[r], kSize[dtype]);
    if (!scratch[r]) { rc = -1; goto done; }
    ring_send_step(&g, right, (size_t)(2 * r), p);        /* :102-103 */
    ring_send_step(&g, right, (size_t)(2 * r + 1), p);
    for (round = 2; round < (int)g.chunks; round++) {     /* :106-158 */
      size_t c = ring_chunk_offset(r, round, g.chunks), off, len;
      step_t rv = {ST_RECV, left, (int)(c & 1), 0, 0, (c & 1) * g.chunk_size};
      ring_chunk(&g, c, &off, &len);
      prog_push(p, rv);
      if (len > 0) {
        step_t red = {ST_REDUCE, 0, 0, off, len, (c & 1) * g.chunk_size};
        prog_push(p, red);
      }
      ring_send_step(&g, right, c, p);
    }
    for (round = 0; round < (int)g.chunks - 2; round++) { /* :163-200 */
      size_t c = ring_chunk_offset(r, round, g.chunks), off, len;
      step_t rv = {ST_RECV, left, (int)(c & 1), 0, 0, (c & 1) * g.chunk_size};
      ring_chunk(&g, c, &off, &len);
      prog_push(p, rv);
      if (len > 0) {
        step_t cp = {ST_COPY, 0, 0, off, len, (c & 1) * g.chunk_size};
        prog_push(p, cp);
      }
      if (round < (int)g.chunks - 4) ring_send_step(&g, right, c, p);
    }
  }
  rc = simulate(P, progs, op, dtype, data, scratch, scratch_elems);
  if (rc == 0) local_broadcast(P, nptrs, dtype, (size_t)count, bufs); /* :209-211 */
done:
  if (progs) for (r = 0; r < P; r++) free(progs[r].v);
  if (scratch) for (r = 0; r < P; r++) free(scratch[r]);
  free(progs);
  free(data);
  free(scratch);
  free(scratch_elems);
  return rc;
}

/* ---- allreduce_halving_doubling (gloo/allreduce_halving_doubling.h) */

/* last n bits of ctr, reversed (:23-34) */
static uint32_t reverse_bits(uint32_t ctr, uint32_t n) {
  uint32_t out = 0, i;
  for (i = 0; i < n; i++) out |= ((ctr >> i) & 1u) << (n - 1 - i);
  return out;
}

static uint32_t ilog2(uint32_t v) { /* floor(log2(v)), v >= 1 */
  uint32_t l = 0;
  while ((v >> 1) != 0) { v >>= 1; l++; }
  return l;
}

typedef struct {
  uint32_t offset_to_block, block_size, steps_in_block, rank_in_block;
  uint32_t smaller, larger;
} hd_blocks_t;

/* Binary-block decomposition of P (:39-64): P's set bits from the lowest
 * upward are blocks laid out from the highest rank downward. */
static hd_blocks_t hd_blocks(int P, int rank) {
  hd_blocks_t b = {0, 0, 0, 0, 0, 0};
  uint32_t offset = (uint32_t)P, bs = 1, cur = 0, prev = 0;
  do {
    if ((uint32_t)P & bs) {
      prev = cur;
      cur = bs;
      offset -= bs;
      if (b.block_size != 0) { b.larger = cur; break; }
      if (offset <= (uint32_t)rank) {
        b.offset_to_block = offset;
        b.block_size = cur;
        b.smaller = prev;
      }
    }
    bs <<= 1;
  } while (offset != 0);
  b.steps_in_block = ilog2(b.block_size);
  b.rank_in_block = (uint32_t)rank % b.block_size;
  return b;
}

int oracle_allreduce_halving_doubling(int op, int dtype, int P, int nptrs,
                                      int count, void** bufs) {
  prog_t* progs;
  unsigned char** data;
  unsigned char** scratch;
  size_t* scratch_elems;
  int r, rc = 0;
  size_t steps, chunks, chunk_size;
  if (P < 1 || nptrs < 1 || count < 0 || dtype < 0 || dtype >= OR_NDTYPES)
    return -1;
  if (count == 0) return 0;                                   /* :225-227 */
  local_reduce_and(P, nptrs, op, dtype, (size_t)count, bufs); /* :232-234 */
  if (P == 1) {
    local_broadcast(P, nptrs, dtype, (size_t)count, bufs);
    return 0;
  }
  steps = ilog2((uint32_t)P);                                 /* :76 */
  chunks = (size_t)1 << steps;
  chunk_size = ((size_t)count + chunks - 1) / chunks;
  progs = (prog_t*)calloc((size_t)P, sizeof(prog_t));
  data = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch_elems = (size_t*)calloc((size_t)P, sizeof(size_t));
  if (!progs || !data || !scratch || !scratch_elems) { rc = -1; goto done; }

  for (r = 0; r < P; r++) {
    hd_blocks_t b = hd_blocks(P, r);
    prog_t* p = &progs[r];
    size_t S = b.steps_in_block, i;
    size_t* send_off = (size_t*)calloc(S + 1, sizeof(size_t));
    size_t* recv_off = (size_t*)calloc(S + 1, sizeof(size_t));
    size_t* send_cnt = (size_t*)calloc(S + 1, sizeof(size_t));
    size_t* recv_cnt = (size_t*)calloc(S + 1, sizeof(size_t));
    size_t* rbuf_base = (size_t*)calloc(S + 1, sizeof(size_t));
    size_t step_chunk = chunk_size << (steps - 1);
    size_t so = 0, ro = 0, boff = 0, bitmask = 1;
    size_t larger_recv_base = 0, smaller_recv_base = 0, send_count_larger = 0;
    size_t n_larger = 0;
    size_t total_to_send;
    size_t smaller_recv_len = 0;
    int smaller_peer = -1;
    if (!send_off || !recv_off || !send_cnt || !recv_cnt || !rbuf_base) {
      rc = -1;
      goto done;
    }
    data[r] = (unsigned char*)bufs[r * nptrs];
    /* geometry from the constructor (:107-157) */
    for (i = 0; i < S; i++) {
      int dest = r ^ (int)bitmask;
      send_off[i] = so + ((dest & bitmask) ? step_chunk : 0);
      recv_off[i] = ro + (((size_t)r & bitmask) ? step_chunk : 0);
      if (send_off[i] < (size_t)count)
        send_cnt[i] = (send_off[i] + step_chunk > (size_t)count)
                          ? (size_t)count - send_off[i] : step_chunk;
      if (recv_off[i] < (size_t)count)
        recv_cnt[i] = (recv_off[i] + step_chunk > (size_t)count)
                          ? (size_t)count - recv_off[i] : step_chunk;
      rbuf_base[i] = boff;
      boff += step_chunk;
      if ((size_t)r & bitmask) { so += step_chunk; ro += step_chunk; }
      bitmask <<= 1;
      step_chunk >>= 1;
    }
    if (b.smaller != 0) {                                     /* :159-176 */
      smaller_peer = (int)(b.offset_to_block + b.block_size +
                           b.rank_in_block % b.smaller);
      smaller_recv_base = boff;
      smaller_recv_len = recv_cnt[S - 1];
    }
    total_to_send = S > 0 ? recv_cnt[S - 1] : (size_t)count;
    if (b.larger != 0) {                                      /* :177-221 */
      n_larger = b.larger / b.block_size;
      send_count_larger = step_chunk >> (ilog2((uint32_t)n_larger) - 1);
      larger_recv_base = boff;
    }
    /* scratch = recvBuf_ (chunkSize << steps, zero-initialised, :81) plus
     * room for the cross-block receive windows. */
    scratch_elems[r] = (chunk_size << steps) + (size_t)count + 1;
    scratch[r] = (unsigned char*)calloc(scratch_elems[r], kSize[dtype]);
    if (!scratch[r]) { rc = -1; goto done; }

    /* run(), :244-259 reduce-scatter */
    {
      size_t buf_off = 0;
      size_t num_items = S > 0 ? chunk_size << (steps - 1) : (size_t)count;
      for (i = 0; i < S; i++) {
        int dest = r ^ (1 << i);
        int tag = 0;
        if (send_off[i] < (size_t)count) {
          step_t s = {ST_SEND, dest, tag, send_off[i], send_cnt[i], 0};
          prog_push(p, s);
        }
        if (recv_off[i] < (size_t)count) {
          step_t rv = {ST_RECV, dest, tag, 0, 0, rbuf_base[i]};
          step_t red = {ST_REDUCE, 0, 0, recv_off[i], recv_cnt[i], buf_off};
          prog_push(p, rv);
          prog_push(p, red);
        }
        buf_off += num_items;
        num_items >>= 1;
      }
      /* receive from smaller block (:266-272) */
      if (b.smaller != 0 && smaller_recv_len > 0) {
        step_t rv = {ST_RECV, smaller_peer, 0, 0, 0, smaller_recv_base};
        step_t red = {ST_REDUCE, 0, 0, recv_off[S - 1], recv_cnt[S - 1], buf_off};
        prog_push(p, rv);
        prog_push(p, red);
      }
      /* scatter to / gather from larger block (:274-305) */
      if (b.larger != 0 && total_to_send != 0) {
        size_t offset = S > 0 ? recv_off[S - 1] : 0, k;
        uint32_t src_ord = reverse_bits(b.rank_in_block, ilog2(b.block_size));
        uint32_t dst_ord = src_ord * (uint32_t)n_larger;
        uint32_t off_larger = b.offset_to_block - b.larger;
        int* peers = (int*)calloc(n_larger, sizeof(int));
        size_t rb = larger_recv_base;
        if (!peers) { rc = -1; goto done; }
        for (k = 0; k < n_larger; k++)
          peers[k] = (int)(off_larger +
                           reverse_bits(dst_ord + (uint32_t)k, ilog2(b.larger)));
        for (k = 0; k < n_larger; k++) {
          if (send_count_larger * k < total_to_send) {
            size_t n = total_to_send - send_count_larger * k;
            step_t s = {ST_SEND, peers[k], 0, offset + k * send_count_larger,
                        n < send_count_larger ? n : send_count_larger, 0};
            prog_push(p, s);
          }
        }
        for (k = 0; k < n_larger; k++) {
          if (send_count_larger * k < total_to_send) {
            size_t n = total_to_send - send_count_larger * k;
            step_t rv = {ST_RECV, peers[k], 0, 0, 0, rb};
            prog_push(p, rv);
            rb += n < send_count_larger ? n : send_count_larger;
          }
        }
        {
          step_t cp = {ST_COPY, 0, 0, offset, total_to_send, larger_recv_base};
          prog_push(p, cp);
        }
        free(peers);
      }
      /* send to smaller block (:308-316) */
      if (b.smaller != 0 && recv_off[S - 1] < (size_t)count) {
        step_t s = {ST_SEND, smaller_peer, 0, recv_off[S - 1], recv_cnt[S - 1], 0};
        prog_push(p, s);
      }
      /* allgather (:319-341) */
      num_items = chunk_size << (steps - S);
      for (i = S; i-- > 0;) {
        int dest = r ^ (1 << i);
        if (recv_off[i] < (size_t)count) {
          step_t s = {ST_SEND, dest, 0, recv_off[i], recv_cnt[i], 0};
          prog_push(p, s);
        }
        buf_off -= num_items;
        if (send_off[i] < (size_t)count) {
          step_t rv = {ST_RECV, dest, 0, 0, 0, rbuf_base[i]};
          step_t cp = {ST_COPY, 0, 0, send_off[i], send_cnt[i], buf_off};
          prog_push(p, rv);
          prog_push(p, cp);
        }
        num_items <<= 1;
      }
    }
    free(send_off);
    free(recv_off);
    free(send_cnt);
    free(recv_cnt);
    free(rbuf_base);
  }
  rc = simulate(P, progs, op, dtype, data, scratch, scratch_elems);
  if (rc == 0) local_broadcast(P, nptrs, dtype, (size_t)count, bufs); /* :344-346 */
done:
  if (progs) for (r = 0; r < P; r++) free(progs[r].v);
  if (scratch) for (r = 0; r < P; r++) free(scratch[r]);
  free(progs);
  free(data);
  free(scratch);
  free(scratch_elems);
  return rc;
}

/* ---- gloo::allreduce(opts) (gloo/allreduce.cc) --------------------- */

/* genLocalReduceFunction (:44-82): the local reduction of [off, off+len)
 * into out[0]. */
static void fn_local_reduce(const fnbufs_t* fb, int r, int op, int dtype,
                            size_t off, size_t len) {
  size_t es = kSize[dtype], b = off * es;
  unsigned char* out0 = (unsigned char*)fb->outs[(size_t)r * fb->nout] + b;
  int i;
  if (fb->nin == 1) {
    memmove(out0, (unsigned char*)fb->ins[(size_t)r * fb->nin] + b, len * es);
  } else if (fb->nin >= 2) {
    oracle_reduce(op, dtype, out0, (unsigned char*)fb->ins[(size_t)r * fb->nin] + b,
                  (unsigned char*)fb->ins[(size_t)r * fb->nin + 1] + b, len);
    for (i = 2; i < fb->nin; i++)
      oracle_reduce(op, dtype, out0, out0,
                    (unsigned char*)fb->ins[(size_t)r * fb->nin + i] + b, len);
  } else {
    for (i = 1; i < fb->nout; i++)
      oracle_reduce(op, dtype, out0, out0,
                    (unsigned char*)fb->outs[(size_t)r * fb->nout + i] + b, len);
  }
}

/* genLocalBroadcastFunction (:87-95) */
static void fn_local_broadcast(const fnbufs_t* fb, int r, int dtype, size_t off,
                               size_t len) {
  size_t es = kSize[dtype], b = off * es;
  unsigned char* out0 = (unsigned char*)fb->outs[(size_t)r * fb->nout] + b;
  int i;
  for (i = 1; i < fb->nout; i++)
    memcpy((unsigned char*)fb->outs[(size_t)r * fb->nout + i] + b, out0, len * es);
}

static void push(prog_t* p, int kind, int peer, size_t off, size_t len, size_t boff) {
  step_t s;
  s.kind = kind;
  s.peer = peer;
  s.tag = 0; /* one slot per operation: messages of a pair match in order */
  s.off = off;
  s.len = len;
  s.boff = boff;
  prog_push(p, s);
}

/* ring (:148-393).  Byte offsets of the reference become element offsets:
 * segmentBytes is a multiple of the element size (:218-219). */
static void fn_ring_prog(int r, int P, size_t count, size_t es, size_t max_seg,
                         prog_t* p, size_t* scratch_elems) {
  size_t total = count * es;
  size_t max_seg_bytes = es * (max_seg / es > 0 ? max_seg / es : 1);    /* :193-194 */
  size_t nseg = (total + max_seg_bytes - 1) / max_seg_bytes;             /* :210-214 */
  size_t spr, seg_bytes, seg, iters, i;
  int recv_rank = (P + r + 1) % P, send_rank = (P + r - 1) % P;          /* :158-159 */
  if (nseg < (size_t)P * 2) nseg = (size_t)P * 2;
  nseg = (nseg + (size_t)P - 1) / (size_t)P * (size_t)P;
  spr = nseg / (size_t)P;
  seg_bytes = (total + nseg - 1) / nseg;                                 /* :217-218 */
  seg_bytes = (seg_bytes + es - 1) / es * es;
  seg = seg_bytes / es;
  *scratch_elems = 2 * seg;                                              /* :221-225 */
  iters = nseg - spr + 2;
#define SEG_OFF(k) ((((k) % nseg) * seg))
#define SEG_LEN(o) ((o) >= count ? 0 : ((count - (o)) < seg ? (count - (o)) : seg))
  for (i = 0; i < iters; i++) {                                          /* :279-322 */
    if (i >= 2) {
      size_t k = i - 2;
      size_t ro = SEG_OFF(((size_t)r + 2) * spr + k), rl = SEG_LEN(ro);  /* :252-254 */
      if (rl > 0) {
        push(p, ST_LOCAL, 0, ro, rl, 0);                                 /* :288 */
        push(p, ST_RECV, recv_rank, 0, rl, (i & 1) * seg);               /* :290 */
        push(p, ST_REDUCE, 0, ro, rl, (i & 1) * seg);                    /* :292-296 */
      }
    }
    if (i < nseg - spr) {
      size_t so = SEG_OFF(((size_t)r + 1) * spr + i), sl = SEG_LEN(so);  /* :249-251 */
      if (sl > 0) {
        if (i < spr) push(p, ST_LOCAL, 0, so, sl, 0);                    /* :314-316 */
        push(p, ST_SEND, send_rank, so, sl, 0);                          /* :318 */
      }
    }
  }
  for (i = 0; i < iters; i++) {                                          /* :362-392 */
    if (i >= 2) {
      size_t k = i - 2;
      size_t ro = SEG_OFF(((size_t)r + 1) * spr + k), rl = SEG_LEN(ro);  /* :336-338 */
      if (rl > 0) {
        push(p, ST_RECV, recv_rank, 0, rl, 0);                           /* :366 */
        push(p, ST_COPY, 0, ro, rl, 0);       /* the reference receives in place */
        push(p, ST_BCAST, 0, ro, rl, 0);                                 /* :368 */
      }
    }
    if (i < nseg - spr) {
      size_t so = SEG_OFF((size_t)r * spr + i), sl = SEG_LEN(so);        /* :333-335 */
      if (sl > 0) {
        push(p, ST_SEND, send_rank, so, sl, 0);                          /* :385 */
        if (i < spr) push(p, ST_BCAST, 0, so, sl, 0);                    /* :387-389 */
      }
    }
  }
#undef SEG_OFF
#undef SEG_LEN
}

/* bcube with n = 2 (:395-669) */
typedef struct {
  size_t buffer_offset, buffer_length, chunk_length, my_off, my_len;
  int group_rank, nranks;
  int ranks[64];
} bgroup_t;

static size_t bgroup_len(const bgroup_t* g, int i) { /* :545-550 */
  long rest = (long)g->buffer_length - (long)((size_t)i * g->chunk_length);
  if (rest < 0) rest = 0;
  return (size_t)rest < g->chunk_length ? (size_t)rest : g->chunk_length;
}

static int bcube_groups(int r, int P, size_t count, bgroup_t* gs) {
  int sizes[64], ns = 0, s, i;
  size_t rest = (size_t)P, dist = 1, boff = 0, blen = count;
  while (rest % 2 == 0) { sizes[ns++] = 2; rest /= 2; }                  /* :398-409 */
  if (rest > 1) sizes[ns++] = (int)rest;
  for (s = 0; s < ns; s++) {                                             /* :466-511 */
    bgroup_t* g = &gs[s];
    size_t gsz = (size_t)sizes[s];
    size_t group_rank = ((size_t)r / dist) % gsz;
    size_t base = (size_t)r - group_rank * dist;
    if (gsz > 64) return -1;
    g->group_rank = (int)group_rank;
    g->nranks = (int)gsz;
    for (i = 0; i < (int)gsz; i++) g->ranks[i] = (int)(base + (size_t)i * dist);
    g->buffer_offset = boff;
    g->buffer_length = blen;
    g->chunk_length = (blen + gsz - 1) / gsz;
    g->my_off = boff + group_rank * g->chunk_length;
    g->my_len = bgroup_len(g, (int)group_rank);
    dist *= gsz;
    boff = g->my_off;
    blen = g->my_len;
  }
  return ns;
}

static int fn_bcube_prog(int r, int P, size_t count, prog_t* p, size_t* scratch_elems) {
  bgroup_t gs[64];
  int ns = bcube_groups(r, P, count, gs), s, i;
  size_t need = count;
  if (ns < 0) return -1;
  for (s = 0; s < ns; s++) {                                             /* :503-509 */
    size_t v = (size_t)gs[s].nranks * gs[s].chunk_length;
    if (v > need) need = v;
  }
  *scratch_elems = need;
  for (s = 0; s < ns; s++) {                                             /* :520-597 */
    const bgroup_t* g = &gs[s];
    for (i = 0; i < g->nranks; i++) {                                    /* :534-556 */
      size_t off = g->buffer_offset + (size_t)i * g->chunk_length, len = bgroup_len(g, i);
      if (g->ranks[i] == r) continue;
      if (s == 0) push(p, ST_LOCAL, 0, off, len, 0);
      push(p, ST_SEND, g->ranks[i], off, len, 0);
    }
    for (i = 0; i < g->nranks; i++) {                                    /* :521-532 */
      if (g->ranks[i] == r) continue;
      push(p, ST_RECV, g->ranks[i], 0, g->my_len, (size_t)i * g->chunk_length);
    }
    if (s == 0) push(p, ST_LOCAL, 0, g->my_off, g->my_len, 0);            /* :575-578 */
    for (i = 0; i < g->nranks; i++) {                                    /* :580-596 */
      if (g->ranks[i] == r) continue;
      push(p, ST_REDUCE, 0, g->my_off, g->my_len, (size_t)i * g->chunk_length);
    }
  }
  push(p, ST_BCAST, 0, gs[ns - 1].my_off, gs[ns - 1].my_len, 0);          /* :599-605 */
  for (s = ns - 1; s >= 0; s--) {                                        /* :606-669 */
    const bgroup_t* g = &gs[s];
    for (i = 0; i < g->nranks; i++) {
      if (g->ranks[i] == r) continue;
      push(p, ST_SEND, g->ranks[i], g->my_off, g->my_len, 0);
    }
    for (i = 0; i < g->nranks; i++) {
      size_t off = g->buffer_offset + (size_t)i * g->chunk_length, len = bgroup_len(g, i);
      if (g->ranks[i] == r) continue;
      push(p, ST_RECV, g->ranks[i], 0, len, 0);
      push(p, ST_COPY, 0, off, len, 0);
    }
    for (i = 0; i < g->nranks; i++) {                                    /* :653-667 */
      size_t off = g->buffer_offset + (size_t)i * g->chunk_length, len = bgroup_len(g, i);
      if (g->ranks[i] == r) continue;
      push(p, ST_BCAST, 0, off, len, 0);
    }
  }
  return 0;
}

/* gloo::allreduce(opts) for P ranks.  algo: 1 = RING (and UNSPECIFIED),
 * 2 = BCUBE.  ins[r * nin + i], outs[r * nout + i] (nout >= 1); the result
 * is left in every rank's outputs.  max_seg: opts.maxSegmentSize in bytes
 * (0: 1 MiB, gloo/allreduce.h:80). */
int oracle_allreduce_fn(int algo, int op, int dtype, int P, int nin, int nout,
                        size_t count, size_t max_seg, void** ins, void** outs) {
  fnbufs_t fb;
  prog_t* progs = NULL;
  unsigned char** data = NULL;
  unsigned char** scratch = NULL;
  size_t* scratch_elems = NULL;
  int r, rc = 0;
  if (P < 1 || nin < 0 || nout < 1 || dtype < 0 || dtype >= OR_NDTYPES) return -1;
  if (algo != 1 && algo != 2) return -1;
  if (max_seg == 0) max_seg = 1024 * 1024;
  fb.nin = nin;
  fb.nout = nout;
  fb.ins = ins;
  fb.outs = outs;
  if (count == 0) return 0;                                              /* :98-100 */
  if (P == 1) {                                                          /* :129-133 */
    fn_local_reduce(&fb, 0, op, dtype, 0, count);
    fn_local_broadcast(&fb, 0, dtype, 0, count);
    return 0;
  }
  progs = (prog_t*)calloc((size_t)P, sizeof(prog_t));
  data = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch = (unsigned char**)calloc((size_t)P, sizeof(void*));
  scratch_elems = (size_t*)calloc((size_t)P, sizeof(size_t));
  if (!progs || !data || !scratch || !scratch_elems) { rc = -1; goto done; }
  for (r = 0; r < P; r++) {
    data[r] = (unsigned char*)outs[(size_t)r * nout];
    if (algo == 1) {
      fn_ring_prog(r, P, count, kSize[dtype], max_seg, &progs[r], &scratch_elems[r]);
    } else if (fn_bcube_prog(r, P, count, &progs[r], &scratch_elems[r]) != 0) {
      rc = -1;
      goto done;
    }
    scratch[r] = (unsigned char*)calloc(scratch_elems[r] + 1, kSize[dtype]);
    if (!scratch[r]) { rc = -1; goto done; }
  }
  rc = simulate_fn(P, progs, op, dtype, data, scratch, scratch_elems, &fb);
done:
  if (progs) for (r = 0; r < P; r++) free(progs[r].v);
  if (scratch) for (r = 0; r < P; r++) free(scratch[r]);
  free(progs);
  free(data);
  free(scratch);
  free(scratch_elems);
  return rc;
}
