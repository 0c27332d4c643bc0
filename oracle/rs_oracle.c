/*
 * CPU oracle (C restatement) of the Reed-Solomon path the reference shredder uses.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/_build/liboracle_rs.so by oracle/Makefile;
 * loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
 * product library (alpenglow_amd/) never links or calls it.
 *
 * Restates reed-solomon-simd 3.1.0 (the crate behind /root/reference/src/shredder/
 * reed_solomon.rs:9; pinned at Cargo.lock:2280-2288), the same algorithm as
 * oracle/rs_oracle.py, scalar log/exp-table arithmetic:
 *   tables            crate engine/tables.rs      
 *   fft / ifft        crate engine (radix-2 form; the crate fuses 2 layers, same math)
 *   shard layout      crate Shards::insert / undo_last_chunk_encoding
 *   encode            crate rate/encoder_{high,low}.rs
 *   decode            crate rate/decoder_{high,low}.rs, every present shard
 *
 * PARITY UNPINNED at the reference boundary (no known-answer vectors exist in the
 * reference and the crate cannot be built here); see oracle/rs_oracle.py header.
 *
 * Multi-block entry points (ro_*_blocks) spread blocks over POSIX threads, one block per
 * task, for the CPU baseline of bench.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GF_BITS 16
#define GF_ORDER 65536u
#define GF_MODULUS 65535u
#define GF_POLYNOMIAL 0x1002Du

static const uint16_t CANTOR_BASIS[GF_BITS] = {
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

static uint16_t g_exp[GF_ORDER], g_log[GF_ORDER], g_skew[GF_MODULUS];
static uint16_t g_log_walsh[GF_ORDER];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

enum {
  RO_OK = 0,
  RO_INVALID_SHARD_SIZE = 1,
  RO_NOT_ENOUGH_SHARDS = 9,
  RO_UNSUPPORTED_SHARD_COUNT = 10,
  RO_NO_MEMORY = 100,
};

static inline uint16_t add_mod(uint32_t x, uint32_t y) {
  uint32_t s = x + y;
  return (uint16_t)(s + (s >> GF_BITS));
}
static inline uint16_t sub_mod(uint32_t x, uint32_t y) {
  uint32_t d = x - y;
  return (uint16_t)(d + (d >> GF_BITS));
}
static inline uint16_t gf_mul(uint16_t x, uint16_t log_m) {
  return x == 0 ? 0 : g_exp[add_mod(g_log[x], log_m)];
}

static void fwht(uint16_t *d, size_t n) {
  for (size_t dist = 1; dist < n; dist <<= 1)
    for (size_t r = 0; r < n; r += 2 * dist)
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t a = d[i], b = d[i + dist];
        d[i] = add_mod(a, b);
        d[i + dist] = sub_mod(a, b);
      }
}

static void init_tables(void) {
  uint32_t state = 1;
  for (uint32_t i = 0; i < GF_MODULUS; ++i) {
    g_exp[state] = (uint16_t)i;
    state <<= 1;
    if (state >= GF_ORDER) state ^= GF_POLYNOMIAL;
  }
  g_exp[0] = GF_MODULUS;
  g_log[0] = 0;
  for (int i = 0; i < GF_BITS; ++i) {
    uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; ++j) g_log[j + w] = g_log[j] ^ CANTOR_BASIS[i];
  }
  for (uint32_t i = 0; i < GF_ORDER; ++i) g_log[i] = g_exp[g_log[i]];
  for (uint32_t i = 0; i < GF_ORDER; ++i) g_exp[g_log[i]] = (uint16_t)i;
  g_exp[GF_MODULUS] = g_exp[0];

  uint16_t temp[GF_BITS - 1];
  for (int i = 1; i < GF_BITS; ++i) temp[i - 1] = (uint16_t)(1u << i);
  for (int m = 0; m < GF_BITS - 1; ++m) {
    size_t step = (size_t)1 << (m + 1);
    g_skew[((size_t)1 << m) - 1] = 0;
    for (int i = m; i < GF_BITS - 1; ++i) {
      size_t s = (size_t)1 << (i + 1);
      for (size_t j = ((size_t)1 << m) - 1; j < s; j += step) g_skew[j + s] = g_skew[j] ^ temp[i];
    }
    temp[m] = (uint16_t)(GF_MODULUS - g_log[gf_mul(temp[m], g_log[temp[m] ^ 1])]);
    for (int i = m + 1; i < GF_BITS - 1; ++i)
      temp[i] = gf_mul(temp[i], add_mod(g_log[temp[i] ^ 1], temp[m]));
  }
  for (uint32_t i = 0; i < GF_MODULUS; ++i) g_skew[i] = g_log[g_skew[i]];

  memcpy(g_log_walsh, g_log, sizeof g_log);
  g_log_walsh[0] = 0;
  fwht(g_log_walsh, GF_ORDER);
}

static void ensure_tables(void) { pthread_once(&g_once, init_tables); }

/* ---- table export (tests compare these with the python oracle) ---- */
void ro_tables(uint16_t *exp, uint16_t *log, uint16_t *skew, uint16_t *log_walsh) {
  ensure_tables();
  if (exp) memcpy(exp, g_exp, sizeof g_exp);
  if (log) memcpy(log, g_log, sizeof g_log);
  if (skew) memcpy(skew, g_skew, sizeof g_skew);
  if (log_walsh) memcpy(log_walsh, g_log_walsh, sizeof g_log_walsh);
}

/* read-only table access for the crate-engine baseline (rs_cpu_avx2.c) */
void ro_internal_tables(const uint16_t **exp, const uint16_t **log, const uint16_t **skew,
                        const uint16_t **log_walsh) {
  ensure_tables();
  *exp = g_exp;
  *log = g_log;
  *skew = g_skew;
  *log_walsh = g_log_walsh;
}

/* ---- rows of u16 symbols: work[row * nsym + j] ---- */
static void mul_row(uint16_t *dst, const uint16_t *src, size_t nsym, uint16_t log_m) {
  for (size_t j = 0; j < nsym; ++j) dst[j] = gf_mul(src[j], log_m);
}
static void xor_rows(uint16_t *x, const uint16_t *y, size_t n) {
  for (size_t j = 0; j < n; ++j) x[j] ^= y[j];
}

static void fft(uint16_t *w, size_t nsym, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = size >> 1; dist >= 1; dist >>= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      uint16_t lm = g_skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t *x = w + (pos + i) * nsym, *y = w + (pos + i + dist) * nsym;
        if (lm != GF_MODULUS)
          for (size_t j = 0; j < nsym; ++j) x[j] ^= gf_mul(y[j], lm);
        xor_rows(y, x, nsym);
      }
    }
    if (dist == 1) break;
  }
}

static void ifft(uint16_t *w, size_t nsym, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = 1; dist < size; dist <<= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      uint16_t lm = g_skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint16_t *x = w + (pos + i) * nsym, *y = w + (pos + i + dist) * nsym;
        xor_rows(y, x, nsym);
        if (lm != GF_MODULUS)
          for (size_t j = 0; j < nsym; ++j) x[j] ^= gf_mul(y[j], lm);
      }
    }
  }
}

static void formal_derivative(uint16_t *w, size_t nsym, size_t n) {
  for (size_t i = 1; i < n; ++i) {
    size_t width = i & (~i + 1);
    xor_rows(w + (i - width) * nsym, w + i * nsym, width * nsym);
  }
}

/* ---- shard layout ---- */
static void shard_to_syms(const uint8_t *b, size_t S, uint16_t *sym) {
  size_t whole = S / 64, tail = S % 64, h = tail / 2;
  for (size_t c = 0; c < whole; ++c)
    for (size_t j = 0; j < 32; ++j)
      sym[c * 32 + j] = (uint16_t)(b[c * 64 + j] | (b[c * 64 + 32 + j] << 8));
  for (size_t j = 0; j < h; ++j)
    sym[whole * 32 + j] = (uint16_t)(b[whole * 64 + j] | (b[whole * 64 + h + j] << 8));
}
static void syms_to_shard(const uint16_t *sym, size_t S, uint8_t *b) {
  size_t whole = S / 64, tail = S % 64, h = tail / 2;
  for (size_t c = 0; c < whole; ++c)
    for (size_t j = 0; j < 32; ++j) {
      b[c * 64 + j] = (uint8_t)sym[c * 32 + j];
      b[c * 64 + 32 + j] = (uint8_t)(sym[c * 32 + j] >> 8);
    }
  for (size_t j = 0; j < h; ++j) {
    b[whole * 64 + j] = (uint8_t)sym[whole * 32 + j];
    b[whole * 64 + h + j] = (uint8_t)(sym[whole * 32 + j] >> 8);
  }
}

static size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

int ro_use_high_rate(size_t k, size_t m) {
  if (k > GF_ORDER || m > GF_ORDER) return -1;
  size_t pk = next_pow2(k), pm = next_pow2(m);
  size_t smaller = pk < pm ? pk : pm, larger = k > m ? k : m;
  if (k == 0 || m == 0 || smaller + larger > GF_ORDER) return -1;
  if (pk < pm) return 0;
  if (pk > pm) return 1;
  return k <= m ? 1 : 0;
}

/* orig: k shards of S bytes, contiguous; rec: m shards of S bytes, contiguous. */
int ro_encode(size_t k, size_t m, size_t S, const uint8_t *orig, uint8_t *rec) {
  ensure_tables();
  int hr = ro_use_high_rate(k, m);
  if (hr < 0) return RO_UNSUPPORTED_SHARD_COUNT;
  if (S == 0 || S % 2) return RO_INVALID_SHARD_SIZE;
  size_t nsym = S / 2;
  size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  size_t cover = hr ? k : m;
  size_t rows = ((cover + chunk - 1) / chunk) * chunk;
  if (rows < chunk) rows = chunk;
  uint16_t *w = (uint16_t *)calloc(rows * nsym, sizeof(uint16_t));
  if (!w) return RO_NO_MEMORY;
  for (size_t i = 0; i < k; ++i) shard_to_syms(orig + i * S, S, w + i * nsym);
  if (hr) {
    size_t first = k < chunk ? k : chunk;
    ifft(w, nsym, 0, chunk, first, chunk);
    if (k > chunk) {
      size_t cs = chunk;
      for (; cs + chunk <= k; cs += chunk) {
        ifft(w, nsym, cs, chunk, chunk, cs + chunk);
        xor_rows(w, w + cs * nsym, chunk * nsym);
      }
      size_t last = k % chunk;
      if (last) {
        memset(w + (cs + last) * nsym, 0, (rows - cs - last) * nsym * sizeof(uint16_t));
        ifft(w, nsym, cs, chunk, last, cs + chunk);
        xor_rows(w, w + cs * nsym, chunk * nsym);
      }
    }
    fft(w, nsym, 0, chunk, m, 0);
  } else {
    ifft(w, nsym, 0, chunk, k, 0);
    for (size_t cs = chunk; cs < m; cs += chunk) memcpy(w + cs * nsym, w, chunk * nsym * sizeof(uint16_t));
    size_t cs = 0;
    for (; cs + chunk <= m; cs += chunk) fft(w, nsym, cs, chunk, chunk, cs + chunk);
    if (m % chunk) fft(w, nsym, cs, chunk, m % chunk, cs + chunk);
  }
  for (size_t i = 0; i < m; ++i) syms_to_shard(w + i * nsym, S, rec + i * S);
  free(w);
  return RO_OK;
}

/* locator[x] = log prod_{e erased, e != x} (x + e) for x < n (direct product; equal, as a
 * field element, to the crate's FWHT eval_poly restricted to the transform window -- the
 * factors from erasures outside the window are one constant that cancels). */
static void locator(const uint8_t *erased, size_t n, uint16_t *loc) {
  for (size_t x = 0; x < n; ++x) {
    uint32_t acc = 0;
    for (size_t e = 0; e < n; ++e)
      if (erased[e] && e != x) acc = add_mod(acc, g_log[x ^ e]);
    loc[x] = (uint16_t)acc;
  }
}

/* orig: k shards (absent ones ignored), rec: m shards; present flags 0/1.  Restored
 * originals are written into out (k shards, only the absent ones are touched). */
int ro_decode(size_t k, size_t m, size_t S, const uint8_t *orig, const uint8_t *orig_present,
              const uint8_t *rec, const uint8_t *rec_present, uint8_t *out) {
  ensure_tables();
  int hr = ro_use_high_rate(k, m);
  if (hr < 0) return RO_UNSUPPORTED_SHARD_COUNT;
  if (S == 0 || S % 2) return RO_INVALID_SHARD_SIZE;
  size_t no = 0, nr = 0;
  for (size_t i = 0; i < k; ++i) no += orig_present[i] != 0;
  for (size_t i = 0; i < m; ++i) nr += rec_present[i] != 0;
  if (no + nr < k) return RO_NOT_ENOUGH_SHARDS;
  if (no == k) return RO_OK;
  size_t nsym = S / 2;
  size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  size_t end = hr ? chunk + k : chunk + m;
  size_t W = next_pow2(end);
  uint8_t *erased = (uint8_t *)calloc(W, 1);
  uint16_t *loc = (uint16_t *)malloc(W * sizeof(uint16_t));
  uint16_t *w = (uint16_t *)calloc(W * nsym, sizeof(uint16_t));
  uint16_t *tmp = (uint16_t *)malloc(nsym * sizeof(uint16_t));
  if (!erased || !loc || !w || !tmp) {
    free(erased); free(loc); free(w); free(tmp);
    return RO_NO_MEMORY;
  }
  /* positions: high rate = recovery 0..m, originals chunk+i; low rate = originals 0..k,
   * recovery chunk+i */
  size_t opos = hr ? chunk : 0, rpos = hr ? 0 : chunk;
  for (size_t i = 0; i < k; ++i) erased[opos + i] = !orig_present[i];
  for (size_t i = 0; i < m; ++i) erased[rpos + i] = !rec_present[i];
  if (hr) for (size_t i = m; i < chunk; ++i) erased[i] = 1;
  else for (size_t i = end; i < W; ++i) erased[i] = 1;
  locator(erased, W, loc);
  for (size_t i = 0; i < k; ++i)
    if (orig_present[i]) {
      shard_to_syms(orig + i * S, S, tmp);
      mul_row(w + (opos + i) * nsym, tmp, nsym, loc[opos + i]);
    }
  for (size_t i = 0; i < m; ++i)
    if (rec_present[i]) {
      shard_to_syms(rec + i * S, S, tmp);
      mul_row(w + (rpos + i) * nsym, tmp, nsym, loc[rpos + i]);
    }
  ifft(w, nsym, 0, W, end, 0);
  formal_derivative(w, nsym, W);
  fft(w, nsym, 0, W, hr ? end : k, 0);
  for (size_t i = 0; i < k; ++i)
    if (!orig_present[i]) {
      mul_row(tmp, w + (opos + i) * nsym, nsym, (uint16_t)(GF_MODULUS - loc[opos + i]));
      syms_to_shard(tmp, S, out + i * S);
    }
  free(erased); free(loc); free(w); free(tmp);
  return RO_OK;
}

/* ---- multi-block, multi-thread drivers (CPU baseline) ---- */
typedef struct {
  int decode;
  size_t k, m, S, nblocks;
  const uint8_t *in;
  size_t in_stride;
  uint8_t *out;
  size_t out_stride;
  const uint8_t *orig_present, *rec_present;
  size_t next;
  pthread_mutex_t mu;
  int status;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->nblocks) break;
    int st;
    if (!j->decode) {
      st = ro_encode(j->k, j->m, j->S, j->in + b * j->in_stride, j->out + b * j->out_stride);
    } else {
      const uint8_t *blk = j->in + b * j->in_stride; /* k originals then m recovery */
      st = ro_decode(j->k, j->m, j->S, blk, j->orig_present, blk + j->k * j->S, j->rec_present,
                     j->out + b * j->out_stride);
    }
    if (st) j->status = st;
  }
  return NULL;
}

static int run_blocks(job_t *j, int threads) {
  ensure_tables();
  if (threads < 1) threads = 1;
  pthread_t tid[256];
  if (threads > 256) threads = 256;
  pthread_mutex_init(&j->mu, NULL);
  for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, worker, j);
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  pthread_mutex_destroy(&j->mu);
  return j->status;
}

int ro_encode_blocks(size_t k, size_t m, size_t S, size_t nblocks, const uint8_t *in,
                     size_t in_stride, uint8_t *out, size_t out_stride, int threads) {
  job_t j = {0, k, m, S, nblocks, in, in_stride, out, out_stride, NULL, NULL, 0, {{0}}, 0};
  return run_blocks(&j, threads);
}

/* Each input block holds k originals followed by m recovery shards; one shared pattern. */
int ro_decode_blocks(size_t k, size_t m, size_t S, size_t nblocks, const uint8_t *in,
                     size_t in_stride, const uint8_t *orig_present, const uint8_t *rec_present,
                     uint8_t *out, size_t out_stride, int threads) {
  job_t j = {1, k, m, S, nblocks, in, in_stride, out, out_stride, orig_present, rec_present,
             0, {{0}}, 0};
  return run_blocks(&j, threads);
}
