/*
 * CPU baseline engine: reed-solomon-simd 3.1.0's Avx2 engine restated in C.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/_build/liboracle_rs.so next to the scalar
 * oracle (rs_oracle.c); used by bench.py's cpu_baseline leg and checked against the
 * scalar oracle by tests/test_oracle.py.  The product library never links or calls it.
 *
 * What the crate does per call (the reference calls it once per slice,
 * /root/reference/src/shredder/reed_solomon.rs:96-125 encode, :150-180 decode):
 *   - shards are copied into the engine's work buffer in the crate's chunk layout (per
 *     64-byte chunk: 32 low bytes, then 32 high bytes of 32 GF(2^16) symbols); for shard
 *     sizes that are a multiple of 64 that is the shard's own byte order;
 *   - x ^= y * c is the Avx2 engine's nibble-table multiply: for each constant c (a log
 *     value) a 128-byte table holds, for the 4 nibbles of a symbol, the 16 products' low and
 *     high bytes; 8 vpshufb per 32 symbols (crate engine/engine_avx2.rs + tables.rs mul128,
 *     a 65536 x 128-byte table built once per process);
 *   - encode: the HighRate / LowRate FFT encoders, radix-2 butterflies
 *     (the crate fuses two layers per pass; same arithmetic);
 *   - decode: the erasure locator with the crate's eval_poly (two 65536-point FWHTs per call,
 *     the first truncated at the window end), every received shard multiplied by its
 *     locator value, IFFT, formal derivative, FFT, restored originals times the inverse
 *      -- the per-call cost profile of the crate, not the GPU's shortcuts.
 * Same math as the scalar oracle, so the bytes are identical (checked in tests).
 * Shard sizes that are not a multiple of 64 (tail chunks) are not served: callers fall
 * back to the scalar oracle.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GF_ORDER 65536u
#define GF_MODULUS 65535u

void ro_internal_tables(const uint16_t **exp, const uint16_t **log, const uint16_t **skew,
                        const uint16_t **log_walsh);
int ro_use_high_rate(size_t k, size_t m);

enum { RB_OK = 0, RB_INVALID_SHARD_SIZE = 1, RB_NOT_ENOUGH_SHARDS = 9, RB_UNSUPPORTED = 10, RB_NO_MEMORY = 100,
       RB_NO_AVX2 = 101 };

static const uint16_t *t_exp, *t_log, *t_skew, *t_log_walsh;
static uint8_t (*g_mul128)[4][2][16]; /* [log_m][nibble][lo/hi byte][value] */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static inline uint16_t add_mod(uint32_t x, uint32_t y) {
  uint32_t s = x + y;
  return (uint16_t)(s + (s >> 16));
}
static inline uint16_t sub_mod(uint32_t x, uint32_t y) {
  uint32_t d = x - y;
  return (uint16_t)(d + (d >> 16));
}
static inline uint16_t gf_mul(uint16_t x, uint16_t log_m) {
  return x == 0 ? 0 : t_exp[add_mod(t_log[x], log_m)];
}

static void init(void) {
  ro_internal_tables(&t_exp, &t_log, &t_skew, &t_log_walsh);
  g_mul128 = malloc(sizeof(*g_mul128) * GF_ORDER);
  if (!g_mul128) return;
  for (uint32_t lm = 0; lm < GF_ORDER; ++lm)
    for (int n = 0; n < 4; ++n)
      for (int v = 0; v < 16; ++v) {
        const uint16_t prod = gf_mul((uint16_t)(v << (4 * n)), (uint16_t)lm);
        g_mul128[lm][n][0][v] = (uint8_t)prod;
        g_mul128[lm][n][1][v] = (uint8_t)(prod >> 8);
      }
}
static pthread_key_t g_work_key;
static void free_work(void *p) { free(p); }
static void init_key(void) { pthread_key_create(&g_work_key, free_work); }
static int ready(void) {
  pthread_once(&g_once, init);
  return g_mul128 != NULL;
}

/* Per-thread work buffer, kept across calls like the crate's encoder / decoder work
 * buffers (reset() reuses them): [size_t capacity][64-byte aligned bytes...]. */
static pthread_once_t g_key_once = PTHREAD_ONCE_INIT;
static uint8_t *work_buffer(size_t bytes) {
  pthread_once(&g_key_once, init_key);
  uint8_t *p = pthread_getspecific(g_work_key);
  if (p && *(size_t *)p >= bytes) return p + 64;
  free(p);
  const size_t cap = bytes + (bytes >> 2);
  p = aligned_alloc(64, (cap + 64 + 63) / 64 * 64);
  if (!p) return NULL;
  *(size_t *)p = cap;
  pthread_setspecific(g_work_key, p);
  return p + 64;
}

int rb_avx2_available(void) { return __builtin_cpu_supports("avx2") ? 1 : 0; }

/* ---- row kernels on n bytes (n % 64 == 0), crate chunk layout ---- */
__attribute__((target("avx2"))) static void xor_row(uint8_t *x, const uint8_t *y, size_t n) {
  for (size_t i = 0; i < n; i += 32)
    _mm256_storeu_si256((__m256i *)(x + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(x + i)),
                                                             _mm256_loadu_si256((const __m256i *)(y + i))));
}

/* dst ^= src * c (ACC) or dst = src * c */
__attribute__((target("avx2"))) static inline void mul_row(uint8_t *dst, const uint8_t *src, size_t n, uint16_t lm,
                                                           int acc) {
  const uint8_t(*T)[2][16] = g_mul128[lm];
  const __m256i lo0 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[0][0]));
  const __m256i lo1 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[1][0]));
  const __m256i lo2 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[2][0]));
  const __m256i lo3 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[3][0]));
  const __m256i hi0 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[0][1]));
  const __m256i hi1 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[1][1]));
  const __m256i hi2 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[2][1]));
  const __m256i hi3 = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)T[3][1]));
  const __m256i mask = _mm256_set1_epi8(0x0F);
  for (size_t i = 0; i < n; i += 64) {
    const __m256i ylo = _mm256_loadu_si256((const __m256i *)(src + i));
    const __m256i yhi = _mm256_loadu_si256((const __m256i *)(src + i + 32));
    const __m256i n0 = _mm256_and_si256(ylo, mask), n1 = _mm256_and_si256(_mm256_srli_epi16(ylo, 4), mask);
    const __m256i n2 = _mm256_and_si256(yhi, mask), n3 = _mm256_and_si256(_mm256_srli_epi16(yhi, 4), mask);
    __m256i plo = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(lo0, n0), _mm256_shuffle_epi8(lo1, n1)),
                                   _mm256_xor_si256(_mm256_shuffle_epi8(lo2, n2), _mm256_shuffle_epi8(lo3, n3)));
    __m256i phi = _mm256_xor_si256(_mm256_xor_si256(_mm256_shuffle_epi8(hi0, n0), _mm256_shuffle_epi8(hi1, n1)),
                                   _mm256_xor_si256(_mm256_shuffle_epi8(hi2, n2), _mm256_shuffle_epi8(hi3, n3)));
    if (acc) {
      plo = _mm256_xor_si256(plo, _mm256_loadu_si256((const __m256i *)(dst + i)));
      phi = _mm256_xor_si256(phi, _mm256_loadu_si256((const __m256i *)(dst + i + 32)));
    }
    _mm256_storeu_si256((__m256i *)(dst + i), plo);
    _mm256_storeu_si256((__m256i *)(dst + i + 32), phi);
  }
}

/* ---- FFT / IFFT over rows of n bytes (radix-2; indices relative to pos) ---- */
static void fft(uint8_t *w, size_t n, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = size >> 1; dist >= 1; dist >>= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t_skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint8_t *x = w + (pos + i) * n, *y = w + (pos + i + dist) * n;
        if (lm != GF_MODULUS) mul_row(x, y, n, lm, 1);
        xor_row(y, x, n);
      }
    }
    if (dist == 1) break;
  }
}
static void ifft(uint8_t *w, size_t n, size_t pos, size_t size, size_t trunc, size_t delta) {
  for (size_t dist = 1; dist < size; dist <<= 1) {
    for (size_t r = 0; r < trunc; r += 2 * dist) {
      const uint16_t lm = t_skew[r + dist + delta - 1];
      for (size_t i = r; i < r + dist; ++i) {
        uint8_t *x = w + (pos + i) * n, *y = w + (pos + i + dist) * n;
        xor_row(y, x, n);
        if (lm != GF_MODULUS) mul_row(x, y, n, lm, 1);
      }
    }
  }
}

static size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

/* orig: k shards of S bytes, contiguous; rec: m shards of S bytes, contiguous.  The work
 * buffer is the engine's own (the crate copies shards in and the caller copies parity out). */
int rb_encode(size_t k, size_t m, size_t S, const uint8_t *orig, uint8_t *rec) {
  if (!rb_avx2_available()) return RB_NO_AVX2;
  if (!ready()) return RB_NO_MEMORY;
  const int hr = ro_use_high_rate(k, m);
  if (hr < 0) return RB_UNSUPPORTED;
  if (S == 0 || S % 64) return RB_INVALID_SHARD_SIZE;
  const size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  const size_t cover = hr ? k : m;
  size_t rows = ((cover + chunk - 1) / chunk) * chunk;
  if (rows < chunk) rows = chunk;
  uint8_t *w = work_buffer(rows * S);
  if (!w) return RB_NO_MEMORY;
  memcpy(w, orig, k * S);
  memset(w + k * S, 0, (rows - k) * S);
  if (hr) {
    const size_t first = k < chunk ? k : chunk;
    ifft(w, S, 0, chunk, first, chunk);
    size_t cs = chunk;
    for (; cs + chunk <= k; cs += chunk) {
      ifft(w, S, cs, chunk, chunk, cs + chunk);
      xor_row(w, w + cs * S, chunk * S);
    }
    if (k > chunk && k % chunk) {
      ifft(w, S, cs, chunk, k % chunk, cs + chunk);
      xor_row(w, w + cs * S, chunk * S);
    }
    fft(w, S, 0, chunk, m, 0);
  } else {
    ifft(w, S, 0, chunk, k, 0);
    for (size_t cs = chunk; cs < m; cs += chunk) memcpy(w + cs * S, w, chunk * S);
    size_t cs = 0;
    for (; cs + chunk <= m; cs += chunk) fft(w, S, cs, chunk, chunk, cs + chunk);
    if (m % chunk) fft(w, S, cs, chunk, m % chunk, cs + chunk);
  }
  memcpy(rec, w, m * S);
  return RB_OK;
}

/* crate fwht: radix-2 add/sub-mod Walsh-Hadamard over GF_ORDER entries; groups starting at
 * or beyond `truncated` hold only zeros and are skipped (exact).  Layers with dist >= 16
 * run on 16 u16 lanes: add_mod = wrapping add + end-around carry, sub_mod = wrapping
 * subtract - borrow (the u32 forms' results, 65535 an alias of 0 as in the crate). */
__attribute__((target("avx2"))) static void fwht(uint16_t *d, size_t truncated) {
  for (size_t dist = 1; dist < GF_ORDER; dist <<= 1) {
    if (dist < 16) {  /* both partners in one vector: swap lanes, blend add / sub results */
      const __m256i hi = dist == 1   ? _mm256_set1_epi32((int)0xFFFF0000)
                         : dist == 2 ? _mm256_set1_epi64x((long long)0xFFFFFFFF00000000ull)
                         : dist == 4 ? _mm256_set_epi64x(-1, 0, -1, 0)
                                     : _mm256_set_epi64x(-1, -1, 0, 0);
      for (size_t i = 0; i < (truncated < 16 ? 16 : truncated); i += 16) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(d + i));
        const __m256i w = dist == 1   ? _mm256_or_si256(_mm256_srli_epi32(v, 16), _mm256_slli_epi32(v, 16))
                          : dist == 2 ? _mm256_shuffle_epi32(v, 0xB1)
                          : dist == 4 ? _mm256_shuffle_epi32(v, 0x4E)
                                      : _mm256_permute2x128_si256(v, v, 0x01);
        /* low lanes: a = v, b = w -> a + b;  high lanes: a = w, b = v -> a - b */
        const __m256i s = _mm256_add_epi16(v, w);
        const __m256i carry = _mm256_xor_si256(_mm256_cmpeq_epi16(_mm256_max_epu16(s, v), s), _mm256_set1_epi16(-1));
        const __m256i df = _mm256_sub_epi16(w, v);
        const __m256i borrow = _mm256_xor_si256(_mm256_cmpeq_epi16(_mm256_max_epu16(w, v), w), _mm256_set1_epi16(-1));
        _mm256_storeu_si256((__m256i *)(d + i),
                            _mm256_blendv_epi8(_mm256_sub_epi16(s, carry), _mm256_add_epi16(df, borrow), hi));
      }
      continue;
    }
    for (size_t r = 0; r < truncated; r += 2 * dist)
      for (size_t i = r; i < r + dist; i += 16) {
        const __m256i a = _mm256_loadu_si256((const __m256i *)(d + i));
        const __m256i b = _mm256_loadu_si256((const __m256i *)(d + i + dist));
        const __m256i s = _mm256_add_epi16(a, b);
        const __m256i carry = _mm256_xor_si256(_mm256_cmpeq_epi16(_mm256_max_epu16(s, a), s), _mm256_set1_epi16(-1));
        const __m256i df = _mm256_sub_epi16(a, b);
        const __m256i borrow = _mm256_xor_si256(_mm256_cmpeq_epi16(_mm256_max_epu16(a, b), a), _mm256_set1_epi16(-1));
        _mm256_storeu_si256((__m256i *)(d + i), _mm256_sub_epi16(s, carry));
        _mm256_storeu_si256((__m256i *)(d + i + dist), _mm256_add_epi16(df, borrow));
      }
  }
}
/* crate eval_poly: erasure flags -> locator logs at every position */
__attribute__((target("avx2"))) static void eval_poly(uint16_t *e, size_t truncated) {
  fwht(e, truncated);
  for (size_t i = 0; i < GF_ORDER; ++i) {
    const uint32_t prod = (uint32_t)e[i] * t_log_walsh[i];
    e[i] = add_mod(prod & GF_MODULUS, prod >> 16);
  }
  fwht(e, GF_ORDER);
}

int rb_decode(size_t k, size_t m, size_t S, const uint8_t *orig, const uint8_t *orig_present, const uint8_t *rec,
              const uint8_t *rec_present, uint8_t *out) {
  if (!rb_avx2_available()) return RB_NO_AVX2;
  if (!ready()) return RB_NO_MEMORY;
  const int hr = ro_use_high_rate(k, m);
  if (hr < 0) return RB_UNSUPPORTED;
  if (S == 0 || S % 64) return RB_INVALID_SHARD_SIZE;
  size_t no = 0, nr = 0;
  for (size_t i = 0; i < k; ++i) no += orig_present[i] != 0;
  for (size_t i = 0; i < m; ++i) nr += rec_present[i] != 0;
  if (no + nr < k) return RB_NOT_ENOUGH_SHARDS;
  if (no == k) return RB_OK;
  const size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  const size_t end = hr ? chunk + k : chunk + m;
  const size_t W = next_pow2(end);
  uint8_t *buf = work_buffer(W * S + GF_ORDER * sizeof(uint16_t));
  if (!buf) return RB_NO_MEMORY;
  uint8_t *w = buf;
  uint16_t *e = (uint16_t *)(buf + W * S);
  memset(e, 0, GF_ORDER * sizeof(uint16_t));
  const size_t opos = hr ? chunk : 0, rpos = hr ? 0 : chunk;
  for (size_t i = 0; i < k; ++i) e[opos + i] = !orig_present[i];
  for (size_t i = 0; i < m; ++i) e[rpos + i] = !rec_present[i];
  if (hr) {
    for (size_t i = m; i < chunk; ++i) e[i] = 1;
  } else {
    for (size_t i = end; i < GF_ORDER; ++i) e[i] = 1;
  }
  eval_poly(e, hr ? end : GF_ORDER);
  memset(w, 0, W * S);
  for (size_t i = 0; i < k; ++i)
    if (orig_present[i]) mul_row(w + (opos + i) * S, orig + i * S, S, e[opos + i], 0);
  for (size_t i = 0; i < m; ++i)
    if (rec_present[i]) mul_row(w + (rpos + i) * S, rec + i * S, S, e[rpos + i], 0);
  ifft(w, S, 0, W, end, 0);
  for (size_t i = 1; i < W; ++i) { /* formal derivative */
    const size_t width = i & (~i + 1);
    xor_row(w + (i - width) * S, w + i * S, width * S);
  }
  fft(w, S, 0, W, hr ? end : k, 0);
  for (size_t i = 0; i < k; ++i)
    if (!orig_present[i]) mul_row(out + i * S, w + (opos + i) * S, S, (uint16_t)(GF_MODULUS - e[opos + i]), 0);
  return RB_OK;
}

/* ---- multi-block drivers: one block per task over POSIX threads ---- */
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
    const size_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->nblocks) break;
    int st;
    if (!j->decode) {
      st = rb_encode(j->k, j->m, j->S, j->in + b * j->in_stride, j->out + b * j->out_stride);
    } else {
      const uint8_t *blk = j->in + b * j->in_stride; /* k originals then m recovery */
      st = rb_decode(j->k, j->m, j->S, blk, j->orig_present, blk + j->k * j->S, j->rec_present,
                     j->out + b * j->out_stride);
    }
    if (st) j->status = st;
  }
  return NULL;
}

static int run_blocks(job_t *j, int threads) {
  if (!ready()) return RB_NO_MEMORY;
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  pthread_mutex_init(&j->mu, NULL);
  for (int t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, worker, j);
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  pthread_mutex_destroy(&j->mu);
  return j->status;
}

int rb_encode_blocks(size_t k, size_t m, size_t S, size_t nblocks, const uint8_t *in, size_t in_stride, uint8_t *out,
                     size_t out_stride, int threads) {
  job_t j = {0, k, m, S, nblocks, in, in_stride, out, out_stride, NULL, NULL, 0, {{0}}, 0};
  return run_blocks(&j, threads);
}

int rb_decode_blocks(size_t k, size_t m, size_t S, size_t nblocks, const uint8_t *in, size_t in_stride,
                     const uint8_t *orig_present, const uint8_t *rec_present, uint8_t *out, size_t out_stride,
                     int threads) {
  job_t j = {1, k, m, S, nblocks, in, in_stride, out, out_stride, orig_present, rec_present, 0, {{0}}, 0};
  return run_blocks(&j, threads);
}
