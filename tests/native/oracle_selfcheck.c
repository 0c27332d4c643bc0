/* Test infrastructure (not part of the library): the C oracle (oracle/rs_oracle.c) and the
 * restated Avx2 engine (oracle/rs_cpu_avx2.c) built with AddressSanitizer and
 * UndefinedBehaviorSanitizer by tests/test_sanitizers.py.  For the reference geometries and
 * random erasure patterns: the two engines' encodes agree byte for byte, each decode restores
 * the originals, and the threaded block entry points match the per-call ones.  Prints "ok". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int ro_encode(size_t k, size_t m, size_t S, const uint8_t *orig, uint8_t *rec);
int ro_decode(size_t k, size_t m, size_t S, const uint8_t *orig, const uint8_t *orig_present,
              const uint8_t *rec, const uint8_t *rec_present, uint8_t *out);
int ro_encode_blocks(size_t k, size_t m, size_t S, size_t nblocks, const uint8_t *in, size_t in_stride,
                     uint8_t *out, size_t out_stride, int threads);
int rb_avx2_available(void);
int rb_encode(size_t k, size_t m, size_t S, const uint8_t *orig, uint8_t *rec);
int rb_decode(size_t k, size_t m, size_t S, const uint8_t *orig, const uint8_t *orig_present, const uint8_t *rec,
              const uint8_t *rec_present, uint8_t *out);

static uint64_t st = 0x5EEDA19Eull;
static uint64_t rnd(void) {
  st += 0x9E3779B97F4A7C15ull;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#define FAIL(...) do { fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); return 1; } while (0)

static int one(size_t k, size_t m, size_t S, int avx) {
  uint8_t *orig = malloc(k * S), *rec = malloc(m * S), *rec2 = malloc(m * S), *out = malloc(k * S);
  uint8_t *op = malloc(k), *rp = malloc(m);
  for (size_t i = 0; i < k * S; ++i) orig[i] = (uint8_t)rnd();
  if (ro_encode(k, m, S, orig, rec)) FAIL("ro_encode %zu:%zu S=%zu", k, m, S);
  if (avx) {
    if (rb_encode(k, m, S, orig, rec2)) FAIL("rb_encode %zu:%zu", k, m);
    if (memcmp(rec, rec2, m * S)) FAIL("avx2 encode differs %zu:%zu S=%zu", k, m, S);
  }
  for (int it = 0; it < 3; ++it) {
    /* random erasures keeping at least k survivors */
    size_t have = 0, lost = 0;
    for (size_t i = 0; i < k; ++i) {
      op[i] = lost < m ? (uint8_t)(rnd() & 1) : 1;
      lost += !op[i];
      have += op[i];
    }
    for (size_t j = 0; j < m; ++j) { rp[j] = 1; have += 1; }
    for (size_t j = 0; j < m && have > k; ++j)
      if (rnd() & 1) { rp[j] = 0; --have; }
    for (int engine = 0; engine <= avx; ++engine) {
      memset(out, 0xEE, k * S);
      for (size_t i = 0; i < k; ++i)
        if (op[i]) memcpy(out + i * S, orig + i * S, S);
      int r = engine ? rb_decode(k, m, S, out, op, rec, rp, out) : ro_decode(k, m, S, out, op, rec, rp, out);
      if (r) FAIL("decode %d rc %d", engine, r);
      if (memcmp(out, orig, k * S)) FAIL("decode %d mismatch %zu:%zu S=%zu", engine, k, m, S);
    }
  }
  free(orig); free(rec); free(rec2); free(out); free(op); free(rp);
  return 0;
}

int main(void) {
  static const size_t geo[][3] = {{32, 32, 1024}, {32, 32, 64}, {16, 4, 128}, {64, 64, 64}, {32, 64, 128},
                                  {32, 33, 64}, {33, 64, 192}, {48, 60, 192}, {17, 32, 2048}, {32, 32, 62}};
  const int avx = rb_avx2_available();
  for (size_t g = 0; g < sizeof geo / sizeof geo[0]; ++g)
    if (one(geo[g][0], geo[g][1], geo[g][2], avx && geo[g][2] % 64 == 0)) return 1;
  /* threaded block entry point vs per-call encode */
  const size_t k = 32, m = 32, S = 256, nb = 9, stride = (k + m) * S;
  uint8_t *blk = malloc(nb * stride), *par = malloc(nb * m * S), *one_rec = malloc(m * S);
  for (size_t i = 0; i < nb * stride; ++i) blk[i] = (uint8_t)rnd();
  if (ro_encode_blocks(k, m, S, nb, blk, stride, par, m * S, 4)) FAIL("encode_blocks");
  for (size_t b = 0; b < nb; ++b) {
    if (ro_encode(k, m, S, blk + b * stride, one_rec)) FAIL("encode");
    if (memcmp(one_rec, par + b * m * S, m * S)) FAIL("encode_blocks block %zu differs", b);
  }
  free(blk); free(par); free(one_rec);
  printf("ok\n");
  return 0;
}
