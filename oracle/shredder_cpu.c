/*
 * CPU baseline of the composed RegularShredder -- TEST INFRASTRUCTURE ONLY (a "port").
 *
 * bench_shredder.py's cpu_baseline leg times this next to the device path; tests check it
 * against oracle/shredder_oracle.py.  The product library never links or calls it.
 *
 * What the reference's own benchmark times per maximum slice (/root/reference/benches/
 * shredder.rs:19-61, RegularShredder):
 *   shred   (shredder.rs:337-345, :533-611): Slice::payload_bytes (types/slice.rs:73-84),
 *           ReedSolomonCoder::shred (reed_solomon.rs:88-128: 0x80 00.. padding, 32 x 1 KiB
 *           data shards, 32 coding shards), build_merkle_tree over the 64 raw shreds
 *           (merkle.rs:281-333: labelled SHA-256 leaves and pairs), the leader's Ed25519
 *           signature of SliceCommitment(header, root) (shredder.rs:206-222), and one output
 *           shred per index with the header, signature and tree.create_proof(j);
 *   deshred (shredder.rs:282-311) from the 32 coding shreds: ReedSolomonCoder::deshred
 *           (decode, padding strip, re-encode of every coding shard: reed_solomon.rs:140-231),
 *           check_merkle_tree (rebuild + root compare), SlicePayload::try_from, and the 32
 *           missing shreds filled in with their proofs.
 * The receive side in front of deshred (ValidatedShred::try_new, validated_shred.rs:52-81:
 * each arriving shred's root derived from its Merkle path, the first one's signature
 * verified, the others compared with the cached commitment) is timed separately, because
 * the device's composed deshred (ag_shredder_deshred_batch) includes it.
 *
 * Arithmetic: Reed-Solomon by rs_cpu_avx2.c (the crate's Avx2 engine restated); SHA-256 and
 * Ed25519 by OpenSSL's libcrypto (SHA-NI / assembly SHA-256, its Ed25519: a production
 * CPU implementation standing in for the reference's sha2 / ed25519 crates).  Ed25519
 * signatures are deterministic (RFC 8032), so the CPU's signatures equal the device's.
 */
#define _GNU_SOURCE
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int rb_encode(size_t k, size_t m, size_t S, const uint8_t *orig, uint8_t *rec);
int rb_decode(size_t k, size_t m, size_t S, const uint8_t *orig, const uint8_t *orig_present, const uint8_t *rec,
              const uint8_t *rec_present, uint8_t *out);

enum { DATA = 32, TOTAL = 64, S_MAX = 1024, HEIGHT = 6, NODES = 127 };

static const char LEAF_LABEL[33] = "ALPENGLOW-MERKLE-TREE  LEAF-NODE";
static const char LEFT_LABEL[33] = "ALPENGLOW-MERKLE-TREE  LEFT-NODE";
static const char RIGHT_LABEL[33] = "ALPENGLOW-MERKLE-TREE RIGHT-NODE";

/* ---- Merkle tree of a 64-leaf slice (merkle.rs:281-333, 351-370, 411-428, 457-468) ---- */
static void hash_leaf(const uint8_t *data, size_t len, uint8_t out[32]) {
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, LEAF_LABEL, 32);
  SHA256_Update(&c, data, len);
  SHA256_Final(out, &c);
}
/* (the low-level SHA256_* calls: OpenSSL 3's one-shot SHA256() goes through an EVP fetch under a
 * process-wide lock, which serialised the threads) */
static void hash_pair(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
  uint8_t buf[128];
  memcpy(buf, LEFT_LABEL, 32);
  memcpy(buf + 32, l, 32);
  memcpy(buf + 64, RIGHT_LABEL, 32);
  memcpy(buf + 96, r, 32);
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, buf, sizeof buf);
  SHA256_Final(out, &c);
}
/* nodes[0..63] leaves, then 32, 16, 8, 4, 2, 1: a power-of-two leaf count never pairs with
 * an EMPTY_ROOTS entry; nodes[126] is the root */
static void build_tree(const uint8_t *shreds, size_t S, uint8_t nodes[NODES][32]) {
  for (int j = 0; j < TOTAL; ++j) hash_leaf(shreds + (size_t)j * S, S, nodes[j]);
  int in = 0, out = TOTAL;
  for (int len = TOTAL; len > 1; len /= 2) {
    for (int i = 0; i < len; i += 2) hash_pair(nodes[in + i], nodes[in + i + 1], nodes[out + i / 2]);
    in = out;
    out += len / 2;
  }
}
static void create_proof(uint8_t nodes[NODES][32], int j, uint8_t proof[HEIGHT][32]) {
  int base = 0, len = TOTAL;
  for (int h = 0; h < HEIGHT; ++h) {
    memcpy(proof[h], nodes[base + (j ^ 1)], 32);
    base += len;
    len /= 2;
    j >>= 1;
  }
}
static void derive_root(const uint8_t *data, size_t S, int j, uint8_t proof[HEIGHT][32], uint8_t root[32]) {
  uint8_t node[32];
  hash_leaf(data, S, node);
  for (int h = 0; h < HEIGHT; ++h, j >>= 1) {
    if (j & 1) hash_pair(proof[h], node, node);
    else hash_pair(node, proof[h], node);
  }
  memcpy(root, node, 32);
}

/* SliceCommitment::new (shredder.rs:206-215): slot u64 LE, slice index u64 LE, is_last, root */
static size_t commitment(uint64_t slot, uint64_t slice_index, int is_last, const uint8_t root[32], uint8_t out[49]) {
  for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(slot >> (8 * i));
  for (int i = 0; i < 8; ++i) out[8 + i] = (uint8_t)(slice_index >> (8 * i));
  out[16] = is_last ? 1 : 0;
  memcpy(out + 17, root, 32);
  return 49;
}

/* ---- per-thread state ---- */
typedef struct {
  EVP_PKEY *sk, *pk;
  EVP_MD_CTX *md, *sign_tmpl, *verify_tmpl;
  uint8_t cw[TOTAL * S_MAX];            /* 32 data then 32 coding shards */
  uint8_t nodes[NODES][32];
  uint8_t proofs[TOTAL][HEIGHT][32];    /* the output shreds' Merkle paths */
} worker_t;

/* OpenSSL 3 fetches the signature implementation on every EVP_Digest{Sign,Verify}Init under a
 * process-wide lock (16 threads signed slower than one); each worker initialises one signing
 * and one verifying context once and copies them per call. */
static int worker_init(worker_t *w, const uint8_t seed[32], const uint8_t pk[32]) {
  w->sk = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seed, 32);
  w->pk = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pk, 32);
  w->md = EVP_MD_CTX_new();
  w->sign_tmpl = EVP_MD_CTX_new();
  w->verify_tmpl = EVP_MD_CTX_new();
  if (!w->sk || !w->pk || !w->md || !w->sign_tmpl || !w->verify_tmpl) return -1;
  if (EVP_DigestSignInit(w->sign_tmpl, NULL, NULL, NULL, w->sk) != 1) return -1;
  if (EVP_DigestVerifyInit(w->verify_tmpl, NULL, NULL, NULL, w->pk) != 1) return -1;
  return 0;
}
static void worker_free(worker_t *w) {
  EVP_PKEY_free(w->sk);
  EVP_PKEY_free(w->pk);
  EVP_MD_CTX_free(w->md);
  EVP_MD_CTX_free(w->sign_tmpl);
  EVP_MD_CTX_free(w->verify_tmpl);
}
static int ed_sign(worker_t *w, const uint8_t *msg, size_t len, uint8_t sig[64]) {
  size_t sl = 64;
  if (EVP_MD_CTX_copy_ex(w->md, w->sign_tmpl) != 1) return -1;
  return EVP_DigestSign(w->md, sig, &sl, msg, len) == 1 && sl == 64 ? 0 : -1;
}
static int ed_verify(worker_t *w, const uint8_t *msg, size_t len, const uint8_t sig[64]) {
  if (EVP_MD_CTX_copy_ex(w->md, w->verify_tmpl) != 1) return -1;
  return EVP_DigestVerify(w->md, sig, 64, msg, len) == 1 ? 0 : -1;
}

/* RegularShredder::shred of one slice whose framed payload is `payload` (len <= 32767):
 * coding shards, root and signature out (the raw shreds stay in w->cw, the proofs in
 * w->proofs).  Returns the shred size or -1. */
static long shred_one(worker_t *w, const uint8_t *payload, size_t len, uint64_t slot, uint64_t slice_index,
                      int is_last, uint8_t root[32], uint8_t sig[64]) {
  if (len > DATA * S_MAX - 1) return -1;
  const size_t padding = 2 * DATA - len % (2 * DATA), S = (len + padding) / DATA;
  if (S % 64) return -1; /* the Avx2 port serves whole 64-byte chunks (maximum slices: S = 1024) */
  memcpy(w->cw, payload, len);
  w->cw[len] = 0x80;
  memset(w->cw + len + 1, 0, padding - 1);
  if (rb_encode(DATA, TOTAL - DATA, S, w->cw, w->cw + DATA * S)) return -1;
  build_tree(w->cw, S, w->nodes);
  memcpy(root, w->nodes[NODES - 1], 32);
  uint8_t msg[49];
  if (ed_sign(w, msg, commitment(slot, slice_index, is_last, root, msg), sig)) return -1;
  for (int j = 0; j < TOTAL; ++j) create_proof(w->nodes, j, w->proofs[j]);
  return (long)S;
}

/* Shredder::deshred of one slice from its 32 coding shreds (the reference bench's shape):
 * w->cw holds the coding shards at DATA * S (the data region is garbage).  Returns the
 * payload length, or -1 (bad padding / Merkle mismatch / framing). */
static long deshred_one(worker_t *w, size_t S, const uint8_t root[32]) {
  static const uint8_t none[DATA] = {0};
  uint8_t all[TOTAL - DATA];
  memset(all, 1, sizeof all);
  /* ReedSolomonCoder::deshred: decode, then strip the padding, then re-encode all coding */
  if (rb_decode(DATA, TOTAL - DATA, S, w->cw, none, w->cw + DATA * S, all, w->cw)) return -1;
  const size_t total = DATA * S;
  size_t z = 0;
  while (z < total && w->cw[total - 1 - z] == 0) ++z;
  if (z == total || w->cw[total - 1 - z] != 0x80) return -1;
  const size_t plen = total - 1 - z;
  if (rb_encode(DATA, TOTAL - DATA, S, w->cw, w->cw + DATA * S)) return -1;
  /* check_merkle_tree */
  build_tree(w->cw, S, w->nodes);
  if (memcmp(w->nodes[NODES - 1], root, 32)) return -1;
  /* SlicePayload::try_from (slice.rs:211-218): tag, optional BlockId, u64 length, data */
  if (plen < 9 || w->cw[0] > 1) return -1;
  const size_t off = w->cw[0] ? 41 : 1;
  uint64_t dl = 0;
  for (int i = 0; i < 8; ++i) dl |= (uint64_t)w->cw[off + i] << (8 * i);
  if (off + 8 + dl != plen) return -1;
  /* fill_missing_shreds: the 32 data shreds' proofs */
  for (int j = 0; j < DATA; ++j) create_proof(w->nodes, j, w->proofs[j]);
  return (long)plen;
}

/* ValidatedShred::try_new for the 32 arriving coding shreds of one slice: each one's root
 * derived from its path, the first one's signature verified, the others compared with the
 * cached commitment.  Returns 0 when all are valid. */
static int receive_one(worker_t *w, size_t S, uint64_t slot, uint64_t slice_index, int is_last, const uint8_t sig[64]) {
  uint8_t cached[49], msg[49], r[32];
  for (int j = DATA; j < TOTAL; ++j) {
    derive_root(w->cw + (size_t)j * S, S, j, w->proofs[j], r);
    commitment(slot, slice_index, is_last, r, msg);
    if (j == DATA) {
      if (ed_verify(w, msg, 49, sig)) return -1;
      memcpy(cached, msg, 49);
    } else if (memcmp(msg, cached, 49)) {
      return -1;
    }
  }
  return 0;
}

/* ---- batch driver: slices over threads ---- */
typedef struct {
  size_t n, S;
  const uint8_t *payloads; /* n x stride framed payloads */
  size_t stride;
  const uint32_t *lens;
  const uint64_t *slots, *slice_idx;
  const uint8_t *is_last;
  const uint8_t *seed, *pk;
  uint8_t *coding_out; /* n x 32 x S (optional) */
  uint8_t *roots, *sigs; /* n x 32, n x 64 (optional) */
  int what;             /* 1 shred, 2 + deshred, 4 + receive */
  size_t next;
  pthread_mutex_t mu;
  int status;
} sjob_t;

static void *sworker(void *arg) {
  sjob_t *j = arg;
  worker_t *w = malloc(sizeof *w);
  if (!w || worker_init(w, j->seed, j->pk)) {
    pthread_mutex_lock(&j->mu);
    j->status = -1;
    pthread_mutex_unlock(&j->mu);
    if (w) worker_free(w);
    free(w);
    return NULL;
  }
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const size_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->n) break;
    uint8_t root[32], sig[64];
    const long S = shred_one(w, j->payloads + b * j->stride, j->lens[b], j->slots[b], j->slice_idx[b], j->is_last[b],
                             root, sig);
    int bad = S < 0;
    if (!bad && j->coding_out) memcpy(j->coding_out + b * DATA * (size_t)S, w->cw + DATA * (size_t)S, DATA * (size_t)S);
    if (!bad && j->roots) memcpy(j->roots + 32 * b, root, 32);
    if (!bad && j->sigs) memcpy(j->sigs + 64 * b, sig, 64);
    if (!bad && (j->what & 4)) bad = receive_one(w, (size_t)S, j->slots[b], j->slice_idx[b], j->is_last[b], sig) != 0;
    if (!bad && (j->what & 2)) {
      memset(w->cw, 0xA5, DATA * (size_t)S); /* the data shreds did not arrive */
      bad = deshred_one(w, (size_t)S, root) != (long)j->lens[b];
    }
    if (bad) {
      pthread_mutex_lock(&j->mu);
      j->status = -2;
      pthread_mutex_unlock(&j->mu);
    }
  }
  worker_free(w);
  free(w);
  return NULL;
}

/* Shred (what & 1, always), then receive (what & 4) and deshred (what & 2) n slices on
 * `threads` threads, one slice per task.  Optional outputs of the shred: coding shards, roots,
 * signatures.  Returns 0, or < 0 on any failure (a round trip that did not restore the payload
 * length). */
int sc_run(int what, int threads, size_t n, const uint8_t *payloads, size_t stride, const uint32_t *lens,
           const uint64_t *slots, const uint64_t *slice_idx, const uint8_t *is_last, const uint8_t seed[32],
           const uint8_t pk[32], uint8_t *coding_out, uint8_t *roots, uint8_t *sigs) {
  sjob_t j = {n, 0, payloads, stride, lens, slots, slice_idx, is_last, seed, pk, coding_out, roots, sigs, what | 1, 0,
              PTHREAD_MUTEX_INITIALIZER, 0};
  if (threads < 1) threads = 1;
  pthread_t *t = malloc(sizeof(pthread_t) * (size_t)threads);
  if (!t) return -1;
  int started = 0;
  for (int i = 0; i < threads; ++i)
    if (pthread_create(&t[i], NULL, sworker, &j) == 0) ++started;
  for (int i = 0; i < started; ++i) pthread_join(t[i], NULL);
  free(t);
  return started ? j.status : -1;
}

/* The phases of one slice timed separately on one thread (the reference bench's two
 * functions and the receive side): microseconds per slice, averaged over `reps`. */
int sc_phase_us(int reps, const uint8_t *payload, size_t len, const uint8_t seed[32], const uint8_t pk[32],
                double out_us[3]) {
  worker_t *w = malloc(sizeof *w);
  if (!w || worker_init(w, seed, pk)) {
    free(w);
    return -1;
  }
  struct timespec a, b;
  double t[3] = {0, 0, 0};
  int st = 0;
  for (int r = 0; r < reps && !st; ++r) {
    uint8_t root[32], sig[64];
    clock_gettime(CLOCK_MONOTONIC, &a);
    const long S = shred_one(w, payload, len, 7, 3, 0, root, sig);
    clock_gettime(CLOCK_MONOTONIC, &b);
    t[0] += (b.tv_sec - a.tv_sec) * 1e6 + (b.tv_nsec - a.tv_nsec) * 1e-3;
    if (S < 0) {
      st = -2;
      break;
    }
    clock_gettime(CLOCK_MONOTONIC, &a);
    st = receive_one(w, (size_t)S, 7, 3, 0, sig) ? -3 : 0;
    clock_gettime(CLOCK_MONOTONIC, &b);
    t[2] += (b.tv_sec - a.tv_sec) * 1e6 + (b.tv_nsec - a.tv_nsec) * 1e-3;
    memset(w->cw, 0xA5, DATA * (size_t)S);
    clock_gettime(CLOCK_MONOTONIC, &a);
    if (!st && deshred_one(w, (size_t)S, root) != (long)len) st = -4;
    clock_gettime(CLOCK_MONOTONIC, &b);
    t[1] += (b.tv_sec - a.tv_sec) * 1e6 + (b.tv_nsec - a.tv_nsec) * 1e-3;
  }
  for (int i = 0; i < 3; ++i) out_us[i] = t[i] / reps;
  worker_free(w);
  free(w);
  return st;
}
