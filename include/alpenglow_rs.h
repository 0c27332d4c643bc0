/*
 * alpenglow_rs.h -- C ABI of the MI355X Reed-Solomon shredder library (libalpenglow_rs.so).
 *
 * Drop-in boundary for the reference's erasure-coding path.  The reference shredder
 * (/root/reference/src/shredder/reed_solomon.rs) gets its arithmetic from the crate
 * reed-solomon-simd 3.1.0 (GF(2^16) Leopard additive-FFT codec).  This library replaces
 * those crate calls with HIP kernels for gfx950; the Rust side keeps its public API
 * (Shredder trait, disseminator, repair unchanged).  INTEGRATION.md shows the Rust
 * facade a maintainer would add over these symbols.
 *
 * Four layers, each mirroring one reference interface:
 *   1. ag_rs_encoder_* / ag_rs_decoder_*  -- the crate API the wrapper calls
 *      (ReedSolomonEncoder / ReedSolomonDecoder, reed_solomon.rs:9,64-66,96-125,150-180,214-226)
 *   2. ag_rs_coder_*   -- ReedSolomonCoder (reed_solomon.rs:47-232): padding, split,
 *      reassembly, padding strip, re-encode
 *   3. ag_rs_encode_batch / ag_rs_decode_batch -- batched, device-resident forms of 1.
 *      (the GPU-shaped entry points: many blocks per launch)
 *   4. context / stream / utility
 *   5. ag_merkle_*     -- the slice Merkle tree over the shreds (crypto/merkle.rs,
 *      shredder.rs:628-632), batched on the device
 *   6. ag_aon_* / ag_cipher_* / ag_sha256_* -- the AONT / PETS shredders' payload
 *      transforms (shredder.rs:403-528, crypto/cipher.rs, crypto/hash.rs)
 *   7. ag_ed25519_* / ag_shred_validate_batch / ag_slice_sign_batch -- the leader's slice
 *      signatures (crypto/signature.rs over ed25519-zebra 4.2.0) and the per-shred check
 *      ValidatedShred::try_new (shredder/validated_shred.rs:52-81)
 *   8. ag_shred_serialize_batch / ag_shred_deserialize_batch -- the Shred datagram
 *      (shredder.rs:113-186 encoded by wincode 0.6; network.rs:52-64)
 *
 * Conventions: the caller owns every buffer; the library borrows them for the call
 * (reed_solomon.rs copies out of the crate's borrowed results, :118,125,187,226).  A
 * context binds one device and one HIP stream; it is not thread-safe, like a
 * ReedSolomonCoder checked out of ShredderPool (pool.rs:33-93).  Encoders, decoders and
 * coders made with *_new_on_device own a private context each, so they may run
 * concurrently on different threads (the reference builds its coders on one thread and
 * drives them from separate tokio tasks, consensus.rs:180-266); those made with *_new on a
 * shared context must not be used concurrently with anything else on it.  Calls fail loudly
 * (AG_RS_ERR_NO_DEVICE / AG_RS_ERR_DEVICE) when no GPU is usable: there is no CPU
 * fallback.  On error, caller-visible outputs are left untouched (shredder.rs:274).
 */
#ifndef ALPENGLOW_RS_H
#define ALPENGLOW_RS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AG_RS_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------------------
 * 1..10 mirror reed_solomon_simd::Error (crate error.rs; the wrapper .expect()s them,
 * reed_solomon.rs:65,67,98,116,124,152,159,164,166).  20..22 are the wrapper's own
 * errors (ReedSolomonShredError / ReedSolomonDeshredError, reed_solomon.rs:18-32, and
 * DeshredError::InvalidLayout, shredder.rs:75). */
enum {
  AG_RS_OK = 0,
  AG_RS_ERR_INVALID_SHARD_SIZE = 1,           /* Error::InvalidShardSize (0 or odd) */
  AG_RS_ERR_DIFFERENT_SHARD_SIZE = 2,         /* Error::DifferentShardSize */
  AG_RS_ERR_TOO_FEW_ORIGINAL_SHARDS = 3,      /* Error::TooFewOriginalShards */
  AG_RS_ERR_TOO_MANY_ORIGINAL_SHARDS = 4,     /* Error::TooManyOriginalShards */
  AG_RS_ERR_INVALID_ORIGINAL_SHARD_INDEX = 5, /* Error::InvalidOriginalShardIndex */
  AG_RS_ERR_INVALID_RECOVERY_SHARD_INDEX = 6, /* Error::InvalidRecoveryShardIndex */
  AG_RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX = 7,
  AG_RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX = 8,
  AG_RS_ERR_NOT_ENOUGH_SHARDS = 9,            /* Error::NotEnoughShards / NotEnoughShreds */
  AG_RS_ERR_UNSUPPORTED_SHARD_COUNT = 10,     /* Error::UnsupportedShardCount */
  AG_RS_ERR_TOO_MUCH_DATA = 20,               /* TooMuchData (reed_solomon.rs:20,29) */
  AG_RS_ERR_INVALID_PADDING = 21,             /* InvalidPadding (reed_solomon.rs:31) */
  AG_RS_ERR_INVALID_LAYOUT = 22,              /* DeshredError::InvalidLayout (shredder.rs:75) */
  AG_RS_ERR_BAD_ENCODING = 23,                /* DeshredError::BadEncoding (decrypt_payload, shredder.rs:518) */
  AG_RS_ERR_INVALID_MERKLE_TREE = 24,         /* DeshredError::InvalidMerkleTree (shredder.rs:616-625) */
  AG_RS_ERR_INVALID_ARGUMENT = 100,
  AG_RS_ERR_NO_DEVICE = 101,                  /* no usable GPU: never a CPU fallback */
  AG_RS_ERR_DEVICE = 102,                     /* HIP runtime / kernel launch failure */
  AG_RS_ERR_OUT_OF_MEMORY = 103,
  AG_RS_ERR_NOT_RESTORED = 104                /* restored_original(i) == None */
};

/* Where the buffers of a batch call live. */
enum { AG_RS_MEM_DEVICE = 0, AG_RS_MEM_HOST = 1 };

/* Decode modes for ag_rs_decode_batch.
 * EXACT: the crate's decoder on every present shard (bit-identical to the crate for
 *        any input, consistent or not).
 * ANY_K: any k present shards suffice; uses the bitsliced kernel when a block's full
 *        recovery set is present.  Bit-identical to EXACT on every valid codeword (MDS:
 *        the originals are unique) -- the only inputs the reference's Merkle check
 *        accepts (shredder.rs:301-303). */
enum { AG_RS_DECODE_EXACT = 0, AG_RS_DECODE_ANY_K = 1 };

const char* ag_rs_status_string(int status);
int ag_rs_abi_version(void);

/* ---- 4. context --------------------------------------------------------------------- */
typedef struct ag_rs_ctx ag_rs_ctx;

int ag_rs_ctx_create(int device, ag_rs_ctx** out);
void ag_rs_ctx_destroy(ag_rs_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch's current stream).  NULL is the HIP
 * null stream; ag_rs_ctx_reset_stream returns to the context's own stream (created
 * blocking, so it is ordered with the null stream). */
int ag_rs_ctx_set_stream(ag_rs_ctx* ctx, void* hip_stream);
int ag_rs_ctx_reset_stream(ag_rs_ctx* ctx);
void* ag_rs_ctx_stream(ag_rs_ctx* ctx);
int ag_rs_ctx_synchronize(ag_rs_ctx* ctx);
int ag_rs_device_count(int* count);

/* Crate rate rule (rate.rs use_high_rate): 1 HighRate, 0 LowRate, <0 -status. */
int ag_rs_use_high_rate(size_t original_count, size_t recovery_count);
/* 1 when the bitsliced (HBM-bound) kernels serve this geometry, else 0 (generic kernel). */
int ag_rs_has_fast_path(size_t original_count, size_t recovery_count, size_t shard_bytes);

/* ---- 3. batched, device-resident ----------------------------------------------------
 * Block b's original shard i is read at original + b*original_block_stride + i*shard_bytes;
 * recovery shard j at recovery + b*recovery_block_stride + j*shard_bytes.
 * AG_RS_MEM_DEVICE: asynchronous on the context stream.  AG_RS_MEM_HOST: staged through
 * pinned buffers, synchronous. */
int ag_rs_encode_batch(ag_rs_ctx* ctx, size_t original_count, size_t recovery_count,
                       size_t shard_bytes, size_t nblocks, const uint8_t* original,
                       size_t original_block_stride, uint8_t* recovery,
                       size_t recovery_block_stride, int memory);

/* Restores the absent originals of every block in place (present ones untouched).
 * original_present / recovery_present are HOST arrays of 0/1 flags,
 * [npatterns][original_count] and [npatterns][recovery_count]; npatterns is 1 (one
 * pattern for the whole batch) or nblocks (pattern b for block b). */
int ag_rs_decode_batch(ag_rs_ctx* ctx, size_t original_count, size_t recovery_count,
                       size_t shard_bytes, size_t nblocks, uint8_t* original,
                       size_t original_block_stride, const uint8_t* recovery,
                       size_t recovery_block_stride, const uint8_t* original_present,
                       const uint8_t* recovery_present, size_t npatterns, int mode,
                       int memory);

/* Synthetic input: splitmix64 u64 LE words, block b seeded seed_base + b. */
int ag_rs_fill_splitmix(ag_rs_ctx* ctx, uint8_t* device_dst, size_t nblocks, size_t block_bytes,
                        size_t dst_block_stride, uint64_t seed_base);

/* ---- 1. crate API mirror (one codeword, host memory) --------------------------------
 * ReedSolomonEncoder::{new,reset,add_original_shard,encode} + EncoderResult::recovery_iter */
typedef struct ag_rs_encoder ag_rs_encoder;
int ag_rs_encoder_new(ag_rs_ctx* ctx, size_t original_count, size_t recovery_count,
                      size_t shard_bytes, ag_rs_encoder** out);
int ag_rs_encoder_reset(ag_rs_encoder* enc, size_t original_count, size_t recovery_count,
                        size_t shard_bytes);
int ag_rs_encoder_add_original_shard(ag_rs_encoder* enc, const uint8_t* shard, size_t len);
int ag_rs_encoder_encode(ag_rs_encoder* enc);
/* Borrowed view of recovery shard `index` after encode (valid until the next reset). */
int ag_rs_encoder_recovery(const ag_rs_encoder* enc, size_t index, const uint8_t** shard,
                           size_t* len);
void ag_rs_encoder_free(ag_rs_encoder* enc);
/* ReedSolomonEncoder::new on a private context of `device` (created here, destroyed by
 * ag_rs_encoder_free): no state shared with any other object. */
int ag_rs_encoder_new_on_device(int device, size_t original_count, size_t recovery_count,
                                size_t shard_bytes, ag_rs_encoder** out);

/* ReedSolomonDecoder::{new,reset,add_original_shard,add_recovery_shard,decode} +
 * DecoderResult::restored_original (AG_RS_ERR_NOT_RESTORED for None). */
typedef struct ag_rs_decoder ag_rs_decoder;
int ag_rs_decoder_new(ag_rs_ctx* ctx, size_t original_count, size_t recovery_count,
                      size_t shard_bytes, ag_rs_decoder** out);
int ag_rs_decoder_reset(ag_rs_decoder* dec, size_t original_count, size_t recovery_count,
                        size_t shard_bytes);
int ag_rs_decoder_add_original_shard(ag_rs_decoder* dec, size_t index, const uint8_t* shard,
                                     size_t len);
int ag_rs_decoder_add_recovery_shard(ag_rs_decoder* dec, size_t index, const uint8_t* shard,
                                     size_t len);
int ag_rs_decoder_decode(ag_rs_decoder* dec);
int ag_rs_decoder_restored_original(const ag_rs_decoder* dec, size_t index,
                                    const uint8_t** shard, size_t* len);
void ag_rs_decoder_free(ag_rs_decoder* dec);
/* ReedSolomonDecoder::new on a private context of `device` (destroyed by ag_rs_decoder_free). */
int ag_rs_decoder_new_on_device(int device, size_t original_count, size_t recovery_count,
                                size_t shard_bytes, ag_rs_decoder** out);

/* ---- 2. ReedSolomonCoder mirror (reed_solomon.rs:47-232) ----------------------------- */
#define AG_RS_DATA_SHREDS 32                 /* shredder.rs:43 */
#define AG_RS_TOTAL_SHREDS 64                /* shredder.rs:48 */
#define AG_RS_MAX_DATA_PER_SHRED 1024        /* shredder.rs:50 */
#define AG_RS_MAX_DATA_PER_SLICE (AG_RS_DATA_SHREDS * AG_RS_MAX_DATA_PER_SHRED - 1)

typedef struct ag_rs_coder ag_rs_coder;
/* ReedSolomonCoder::new(num_coding) -- 32 data shreds, num_coding <= 64. */
int ag_rs_coder_new(ag_rs_ctx* ctx, size_t num_coding, ag_rs_coder** out);
void ag_rs_coder_free(ag_rs_coder* coder);
/* ReedSolomonCoder::new on a private context of `device` (its encoder and decoder share it;
 * destroyed by ag_rs_coder_free): one per ShredderPool entry (pool.rs:33-93). */
int ag_rs_coder_new_on_device(int device, size_t num_coding, ag_rs_coder** out);
/* The coder's num_coding (the coding_out capacity ag_rs_coder_shred / _deshred fill is
 * num_coding * shred bytes): lets bindings size their buffers from the coder itself. */
int ag_rs_coder_num_coding(const ag_rs_coder* coder, size_t* out);

/* ReedSolomonCoder::shred: pads payload with 0x80 00.. to a multiple of 64 bytes, splits
 * it into 32 shards of *shred_bytes and encodes num_coding coding shards.  data_out must
 * hold 32 * 1024 bytes, coding_out num_coding * 1024; shards are packed with stride
 * *shred_bytes.  Errors: AG_RS_ERR_TOO_MUCH_DATA (payload_len > 32767). */
int ag_rs_coder_shred(ag_rs_coder* coder, const uint8_t* payload, size_t payload_len,
                      uint8_t* data_out, uint8_t* coding_out, size_t* shred_bytes);

/* Shredder::deshred + ReedSolomonCoder::deshred for one slice.  shreds[i] (i < 64) is
 * NULL when absent; shreds 0..data_shreds-1 are data shreds (original index i), the rest
 * coding shreds (recovery index i - data_shreds) -- validated_shreds.rs:87-114.
 * shred_is_data (optional, 64 flags) is checked against that layout and shred_lens must
 * all be equal, non-zero and even (validated_shreds.rs:34-70).  Outputs: payload
 * (<= 32767 bytes), all 32 data shards and num_coding re-encoded coding shards (packed,
 * stride *shred_bytes).  Errors: NOT_ENOUGH_SHARDS, INVALID_LAYOUT, TOO_MUCH_DATA,
 * INVALID_PADDING -- outputs untouched on error. */
int ag_rs_coder_deshred(ag_rs_coder* coder, size_t data_shreds, const uint8_t* const* shreds,
                        const size_t* shred_lens, const uint8_t* shred_is_data,
                        uint8_t* payload_out, size_t* payload_len, uint8_t* data_out,
                        uint8_t* coding_out, size_t* shred_bytes);

/* ---- 2b. ReedSolomonCoder over batches of slices (device-resident) -------------------
 * All slices of a call share one shred size S (even, <= 1024).  Slice b's codeword is 32
 * data shards then num_coding coding shards, contiguous, at codewords + b*codeword_stride
 * (stride >= (32 + num_coding) * S).  A batch form of reed_solomon.rs:88-128 / :140-208 for
 * callers holding many slices (block production, repair catch-up): the same bytes as
 * ag_rs_coder_shred / ag_rs_coder_deshred per slice.
 *
 * shred_batch: payload_lens (HOST, nslices) must each pad to S (64-byte multiple / 32);
 * payload b (device, payloads + b*payload_stride) is copied into the data region, padded
 * with 0x80 00.., then the coding shards are encoded.  payloads NULL: the payloads already
 * sit in the data regions.  Asynchronous on the context stream.
 * Errors (nothing launched): TOO_MUCH_DATA (a length > 32767), INVALID_ARGUMENT. */
int ag_rs_coder_shred_batch(ag_rs_ctx* ctx, size_t num_coding, size_t nslices, size_t shred_bytes,
                            const uint8_t* payloads, size_t payload_stride,
                            const uint32_t* payload_lens, uint8_t* codewords,
                            size_t codeword_stride);

/* deshred_batch: data_present [nslices][32] and coding_present [nslices][num_coding] are
 * HOST 0/1 flags.  Restores the absent data shards in place, strips the padding and
 * re-encodes all num_coding coding shards of every slice that succeeded (RawShreds of the
 * reference).  payload_len_out (HOST, nslices): the payload length (the payload is the
 * first len bytes of the slice's data region), or -AG_RS_ERR_NOT_ENOUGH_SHARDS /
 * -AG_RS_ERR_INVALID_PADDING for a slice whose received shards are left untouched (its absent
 * shard slots hold unspecified bytes: a slice with exactly 32 kept 1 KiB shreds restores its
 * absent data and coding shards in one decode, before the padding check).  mode:
 * AG_RS_DECODE_EXACT (crate semantics) or AG_RS_DECODE_ANY_K.  Synchronous.  Whole-call
 * errors: TOO_MUCH_DATA (S > 1024), INVALID_SHARD_SIZE. */
int ag_rs_coder_deshred_batch(ag_rs_ctx* ctx, size_t num_coding, size_t nslices,
                              size_t shred_bytes, uint8_t* codewords, size_t codeword_stride,
                              const uint8_t* data_present, const uint8_t* coding_present,
                              int mode, int64_t* payload_len_out);

/* ---- 4b. slice payload framing ---------------------------------------------------------
 * Slice::payload_bytes (types/slice.rs:73-84) and SlicePayload::try_from (slice.rs:211-218)
 * on the batched coder's codeword buffers (device), the data region of codeword b being
 * its 32 data shards.  Metadata arrays are HOST memory; synchronous.
 * Framing: wincode(parent: Option<BlockId>) || u64 LE data length || data, BlockId = (Slot
 * u64, BlockHash [u8; 32]) = 40 bytes (lib.rs:65).  The framed payload then goes through
 * ag_rs_coder_shred_batch with payloads = NULL (padded and encoded in place). */
#define AG_SLICE_MAX_DATA 32767      /* MAX_DATA_PER_SLICE (shredder.rs:54) */
#define AG_SLICE_BLOCK_ID_BYTES 40
enum {
  AG_SLICE_OK = 0,
  AG_SLICE_TOO_LARGE = 1,    /* SlicePayloadError::TooLarge (slice.rs:195) */
  AG_SLICE_BAD_ENCODING = 2, /* SlicePayloadError::BadEncoding (slice.rs:198) */
  AG_SLICE_NO_PAYLOAD = 3    /* the slice's deshred failed (payload_len < 0) */
};

/* frame_batch: parent_flags [nslices] (0 None / 1 Some), parent_ids [nslices][40] (slot LE,
 * then the block hash), data_lens [nslices]: HOST.  data: device, slice b at data +
 * b * data_stride.  codewords: device, 4-byte aligned, codeword_stride % 4 == 0.
 * payload_lens_out (HOST, nslices): framed length = ag_rs_coder_shred_batch's payload_lens.
 * shred_bytes: the coder batch's shred size; every framed payload must be <=
 * AG_SLICE_MAX_DATA and < 32 * shred_bytes (ReedSolomonCoder::shred's TooMuchData,
 * reed_solomon.rs:89-91), else AG_RS_ERR_TOO_MUCH_DATA with nothing written. */
int ag_slice_frame_batch(ag_rs_ctx* ctx, size_t nslices, size_t shred_bytes, const uint8_t* parent_flags,
                         const uint8_t* parent_ids, const uint8_t* data, size_t data_stride,
                         const uint32_t* data_lens, uint8_t* codewords, size_t codeword_stride,
                         uint32_t* payload_lens_out);

/* parse_batch: SlicePayload::try_from on the first payload_lens[b] bytes of codeword b
 * (payload_lens HOST, as ag_rs_coder_deshred_batch returns them; < 0 = failed slice).
 * Outputs HOST: status AG_SLICE_*, parent_flags, parent_ids [nslices][40], and the data
 * (left in place) as codeword + data_offsets[b], data_lens[b] bytes. */
int ag_slice_parse_batch(ag_rs_ctx* ctx, size_t nslices, const uint8_t* codewords, size_t codeword_stride,
                         const int64_t* payload_lens, uint8_t* status, uint8_t* parent_flags,
                         uint8_t* parent_ids, uint32_t* data_offsets, uint32_t* data_lens);

/* ---- 5. slice Merkle trees -----------------------------------------------------------
 * The SHA-256 Merkle tree the shredder builds over each slice's 64 shreds (data shreds,
 * then coding shreds; shredder.rs:628-632) -- crypto/merkle.rs MerkleTree:
 *   leaf  = SHA-256("ALPENGLOW-MERKLE-TREE  LEAF-NODE" || shred)      (merkle.rs:457-460)
 *   inner = SHA-256(LEFT_LABEL || left || RIGHT_LABEL || right)       (merkle.rs:466-468)
 *   odd node at height h pairs with EMPTY_ROOTS[h]                    (merkle.rs:303-328)
 * Device-resident batches (all pointers device memory, on the context's stream). */
#define AG_MERKLE_MAX_LEAVES 64

/* EMPTY_ROOTS[height] (merkle.rs:62-157) computed by the library's SHA-256; no GPU needed. */
int ag_merkle_empty_root(size_t height, uint8_t out[32]);
/* Height and node count (reference `nodes.len()`) of a tree of n_leaves leaves. */
size_t ag_merkle_height(size_t n_leaves);
size_t ag_merkle_node_count(size_t n_leaves);
/* MerkleTree::new + get_root + create_proof for every leaf (merkle.rs:281-370), nslices
 * slices.  Leaf j of slice s: leaves + s*slice_stride + j*leaf_stride, leaf_bytes long
 * (1 <= n_leaves <= 64).  roots: 32 B per slice.  nodes (nullable): node_count digests per
 * slice at nodes_stride.  proofs (nullable): height digests per leaf, n_leaves*height*32 B
 * per slice at proofs_stride. */
int ag_merkle_build_batch(ag_rs_ctx* ctx, size_t n_leaves, size_t leaf_bytes, size_t nslices,
                          const uint8_t* leaves, size_t leaf_stride, size_t slice_stride, uint8_t* roots,
                          uint8_t* nodes, size_t nodes_stride, uint8_t* proofs, size_t proofs_stride);
/* check_proof (merkle.rs:374-387) for n leaves: leaf t at leaves + t*leaf_stride, index[t],
 * root at roots + t*roots_stride, height digests at proofs + t*proofs_stride;
 * ok[t] = 1 if the proof derives the root, else 0. */
int ag_merkle_verify_batch(ag_rs_ctx* ctx, size_t n, size_t leaf_bytes, const uint8_t* leaves,
                           size_t leaf_stride, const uint32_t* index, const uint8_t* roots,
                           size_t roots_stride, const uint8_t* proofs, size_t proofs_stride, size_t height,
                           uint8_t* ok);

/* ---- 6. all-or-nothing payload transforms (AONT / PETS shredders) ---------------------
 * AontShredder::shred (shredder.rs:463-470): payload := AES-128-CTR_key(payload) ||
 * (key ^ SHA-256(ciphertext)[0..16)); PetsShredder::shred (:414-418): ... || key.  The
 * deshred side (decrypt_payload, :509-528) splits the 16-byte tail, derives the key (AONT:
 * tail ^ SHA-256(ciphertext); PETS: the tail) and decrypts in place.  AES-128-CTR is
 * cipher::apply_keystream (crypto/cipher.rs:25-30: ctr::Ctr64LE, all-zero IV); SHA-256 is
 * hash::hash (crypto/hash.rs:64-67).  Buffers/keys/digests: device memory; lengths: HOST
 * arrays.  Asynchronous on the context stream unless stated. */
enum { AG_AON_AONT = 0, AG_AON_PETS = 1 };
/* One AES-128 block with the library's tables (host; known-answer checks). */
int ag_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]);
/* apply_keystream to n buffers (buffer b: buffers + b*stride, lens[b] bytes, key keys + 16*b). */
int ag_cipher_apply_keystream_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* keys, uint8_t* buffers, size_t stride,
                                    const uint32_t* lens);
/* hash::hash of n buffers -> digests + 32*b. */
int ag_sha256_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* buffers, size_t stride, const uint32_t* lens,
                    uint8_t* digests);
/* The shred side: encrypt buffer b's lens[b] payload bytes in place under keys + 16*b and
 * write the 16-byte tail after them (the buffer then holds lens[b] + 16 bytes). */
int ag_aon_encrypt_batch(ag_rs_ctx* ctx, int scheme, size_t n, const uint8_t* keys, uint8_t* buffers, size_t stride,
                         const uint32_t* lens);
/* The deshred side: buffer b holds lens[b] bytes (ciphertext || tail); decrypts in place.
 * plain_len_out (HOST): lens[b] - 16, or -AG_RS_ERR_BAD_ENCODING when lens[b] < 16.
 * Synchronous. */
int ag_aon_decrypt_batch(ag_rs_ctx* ctx, int scheme, size_t n, uint8_t* buffers, size_t stride, const uint32_t* lens,
                         int64_t* plain_len_out);

/* ---- 7. shred signatures (Ed25519) ----------------------------------------------------
 * crypto/signature.rs wraps ed25519-zebra 4.2.0: RFC 8032 keys and signatures, ZIP-215
 * verification (s < l required; A and R need only decode to curve points, non-canonical y
 * accepted; accept iff [8]([s]B - [k]A - R) = 0 with k = SHA-512(R || A || M) mod l).
 * Device-resident batches on the context stream; every pointer is device memory. */
#define AG_SLICE_COMMITMENT_LEN 49
enum { AG_SHRED_OK = 0, AG_SHRED_INVALID_SIGNATURE = 1, AG_SHRED_EQUIVOCATION = 2 };
/* SecretKey::to_pk (signature.rs:54-58): 32-byte seeds -> 32-byte public keys. */
int ag_ed25519_public_key_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* seeds, uint8_t* pks);
/* SecretKey::sign_bytes (signature.rs:69-72): sig t (64 B at sigs + 64*t) over msg_len bytes
 * at msgs + t*msg_stride with seed seeds + t*seed_stride and its public key pks +
 * t*pk_stride (strides 0: one key for the batch). */
int ag_ed25519_sign_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* seeds, size_t seed_stride, const uint8_t* pks,
                          size_t pk_stride, const uint8_t* msgs, size_t msg_stride, size_t msg_len, uint8_t* sigs);
/* Signature::verify_bytes (signature.rs:100-103): ok[t] = 1 / 0 for key pks + t*pk_stride,
 * message msgs + t*msg_stride of msg_lens[t] bytes (msg_lens null: msg_len each), signature
 * sigs + t*sig_stride. */
int ag_ed25519_verify_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* pks, size_t pk_stride, const uint8_t* msgs,
                            size_t msg_stride, const uint32_t* msg_lens, size_t msg_len, const uint8_t* sigs,
                            size_t sig_stride, uint8_t* ok);
/* ValidatedShred::try_new (validated_shred.rs:52-81) for n shreds of one leader (pk):
 * shred t has payload data + t*data_stride (data_bytes), index shred_index[t], Merkle path
 * proofs + t*proofs_stride (height digests), header slots[t] / slice_indices[t] / is_last[t]
 * and slice_sig sigs + t*sig_stride.  Its root is derived from the path (Shred::slice_root,
 * shredder.rs:168-175), the SliceCommitment built (shredder.rs:206-215), and, when
 * has_cached[t] (cached + 49*t is the commitment of an earlier shred of that slice), a match
 * is OK without a signature check, a valid signature over a different commitment is
 * AG_SHRED_EQUIVOCATION; otherwise the signature decides OK / AG_SHRED_INVALID_SIGNATURE.
 * status[t] gets the verdict; roots_out (32 B each) and commitments_out (49 B each) are
 * optional.  cached and has_cached are both null or both set. */
int ag_shred_validate_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* data, size_t data_stride, size_t data_bytes,
                            const uint32_t* shred_index, const uint8_t* proofs, size_t proofs_stride, size_t height,
                            const uint64_t* slots, const uint64_t* slice_indices, const uint8_t* is_last,
                            const uint8_t* sigs, size_t sig_stride, const uint8_t* pk, const uint8_t* cached,
                            const uint8_t* has_cached, uint8_t* status, uint8_t* roots_out, uint8_t* commitments_out);
/* The shred side (shredder.rs:540): slice_sig = sign(SliceCommitment(header, root)) for
 * nslices slices with one leader key (seed, pk: 32 B each); roots 32 B per slice; sigs 64 B
 * per slice; commitments_out (49 B per slice) optional. */
int ag_slice_sign_batch(ag_rs_ctx* ctx, size_t nslices, const uint8_t* seed, const uint8_t* pk, const uint64_t* slots,
                        const uint64_t* slice_indices, const uint8_t* is_last, const uint8_t* roots, uint8_t* sigs,
                        uint8_t* commitments_out);

/* ---- 8. shred wire format --------------------------------------------------------------
 * One UDP datagram per Shred (shredder.rs:113-186), wincode 0.6 (bincode-compatible):
 *   u32 variant (0 Data, 1 Coding) | u64 slot | u64 slice_index | u8 is_last |
 *   u64 shred_index | u64 data_len | data | 64 B slice_sig | u64 proof_len | proof_len x 32 B
 * decoded like network::deserialize (network.rs:52-64): preallocation capped at MTU (1500
 * bytes), trailing bytes rejected; slice_index < 1024 and shred_index < 64
 * (types/slice_index.rs:115-132, shred_index.rs:91-108).  Columns are device arrays. */
typedef struct ag_shred_columns {
  uint8_t* kind;          /* ShredPayloadType: 0 Data, 1 Coding */
  uint64_t* slot;
  uint64_t* slice_index;
  uint8_t* is_last;
  uint32_t* shred_index;
  uint8_t* data;          /* row t at data + t*data_stride (capacity data_stride bytes) */
  size_t data_stride;
  uint32_t* data_len;
  uint8_t* sig;           /* 64 B per shred */
  uint8_t* proof;         /* row t at proof + t*proof_stride: height digests of 32 B */
  size_t proof_stride;
  uint32_t* height;
} ag_shred_columns;
enum { AG_WIRE_OK = 0, AG_WIRE_MALFORMED = 1, AG_WIRE_TOO_LARGE = 2 };
/* Packets (device; packet t at packets + t*packet_stride, packet_lens[t] bytes) -> columns.
 * status[t]: AG_WIRE_OK, AG_WIRE_MALFORMED (the reference's deserialize rejects it) or
 * AG_WIRE_TOO_LARGE (valid, but wider than the caller's rows); columns are written only
 * for AG_WIRE_OK. */
int ag_shred_deserialize_batch(ag_rs_ctx* ctx, size_t n, const uint8_t* packets, size_t packet_stride,
                               const uint32_t* packet_lens, const ag_shred_columns* cols, uint8_t* status);
/* Columns -> packets; packet_lens[t] = encoded length, or 0 (packet untouched) when the
 * shred does not fit packet_stride or its own rows. */
int ag_shred_serialize_batch(ag_rs_ctx* ctx, size_t n, const ag_shred_columns* cols, uint8_t* packets,
                             size_t packet_stride, uint32_t* packet_lens);

/* ---- 9. composed Shredder (RegularShredder, 32 data + 32 coding shreds) ----------------
 * One call per direction for nslices slices of one shred size S (even, <= 1024), every
 * stage on the device, one leader key.  Slice s owns 64 datagram slots (packets +
 * (64 s + j) * packet_stride, j = shred index; packet_stride >= 1325 for S = 1024) and one
 * codeword of 64 raw shreds (codewords + s * 64 * S: 32 data shreds, then 32 coding
 * shreds, 16-byte aligned).  Slice headers (slots, slice_indices, is_last: one entry per
 * slice) and the key (seed, pk: 32 B) are device arrays; the rest is stated per argument.
 *
 * shred_batch -- RegularShredder::shred (shredder.rs:337-345): Slice::payload_bytes (the
 * framing of section 4b; parent_flags / parent_ids / data_lens HOST, data device) ->
 * ReedSolomonCoder::shred -> slice Merkle tree (roots_out, 32 B per slice, nullable) ->
 * sign(SliceCommitment) (sigs_out, 64 B per slice, nullable) -> the 64 Shred datagrams of
 * every slice, data shreds first (data_and_coding_to_output_shreds, :533-560);
 * packet_lens (device) gets each datagram's length.  Errors (nothing launched):
 * TOO_MUCH_DATA (a framed slice does not fit 32 * S or 32767 bytes), INVALID_ARGUMENT.
 *
 * deshred_batch -- Shredder::deshred (shredder.rs:282-311) behind the receiver's checks:
 * the datagrams present (packet_lens > 0) are parsed (network::deserialize), their fields
 * checked against their slot (shred index j, kind, S bytes, 6-digest path) and validated
 * (ValidatedShred::try_new, validated_shred.rs:52-81: Merkle path -> root -> commitment ->
 * Ed25519 under pk; the first such shred of a slice is verified by signature and the
 * others compared with its commitment, as the blockstore's cache does); datagrams failing
 * any check count as absent.  Then ReedSolomonCoder::deshred (any 32 survivors, ANY_K),
 * check_merkle_tree, SlicePayload::try_from, and fill_missing_shreds: every absent slot of
 * a slice that succeeded receives its datagram (packet and packet_lens written; the
 * present ones are left as they were).  Per slice (HOST outputs): status[s] = AG_RS_OK or
 * AG_RS_ERR_NOT_ENOUGH_SHARDS / _TOO_MUCH_DATA / _BAD_ENCODING (invalid padding or
 * SlicePayload encoding) / _INVALID_MERKLE_TREE; for AG_RS_OK the header (slots_out,
 * slice_indices_out, is_last_out), the parent (parent_flags_out, parent_ids_out 40 B) and
 * the data at codewords + s * 64 * S + data_offsets_out[s], data_lens_out[s] bytes.  The
 * codewords hold the 64 raw shreds of every successful slice.  Synchronous. */
int ag_shredder_shred_batch(ag_rs_ctx* ctx, size_t nslices, size_t shred_bytes, const uint8_t* parent_flags,
                            const uint8_t* parent_ids, const uint8_t* data, size_t data_stride,
                            const uint32_t* data_lens, const uint64_t* slots, const uint64_t* slice_indices,
                            const uint8_t* is_last, const uint8_t* seed, const uint8_t* pk, uint8_t* codewords,
                            uint8_t* roots_out, uint8_t* sigs_out, uint8_t* packets, size_t packet_stride,
                            uint32_t* packet_lens);
int ag_shredder_deshred_batch(ag_rs_ctx* ctx, size_t nslices, size_t shred_bytes, uint8_t* packets,
                              size_t packet_stride, uint32_t* packet_lens, const uint8_t* pk, uint8_t* codewords,
                              int32_t* status, uint64_t* slots_out, uint64_t* slice_indices_out,
                              uint8_t* is_last_out, uint8_t* parent_flags_out, uint8_t* parent_ids_out,
                              uint32_t* data_offsets_out, uint32_t* data_lens_out);

/* The other shredders of shredder.rs, composed the same way (round 6):
 *   AG_SHREDDER_CODING_ONLY  CodingOnlyShredder (:361-394): ReedSolomonCoder::new(64), the 64
 *                            coding shreds are the output (no data shreds);
 *   AG_SHREDDER_PETS         PetsShredder (:396-444): payload := AES-128-CTR_key(payload) || key,
 *                            ReedSolomonCoder::new(33), the data shred holding the key dropped:
 *                            31 data + 33 coding output shreds;
 *   AG_SHREDDER_AONT         AontShredder (:446-500): ... || (key ^ SHA-256(ciphertext)[0..16)),
 *                            ReedSolomonCoder::new(32): 32 data + 32 coding output shreds;
 *   AG_SHREDDER_REGULAR      forwards to ag_shredder_shred_batch / _deshred_batch
 *                            (codeword_stride must then be 64 * S).
 * Output shred j is codeword row j (AONT), 32 + j (CodingOnly), or j < 31 / 32 + (j - 31)
 * (PETS) of a codeword of 32 data + m coding shards at codewords + s * codeword_stride
 * (codeword_stride >= (32 + m) * S, a multiple of 4).  keys (DEVICE, 16 bytes per slice; PETS /
 * AONT only): the key cipher::encrypt_with_random_key drew (crypto/cipher.rs) -- the caller
 * supplies it, so the output is reproducible.  MAX_DATA_SIZE is 16 bytes less for PETS / AONT
 * (TooMuchData).  The deshred side gives the verdicts of the crate's decoder over every kept
 * shred (EXACT: a batch decodes ANY_K on the device and is redone with EXACT when a slice with
 * surplus shreds fails), decrypts after the raw shreds are taken (decrypt_payload: BadEncoding
 * for a buffer shorter than the key or a failed key check, :512-528), then check_merkle_tree,
 * SlicePayload::try_from and fill_missing_shreds as ag_shredder_deshred_batch; the parsed data
 * is at codewords + s * codeword_stride + data_offsets_out[s].  The datagrams are parsed into
 * and serialized from their codeword rows.  PETS / AONT serialize the absent datagrams before
 * decrypting, so a slice that fails only at decryption or SlicePayload may find bytes written
 * in its absent (length-0) slots; lengths change only for successful slices.  Arguments
 * otherwise as the Regular calls. */
enum { AG_SHREDDER_REGULAR = 0, AG_SHREDDER_CODING_ONLY = 1, AG_SHREDDER_PETS = 2, AG_SHREDDER_AONT = 3 };
int ag_shredder_shred_batch_kind(ag_rs_ctx* ctx, int kind, size_t nslices, size_t shred_bytes,
                                 const uint8_t* parent_flags, const uint8_t* parent_ids, const uint8_t* data,
                                 size_t data_stride, const uint32_t* data_lens, const uint64_t* slots,
                                 const uint64_t* slice_indices, const uint8_t* is_last, const uint8_t* seed,
                                 const uint8_t* pk, const uint8_t* keys, uint8_t* codewords, size_t codeword_stride,
                                 uint8_t* roots_out, uint8_t* sigs_out, uint8_t* packets, size_t packet_stride,
                                 uint32_t* packet_lens);
int ag_shredder_deshred_batch_kind(ag_rs_ctx* ctx, int kind, size_t nslices, size_t shred_bytes, uint8_t* packets,
                                   size_t packet_stride, uint32_t* packet_lens, const uint8_t* pk,
                                   uint8_t* codewords, size_t codeword_stride, int32_t* status, uint64_t* slots_out,
                                   uint64_t* slice_indices_out, uint8_t* is_last_out, uint8_t* parent_flags_out,
                                   uint8_t* parent_ids_out, uint32_t* data_offsets_out, uint32_t* data_lens_out);

#ifdef __cplusplus
}
#endif
#endif /* ALPENGLOW_RS_H */
