// Kernel parameter blocks and launchers (host side of rs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ag {

// Bitsliced single-chunk transform over one 32-shard (or 64-shard) position block:
//   out = FFT_{delta_out}( IFFT_{delta_in}( in ) )
// encode (HighRate, k <= m = N): in = originals (points N..2N), out = recovery (points 0..N)
// decode from a full recovery set: in = recovery, out = originals (masked per block).
struct XformParams {
  const uint8_t* in;
  uint64_t in_block_stride;
  uint64_t in_shard_stride;
  uint8_t* out;
  uint64_t out_block_stride;
  uint64_t out_shard_stride;
  const uint64_t* out_mask;    // device, one word per pattern: bit s set => store shard s
  uint32_t pattern_per_block;  // pattern(b) = pattern_per_block ? b : 0
  uint32_t n_in;               // shards 0..n_in-1 are loaded, the rest are zero
  uint32_t n_out;              // shards 0..n_out-1 may be stored
  uint32_t chunks_per_shard;   // shard_bytes / 64
  uint64_t total_columns;         // nblocks * chunks_per_shard
  uint32_t out_low_half;          // decode: every stored shard is < N / 2 (pruned FFT)
  uint32_t skip_idle;             // xform<4> with per-block masks: tiles whose blocks all have
                                  // mask 0 exit before loading (re-encodes of a few slices)
  uint32_t tail_bytes;            // T = S mod 64 (even), TAIL kernels: chunk chunks_per_shard - 1 of
                                  // every shard is the crate's split tail (T/2 low bytes, then T/2
                                  // high bytes), read and written in place
};

enum class XformKind { kEncode32, kDecode32, kEncode64, kDecode64 };

// Encode kernels, as bits of the per-context record of the last encode call (test aid:
// ag_rs_internal_last_encode_kernels).
enum EncodeKernelBit : uint32_t {
  kEkXform4 = 1u << 0,    // xform_kernel<4, 32, 0>: the headline 32-point encode
  kEkXform8 = 1u << 1,    // xform8_kernel<32, 0>: small batches, 8 / 16 KiB shards
  kEkXformH8 = 1u << 2,   // xform_h8: 64-point encode
  kEkEncodeMc = 1u << 3,  // encode_mc: multi-chunk HighRate (16:4)
  kEkLowRate = 1u << 4,   // xform_lowrate: one LowRate recovery chunk
  kEkLowRate2 = 1u << 5,  // xform_h8 LR2: two LowRate chunks of a 32-point code
  kEkGeneric = 1u << 6,   // generic_encode_kernel (table-driven)
  kEkRestride = 1u << 7,  // tail bytes restrided through padded shards
};
// The 32-point encode kernel launch_xform(kEncode32, p) runs: xform8 for batches of fewer
// than 256 tiles and for 8 / 16 KiB shards (chunks_per_shard 128 / 256), else xform<4>.
inline EncodeKernelBit encode32_kernel(const XformParams& p) {
  const uint64_t groups = (p.total_columns + 63) / 64;
  return groups < 256 || p.chunks_per_shard == 128 || p.chunks_per_shard == 256 ? kEkXform8 : kEkXform4;
}

hipError_t launch_xform(XformKind kind, const XformParams& p, hipStream_t stream);
// True when the bitsliced transform exists for this transform size.
bool xform_supported(unsigned n);
// The 64-point transform (xform_h8): (din, dout) in {(64, 0), (0, 64), (0, 128), (0, 192)}.
hipError_t launch_xform64(unsigned din, unsigned dout, const XformParams& p, hipStream_t stream);
// LowRate encode, recovery chunk j: out = FFT_n(IFFT_n(in, 0), n * (j + 1)) for
// n = next_pow2(k) in {32 (j < 4), 64 (j < 3)} -- the crate's LowRate encoder per chunk.
hipError_t launch_xform_lowrate(unsigned n, unsigned j, const XformParams& p, hipStream_t stream);
// LowRate recovery chunks 2 pair and 2 pair + 1 of a 32-point code (k <= 32) in one launch
// (xform_h8 LR2): in = the k originals, out = recovery shard 64 pair, n_out <= 64.
hipError_t launch_xform_lowrate2(unsigned pair, const XformParams& p, hipStream_t stream);
// LowRate decode from a fully present recovery chunk j < 4 (next_pow2(k) = 32):
// originals = FFT_0(IFFT_{32(j+1)}(chunk j)); in = chunk j, out = originals (masked).
hipError_t launch_xform_lowrate_decode(unsigned j, const XformParams& p, hipStream_t stream);
// Multi-chunk HighRate encode with chunk = next_pow2(m) in {1, 2, 4} and k <= 64:
// in = originals (n_in = k), out = recovery (n_out = m).  out_mask unused.
hipError_t launch_encode_mc(unsigned chunk, const XformParams& p, hipStream_t stream);

// Syndrome decoder for HighRate geometries with chunk = next_pow2(m) <= 4, k <= 64 (the
// encode_mc domain), any k survivors: re-encode the present originals (erased ones read as
// zero), XOR with e received recovery shards -> syndromes S, restore the e <= 4 erased
// originals as Minv S (Minv = inverse of the generator's e x e erased/used submatrix).
struct SynPattern {
  uint64_t dmask;           // originals present (loaded)
  uint32_t e;               // originals restored (<= 4)
  uint8_t rec[4];           // recovery shards used for the syndromes
  uint8_t out[4];           // erased originals
  uint32_t pad;
  uint32_t rows[4][4][16];  // Minv[a][b] as 16x16 GF(2) matrices (rows[o] bit i)
};
struct DecodeSynParams {
  const uint8_t* rec;
  uint64_t rec_block_stride;
  uint64_t rec_shard_stride;
  uint8_t* orig;  // present originals are read, restored ones written here
  uint64_t orig_block_stride;
  uint64_t orig_shard_stride;
  const SynPattern* pat;      // [pattern]
  const uint32_t* block_ids;  // per_block: blocks processed (null = 0..)
  uint32_t per_block;         // 1: pattern = block; tiles_per_block 64-column tiles per block
  uint32_t tiles_per_block;
  uint32_t k;
  uint32_t chunks_per_shard;
  uint64_t total_columns;  // batch blocks * chunks_per_shard
  uint64_t ntiles;         // 64-column tiles processed
};
hipError_t launch_decode_syn(unsigned chunk, const DecodeSynParams& p, hipStream_t stream);

// Correction decoder (decode_c_kernel, rs_decode_c.hip) for the 32-point full-window
// geometries (HighRate, m = 32, k <= 32) with lost recovery shards, any k survivors:
//   d = X r is the full-recovery transform (X = FFT_32 o IFFT_0, the inverse of the 32:32
//   encoder; original-coset points k..31 are virtual zeros).  With the lost recovery shards
//   L read as zero, X r' differs from d by X[:, L] g, g = the lost values.  At |L| known
//   original-coset points (present originals or virtual zeros) the syndromes
//   s = d - X r' give g = N^-1 s (N = X[Dsel, L]), so the erased originals are
//   d_E = (X r')_E + K s with K = X[E, L] N^-1 (|E| x |L| runtime multiplies).
constexpr int kCorrMaxSyn = 16;    // |L| <= 16 (syndrome planes staged in 64 KiB of LDS)
constexpr int kCorrMaxPairs = 256;  // |E| * |L| <= 256 (|E| + |L| <= 32)
constexpr int kCorrPairWords = 64;  // table picks per (a, b) pair
struct CorrPattern {
  uint64_t rmask;  // recovery shards present (loaded); lost ones read as zero
  uint64_t emask;  // originals restored (E)
  uint64_t smask;  // original-coset points used as syndromes: present originals (< k) or virtual zeros
  uint32_t ne, ns;  // |E|, |L| = number of syndromes
  uint64_t kofs;    // K picks at kpool + kofs, pair (a, b) (a < ne, b < ns) at + 64 * (a * ns + b)
  // The balanced correction's assignment (decode_c, layout H0), per wave w:
  //   wsum[w]: bits 0-3 slots that accumulate K s (own kept or foreign), 4-7 slots holding own
  //            restored originals (stored at the end), 8-11 own outputs donated to other
  //            waves, 12-15 slots accumulating a foreign output; bit 16: the pattern donates
  //   wslot[w][t]: bits 0-19 the slot's K row offset (kCorrPairWords * rank * ns), bits
  //            20-24 its LDS exchange slot (foreign: written; donated: read)
  uint32_t wsum[8];
  uint32_t wslot[8][4];
};
// K[a][b] as table picks: for group pair gp (input planes 8gp..8gp+7) and output plane o,
// dwords [32 gp + 2 o] and [32 gp + 2 o + 1] are the 4-bit indices (row o of K[a][b]'s
// 16x16 GF(2) matrix, input planes 8gp..8gp+3 and 8gp+4..8gp+7; row o bit i = bit o of
// K * 2^i) into the two 16-entry XOR tables of the syndrome's planes.
struct DecodeCParams {
  const uint8_t* rec;
  uint64_t rec_block_stride;
  uint64_t rec_shard_stride;
  uint8_t* orig;  // present originals are read (syndromes), restored ones written here
  uint64_t orig_block_stride;
  uint64_t orig_shard_stride;
  const CorrPattern* pat;     // [pattern]
  const uint32_t* kpool;      // table picks of every pattern
  const uint32_t* block_ids;  // per_block: blocks processed (null = 0..)
  uint32_t per_block;         // 1: pattern = block; tiles_per_block 64-column tiles per block
  uint32_t tiles_per_block;
  uint32_t k;
  uint32_t chunks_per_shard;
  uint64_t total_columns;  // batch blocks * chunks_per_shard
  uint64_t ntiles;         // 64-column tiles processed
};
hipError_t launch_decode_c(const DecodeCParams& p, hipStream_t stream);

struct GfDeviceTables {
  const uint16_t* exp;
  const uint16_t* log;
  const uint16_t* skew;
  const uint16_t* log_walsh;
};

// Bitsliced HighRate decode for any erasure pattern over a W = 32 / 64 point window.
// Positions: recovery j < chunk (shard j), originals chunk + i (shard i).
struct DecodeXParams {
  const uint8_t* rec;
  uint64_t rec_block_stride;
  uint64_t rec_shard_stride;
  uint8_t* orig;  // present originals are read, restored ones written here
  uint64_t orig_block_stride;
  uint64_t orig_shard_stride;
  const uint64_t* pmask;      // [pattern][2]: positions present (loaded), positions restored
  const uint32_t* rows;       // [pattern][W][16] multiply matrices (decode_rows_kernel); per_lane:
                              // [pattern][W] polynomial-basis constants (decode_rows poly)
  const uint32_t* block_ids;  // per_block: blocks processed (null = 0..)
  uint32_t per_block;         // 1: pattern = block, tiles_per_block tiles per block
  uint32_t tiles_per_block;   // chunks_per_shard / 64 (per_block mode)
  uint32_t per_lane;          // 1: pattern = block of each lane's chunk (tiles straddle blocks)
  uint32_t k, m, chunk;       // m: recovery shards inside the window
  uint32_t low_rate;          // 0: recovery j at position j, original i at chunk + i (HighRate);
                              // 1: original i at i, recovery j at chunk + j (LowRate sub-window)
  uint32_t chunks_per_shard;
  uint64_t total_columns;  // batch blocks * chunks_per_shard
  uint32_t rows_w;         // constants per pattern in rows (W = 64: 64; W = 128: 128)
  uint32_t any_k;          // 1: every pattern loads at most k survivors (ANY_K; the packed kernel)
  uint32_t fuse;           // packed kernel, HighRate: the restored set may include recovery positions
                           // (every erased position of an exactly-k pattern: decode_pk<-1>)
  uint32_t tail_bytes;     // T = S mod 64 (even, >= 16; W = 64 per-lane HighRate only): column
                           // chunks_per_shard - 1 of every shard is its T-byte tail (decode_h8 TAIL)
};
// W = 32 / 64: pass 0.  W = 128: pass 1 (the other half's inputs, raw partial outputs), then
// pass 2 (the output half's inputs, the partial added, output multiply); masks per pass.
// which (optional): ORed with the DecodeXKernelBit of the W = 64 kernel launched (test aid)
enum DecodeXKernelBit : uint32_t { kDxPkFused = 1, kDxPk = 2, kDxH8Fused = 4, kDxH8 = 8, kDxX16 = 16 };
hipError_t launch_decode_x(unsigned W, int pass, const DecodeXParams& p, uint64_t ntiles, hipStream_t stream,
                           uint32_t* which = nullptr);
hipError_t launch_decode_rows128(const uint64_t* m6, uint32_t npat, const GfDeviceTables& t, uint32_t* rows,
                                 hipStream_t stream);
// rows for npat patterns: emask[p] = erased positions (locator), pmask as above.
hipError_t launch_decode_rows(const uint64_t* emask, const uint64_t* pmask, uint32_t npat, uint32_t W,
                              const GfDeviceTables& t, uint32_t* rows, bool poly, hipStream_t stream);

// The per-call server (latency_server_kernel): one resident workgroup per context serves
// single-tile 32-point transforms posted through a mailbox in mapped, fine-grained host
// memory, so a per-slice call costs no kernel dispatch and no completion signal.
//   host:   writes kind / mask / p, then doorbell = seq; spins until done == seq
//   server: polls doorbell, runs the job, releases its stores, writes done = seq; exits
//           (alive = 0) on kJobQuit or after idle_ticks of the 100 MHz wall clock with no job
// kJobDecodePk: one 32:32 slice of 1 KiB shreds with exactly 32 shreds present (the follower's
// deshred at its 32nd arriving shred, slot_block_data.rs:353): decode_pk<-1>'s window decode on
// a one-slice tile, restoring every absent data and coding shred in place; `mask` = the present
// window positions (bit j < 32: coding shred j, bit 32 + i: data shred i); the server computes
// the locator constants itself (decode_rows' Walsh route, PkLocTables).
enum LatencyJob : uint32_t {
  kJobEncode32 = 0,
  kJobDecode32 = 1,
  kJobDecode32Half = 2,
  kJobDecodePk = 3,
  kJobQuit = 4
};
struct LatencyMailbox {
  uint32_t doorbell;  // host: sequence number of the posted job
  uint32_t done;      // server: sequence number of the last finished job
  uint32_t alive;     // 0 no server, 1 server running, 2 launch requested (host)
  uint32_t kind;      // LatencyJob
  uint64_t mask;      // decode: store mask (bit s: shard s restored); pk: present positions
  uint32_t p_seq;     // host: version of p / dp (bumped when the bytes change; the server keeps
  uint32_t dp_seq;    // its last copy in LDS, so a call with unchanged parameters skips that read)
  XformParams p;      // in / out: device addresses of mapped host memory; p.out_mask ignored
  DecodeXParams dp;   // kJobDecodePk: rec / orig / strides (pmask set by the server; rows unused)
  uint64_t job_ticks; // server: wall-clock ticks (100 MHz) of the last job, doorbell seen -> stores
                      // released (diagnostic: the in-kernel share of a per-call latency)
  uint32_t phase_ticks[4];  // the same job's phases: kind read, parameters read + cache
                            // invalidate, the tile (loads, transform, stores issued), the release
};
// log_t: the device log table (the server caches log x for x < 64 at start)
hipError_t launch_latency_server(LatencyMailbox* mb_dev, uint64_t idle_ticks, const uint16_t* log_t,
                                 hipStream_t stream);

// Generic (any geometry) table-driven kernels.  One thread per (block, symbol).

struct GenericEncodeParams {
  const uint8_t* orig;
  uint64_t orig_block_stride;
  uint64_t orig_shard_stride;
  uint8_t* rec;
  uint64_t rec_block_stride;
  uint64_t rec_shard_stride;
  uint32_t k, m, high_rate, chunk, rows;
  uint32_t shard_bytes, nsym;
  uint64_t nblocks;  // blocks in this launch
  uint16_t* scratch;  // nblocks * rows * nsym
  GfDeviceTables t;
};
hipError_t launch_generic_encode(const GenericEncodeParams& p, hipStream_t stream);

struct GenericDecodeParams {
  uint8_t* orig;  // restored originals are written here (absent positions only)
  uint64_t orig_block_stride;
  uint64_t orig_shard_stride;
  const uint8_t* rec;
  uint64_t rec_block_stride;
  uint64_t rec_shard_stride;
  const uint8_t* orig_present;  // [pattern][k]
  const uint8_t* rec_present;   // [pattern][m]
  uint32_t pattern_per_block;     // pattern(b) = pattern_per_block ? b : 0
  const uint32_t* block_ids;      // blocks to process (null => block_base + 0..nblocks-1)
  uint64_t block_base;
  const uint16_t* loc;            // [pattern][W] locator logs
  uint32_t k, m, high_rate, chunk, end, W;
  uint32_t shard_bytes, nsym;
  uint64_t nblocks;   // entries processed in this launch
  uint16_t* scratch;  // nblocks * W * nsym
  GfDeviceTables t;
};
hipError_t launch_generic_decode(const GenericDecodeParams& p, hipStream_t stream);

// locator logs for npatterns erasure patterns: erased[p * W + x] (x < W); positions
// >= fill_from up to 65535 are also erased (LowRate virtual recovery); loc[p * W + x].
hipError_t launch_locator(const uint8_t* erased, uint32_t npatterns, uint32_t W, uint32_t fill_from,
                          const uint16_t* log_walsh, uint16_t* loc, hipStream_t stream);

// Shard restride (sizes that are not whole 64-byte chunks): pack = crate layout (tail chunk
// split into low / high halves) -> padded shards of ceil(S/64)*64 bytes (whole-chunk
// layout, zero symbols after the tail); unpack = the inverse, shards selected by mask.
hipError_t launch_restride(const uint8_t* src, uint64_t src_block_stride, uint64_t src_shard_stride, uint8_t* dst,
                           uint64_t dst_block_stride, uint64_t dst_shard_stride, uint32_t S, uint32_t nshards,
                           uint64_t nblocks, bool unpack, const uint64_t* mask, bool mask_per_block,
                           hipStream_t stream);

// ReedSolomonCoder batches: padding writer (payload null = in place) and padding strip
// (out[b] = payload length, or -1 for invalid padding).  data_bytes = 32 * S, % 16 == 0.
hipError_t launch_coder_pad(const uint8_t* payload, uint64_t payload_stride, const uint32_t* lens, uint8_t* cw,
                            uint64_t cw_stride, uint32_t data_bytes, uint64_t nslices, hipStream_t stream);
hipError_t launch_coder_strip(const uint8_t* cw, uint64_t cw_stride, uint32_t data_bytes, uint64_t nslices,
                              int64_t* out, hipStream_t stream);

// Synthetic blocks: splitmix64 u64 little-endian words, block b seeded seed_base + b.
hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nblocks, uint64_t block_bytes,
                                uint64_t dst_block_stride, uint64_t seed_base, hipStream_t stream);

}  // namespace ag
