// Host side of libalpenglow_rs.so: the C ABI declared in include/alpenglow_rs.h.
//
// Mirrors three reference interfaces on top of the HIP kernels (rs_kernels.hip):
//   * the reed-solomon-simd 3.1.0 encoder/decoder API the reference wrapper calls
//     (reed_solomon.rs:9,64-66,96-125,150-180,214-226)
//   * ReedSolomonCoder (reed_solomon.rs:47-232) and the ValidatedShreds checks
//     (validated_shreds.rs:34-114) in front of it
//   * batched, device-resident forms of the encode/decode for throughput
// All Reed-Solomon arithmetic runs on the GPU; the host does argument validation,
// padding/splitting (byte copies), pattern bookkeeping and table setup only.  There is
// no CPU compute fallback: without a device every call fails with AG_RS_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <memory>
#include <new>
#include <vector>

#include "../../include/alpenglow_rs.h"
#include "gf16.hpp"
#include "cipher.hpp"
#include "ed25519.hpp"
#include "slice.hpp"
#include "wire.hpp"
#include "merkle.hpp"
#include "rs_launch.hpp"
#include "rs_patterns.hpp"
#include "shredder.hpp"

using ag::build_corr_pattern;
using ag::build_syn_pattern;
using ag::corr_fits;
using ag::count_flags;
using ag::gf_invert;
using ag::next_pow2;
using ag::pack_flags;
using ag::window128_masks;
using ag::window64_masks;

namespace {

#define AG_HIP(expr)                                  \
  do {                                                \
    if ((expr) != hipSuccess) return AG_RS_ERR_DEVICE; \
  } while (0)

// Grow-only device buffer.
struct DevBuf {
  void* ptr = nullptr;
  size_t size = 0;
  int ensure(size_t n, hipStream_t stream) {
    if (n <= size) return AG_RS_OK;
    if (ptr) {
      if (hipStreamSynchronize(stream) != hipSuccess) return AG_RS_ERR_DEVICE;
      (void)hipFree(ptr);
      ptr = nullptr;
      size = 0;
    }
    if (hipMalloc(&ptr, n) != hipSuccess) return AG_RS_ERR_OUT_OF_MEMORY;
    size = n;
    return AG_RS_OK;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(ptr);
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    size = 0;
  }
};

// Grow-only pinned host buffer, mapped and coherent (fine-grained: never cached in the GPU's
// L2, so one call's kernels cannot read another call's stale bytes): the crate-API
// single-call kernels read and write it directly (zero-copy).
struct PinBuf {
  void* ptr = nullptr;
  size_t size = 0;
  int ensure(size_t n) {
    if (n <= size) return AG_RS_OK;
    release();
    if (hipHostMalloc(&ptr, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      ptr = nullptr;
      return AG_RS_ERR_OUT_OF_MEMORY;
    }
    if (hipHostGetDevicePointer(&dptr, ptr, 0) != hipSuccess) {
      release();
      return AG_RS_ERR_DEVICE;
    }
    size = n;
    return AG_RS_OK;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(ptr);
  }
  template <typename T>
  T* dev() const {  // the same bytes as the device addresses them (zero-copy over PCIe)
    return static_cast<T*>(dptr);
  }
  void* dptr = nullptr;
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    ptr = dptr = nullptr;
    size = 0;
  }
};

int check_geometry(size_t k, size_t m, size_t S) {
  if (ag::use_high_rate(k, m) < 0) return AG_RS_ERR_UNSUPPORTED_SHARD_COUNT;
  if (S == 0 || S % 2) return AG_RS_ERR_INVALID_SHARD_SIZE;
  if (S > 0xFFFFFFFEull) return AG_RS_ERR_INVALID_ARGUMENT;
  return AG_RS_OK;
}


// Single-chunk HighRate geometries served by the bitsliced N-point transform kernel:
// k <= N, next_pow2(m) == N, N in {32, 64}, whole 64-byte chunks.  Returns N or 0.
// (HighRate with a single chunk implies next_pow2(k) == N and k <= m.)
unsigned xform_points(size_t k, size_t m, size_t S) {
  if (S == 0 || S % 64 || ag::use_high_rate(k, m) != 1) return 0;
  const size_t n = next_pow2(m);
  return (n == 32 || n == 64) && k <= n ? static_cast<unsigned>(n) : 0;
}

// Multi-chunk HighRate encode with a small recovery chunk (encode_mc kernel): returns the
// chunk next_pow2(m) in {1, 2, 4} when k > chunk, k <= 64, whole 64-byte chunks; else 0.
unsigned mc_chunk(size_t k, size_t m, size_t S) {
  if (S == 0 || S % 64 || ag::use_high_rate(k, m) != 1 || k > 64) return 0;
  const size_t c = next_pow2(m);
  return c <= 4 && k > c ? static_cast<unsigned>(c) : 0;
}

// LowRate encode through the transform kernel, one launch per recovery chunk: returns the
// chunk next_pow2(k) in {32, 64} when the recovery chunks fit the launcher, else 0.
unsigned lowrate_chunk(size_t k, size_t m, size_t S) {
  if (S == 0 || S % 64 || ag::use_high_rate(k, m) != 0) return 0;
  const size_t c = next_pow2(k);
  const size_t chunks = (m + c - 1) / c;
  if (c == 32 && chunks <= 4) return 32;
  if (c == 64 && chunks <= 3) return 64;
  return 0;
}

}  // namespace

struct ag_rs_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  bool tables_ready = false;
  DevBuf d_exp, d_log, d_skew, d_log_walsh;
  DevBuf scratch;                         // generic-kernel work rows
  DevBuf d_flags, d_loc, d_blocks, d_mask;  // decode bookkeeping
  DevBuf d_xmask, d_rows, d_xblocks;        // bitsliced general decode: masks, matrices
  DevBuf d_x128, d_rows128;                 // W = 128 two-pass decode: masks, constants
  uint64_t last_classes[16] = {};           // patterns per decoder class of the last decode call
  int decode_depth = 0;                     // decode_device nesting (tail restrides decode inside)
  uint32_t last_encode_kernels = 0;         // EncodeKernelBit of the last ag_rs_encode_batch / coder deshred batch
  uint32_t last_window_kernels = 0;         // DecodeXKernelBit of the last coder deshred batch's window decode
  DevBuf d_syn, d_synblocks;                // syndrome decoder: patterns, block ids
  DevBuf d_corr, d_corrk, d_corrblocks;     // correction decoder: patterns, K picks, block ids
  DevBuf d_empty_roots;                     // Merkle EMPTY_ROOTS [32][8] words
  DevBuf d_merkle_nodes;                    // Merkle node scratch (callers without a nodes buffer)
  DevBuf d_aon_lens, d_aon_digests, d_aon_keys;  // all-or-nothing transforms
  DevBuf d_aon_lens2;                            // the side stream's SHA-256 lengths (AONT deshred)
  hipStream_t side = nullptr;                    // a second compute stream (AONT deshred's SHA-256)
  hipEvent_t side_fork = nullptr, side_join = nullptr;
  DevBuf d_slice_meta;                           // slice framing / parsing metadata
  DevBuf stage_pad, stage_mask;                  // restrided shards (sizes not whole 64-byte chunks)
  DevBuf d_lens, d_strip;                   // coder batches: payload lengths, strip results
  DevBuf d_reenc_mask;                      // uniform coder deshreds: the re-encode's store mask word
  DevBuf d_pipe_few, d_pipe_mask;           // composed deshred: too-few flags, re-encode store masks
  DevBuf d_present;                         // coder batches: per-slice present masks
  PinBuf h_present;                         // their pinned host staging
  hipEvent_t present_ev = nullptr;          // recorded after its upload
  PinBuf h_lens;                            // coder shred batches: pinned staging of the lengths
  hipEvent_t lens_ev = nullptr;             // recorded after its upload
  PinBuf h_strip;                           // coder deshred batches: pinned staging of the results
  PinBuf h_slice_meta;                      // slice parse batches: pinned staging of the results
  PinBuf h_pipe_meta;                       // composed deshreds: pinned staging of the per-slice columns
  DevBuf d_ed_base;                         // Ed25519 fixed-base table (ed25519.hpp)
  static constexpr int kPipeBufs = 28;
  DevBuf pipe[kPipeBufs];                   // composed shredder scratch (ag_shredder_*_batch)
  DevBuf d_sh_roots, d_sh_commit, d_sh_onvalid, d_sh_list;  // shred validation scratch
  DevBuf stage_in, stage_out;             // host-memory calls (unused; see slots)
  // host-memory calls: two staging slots, H2D / D2H streams next to the compute stream
  struct Slot {
    DevBuf in, out;
    hipEvent_t up = nullptr, done = nullptr, down = nullptr;
  } slot[2];
  hipStream_t h2d = nullptr, d2h = nullptr;
  DevBuf one_in, one_out;                 // crate-API single codeword
  // per-call server (latency_server_kernel): mailbox in mapped host memory, its own stream
  ag::LatencyMailbox* mb = nullptr;
  ag::LatencyMailbox* mb_dev = nullptr;
  hipStream_t server_stream = nullptr;
  uint32_t server_seq = 0;
  uint32_t server_p_seq = 0, server_dp_seq = 0;  // versions of the parameters last posted
  bool server_broken = false;  // a job timed out: the server path is off for this context
  bool fail_next_server_job = false;  // test aid: the next server job takes the timeout path
  uint64_t server_jobs[4] = {};        // jobs posted per LatencyJob kind (test aid)
  std::vector<PinBuf> abandoned_pins;  // staging a timed-out job named (freed once the server is gone)
  std::vector<uint64_t> mask_host;        // last store-mask words uploaded to d_mask
  std::vector<uint64_t> stage_mask_host;  // last restride masks uploaded to stage_mask
  std::vector<uint64_t> xmask_host;       // last general-decode masks (d_xmask), W = xmask_w
  size_t xmask_w = 0;
  bool xmask_poly = false;                // d_rows holds polynomial-basis constants (per-lane)
  std::vector<uint8_t> syn_key;             // (k, m, present flags) of the patterns in d_syn
  std::vector<uint8_t> corr_key;            // (k, m, present flags) of the patterns in d_corr
  std::vector<uint64_t> x128_host;          // last W = 128 masks uploaded to d_x128
  std::vector<uint32_t> x128_ids;           // their per-block ids (d_xblocks)

  int enter() { return hipSetDevice(device) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE; }

  int ensure_tables() {
    if (tables_ready) return AG_RS_OK;
    const ag::Gf16Tables& t = ag::gf16_tables();
    // log_walsh: Walsh-Hadamard transform (mod 65535) of the log table with log[0] := 0
    // (crate engine/tables.rs initialize_log_walsh).
    std::vector<uint16_t> lw(t.log, t.log + ag::kGfOrder);
    lw[0] = 0;
    for (size_t dist = 1; dist < ag::kGfOrder; dist <<= 1)
      for (size_t r = 0; r < ag::kGfOrder; r += 2 * dist)
        for (size_t i = r; i < r + dist; ++i) {
          const uint32_t a = lw[i], b = lw[i + dist];
          const uint32_t s = a + b, d = a - b;
          lw[i] = static_cast<uint16_t>(s + (s >> 16));
          lw[i + dist] = static_cast<uint16_t>(d + (d >> 16));
        }
    int st;
    if ((st = d_exp.ensure(sizeof t.exp, stream)) || (st = d_log.ensure(sizeof t.log, stream)) ||
        (st = d_skew.ensure(sizeof t.skew, stream)) || (st = d_log_walsh.ensure(lw.size() * 2, stream)))
      return st;
    AG_HIP(hipMemcpy(d_exp.ptr, t.exp, sizeof t.exp, hipMemcpyHostToDevice));
    AG_HIP(hipMemcpy(d_log.ptr, t.log, sizeof t.log, hipMemcpyHostToDevice));
    AG_HIP(hipMemcpy(d_skew.ptr, t.skew, sizeof t.skew, hipMemcpyHostToDevice));
    AG_HIP(hipMemcpy(d_log_walsh.ptr, lw.data(), lw.size() * 2, hipMemcpyHostToDevice));
    tables_ready = true;
    return AG_RS_OK;
  }

  ag::GfDeviceTables dtables() const {
    return {d_exp.as<uint16_t>(), d_log.as<uint16_t>(), d_skew.as<uint16_t>(), d_log_walsh.as<uint16_t>()};
  }

  int ensure_side_stream() {
    if (side) return AG_RS_OK;
    AG_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    AG_HIP(hipEventCreateWithFlags(&side_fork, hipEventDisableTiming));
    AG_HIP(hipEventCreateWithFlags(&side_join, hipEventDisableTiming));
    return AG_RS_OK;
  }

  int ensure_copy_streams() {
    if (h2d) return AG_RS_OK;
    AG_HIP(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
    AG_HIP(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
    for (Slot& s : slot) {
      AG_HIP(hipEventCreateWithFlags(&s.up, hipEventDisableTiming));
      AG_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
      AG_HIP(hipEventCreateWithFlags(&s.down, hipEventDisableTiming));
      AG_HIP(hipEventRecord(s.down, d2h));  // slots start free
    }
    return AG_RS_OK;
  }

  void server_stop() {
    if (!mb) return;
    (void)hipSetDevice(device);
    const auto t0 = std::chrono::steady_clock::now();
    if (__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE) != 0) {
      mb->kind = ag::kJobQuit;
      __atomic_store_n(&mb->doorbell, ++server_seq, __ATOMIC_RELEASE);
      while (__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE) != 0 &&
             std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
      }
    }
    if (__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE) != 0) {
      // a server that neither served nor quit (server_broken): waiting on its stream could
      // block forever, and it may still write the mailbox or an abandoned staging buffer,
      // so those stay allocated
      mb = mb_dev = nullptr;
      server_stream = nullptr;
      abandoned_pins.clear();
      return;
    }
    (void)hipStreamSynchronize(server_stream);  // the server has exited (quit or idle timeout)
    for (PinBuf& b : abandoned_pins) b.release();
    abandoned_pins.clear();
    (void)hipStreamDestroy(server_stream);
    (void)hipHostFree(mb);
    mb = mb_dev = nullptr;
    server_stream = nullptr;
  }

  ~ag_rs_ctx() {
    server_stop();
    if (side) {
      (void)hipSetDevice(device);
      (void)hipStreamSynchronize(side);
      (void)hipEventDestroy(side_fork);
      (void)hipEventDestroy(side_join);
      (void)hipStreamDestroy(side);
    }
    if (own_stream) {
      (void)hipSetDevice(device);
      (void)hipStreamSynchronize(own_stream);
    }
    if (h2d) {
      (void)hipStreamSynchronize(h2d);
      (void)hipStreamSynchronize(d2h);
      for (Slot& s : slot) {
        s.in.release();
        s.out.release();
        for (hipEvent_t e : {s.up, s.done, s.down})
          if (e) (void)hipEventDestroy(e);
      }
      (void)hipStreamDestroy(h2d);
      (void)hipStreamDestroy(d2h);
    }
    for (DevBuf* b : {&d_exp, &d_log, &d_skew, &d_log_walsh, &scratch, &d_flags, &d_loc, &d_blocks, &d_mask,
                      &d_xmask, &d_rows, &d_xblocks, &d_x128, &d_rows128, &d_syn, &d_synblocks, &d_corr, &d_corrk, &d_corrblocks, &d_empty_roots, &d_merkle_nodes, &d_aon_lens, &d_aon_digests, &d_aon_keys, &d_aon_lens2, &d_lens, &d_strip, &d_reenc_mask, &d_ed_base, &d_sh_roots, &d_sh_commit, &d_sh_onvalid, &d_sh_list, &stage_in, &stage_out, &stage_pad, &stage_mask, &d_slice_meta, &one_in,
                      &one_out, &d_pipe_few, &d_pipe_mask, &d_present})
      b->release();
    for (DevBuf& b : pipe) b.release();
    if (present_ev) {
      (void)hipEventSynchronize(present_ev);
      (void)hipEventDestroy(present_ev);
    }
    h_present.release();
    if (lens_ev) {
      (void)hipEventSynchronize(lens_ev);
      (void)hipEventDestroy(lens_ev);
    }
    h_lens.release();
    h_strip.release();
    h_slice_meta.release();
    h_pipe_meta.release();
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }
};

namespace {

// Host-memory calls: bytes (in + out) per staging group; two groups in flight.
constexpr size_t kStageGroupBytes = size_t{64} << 20;

// Scratch budget of the generic kernels (per launch).
constexpr size_t kGenericScratchBytes = size_t{512} << 20;

// Restrided shard buffer (shard sizes that are not whole 64-byte chunks), per group.
constexpr size_t kRestrideGroupBytes = size_t{2048} << 20;

int encode_device(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, const uint8_t* orig,
                  size_t ostride, uint8_t* rec, size_t rstride);

// Shard sizes that are not whole 64-byte chunks (a slice's tail, reed_solomon.rs:94-95):
// the whole chunks of every shard run in place on the bitsliced kernels (shard stride S,
// chunks_per_shard = S / 64: the kernels take any alignment), and only the T = S mod 64 tail
// bytes of each shard -- in the crate's tail layout exactly a T-byte shard --
// are restrided into a padded 64-byte chunk per shard (restride_kernel), run there and
// restrided back.  Taken when the padded geometry has a bitsliced path.
size_t padded_shard(size_t S) { return (S + 63) / 64 * 64; }
// Byte-odd buffers or strides: every shard goes through the restride (its byte path)
bool odd_layout(const void* a, const void* b, size_t sa, size_t sb) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | sa | sb) & 1) != 0;
}

// Virtual shards of Sv bytes at byte `off` of every shard (shard stride sstride) are packed
// into padded shards, encoded there, and the recovery shards' pieces unpacked.
int encode_restrided(ag_rs_ctx* c, size_t k, size_t m, size_t Sv, size_t sstride, size_t off, size_t nblocks,
                     const uint8_t* orig, size_t ostride, uint8_t* rec, size_t rstride) {
  const size_t Sp = padded_shard(Sv), per_block = (k + m) * Sp;
  const size_t group = std::max<size_t>(1, kRestrideGroupBytes / per_block);
  int st = c->stage_pad.ensure(std::min(group, nblocks) * per_block, c->stream);
  if (st) return st;
  c->last_encode_kernels |= ag::kEkRestride;
  uint8_t* pad = c->stage_pad.as<uint8_t>();
  for (size_t b0 = 0; b0 < nblocks; b0 += group) {
    const size_t nb = std::min(group, nblocks - b0);
    if (ag::launch_restride(orig + b0 * ostride + off, ostride, sstride, pad, per_block, Sp, static_cast<uint32_t>(Sv),
                            static_cast<uint32_t>(k), nb, false, nullptr, false, c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
    if ((st = encode_device(c, k, m, Sp, nb, pad, per_block, pad + k * Sp, per_block))) return st;
    if (ag::launch_restride(pad + k * Sp, per_block, Sp, rec + b0 * rstride + off, rstride, sstride,
                            static_cast<uint32_t>(Sv), static_cast<uint32_t>(m), nb, true, nullptr, false,
                            c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
  }
  return AG_RS_OK;
}

// The encode over the first S bytes of every shard (S % 64 == 0 on the bitsliced paths;
// shards sstride >= S bytes apart).
int encode_cols(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t sstride, size_t nblocks, const uint8_t* orig,
                size_t ostride, uint8_t* rec, size_t rstride) {
  const unsigned npts = xform_points(k, m, S);
  const unsigned mc = mc_chunk(k, m, S);
  const unsigned lr = lowrate_chunk(k, m, S);
  if (npts || mc || lr) {
    ag::XformParams p{};
    p.in = orig;
    p.in_block_stride = ostride;
    p.in_shard_stride = sstride;
    p.out = rec;
    p.out_block_stride = rstride;
    p.out_shard_stride = sstride;
    p.n_in = static_cast<uint32_t>(k);
    p.n_out = static_cast<uint32_t>(m);
    p.chunks_per_shard = static_cast<uint32_t>(S / 64);
    p.total_columns = static_cast<uint64_t>(nblocks) * (S / 64);
    hipError_t e = hipSuccess;
    if (npts) {
      c->last_encode_kernels |= npts == 32 ? ag::encode32_kernel(p) : ag::kEkXformH8;
      e = ag::launch_xform(npts == 32 ? ag::XformKind::kEncode32 : ag::XformKind::kEncode64, p, c->stream);
    } else if (mc) {
      c->last_encode_kernels |= ag::kEkEncodeMc;
      e = ag::launch_encode_mc(mc, p, c->stream);
    } else {
      for (size_t j = 0; j * lr < m && e == hipSuccess;) {  // one launch per recovery chunk
        ag::XformParams pj = p;
        pj.out = rec + j * lr * sstride;
        if (lr == 32 && j % 2 == 0 && (j + 1) * lr < m && j < 4) {  // chunks j, j + 1 in one launch
          pj.n_out = static_cast<uint32_t>(std::min<size_t>(2 * lr, m - j * lr));
          c->last_encode_kernels |= ag::kEkLowRate2;
          e = ag::launch_xform_lowrate2(static_cast<unsigned>(j / 2), pj, c->stream);
          j += 2;
          continue;
        }
        pj.n_out = static_cast<uint32_t>(std::min<size_t>(lr, m - j * lr));
        c->last_encode_kernels |= ag::kEkLowRate;
        e = ag::launch_xform_lowrate(lr, static_cast<unsigned>(j), pj, c->stream);
        ++j;
      }
    }
    return e == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
  }
  int st = c->ensure_tables();
  if (st) return st;
  const int hr = ag::use_high_rate(k, m);
  const size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  const size_t cover = hr ? k : m;
  const size_t rows = std::max(chunk, (cover + chunk - 1) / chunk * chunk);
  const size_t nsym = S / 2;
  const size_t per_block = rows * nsym * 2;
  const size_t per_launch = std::max<size_t>(1, kGenericScratchBytes / per_block);
  if ((st = c->scratch.ensure(std::min(per_launch, nblocks) * per_block, c->stream))) return st;
  for (size_t b0 = 0; b0 < nblocks; b0 += per_launch) {
    ag::GenericEncodeParams p{};
    p.orig = orig + b0 * ostride;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.rec = rec + b0 * rstride;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.k = static_cast<uint32_t>(k);
    p.m = static_cast<uint32_t>(m);
    p.high_rate = static_cast<uint32_t>(hr);
    p.chunk = static_cast<uint32_t>(chunk);
    p.rows = static_cast<uint32_t>(rows);
    p.shard_bytes = static_cast<uint32_t>(S);
    p.nsym = static_cast<uint32_t>(nsym);
    p.nblocks = std::min(per_launch, nblocks - b0);
    p.scratch = c->scratch.as<uint16_t>();
    p.t = c->dtables();
    c->last_encode_kernels |= ag::kEkGeneric;
    if (ag::launch_generic_encode(p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  return AG_RS_OK;
}

// A 32-point transform over shards that end in a split tail chunk, one launch on the caller's
// buffers (no restride): chunks_per_shard = ceil(S / 64), the last chunk of every shard read
// and written as 16-byte windows of its tail (rs_xform.hpp tile_io_g).  (Two launches -- the
// whole chunks with the tails skipped, then the tails alone -- measured slower: 3.76 / 4.06
// TB/s at S = 1000 against 3.8-4.0 / 4.2-4.4; the whole-chunk pass alone ran at 4.35 TB/s,
// its shards' last 64-byte sectors left partial for the second pass to complete,
// profiles/r05_tail_split_kernel_stats.csv.)
int launch_tail(ag_rs_ctx* c, ag::XformKind kind, const ag::XformParams& p, bool encode) {
  if (encode) c->last_encode_kernels |= ag::encode32_kernel(p);
  return ag::launch_xform(kind, p, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

// 32-point encodes of shards ending in a split tail chunk (S % 64 != 0, S even): the TAIL
// transforms read and write the tail in place (launch_tail), no restride
int encode_tail32(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, const uint8_t* orig, size_t ostride,
                  uint8_t* rec, size_t rstride) {
  const size_t cps = padded_shard(S) / 64;
  ag::XformParams p{};
  p.in = orig;
  p.in_block_stride = ostride;
  p.in_shard_stride = S;
  p.out = rec;
  p.out_block_stride = rstride;
  p.out_shard_stride = S;
  p.n_in = static_cast<uint32_t>(k);
  p.n_out = static_cast<uint32_t>(m);
  p.chunks_per_shard = static_cast<uint32_t>(cps);
  p.total_columns = static_cast<uint64_t>(nblocks) * cps;
  p.tail_bytes = static_cast<uint32_t>(S % 64);
  return launch_tail(c, ag::XformKind::kEncode32, p, true);
}

int encode_device(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, const uint8_t* orig,
                  size_t ostride, uint8_t* rec, size_t rstride) {
  if (nblocks == 0) return AG_RS_OK;
  const size_t Sp = padded_shard(S);
  if (S % 2 == 0 && (xform_points(k, m, Sp) || mc_chunk(k, m, Sp) || lowrate_chunk(k, m, Sp))) {
    if (odd_layout(orig, rec, ostride, rstride))
      return encode_restrided(c, k, m, S, S, 0, nblocks, orig, ostride, rec, rstride);
    const size_t full = S / 64 * 64, tail = S - full;
    if (tail >= 16 && xform_points(k, m, Sp) == 32)  // (tail windows are 16 bytes of the tail itself)
      return encode_tail32(c, k, m, S, nblocks, orig, ostride, rec, rstride);
    int st;
    if (full && (st = encode_cols(c, k, m, full, S, nblocks, orig, ostride, rec, rstride))) return st;
    if (tail && (st = encode_restrided(c, k, m, tail, S, full, nblocks, orig, ostride, rec, rstride))) return st;
    return AG_RS_OK;
  }
  return encode_cols(c, k, m, S, S, nblocks, orig, ostride, rec, rstride);
}

int decode_device(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                  const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres, size_t npat,
                  int mode);

// ag_rs_coder_deshred_batch's flag packer (below): word b = data flags | coding 0..31 << 32
bool pack_present_words(const uint8_t* dpres, const uint8_t* cpres, size_t m, size_t n, uint64_t* pres,
                        bool* any_full_data);

// The decode counterpart of encode_restrided: originals and recovery shards of a group of
// blocks go to one padded buffer, the bitsliced decoders run there, and only the restored
// originals are restrided back (a store mask per pattern).
int decode_restrided(ag_rs_ctx* c, size_t k, size_t m, size_t Sv, size_t sstride, size_t off, size_t nblocks,
                     uint8_t* orig, size_t ostride, const uint8_t* rec, size_t rstride, const uint8_t* opres,
                     const uint8_t* rpres, size_t npat, int mode) {
  const size_t Sp = padded_shard(Sv), per_block = (k + m) * Sp;
  // store masks: the absent originals of each pattern (k <= 64 on every bitsliced path)
  // and the pack masks: only present shards are packed (decoders never read absent ones)
  std::vector<uint64_t> mask(3 * npat);
  const uint64_t kmask = k >= 64 ? ~uint64_t{0} : (uint64_t{1} << k) - 1;
  const bool rmask = m <= 64;
  if (k == 32 && m == 32) {  // the flags packed 32 at a time (AVX2 where the host has it)
    std::vector<uint64_t> w(npat);
    bool full_data = false;
    (void)pack_present_words(opres, rpres, m, npat, w.data(), &full_data);
    for (size_t p = 0; p < npat; ++p) {
      if (__builtin_popcountll(w[p]) < 32) return AG_RS_ERR_NOT_ENOUGH_SHARDS;  // nothing launched yet
      mask[p] = ~w[p] & kmask;
      mask[npat + p] = w[p] & kmask;
      mask[2 * npat + p] = w[p] >> 32;
    }
  } else {
    for (size_t p = 0; p < npat; ++p)  // NotEnoughShards before anything is launched
      if (count_flags(opres + p * k, k) + count_flags(rpres + p * m, m) < k) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
    for (size_t p = 0; p < npat; ++p) {
      mask[p] = ~pack_flags(opres + p * k, k) & kmask;
      mask[npat + p] = pack_flags(opres + p * k, k);
      mask[2 * npat + p] = rmask ? pack_flags(rpres + p * m, m) : 0;
    }
  }
  // upload only when the masks changed (steady-state batches reuse them, no sync)
  int st;
  if (mask != c->stage_mask_host) {
    AG_HIP(hipStreamSynchronize(c->stream));  // queued restrides / a pending upload may read the old masks
    if ((st = c->stage_mask.ensure(3 * npat * 8, c->stream))) return st;
    c->stage_mask_host = std::move(mask);
    if (hipMemcpyAsync(c->stage_mask.ptr, c->stage_mask_host.data(), 3 * npat * 8, hipMemcpyHostToDevice,
                       c->stream) != hipSuccess) {
      c->stage_mask_host.clear();  // never matches a mask set (3 * npat >= 3 words)
      return AG_RS_ERR_DEVICE;
    }
  }
  const uint64_t* d_omask = c->stage_mask.as<uint64_t>() + npat;
  const uint64_t* d_rmask = rmask ? c->stage_mask.as<uint64_t>() + 2 * npat : nullptr;
  const size_t group = std::max<size_t>(1, kRestrideGroupBytes / per_block);
  if ((st = c->stage_pad.ensure(std::min(group, nblocks) * per_block, c->stream))) return st;
  uint8_t* pad = c->stage_pad.as<uint8_t>();
  for (size_t b0 = 0; b0 < nblocks; b0 += group) {
    const size_t nb = std::min(group, nblocks - b0);
    const size_t p0 = npat > 1 ? b0 : 0, np = npat > 1 ? nb : 1;
    if (ag::launch_restride(orig + b0 * ostride + off, ostride, sstride, pad, per_block, Sp, static_cast<uint32_t>(Sv),
                            static_cast<uint32_t>(k), nb, false, d_omask + p0, npat > 1, c->stream) != hipSuccess ||
        ag::launch_restride(rec + b0 * rstride + off, rstride, sstride, pad + k * Sp, per_block, Sp,
                            static_cast<uint32_t>(Sv), static_cast<uint32_t>(m), nb, false,
                            d_rmask ? d_rmask + p0 : nullptr, npat > 1, c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
    if ((st = decode_device(c, k, m, Sp, nb, pad, per_block, pad + k * Sp, per_block, opres + p0 * k, rpres + p0 * m,
                            np, mode)))
      return st;
    if (ag::launch_restride(pad, per_block, Sp, orig + b0 * ostride + off, ostride, sstride, static_cast<uint32_t>(Sv),
                            static_cast<uint32_t>(k), nb, true, c->stage_mask.as<uint64_t>() + p0, npat > 1,
                            c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
  }
  return AG_RS_OK;
}

// The decode over the first S bytes of every shard (S % 64 == 0 on the bitsliced paths;
// shards sstride >= S bytes apart; any alignment).
int decode_cols(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t sstride, size_t nblocks, uint8_t* orig,
                size_t ostride, const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres,
                size_t npat, int mode);

int decode_device_body(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                       const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres, size_t npat,
                       int mode);
int decode_cols_device_patterns(ag_rs_ctx* c, size_t S, size_t sstride, size_t nblocks, uint8_t* orig,
                                size_t ostride, const uint8_t* rec, size_t rstride, const uint8_t* opres,
                                const uint8_t* rpres);
constexpr int kNotApplicable = -1;

// last_classes counts every pattern of the outermost call: the whole-chunk decode and the
// tail restride's inner decode of a shard size with S % 64 != 0 add up (reset once per call)
int decode_device(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                  const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres, size_t npat,
                  int mode) {
  if (c->decode_depth == 0) std::fill(std::begin(c->last_classes), std::end(c->last_classes), uint64_t{0});
  ++c->decode_depth;
  const int st = decode_device_body(c, k, m, S, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode);
  --c->decode_depth;
  return st;
}

// The 32-point full-recovery reconstruct (decode class "transform") of shards ending in a split
// tail chunk: xform8's TAIL variant restores the erased originals, tail included, in place.
int decode_tail32(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                  const uint8_t* rec, size_t rstride, const uint8_t* opres, size_t npat) {
  if (npat > 1) {
    bool same = true;
    for (size_t p = 1; p < npat && same; ++p) same = std::memcmp(opres, opres + p * k, k) == 0;
    if (same) npat = 1;
  }
  std::vector<uint64_t> mask(npat);
  const uint64_t kmask = (uint64_t{1} << k) - 1;  // k <= 32
  bool any = false;
  for (size_t p = 0; p < npat; ++p) {
    mask[p] = ~pack_flags(opres + p * k, k) & kmask;
    ++c->last_classes[mask[p] ? 1 : 0];
    any = any || mask[p];
  }
  if (!any) return AG_RS_OK;
  int st;
  if (mask != c->mask_host) {
    AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read mask_host
    if ((st = c->d_mask.ensure(mask.size() * 8, c->stream))) return st;
    c->mask_host = mask;
    AG_HIP(hipMemcpyAsync(c->d_mask.ptr, c->mask_host.data(), mask.size() * 8, hipMemcpyHostToDevice, c->stream));
  }
  const size_t cps = padded_shard(S) / 64;
  ag::XformParams p{};
  p.in = rec;
  p.in_block_stride = rstride;
  p.in_shard_stride = S;
  p.out = orig;
  p.out_block_stride = ostride;
  p.out_shard_stride = S;
  p.out_mask = c->d_mask.as<uint64_t>();
  p.pattern_per_block = npat > 1 ? 1u : 0u;
  p.n_in = static_cast<uint32_t>(m);
  p.n_out = static_cast<uint32_t>(k);
  p.chunks_per_shard = static_cast<uint32_t>(cps);
  p.total_columns = static_cast<uint64_t>(nblocks) * cps;
  p.tail_bytes = static_cast<uint32_t>(S % 64);
  p.out_low_half = std::all_of(mask.begin(), mask.end(), [](uint64_t w) { return (w >> 16) == 0; });
  return launch_tail(c, ag::XformKind::kDecode32, p, false);
}

int decode_device_body(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                       const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres, size_t npat,
                       int mode) {
  if (nblocks == 0) return AG_RS_OK;
  const bool odd = odd_layout(orig, rec, ostride, rstride);
  if (k <= 64 && (S % 64 != 0 || odd) && S % 2 == 0) {
    const size_t Sp = padded_shard(S);
    const int hr = ag::use_high_rate(k, m);
    const size_t xw = hr == 1 ? next_pow2(next_pow2(m) + k) : 0;
    if (xform_points(k, m, Sp) || mc_chunk(k, m, Sp) || lowrate_chunk(k, m, Sp) || xw == 32 || xw == 64) {
      if (odd) return decode_restrided(c, k, m, S, S, 0, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode);
      const size_t full = S / 64 * 64, tail = S - full;
      // every pattern restores from the full 32-point recovery set (or restores nothing): the
      // TAIL transform decodes the whole shards, tail included, in place in one launch
      if (tail >= 16 && xform_points(k, m, Sp) == 32 && m == 32 && mode == AG_RS_DECODE_ANY_K) {
        bool all_full = true;
        for (size_t p = 0; p < npat && all_full; ++p) all_full = count_flags(rpres + p * m, m) == m;
        if (all_full) return decode_tail32(c, k, m, S, nblocks, orig, ostride, rec, rstride, opres, npat);
      }
      int st;
      // per-block 32:32 patterns with lost recovery shards (ANY_K): the per-lane window decode
      // takes the whole shards, the T-byte tail as one more column (decode_h8 TAIL), no restride
      if (tail != 0 && npat > 1 && npat == nblocks && k == 32 && m == 32 && hr == 1 && mode == AG_RS_DECODE_ANY_K) {
        st = decode_cols_device_patterns(c, S, S, nblocks, orig, ostride, rec, rstride, opres, rpres);
        if (st != kNotApplicable) return st;
      }
      if (full && (st = decode_cols(c, k, m, full, S, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode)))
        return st;
      return decode_restrided(c, k, m, tail, S, full, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode);
    }
  }
  return decode_cols(c, k, m, S, S, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode);
}


// Per-block patterns of the 32:32 code on tiles that straddle blocks (chunks per shard not a
// multiple of 64: the follower's slices, tail shreds' whole chunks and their restrided tails),
// ANY_K, where some recovery shards are lost: the per-lane window decode with its masks built
// on the device (launch_pipe_patterns, the coder batches' kernel), so the host only packs the
// presence flags (AVX2) -- the per-pattern classification, window masks and mask compares cost
// ~25 ns per pattern and call on the host, 3-7 ms per 131 072-block call
// (profiles/r06_kt_tail_lose4_kernel_stats.csv against the call's wall time).  kNotApplicable
// when some pattern has its full recovery set and lost data (the transform decodes those) --
// the host route below takes the call then.
int decode_cols_device_patterns(ag_rs_ctx* c, size_t S, size_t sstride, size_t nblocks, uint8_t* orig,
                                size_t ostride, const uint8_t* rec, size_t rstride, const uint8_t* opres,
                                const uint8_t* rpres) {
  constexpr size_t k = 32, m = 32, W = 64;
  // S = 64 C, or 64 C + T with a tail of T >= 16 bytes as the last column (decode_h8 TAIL)
  const size_t n = nblocks, cps = (S + 63) / 64;
  int st;
  if (c->present_ev) AG_HIP(hipEventSynchronize(c->present_ev));  // the previous upload has read h_present
  else AG_HIP(hipEventCreateWithFlags(&c->present_ev, hipEventDisableTiming));
  if ((st = c->h_present.ensure(n * 8))) return st;
  uint64_t* pres = c->h_present.as<uint64_t>();
  bool full_data = false;
  (void)pack_present_words(opres, rpres, m, n, pres, &full_data);
  size_t restore = 0;
  for (size_t b = 0; b < n; ++b) {
    const uint64_t w = pres[b];
    if (__builtin_popcountll(w) < static_cast<int>(k)) return AG_RS_ERR_NOT_ENOUGH_SHARDS;  // nothing launched
    const bool data_full = (w & 0xFFFFFFFFull) == 0xFFFFFFFFull;
    if (!data_full && (w >> 32) == 0xFFFFFFFFull) return kNotApplicable;
    restore += data_full ? 0 : 1;
  }
  c->last_classes[0] += n - restore;
  c->last_classes[3] += restore;
  if (!restore) return AG_RS_OK;
  if ((st = c->ensure_tables()) || (st = c->d_present.ensure(n * 8, c->stream)) ||
      (st = c->d_pipe_few.ensure(n, c->stream)) || (st = c->d_xmask.ensure(3 * n * 8, c->stream)) ||
      (st = c->d_rows.ensure(n * W * 4, c->stream)))
    return st;
  c->xmask_host.clear();  // d_xmask / d_rows no longer hold the host route's cached patterns
  c->xmask_w = 0;
  AG_HIP(hipMemcpyAsync(c->d_present.ptr, pres, n * 8, hipMemcpyHostToDevice, c->stream));
  AG_HIP(hipEventRecord(c->present_ev, c->stream));
  uint64_t* xm = c->d_xmask.as<uint64_t>();
  uint32_t* rows = c->d_rows.as<uint32_t>();
  if (ag::launch_pipe_patterns(c->d_present.as<uint64_t>(), n, xm, c->d_pipe_few.as<uint8_t>(), false, c->stream) !=
          hipSuccess ||
      ag::launch_decode_rows(xm, xm + n, static_cast<uint32_t>(n), static_cast<uint32_t>(W), c->dtables(), rows, true,
                             c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  ag::DecodeXParams p{};
  p.rec = rec;
  p.rec_block_stride = rstride;
  p.rec_shard_stride = sstride;
  p.orig = orig;
  p.orig_block_stride = ostride;
  p.orig_shard_stride = sstride;
  p.pmask = xm + n;
  p.rows = rows;
  p.k = static_cast<uint32_t>(k);
  p.m = static_cast<uint32_t>(m);
  p.chunk = 32;
  p.low_rate = 0;
  p.chunks_per_shard = static_cast<uint32_t>(cps);
  p.total_columns = static_cast<uint64_t>(n) * cps;
  p.per_lane = 1;
  p.rows_w = static_cast<uint32_t>(W);
  p.any_k = 1;  // launch_pipe_patterns keeps exactly k survivors
  p.tail_bytes = static_cast<uint32_t>(S % 64);
  if (ag::launch_decode_x(static_cast<unsigned>(W), 0, p, (p.total_columns + 63) / 64, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  return AG_RS_OK;
}

int decode_cols(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t sstride, size_t nblocks, uint8_t* orig,
                size_t ostride, const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres,
                size_t npat, int mode) {
  const int hr = ag::use_high_rate(k, m);
  // one erasure pattern repeated for every block (a repair batch, a uniform loss) is one
  // pattern: uniform store masks, and the bitsliced kernels regardless of block alignment
  if (npat > 1) {
    bool same = true;
    for (size_t p = 1; p < npat && same; ++p)
      same = std::memcmp(opres, opres + p * k, k) == 0 && std::memcmp(rpres, rpres + p * m, m) == 0;
    if (same) npat = 1;
  }
  // classify patterns: 0 = nothing to restore, 1 = transform kernel (full recovery set),
  // 3 = bitsliced general decoder, 2 = table-driven generic kernel.
  // The transform inverts the encoder only when all N recovery points exist (m == N):
  // with m < N the points m..N-1 were never stored.
  std::vector<uint8_t> cls(npat);
  const bool aligned = true;  // the bitsliced kernels take any alignment (16-byte pieces, unaligned mode)
  const unsigned npts = xform_points(k, m, S);
  const bool fast_geo = mode == AG_RS_DECODE_ANY_K && npts != 0 && m == npts && aligned;
  // decode_x window: HighRate, W = next_pow2(chunk + k) in {32, 64}; or the LowRate
  // sub-window [0, 64) when next_pow2(k) = 32 (CodingOnly 32:64, PETS 32:33): originals
  // at 0..k-1, their zero padding k..31 (known zeros, survivors for free), recovery
  // 0..31 at 32..63.  The LowRate polynomial has degree < 32, so any 32 survivors inside
  // the window decode it there (ANY_K; patterns with fewer survivors inside take another
  // path).
  const bool x_lr = hr == 0 && next_pow2(k) == 32 && mode == AG_RS_DECODE_ANY_K;
  const size_t xchunk = hr == 1 ? next_pow2(m) : x_lr ? 32 : 0;
  const size_t xw = hr == 1 ? next_pow2(xchunk + k) : x_lr ? 64 : 0;
  const size_t xm_rec = hr == 1 ? m : std::min<size_t>(m, 32);  // recovery shards inside the window
  const size_t cps = S / 64;
  if (npat > 1 && npat == nblocks && hr == 1 && k == 32 && m == 32 && mode == AG_RS_DECODE_ANY_K && S % 64 == 0 &&
      cps % 64 != 0 && aligned) {
    const int st = decode_cols_device_patterns(c, S, sstride, nblocks, orig, ostride, rec, rstride, opres, rpres);
    if (st != kNotApplicable) return st;
  }
  // decode_x: one pattern per tile (single pattern, or tiles that never straddle blocks),
  // else per-lane patterns (each lane one chunk of one block: the follower's per-slice
  // patterns on 1 KiB shreds)
  const bool x_geo = (hr == 1 || x_lr) && S % 64 == 0 && (xw == 32 || xw == 64) && aligned;
  const bool x_per_lane = npat > 1 && cps % 64 != 0;
  // decode_syn: the encode_mc geometries (chunk <= 4), any k survivors, same tiling rule
  const unsigned syn_chunk = mode == AG_RS_DECODE_ANY_K && aligned && (npat == 1 || cps % 64 == 0)
                                 ? mc_chunk(k, m, S) : 0;
  std::vector<uint16_t> G;
  if (syn_chunk) {
    G.resize(m * k);
    ag::hr_generator(k, m, G.data());
  }
  std::vector<ag::SynPattern> syn;
  if (syn_chunk) syn.resize(npat);
  // LowRate (next_pow2(k) = 32): recovery chunk j = FFT_{32(j+1)}(IFFT_0(originals)), so a
  // fully present chunk inverts through the transform kernel: originals =
  // FFT_0(IFFT_{32(j+1)}(chunk j)).  ANY_K only (MDS uniqueness), chunks j < 4.
  const bool lr_geo = mode == AG_RS_DECODE_ANY_K && hr == 0 && next_pow2(k) == 32 && S % 64 == 0 && aligned;
  std::vector<uint8_t> lr_chunk(npat, 0xFF);
  bool any_lr = false;
  // decode_c: the 32-point full-window geometries (HighRate, m = 32, k <= 32) with lost
  // recovery shards; any k survivors, same tiling rule
  // (a batch of fewer tiles than CUs is latency-bound -- a single slice per call -- and the
  // correction's serial SALU phase made one tile a 43 us kernel: those take the window decoder)
  const uint64_t ncols = static_cast<uint64_t>(nblocks) * cps;
  const bool corr_geo = mode == AG_RS_DECODE_ANY_K && hr == 1 && m == 32 && k <= 32 && S % 64 == 0 && aligned &&
                        (npat == 1 || cps % 64 == 0) && ncols < (uint64_t{1} << 31) && ncols >= 64 * 256;
  // W = 128 windows as two 64-point passes (decode_x16 PASS 1 / 2): the originals in one
  // window half -- HighRate with next_pow2(m) = 64 (originals at 64..127), LowRate with
  // next_pow2(k) <= 64 and next_pow2(k) + m in (64, 128] (originals at 0..k-1).  Any k
  // survivors (exactly k: the codeword is then unique, so the pass split's own erasure set
  // gives the crate's bytes)
  const size_t c128 = hr == 1 ? next_pow2(m) : next_pow2(k);
  const bool x128_geo = S % 64 == 0 && k <= 64 &&
                        (hr == 1 ? c128 == 64 : (c128 <= 64 && c128 + m > 64 && c128 + m <= 128));
  bool any_fast = false, any_generic = false, any_x = false, any_syn = false, any_corr = false, any_x128 = false;
  for (size_t p = 0; p < npat; ++p) {
    const size_t no = count_flags(opres + p * k, k), nr = count_flags(rpres + p * m, m);
    if (no + nr < k) return AG_RS_ERR_NOT_ENOUGH_SHARDS;  // nothing launched yet
    if (no == k) {
      cls[p] = 0;
    } else if (fast_geo && nr == m) {
      cls[p] = 1;
      any_fast = true;
    } else if (lr_geo && [&] {
                 for (size_t j = 0; j < 4 && 32 * (j + 1) <= m; ++j) {
                   bool full = true;
                   for (size_t i = 32 * j; i < 32 * (j + 1) && full; ++i) full = rpres[p * m + i] != 0;
                   if (full) {
                     lr_chunk[p] = static_cast<uint8_t>(j);
                     return true;
                   }
                 }
                 return false;
               }()) {
      cls[p] = 5;
      any_lr = true;
    } else if (syn_chunk && build_syn_pattern(k, m, opres + p * k, rpres + p * m, G.data(), &syn[p])) {
      cls[p] = 4;
      any_syn = true;
    } else if (corr_geo && corr_fits(k, no, nr)) {
      cls[p] = 6;
      any_corr = true;
    } else if (x_geo && (hr == 1 || count_flags(opres + p * k, k) + count_flags(rpres + p * m, xm_rec) >= k)) {
      cls[p] = 3;
      any_x = true;
    } else if (x128_geo && (mode == AG_RS_DECODE_ANY_K || no + nr == k)) {
      cls[p] = 8;
      any_x128 = true;
    } else {
      cls[p] = 2;
      any_generic = true;
    }
  }
  for (size_t p = 0; p < npat; ++p) ++c->last_classes[cls[p]];
  int st;
  if (any_fast) {
    // store mask word per pattern: restore original i iff the pattern is fast and i is absent
    std::vector<uint64_t> mask(npat, 0);
    const uint64_t kmask = k >= 64 ? ~uint64_t{0} : (uint64_t{1} << k) - 1;  // npts <= 64: k <= 64
    for (size_t p = 0; p < npat; ++p)
      if (cls[p] == 1) mask[p] = ~pack_flags(opres + p * k, k) & kmask;
    // upload only when the pattern set changed (steady-state batches reuse it, no sync)
    if (mask != c->mask_host) {
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read mask_host
      if ((st = c->d_mask.ensure(mask.size() * 8, c->stream))) return st;
      c->mask_host = mask;
      AG_HIP(hipMemcpyAsync(c->d_mask.ptr, c->mask_host.data(), mask.size() * 8, hipMemcpyHostToDevice, c->stream));
    }
    ag::XformParams p{};
    p.in = rec;
    p.in_block_stride = rstride;
    p.in_shard_stride = sstride;
    p.out = orig;
    p.out_block_stride = ostride;
    p.out_shard_stride = sstride;
    p.out_mask = c->d_mask.as<uint64_t>();
    p.pattern_per_block = npat > 1 ? 1u : 0u;
    p.n_in = static_cast<uint32_t>(m);
    p.n_out = static_cast<uint32_t>(k);
    p.chunks_per_shard = static_cast<uint32_t>(S / 64);
    p.total_columns = static_cast<uint64_t>(nblocks) * (S / 64);
    // all restored originals among shards 0..15: the output-pruned 32-point transform
    // (64-point: every restored original among shards 0..31, xform_h8's pruned FFT)
    p.out_low_half = (npts == 32 && std::all_of(mask.begin(), mask.end(), [](uint64_t w) { return (w >> 16) == 0; })) ||
                     (npts == 64 && std::all_of(mask.begin(), mask.end(), [](uint64_t w) { return (w >> 32) == 0; }));
    const auto kind = npts == 32 ? ag::XformKind::kDecode32 : ag::XformKind::kDecode64;
    if (ag::launch_xform(kind, p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  if (any_lr) {
    // one launch per recovery chunk in use; store masks select that chunk's patterns
    for (unsigned j = 0; j < 4; ++j) {
      std::vector<uint64_t> mask(npat, 0);
      bool used = false;
      for (size_t p = 0; p < npat; ++p)
        if (cls[p] == 5 && lr_chunk[p] == j) {
          used = true;
          for (size_t i = 0; i < k; ++i)
            if (!opres[p * k + i]) mask[p] |= uint64_t{1} << i;
        }
      if (!used) continue;
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read mask_host
      if ((st = c->d_mask.ensure(mask.size() * 8, c->stream))) return st;
      c->mask_host = mask;
      AG_HIP(hipMemcpyAsync(c->d_mask.ptr, c->mask_host.data(), mask.size() * 8, hipMemcpyHostToDevice, c->stream));
      ag::XformParams p{};
      p.in = rec + static_cast<size_t>(32) * j * sstride;
      p.in_block_stride = rstride;
      p.in_shard_stride = sstride;
      p.out = orig;
      p.out_block_stride = ostride;
      p.out_shard_stride = sstride;
      p.out_mask = c->d_mask.as<uint64_t>();
      p.pattern_per_block = npat > 1 ? 1u : 0u;
      p.n_in = 32;
      p.n_out = static_cast<uint32_t>(k);
      p.chunks_per_shard = static_cast<uint32_t>(S / 64);
      p.total_columns = static_cast<uint64_t>(nblocks) * (S / 64);
      if (ag::launch_xform_lowrate_decode(j, p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    }
  }
  if (any_syn) {
    // pattern upload only when (k, m, flags) changed; non-syndrome patterns stay zeroed
    std::vector<uint8_t> key(16 + npat * (k + m));
    const uint64_t km[2] = {k, m};
    std::memcpy(key.data(), km, 16);
    for (size_t p = 0; p < npat; ++p) {
      if (cls[p] != 4) continue;
      std::memcpy(&key[16 + p * (k + m)], opres + p * k, k);
      std::memcpy(&key[16 + p * (k + m) + k], rpres + p * m, m);
    }
    if (key != c->syn_key) {
      for (size_t p = 0; p < npat; ++p)
        if (cls[p] != 4) std::memset(&syn[p], 0, sizeof syn[p]);
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read d_syn
      if ((st = c->d_syn.ensure(npat * sizeof(ag::SynPattern), c->stream))) return st;
      AG_HIP(hipMemcpy(c->d_syn.ptr, syn.data(), npat * sizeof(ag::SynPattern), hipMemcpyHostToDevice));
      c->syn_key = key;
    }
    ag::DecodeSynParams p{};
    p.rec = rec;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.orig = orig;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.pat = c->d_syn.as<ag::SynPattern>();
    p.k = static_cast<uint32_t>(k);
    p.chunks_per_shard = static_cast<uint32_t>(cps);
    p.total_columns = static_cast<uint64_t>(nblocks) * cps;
    if (npat == 1) {
      p.ntiles = (p.total_columns + 63) / 64;
    } else {
      p.per_block = 1;
      p.tiles_per_block = static_cast<uint32_t>(cps / 64);
      std::vector<uint32_t> ids;
      for (size_t b = 0; b < nblocks; ++b)
        if (cls[b] == 4) ids.push_back(static_cast<uint32_t>(b));
      if (ids.size() != nblocks) {
        AG_HIP(hipStreamSynchronize(c->stream));  // a previous id upload may be pending
        if ((st = c->d_synblocks.ensure(ids.size() * 4, c->stream))) return st;
        AG_HIP(hipMemcpy(c->d_synblocks.ptr, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
        p.block_ids = c->d_synblocks.as<uint32_t>();
      }
      p.ntiles = static_cast<uint64_t>(ids.size()) * p.tiles_per_block;
    }
    if (ag::launch_decode_syn(syn_chunk, p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  if (any_corr) {
    // patterns are built and uploaded only when (k, m, flags) changed
    std::vector<uint8_t> key(16 + npat * (k + m));
    const uint64_t km[2] = {k, m};
    std::memcpy(key.data(), km, 16);
    for (size_t p = 0; p < npat; ++p) {
      if (cls[p] != 6) continue;
      std::memcpy(&key[16 + p * (k + m)], opres + p * k, k);
      std::memcpy(&key[16 + p * (k + m) + k], rpres + p * m, m);
    }
    if (key != c->corr_key) {
      std::vector<ag::CorrPattern> corr(npat);
      std::vector<uint32_t> pool;
      for (size_t p = 0; p < npat; ++p) {
        if (cls[p] != 6) {
          std::memset(&corr[p], 0, sizeof corr[p]);
          continue;
        }
        // corr_fits admitted the pattern; the MDS property makes N invertible
        if (!build_corr_pattern(k, opres + p * k, rpres + p * m, &corr[p], pool)) return AG_RS_ERR_DEVICE;
      }
      c->corr_key.clear();
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read d_corr
      if ((st = c->d_corr.ensure(npat * sizeof(ag::CorrPattern), c->stream))) return st;
      if ((st = c->d_corrk.ensure(std::max<size_t>(pool.size(), 1) * 4, c->stream))) return st;
      AG_HIP(hipMemcpy(c->d_corr.ptr, corr.data(), npat * sizeof(ag::CorrPattern), hipMemcpyHostToDevice));
      if (!pool.empty()) AG_HIP(hipMemcpy(c->d_corrk.ptr, pool.data(), pool.size() * 4, hipMemcpyHostToDevice));
      c->corr_key = key;
    }
    ag::DecodeCParams p{};
    p.rec = rec;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.orig = orig;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.pat = c->d_corr.as<ag::CorrPattern>();
    p.kpool = c->d_corrk.as<uint32_t>();
    p.k = static_cast<uint32_t>(k);
    p.chunks_per_shard = static_cast<uint32_t>(cps);
    p.total_columns = static_cast<uint64_t>(nblocks) * cps;
    if (npat == 1) {
      p.ntiles = (p.total_columns + 63) / 64;
    } else {
      p.per_block = 1;
      p.tiles_per_block = static_cast<uint32_t>(cps / 64);
      std::vector<uint32_t> ids;
      for (size_t b = 0; b < nblocks; ++b)
        if (cls[b] == 6) ids.push_back(static_cast<uint32_t>(b));
      if (ids.size() != nblocks) {
        AG_HIP(hipStreamSynchronize(c->stream));  // a previous id upload may be pending
        if ((st = c->d_corrblocks.ensure(ids.size() * 4, c->stream))) return st;
        AG_HIP(hipMemcpy(c->d_corrblocks.ptr, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
        p.block_ids = c->d_corrblocks.as<uint32_t>();
      }
      p.ntiles = static_cast<uint64_t>(ids.size()) * p.tiles_per_block;
    }
    if (ag::launch_decode_c(p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  if (any_x) {
    if ((st = c->ensure_tables())) return st;
    // per pattern: [erased (locator) | present (loaded) | restored] position bits
    std::vector<uint64_t> xm(3 * npat, 0);
    for (size_t p = 0; p < npat; ++p) {
      if (cls[p] != 3) continue;
      uint64_t e, in, out;
      window64_masks(hr == 1, k, m, xchunk, xm_rec, opres + p * k, rpres + p * m, mode == AG_RS_DECODE_ANY_K, &e, &in,
                     &out);
      xm[p] = e;
      xm[npat + 2 * p] = in;
      xm[npat + 2 * p + 1] = out;
    }
    // polynomial-basis constants (one word per position) for decode_x16 (W = 64) and for
    // per-lane patterns; bitsliced matrices for decode_x<4>'s wave-uniform four-Russians products
    const bool poly = xw == 64 || (npat > 1 && x_per_lane);
    if (xm != c->xmask_host || xw != c->xmask_w || poly != c->xmask_poly) {
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read xmask_host
      if ((st = c->d_xmask.ensure(xm.size() * 8, c->stream))) return st;
      if ((st = c->d_rows.ensure(npat * xw * (poly ? 1 : 16) * 4, c->stream))) return st;
      c->xmask_host = xm;
      c->xmask_w = xw;
      c->xmask_poly = poly;
      AG_HIP(hipMemcpyAsync(c->d_xmask.ptr, c->xmask_host.data(), xm.size() * 8, hipMemcpyHostToDevice, c->stream));
      const uint64_t* dx = c->d_xmask.as<uint64_t>();
      if (ag::launch_decode_rows(dx, dx + npat, static_cast<uint32_t>(npat), static_cast<uint32_t>(xw), c->dtables(),
                                 c->d_rows.as<uint32_t>(), poly, c->stream) != hipSuccess)
        return AG_RS_ERR_DEVICE;
    }
    ag::DecodeXParams p{};
    p.rec = rec;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.orig = orig;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.pmask = c->d_xmask.as<uint64_t>() + npat;
    p.rows = c->d_rows.as<uint32_t>();
    p.k = static_cast<uint32_t>(k);
    p.m = static_cast<uint32_t>(xm_rec);
    p.chunk = static_cast<uint32_t>(xchunk);
    p.low_rate = hr == 1 ? 0u : 1u;
    p.chunks_per_shard = static_cast<uint32_t>(cps);
    p.total_columns = static_cast<uint64_t>(nblocks) * cps;
    p.rows_w = static_cast<uint32_t>(xw);
    p.any_k = mode == AG_RS_DECODE_ANY_K ? 1u : 0u;
    uint64_t ntiles;
    if (npat == 1) {
      ntiles = (p.total_columns + 63) / 64;
    } else if (x_per_lane) {
      p.per_lane = 1;  // lanes of blocks outside class 3 find all-zero masks: no loads, no stores
      ntiles = (p.total_columns + 63) / 64;
    } else {
      p.per_block = 1;
      p.tiles_per_block = static_cast<uint32_t>(cps / 64);
      std::vector<uint32_t> ids;
      for (size_t b = 0; b < nblocks; ++b)
        if (cls[b] == 3) ids.push_back(static_cast<uint32_t>(b));
      if (ids.size() != nblocks) {
        AG_HIP(hipStreamSynchronize(c->stream));  // a previous id upload may be pending
        if ((st = c->d_xblocks.ensure(ids.size() * 4, c->stream))) return st;
        AG_HIP(hipMemcpy(c->d_xblocks.ptr, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
        p.block_ids = c->d_xblocks.as<uint32_t>();
      }
      ntiles = static_cast<uint64_t>(ids.size()) * p.tiles_per_block;
    }
    if (ag::launch_decode_x(static_cast<unsigned>(xw), 0, p, ntiles, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  if (any_x128) {
    if ((st = c->ensure_tables())) return st;
    // per pattern: m6 = {erased, present, restored} as (positions 0..63, 64..127) pairs, then
    // the two passes' (present in the loaded half, restored) pairs
    const size_t oh = hr == 1 ? 1 : 0;  // the output (originals') window half
    std::vector<uint64_t> xm(10 * npat, 0);
    for (size_t p = 0; p < npat; ++p) {
      if (cls[p] != 8) continue;
      window128_masks(hr == 1, k, m, c128, opres + p * k, rpres + p * m, &xm[10 * p]);
    }
    // device: m6 [npat][6], pass-1 pairs [npat][2], pass-2 pairs [npat][2]
    std::vector<uint64_t> dev(10 * npat);
    for (size_t p = 0; p < npat; ++p) {
      for (int i = 0; i < 6; ++i) dev[6 * p + i] = xm[10 * p + i];
      dev[6 * npat + 2 * p] = xm[10 * p + 6];
      dev[6 * npat + 2 * p + 1] = xm[10 * p + 7];
      dev[8 * npat + 2 * p] = xm[10 * p + 8];
      dev[8 * npat + 2 * p + 1] = xm[10 * p + 9];
    }
    // upload (and rebuild the constants) only when the masks changed; the copy is ordered on
    // the stream and reads the context's own host vector, so nothing waits for it
    if (dev != c->x128_host) {
      AG_HIP(hipStreamSynchronize(c->stream));  // a pending upload may still read x128_host
      if ((st = c->d_x128.ensure(dev.size() * 8, c->stream)) || (st = c->d_rows128.ensure(npat * 128 * 4, c->stream)))
        return st;
      c->x128_host = std::move(dev);
      if (hipMemcpyAsync(c->d_x128.ptr, c->x128_host.data(), c->x128_host.size() * 8, hipMemcpyHostToDevice,
                         c->stream) != hipSuccess) {
        c->x128_host.clear();
        return AG_RS_ERR_DEVICE;
      }
      if (ag::launch_decode_rows128(c->d_x128.as<uint64_t>(), static_cast<uint32_t>(npat), c->dtables(),
                                    c->d_rows128.as<uint32_t>(), c->stream) != hipSuccess)
        return AG_RS_ERR_DEVICE;
    }
    const uint64_t* d6 = c->d_x128.as<uint64_t>();
    ag::DecodeXParams p{};
    p.rec = rec;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.orig = orig;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.rows = c->d_rows128.as<uint32_t>();
    p.rows_w = 128;
    p.k = static_cast<uint32_t>(k);
    p.m = static_cast<uint32_t>(m);
    p.chunk = static_cast<uint32_t>(c128);
    p.low_rate = hr == 1 ? 0u : 1u;
    p.chunks_per_shard = static_cast<uint32_t>(cps);
    p.total_columns = static_cast<uint64_t>(nblocks) * cps;
    uint64_t ntiles;
    std::vector<uint32_t> ids;
    if (npat == 1) {
      ntiles = (p.total_columns + 63) / 64;
    } else if (x_per_lane) {
      p.per_lane = 1;  // lanes of blocks outside class 8 find all-zero masks: no loads, no stores
      ntiles = (p.total_columns + 63) / 64;
    } else {
      p.per_block = 1;
      p.tiles_per_block = static_cast<uint32_t>(cps / 64);
      for (size_t b = 0; b < nblocks; ++b)
        if (cls[b] == 8) ids.push_back(static_cast<uint32_t>(b));
      // count before the upload below moves `ids` into the context
      ntiles = static_cast<uint64_t>(ids.size()) * p.tiles_per_block;
      if (ids.size() != nblocks) {
        AG_HIP(hipStreamSynchronize(c->stream));  // a pending id upload may still read x128_ids
        if ((st = c->d_xblocks.ensure(ids.size() * 4, c->stream))) return st;
        c->x128_ids = std::move(ids);
        AG_HIP(hipMemcpyAsync(c->d_xblocks.ptr, c->x128_ids.data(), c->x128_ids.size() * 4, hipMemcpyHostToDevice,
                              c->stream));
        p.block_ids = c->d_xblocks.as<uint32_t>();
      }
    }
    // recovery shards beyond the window half the kernel loads are addressed from p.rec with
    // the window position; launch_decode_x checks the geometry
    p.m = static_cast<uint32_t>(std::min<size_t>(m, p.chunk));
    for (int pass = 1; pass <= 2; ++pass) {
      p.pmask = d6 + (pass == 1 ? 6 : 8) * npat;
      if (ag::launch_decode_x(128, pass, p, ntiles, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    }
  }
  if (!any_generic) return AG_RS_OK;

  if ((st = c->ensure_tables())) return st;
  const size_t chunk = hr ? next_pow2(m) : next_pow2(k);
  const size_t end = chunk + (hr ? k : m);
  const size_t W = next_pow2(end);
  // erasure flags per pattern over the transform window (crate decoder_high/low.rs)
  std::vector<uint8_t> erased(npat * W, 0);
  for (size_t p = 0; p < npat; ++p) {
    if (cls[p] != 2) continue;
    uint8_t* e = &erased[p * W];
    const size_t opos = hr ? chunk : 0, rpos = hr ? 0 : chunk;
    for (size_t i = 0; i < k; ++i) e[opos + i] = opres[p * k + i] ? 0 : 1;
    for (size_t i = 0; i < m; ++i) e[rpos + i] = rpres[p * m + i] ? 0 : 1;
    if (hr) {
      for (size_t i = m; i < chunk; ++i) e[i] = 1;  // virtual recovery points
    } else {
      for (size_t i = end; i < W; ++i) e[i] = 1;  // beyond the recovery block
    }
  }
  // per-pattern device copies of the present flags and erasures
  const size_t flag_bytes = npat * (k + m) + erased.size();
  if ((st = c->d_flags.ensure(flag_bytes, c->stream))) return st;
  if ((st = c->d_loc.ensure(npat * W * 2, c->stream))) return st;
  std::vector<uint8_t> hostflags(flag_bytes);
  std::memcpy(hostflags.data(), opres, npat * k);
  std::memcpy(hostflags.data() + npat * k, rpres, npat * m);
  std::memcpy(hostflags.data() + npat * (k + m), erased.data(), erased.size());
  uint8_t* dflags = c->d_flags.as<uint8_t>();
  AG_HIP(hipMemcpyAsync(dflags, hostflags.data(), flag_bytes, hipMemcpyHostToDevice, c->stream));
  if (ag::launch_locator(dflags + npat * (k + m), static_cast<uint32_t>(npat), static_cast<uint32_t>(W),
                         hr ? 65536u : static_cast<uint32_t>(end), c->d_log_walsh.as<uint16_t>(),
                         c->d_loc.as<uint16_t>(), c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  // blocks handled by the generic kernel
  std::vector<uint32_t> ids;
  if (npat > 1) {
    for (size_t b = 0; b < nblocks; ++b)
      if (cls[b] == 2) ids.push_back(static_cast<uint32_t>(b));
    if ((st = c->d_blocks.ensure(ids.size() * 4, c->stream))) return st;
    AG_HIP(hipMemcpyAsync(c->d_blocks.ptr, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, c->stream));
  }
  const size_t ngen = npat > 1 ? ids.size() : nblocks;
  const size_t nsym = S / 2;
  const size_t per_block = W * nsym * 2;
  const size_t per_launch = std::max<size_t>(1, kGenericScratchBytes / per_block);
  if ((st = c->scratch.ensure(std::min(per_launch, ngen) * per_block, c->stream))) return st;
  for (size_t b0 = 0; b0 < ngen; b0 += per_launch) {
    ag::GenericDecodeParams p{};
    p.orig = orig;
    p.orig_block_stride = ostride;
    p.orig_shard_stride = sstride;
    p.rec = rec;
    p.rec_block_stride = rstride;
    p.rec_shard_stride = sstride;
    p.orig_present = dflags;
    p.rec_present = dflags + npat * k;
    p.pattern_per_block = npat > 1 ? 1u : 0u;
    p.block_ids = npat > 1 ? c->d_blocks.as<uint32_t>() + b0 : nullptr;
    p.block_base = npat > 1 ? 0 : b0;
    p.loc = c->d_loc.as<uint16_t>();
    p.k = static_cast<uint32_t>(k);
    p.m = static_cast<uint32_t>(m);
    p.high_rate = static_cast<uint32_t>(hr);
    p.chunk = static_cast<uint32_t>(chunk);
    p.end = static_cast<uint32_t>(end);
    p.W = static_cast<uint32_t>(W);
    p.shard_bytes = static_cast<uint32_t>(S);
    p.nsym = static_cast<uint32_t>(nsym);
    p.nblocks = std::min(per_launch, ngen - b0);
    p.scratch = c->scratch.as<uint16_t>();
    p.t = c->dtables();
    if (ag::launch_generic_decode(p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  // host vectors above are read by async copies: finish before they go out of scope
  AG_HIP(hipStreamSynchronize(c->stream));
  return AG_RS_OK;
}

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

const char* ag_rs_status_string(int s) {
  switch (s) {
    case AG_RS_OK: return "ok";
    case AG_RS_ERR_INVALID_SHARD_SIZE: return "invalid shard size";
    case AG_RS_ERR_DIFFERENT_SHARD_SIZE: return "different shard size";
    case AG_RS_ERR_TOO_FEW_ORIGINAL_SHARDS: return "too few original shards";
    case AG_RS_ERR_TOO_MANY_ORIGINAL_SHARDS: return "too many original shards";
    case AG_RS_ERR_INVALID_ORIGINAL_SHARD_INDEX: return "invalid original shard index";
    case AG_RS_ERR_INVALID_RECOVERY_SHARD_INDEX: return "invalid recovery shard index";
    case AG_RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX: return "duplicate original shard index";
    case AG_RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX: return "duplicate recovery shard index";
    case AG_RS_ERR_NOT_ENOUGH_SHARDS: return "not enough shards";
    case AG_RS_ERR_UNSUPPORTED_SHARD_COUNT: return "unsupported shard count";
    case AG_RS_ERR_TOO_MUCH_DATA: return "too much data";
    case AG_RS_ERR_INVALID_PADDING: return "invalid padding";
    case AG_RS_ERR_INVALID_LAYOUT: return "invalid layout";
    case AG_RS_ERR_BAD_ENCODING: return "bad encoding";
    case AG_RS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case AG_RS_ERR_NO_DEVICE: return "no HIP device";
    case AG_RS_ERR_DEVICE: return "HIP runtime error";
    case AG_RS_ERR_OUT_OF_MEMORY: return "out of device memory";
    case AG_RS_ERR_NOT_RESTORED: return "shard not restored";
    default: return "unknown status";
  }
}

int ag_rs_abi_version(void) { return AG_RS_ABI_VERSION; }

int ag_rs_device_count(int* count) {
  if (!count) return AG_RS_ERR_INVALID_ARGUMENT;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return AG_RS_OK;
}

int ag_rs_ctx_create(int device, ag_rs_ctx** out) {
  if (!out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return AG_RS_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return AG_RS_ERR_NO_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return AG_RS_ERR_DEVICE;
  auto* c = new (std::nothrow) ag_rs_ctx();
  if (!c) return AG_RS_ERR_OUT_OF_MEMORY;
  c->device = device;
  if (hipStreamCreate(&c->own_stream) != hipSuccess) {
    delete c;
    return AG_RS_ERR_DEVICE;
  }
  c->stream = c->own_stream;
  *out = c;
  return AG_RS_OK;
}

void ag_rs_ctx_destroy(ag_rs_ctx* c) { delete c; }

// A stream switch first drains the old stream (its queued kernels may still read the cached
// pattern uploads and scratch) and forgets the upload caches, whose copies were ordered on it.
static int switch_stream(ag_rs_ctx* c, hipStream_t s) {
  if (s == c->stream) return AG_RS_OK;
  if (c->enter() || hipStreamSynchronize(c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  c->stream = s;
  c->mask_host.clear();
  c->stage_mask_host.clear();
  c->xmask_host.clear();
  c->x128_host.clear();
  c->syn_key.clear();
  c->corr_key.clear();
  return AG_RS_OK;
}

int ag_rs_ctx_set_stream(ag_rs_ctx* c, void* s) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  return switch_stream(c, static_cast<hipStream_t>(s));
}

int ag_rs_ctx_reset_stream(ag_rs_ctx* c) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  return switch_stream(c, c->own_stream);
}

void* ag_rs_ctx_stream(ag_rs_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int ag_rs_ctx_synchronize(ag_rs_ctx* c) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_rs_use_high_rate(size_t k, size_t m) {
  const int hr = ag::use_high_rate(k, m);
  return hr < 0 ? -AG_RS_ERR_UNSUPPORTED_SHARD_COUNT : hr;
}

// Test aid (not in the public header's contract): patterns per decoder class in the last
// decode on this context -- 0 nothing to restore, 1 full-recovery transform, 2 table-driven
// generic, 3 W <= 64 window (decode_x / decode_x16), 4 syndrome, 5 LowRate chunk transform,
// 6 correction (decode_c), 8 W = 128 two-pass window.
int ag_rs_internal_last_decode_classes(ag_rs_ctx* c, uint64_t* out16) {
  if (!c || !out16) return AG_RS_ERR_INVALID_ARGUMENT;
  std::memcpy(out16, c->last_classes, sizeof c->last_classes);
  return AG_RS_OK;
}

// Test aid (not in the header): the encode kernels (ag::EncodeKernelBit) the last
// ag_rs_encode_batch call on this context launched.
// Test aid (not in the header): the W = 64 window kernels (DecodeXKernelBit) the last coder
// deshred batch on the context launched.
int ag_rs_internal_last_window_kernels(ag_rs_ctx* c, uint32_t* out) {
  if (!c || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = c->last_window_kernels;
  return AG_RS_OK;
}

// Test aid (not in the header): per-call server jobs posted on the context, per LatencyJob kind
// (encode, decode, decode half, decode_pk).
int ag_rs_internal_server_jobs(ag_rs_ctx* c, uint64_t* out4) {
  if (!c || !out4) return AG_RS_ERR_INVALID_ARGUMENT;
  std::copy(std::begin(c->server_jobs), std::end(c->server_jobs), out4);
  return AG_RS_OK;
}

// Diagnostic (not in the header): the in-kernel duration of the last per-call server job on the
// coder's context, doorbell seen -> its stores released, then its four phases (kind read,
// parameters + cache invalidate, tile, release): ns[5], 0 before any job.
int ag_rs_internal_coder_last_job_ns(ag_rs_coder* coder, uint64_t* ns);

// Test aid (not in the header): the context's next per-call server job takes the timeout path
// (retired, staging abandoned, server path off) without waiting 5 s.
int ag_rs_internal_fail_next_server_job(ag_rs_ctx* c) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  c->fail_next_server_job = true;
  return AG_RS_OK;
}

int ag_rs_internal_last_encode_kernels(ag_rs_ctx* c, uint32_t* out) {
  if (!c || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = c->last_encode_kernels;
  return AG_RS_OK;
}

int ag_rs_has_fast_path(size_t k, size_t m, size_t S) {
  // shard sizes that are not whole 64-byte chunks run restrided (padded) on the same kernels
  if (S == 0 || S % 2) return 0;
  const size_t Sp = padded_shard(S);
  return xform_points(k, m, Sp) || mc_chunk(k, m, Sp) || lowrate_chunk(k, m, Sp) ? 1 : 0;
}

int ag_rs_encode_batch(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, const uint8_t* orig,
                       size_t ostride, uint8_t* rec, size_t rstride, int memory) {
  if (!c || (nblocks && (!orig || !rec))) return AG_RS_ERR_INVALID_ARGUMENT;
  int st = check_geometry(k, m, S);
  if (st) return st;
  if (ostride < k * S || rstride < m * S) return AG_RS_ERR_INVALID_ARGUMENT;
  if ((st = c->enter())) return st;
  c->last_encode_kernels = 0;
  if (memory == AG_RS_MEM_DEVICE) return encode_device(c, k, m, S, nblocks, orig, ostride, rec, rstride);
  if (memory != AG_RS_MEM_HOST) return AG_RS_ERR_INVALID_ARGUMENT;
  // host memory: groups of blocks through two device staging slots, H2D / compute / D2H
  // overlapped across groups (pinned host buffers give the full PCIe rate)
  const size_t in_b = k * S, out_b = m * S;
  const size_t group = std::max<size_t>(1, kStageGroupBytes / (in_b + out_b));
  if ((st = c->ensure_copy_streams())) return st;
  size_t g = 0;
  for (size_t b0 = 0; b0 < nblocks; b0 += group, ++g) {
    const size_t n = std::min(group, nblocks - b0);
    auto& sl = c->slot[g & 1];
    AG_HIP(hipStreamWaitEvent(c->h2d, sl.down, 0));  // slot free: its previous download is done
    if ((st = sl.in.ensure(group * in_b, c->h2d)) || (st = sl.out.ensure(group * out_b, c->h2d))) return st;
    AG_HIP(hipMemcpy2DAsync(sl.in.ptr, in_b, orig + b0 * ostride, ostride, in_b, n, hipMemcpyHostToDevice, c->h2d));
    AG_HIP(hipEventRecord(sl.up, c->h2d));
    AG_HIP(hipStreamWaitEvent(c->stream, sl.up, 0));
    if ((st = encode_device(c, k, m, S, n, sl.in.as<uint8_t>(), in_b, sl.out.as<uint8_t>(), out_b))) break;
    AG_HIP(hipEventRecord(sl.done, c->stream));
    AG_HIP(hipStreamWaitEvent(c->d2h, sl.done, 0));
    AG_HIP(hipMemcpy2DAsync(rec + b0 * rstride, rstride, sl.out.ptr, out_b, out_b, n, hipMemcpyDeviceToHost, c->d2h));
    AG_HIP(hipEventRecord(sl.down, c->d2h));
  }
  AG_HIP(hipStreamSynchronize(c->stream));
  AG_HIP(hipStreamSynchronize(c->d2h));
  return st;
}

int ag_rs_decode_batch(ag_rs_ctx* c, size_t k, size_t m, size_t S, size_t nblocks, uint8_t* orig, size_t ostride,
                       const uint8_t* rec, size_t rstride, const uint8_t* opres, const uint8_t* rpres, size_t npat,
                       int mode, int memory) {
  if (!c || !opres || !rpres || (nblocks && (!orig || !rec))) return AG_RS_ERR_INVALID_ARGUMENT;
  int st = check_geometry(k, m, S);
  if (st) return st;
  if (npat != 1 && npat != nblocks) return AG_RS_ERR_INVALID_ARGUMENT;
  if (mode != AG_RS_DECODE_EXACT && mode != AG_RS_DECODE_ANY_K) return AG_RS_ERR_INVALID_ARGUMENT;
  if (ostride < k * S || rstride < m * S) return AG_RS_ERR_INVALID_ARGUMENT;
  if ((st = c->enter())) return st;
  if (memory == AG_RS_MEM_DEVICE)
    return decode_device(c, k, m, S, nblocks, orig, ostride, rec, rstride, opres, rpres, npat, mode);
  if (memory != AG_RS_MEM_HOST) return AG_RS_ERR_INVALID_ARGUMENT;
  // pattern validity is checked up front so that an error leaves `orig` untouched
  for (size_t p = 0; p < npat; ++p) {
    size_t cnt = 0;
    for (size_t i = 0; i < k; ++i) cnt += opres[p * k + i] != 0;
    for (size_t i = 0; i < m; ++i) cnt += rpres[p * m + i] != 0;
    if (cnt < k) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  }
  const size_t o_b = k * S, r_b = m * S;
  const size_t group = std::max<size_t>(1, kStageGroupBytes / (o_b + r_b));
  if ((st = c->ensure_copy_streams())) return st;
  // One pattern: move only what the kernels read and write -- present originals up (none
  // when the transform path restores from the full recovery set), erased originals down.
  bool up_orig_all = npat > 1, down_all = npat > 1;
  bool need_orig = true;
  if (npat == 1) {
    size_t nr = 0, no = 0;
    for (size_t i = 0; i < m; ++i) nr += rpres[i] != 0;
    for (size_t i = 0; i < k; ++i) no += opres[i] != 0;
    if (no == k) return AG_RS_OK;  // nothing to restore
    const unsigned npts = xform_points(k, m, S);
    need_orig = !(mode == AG_RS_DECODE_ANY_K && npts && m == npts && nr == m);
  }
  size_t g = 0;
  for (size_t b0 = 0; b0 < nblocks; b0 += group, ++g) {
    const size_t n = std::min(group, nblocks - b0);
    auto& sl = c->slot[g & 1];
    AG_HIP(hipStreamWaitEvent(c->h2d, sl.down, 0));
    if ((st = sl.in.ensure(group * r_b, c->h2d)) || (st = sl.out.ensure(group * o_b, c->h2d))) return st;
    AG_HIP(hipMemcpy2DAsync(sl.in.ptr, r_b, rec + b0 * rstride, rstride, r_b, n, hipMemcpyHostToDevice, c->h2d));
    if (up_orig_all) {
      AG_HIP(hipMemcpy2DAsync(sl.out.ptr, o_b, orig + b0 * ostride, ostride, o_b, n, hipMemcpyHostToDevice, c->h2d));
    } else if (need_orig) {
      for (size_t i = 0; i < k; ++i)
        if (opres[i])
          AG_HIP(hipMemcpy2DAsync(sl.out.as<uint8_t>() + i * S, o_b, orig + b0 * ostride + i * S, ostride, S, n,
                                  hipMemcpyHostToDevice, c->h2d));
    }
    AG_HIP(hipEventRecord(sl.up, c->h2d));
    AG_HIP(hipStreamWaitEvent(c->stream, sl.up, 0));
    const uint8_t* op = npat > 1 ? opres + b0 * k : opres;
    const uint8_t* rp = npat > 1 ? rpres + b0 * m : rpres;
    if ((st = decode_device(c, k, m, S, n, sl.out.as<uint8_t>(), o_b, sl.in.as<uint8_t>(), r_b, op, rp,
                            npat > 1 ? n : 1, mode)))
      break;
    AG_HIP(hipEventRecord(sl.done, c->stream));
    AG_HIP(hipStreamWaitEvent(c->d2h, sl.done, 0));
    if (down_all) {
      AG_HIP(hipMemcpy2DAsync(orig + b0 * ostride, ostride, sl.out.ptr, o_b, o_b, n, hipMemcpyDeviceToHost, c->d2h));
    } else {
      for (size_t i = 0; i < k; ++i)
        if (!opres[i])
          AG_HIP(hipMemcpy2DAsync(orig + b0 * ostride + i * S, ostride, sl.out.as<uint8_t>() + i * S, o_b, S, n,
                                  hipMemcpyDeviceToHost, c->d2h));
    }
    AG_HIP(hipEventRecord(sl.down, c->d2h));
  }
  AG_HIP(hipStreamSynchronize(c->stream));
  AG_HIP(hipStreamSynchronize(c->d2h));
  return st;
}

int ag_rs_fill_splitmix(ag_rs_ctx* c, uint8_t* dst, size_t nblocks, size_t block_bytes, size_t dst_stride,
                        uint64_t seed_base) {
  if (!c || (nblocks && !dst) || block_bytes % 8 || dst_stride < block_bytes) return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  return ag::launch_fill_splitmix(dst, nblocks, block_bytes, dst_stride, seed_base, c->stream) == hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}

// ---- slice Merkle trees --------------------------------------------------------------

size_t ag_merkle_height(size_t n) {
  size_t h = 0;
  for (size_t len = n; len > 1; len = (len + 1) / 2) ++h;
  return h;
}

size_t ag_merkle_node_count(size_t n) {
  size_t total = n;
  for (size_t len = n; len > 1;) {
    len = (len + 1) / 2;
    total += len;
  }
  return total;
}

int ag_merkle_empty_root(size_t height, uint8_t out[32]) {
  if (!out || height >= static_cast<size_t>(ag::kMerkleMaxHeight)) return AG_RS_ERR_INVALID_ARGUMENT;
  uint32_t er[ag::kMerkleMaxHeight][8];
  ag::merkle_empty_roots(er);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) out[4 * i + b] = static_cast<uint8_t>(er[height][i] >> (24 - 8 * b));
  return AG_RS_OK;
}

namespace {
int ensure_empty_roots(ag_rs_ctx* c) {
  if (c->d_empty_roots.ptr) return AG_RS_OK;
  uint32_t er[ag::kMerkleMaxHeight][8];
  ag::merkle_empty_roots(er);
  int st = c->d_empty_roots.ensure(sizeof er, c->stream);
  if (st) return st;
  AG_HIP(hipMemcpy(c->d_empty_roots.ptr, er, sizeof er, hipMemcpyHostToDevice));
  return AG_RS_OK;
}
}  // namespace

int ag_merkle_build_batch(ag_rs_ctx* c, size_t n_leaves, size_t leaf_bytes, size_t nslices, const uint8_t* leaves,
                          size_t leaf_stride, size_t slice_stride, uint8_t* roots, uint8_t* nodes,
                          size_t nodes_stride, uint8_t* proofs, size_t proofs_stride) {
  if (!c || n_leaves == 0 || n_leaves > AG_MERKLE_MAX_LEAVES || leaf_bytes >= (size_t{1} << 28))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if ((leaf_bytes && !leaves) || !roots || (n_leaves > 1 && leaf_stride < leaf_bytes) ||
      (nslices > 1 && slice_stride < (n_leaves - 1) * leaf_stride + leaf_bytes))
    return AG_RS_ERR_INVALID_ARGUMENT;
  const size_t h = ag_merkle_height(n_leaves);
  if ((nodes && (nodes_stride % 16 || (nslices > 1 && nodes_stride < 32 * ag_merkle_node_count(n_leaves)))) ||
      (proofs && (proofs_stride % 16 || (nslices > 1 && proofs_stride < 32 * h * n_leaves))) ||
      reinterpret_cast<uintptr_t>(roots) % 16 || reinterpret_cast<uintptr_t>(nodes) % 16 ||
      reinterpret_cast<uintptr_t>(proofs) % 16)
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_empty_roots(c);
  if (st) return st;
  ag::MerkleBuildParams p{};
  p.leaves = leaves;
  p.leaf_stride = leaf_stride;
  p.slice_stride = slice_stride;
  p.leaf_bytes = static_cast<uint32_t>(leaf_bytes);
  p.n_leaves = static_cast<uint32_t>(n_leaves);
  p.nslices = nslices;
  p.empty_roots = c->d_empty_roots.as<uint32_t>();
  p.roots = roots;
  p.proofs = proofs;
  p.proofs_stride = proofs_stride;
  if (!nodes) {  // the levels are built in memory: scratch when the caller wants no nodes
    nodes_stride = (32 * ag_merkle_node_count(n_leaves) + 255) / 256 * 256;
    if ((st = c->d_merkle_nodes.ensure(nslices * nodes_stride, c->stream))) return st;
    nodes = c->d_merkle_nodes.as<uint8_t>();
  }
  return ag::launch_merkle_build(p, nodes, nodes_stride, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_merkle_verify_batch(ag_rs_ctx* c, size_t n, size_t leaf_bytes, const uint8_t* leaves, size_t leaf_stride,
                           const uint32_t* index, const uint8_t* roots, size_t roots_stride, const uint8_t* proofs,
                           size_t proofs_stride, size_t height, uint8_t* ok) {
  if (!c || leaf_bytes >= (size_t{1} << 28) || height > static_cast<size_t>(ag::kMerkleMaxHeight))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if ((leaf_bytes && !leaves) || !index || !roots || !ok || (height && !proofs) || roots_stride % 16 ||
      proofs_stride % 16 || reinterpret_cast<uintptr_t>(roots) % 16 || reinterpret_cast<uintptr_t>(proofs) % 16 ||
      (n > 1 && leaf_stride < leaf_bytes))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  ag::MerkleVerifyParams p{};
  p.leaves = leaves;
  p.leaf_stride = leaf_stride;
  p.leaf_bytes = static_cast<uint32_t>(leaf_bytes);
  p.height = static_cast<uint32_t>(height);
  p.index = index;
  p.roots = roots;
  p.roots_stride = roots_stride;
  p.proofs = proofs;
  p.proofs_stride = proofs_stride;
  p.n = n;
  p.ok = ok;
  return ag::launch_merkle_verify(p, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

// ---- all-or-nothing payload transforms ------------------------------------------------

int ag_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  if (!key || !in || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  ag::aes128_encrypt_block(key, in, out);
  return AG_RS_OK;
}

namespace {
// lengths (host) -> device; the batch descriptor
int aon_batch(ag_rs_ctx* c, size_t n, uint8_t* buffers, size_t stride, const uint32_t* lens, uint32_t extra,
              ag::BufferBatch* bb) {
  uint32_t mx = 0;
  for (size_t b = 0; b < n; ++b) {
    if (lens[b] > (1u << 28)) return AG_RS_ERR_INVALID_ARGUMENT;
    mx = std::max(mx, lens[b]);
  }
  if (n > 1 && stride < static_cast<size_t>(mx) + extra) return AG_RS_ERR_INVALID_ARGUMENT;
  int st = c->d_aon_lens.ensure(n * 4, c->stream);
  if (st) return st;
  AG_HIP(hipStreamSynchronize(c->stream));  // a previous call's upload may still be pending
  AG_HIP(hipMemcpy(c->d_aon_lens.ptr, lens, n * 4, hipMemcpyHostToDevice));
  bb->base = buffers;
  bb->stride = stride;
  bb->lens = c->d_aon_lens.as<uint32_t>();
  bb->n = n;
  bb->max_len = mx;
  return AG_RS_OK;
}
}  // namespace

int ag_cipher_apply_keystream_batch(ag_rs_ctx* c, size_t n, const uint8_t* keys, uint8_t* buffers, size_t stride,
                                    const uint32_t* lens) {
  if (!c || (n && (!keys || !buffers || !lens))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  ag::BufferBatch bb;
  int st = aon_batch(c, n, buffers, stride, lens, 0, &bb);
  if (st) return st;
  return ag::launch_apply_keystream(bb, keys, 0, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_sha256_batch(ag_rs_ctx* c, size_t n, const uint8_t* buffers, size_t stride, const uint32_t* lens,
                    uint8_t* digests) {
  if (!c || (n && (!buffers || !lens || !digests))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  ag::BufferBatch bb;
  int st = aon_batch(c, n, const_cast<uint8_t*>(buffers), stride, lens, 0, &bb);
  if (st) return st;
  return ag::launch_sha256(bb, 0, digests, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_aon_encrypt_batch(ag_rs_ctx* c, int scheme, size_t n, const uint8_t* keys, uint8_t* buffers, size_t stride,
                         const uint32_t* lens) {
  if (!c || (scheme != AG_AON_AONT && scheme != AG_AON_PETS) || (n && (!keys || !buffers || !lens)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  ag::BufferBatch bb;
  int st = aon_batch(c, n, buffers, stride, lens, ag::kCipherKeyBytes, &bb);
  if (st) return st;
  const bool aont = scheme == AG_AON_AONT;
  if (aont && (st = c->d_aon_digests.ensure(n * 32, c->stream))) return st;
  if (ag::launch_apply_keystream(bb, keys, 0, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  if (aont && ag::launch_sha256(bb, 0, c->d_aon_digests.as<uint8_t>(), c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  return ag::launch_write_key_tail(bb, aont, keys, aont ? c->d_aon_digests.as<uint8_t>() : nullptr, c->stream) ==
                 hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}

int ag_aon_decrypt_batch(ag_rs_ctx* c, int scheme, size_t n, uint8_t* buffers, size_t stride, const uint32_t* lens,
                         int64_t* plain_len_out) {
  if (!c || (scheme != AG_AON_AONT && scheme != AG_AON_PETS) || (n && (!buffers || !lens || !plain_len_out)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  // buffers too short for a key: BadEncoding, left untouched (length 16 => empty payload)
  std::vector<uint32_t> lv(lens, lens + n);
  for (size_t b = 0; b < n; ++b) {
    plain_len_out[b] = lens[b] < ag::kCipherKeyBytes ? -AG_RS_ERR_BAD_ENCODING
                                                      : static_cast<int64_t>(lens[b]) - ag::kCipherKeyBytes;
    if (lens[b] < ag::kCipherKeyBytes) lv[b] = ag::kCipherKeyBytes;  // no-op (empty ciphertext, key unused)
  }
  ag::BufferBatch bb;
  int st = aon_batch(c, n, buffers, stride, lv.data(), 0, &bb);
  if (st) return st;
  const bool aont = scheme == AG_AON_AONT;
  if ((st = c->d_aon_keys.ensure(n * 16, c->stream))) return st;
  if (aont) {
    if ((st = c->d_aon_digests.ensure(n * 32, c->stream))) return st;
    if (ag::launch_sha256(bb, ag::kCipherKeyBytes, c->d_aon_digests.as<uint8_t>(), c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
  }
  if (ag::launch_derive_keys(bb, aont, aont ? c->d_aon_digests.as<uint8_t>() : nullptr, c->d_aon_keys.as<uint8_t>(),
                             c->stream) != hipSuccess ||
      ag::launch_apply_keystream(bb, c->d_aon_keys.as<uint8_t>(), ag::kCipherKeyBytes, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  AG_HIP(hipStreamSynchronize(c->stream));
  return AG_RS_OK;
}

}  // extern "C"

// =====================================================================================
// Crate API mirror: ReedSolomonEncoder / ReedSolomonDecoder (one codeword, host memory)
// =====================================================================================
// An object made by *_new_on_device owns its context (`owned`: created with it, destroyed by
// its _free), so objects made that way share no state and may run on different threads at
// once; *_new borrows the caller's context, shared with whatever else uses it.
// Each encoder / decoder stages its codeword in its own mapped pinned buffer (the shards are
// copied there by add_*_shard, the device reads and writes it in place, and the result
// accessors point into it), so no call re-copies or re-zeroes a 64 KiB slice.
struct ag_rs_encoder {
  ag_rs_ctx* ctx = nullptr;
  ag_rs_ctx* owned = nullptr;
  size_t k = 0, m = 0, S = 0;
  size_t received = 0;
  bool encoded = false;
  PinBuf pin;  // originals [k * S] then recovery shards [m * S]
  uint8_t* orig() const { return pin.as<uint8_t>(); }
  uint8_t* rec() const { return pin.as<uint8_t>() + k * S; }
  ~ag_rs_encoder() {
    pin.release();
    ag_rs_ctx_destroy(owned);
  }
};

struct ag_rs_decoder {
  ag_rs_ctx* ctx = nullptr;
  ag_rs_ctx* owned = nullptr;
  size_t k = 0, m = 0, S = 0;
  std::vector<uint8_t> opres, rpres;
  size_t no = 0, nr = 0;
  bool decoded = false;
  std::vector<uint8_t> restored;  // 1 where original i was restored by the last decode
  PinBuf pin;  // originals [k * S], recovery shards [m * S], re-encoded coding shards [m * S]
  uint8_t* orig() const { return pin.as<uint8_t>(); }
  uint8_t* rec() const { return pin.as<uint8_t>() + k * S; }
  ~ag_rs_decoder() {
    pin.release();
    ag_rs_ctx_destroy(owned);
  }
};

namespace {
// One codeword through the device, zero-copy: the kernels read the originals from and
// write the recovery shards to mapped pinned host memory (a 32-shard slice is 32 KiB each
// way; two DMA copies and their scheduling cost more than the kernel's PCIe accesses).
// The single-codeword calls (one slice per call, the reference's pattern) wait for their
// microseconds of device work by polling the stream: hipStreamSynchronize's blocking wait
// added ~9 us per call over the kernel time (profiles/r04_call_latency_hip_api_stats.csv).
int spin_sync(ag_rs_ctx* c) {
  for (;;) {
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) return AG_RS_OK;
    if (e != hipErrorNotReady) return AG_RS_ERR_DEVICE;
  }
}

// ---- per-call server: one single-tile 32-point job through the mailbox ----------------
// A 32:32 codeword of S <= 4 KiB (S % 64 == 0) is one tile of xform8: the resident server
// runs it without a kernel dispatch or completion signal (tools/latency: one slice's shred
// was dispatch + kernel + signal).  Started on first use, restarted when it has idled out.
constexpr uint64_t kServerIdleTicks = 2000000;  // 20 ms of the 100 MHz wall clock
bool server_fits(ag_rs_ctx* c, size_t k, size_t m, size_t S) {
  return !c->server_broken && k == 32 && m == 32 && S % 64 == 0 && S >= 64 && S <= 64 * 64;
}
ag::XformParams one_tile(const uint8_t* in, size_t in_stride, uint8_t* out, size_t out_stride, size_t S) {
  ag::XformParams p{};
  p.in = in;
  p.in_block_stride = in_stride;
  p.in_shard_stride = S;
  p.out = out;
  p.out_block_stride = out_stride;
  p.out_shard_stride = S;
  p.n_in = 32;
  p.n_out = 32;
  p.chunks_per_shard = static_cast<uint32_t>(S / 64);
  p.total_columns = S / 64;
  return p;
}
// `stage`: the pinned buffer the job reads and writes (abandoned on a timeout).  `dp`: the
// kJobDecodePk parameters (then `p` is unused).
int server_job(ag_rs_ctx* c, uint32_t kind, const ag::XformParams& p, uint64_t mask, PinBuf& stage,
               const ag::DecodeXParams* dp = nullptr) {
  if (!c->mb) {
    void* h = nullptr;
    AG_HIP(hipHostMalloc(&h, sizeof(ag::LatencyMailbox), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, sizeof(ag::LatencyMailbox));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&c->server_stream, hipStreamNonBlocking) != hipSuccess) {
      (void)hipHostFree(h);
      c->server_stream = nullptr;
      return AG_RS_ERR_DEVICE;
    }
    c->mb = static_cast<ag::LatencyMailbox*>(h);
    c->mb_dev = static_cast<ag::LatencyMailbox*>(d);
  }
  // the server caches part of the log table at launch (kJobDecodePk's locator)
  int st = c->ensure_tables();
  if (st) return st;
  ag::LatencyMailbox* mb = c->mb;
  // Retire a job that did not complete: a queued or slow server that wakes later finds a quit
  // job instead.  It may already be inside the job, so the staging buffer the job names is
  // abandoned (kept allocated, never reused: `stage` is left empty, and the encoder / decoder
  // that owned it drops its received shards, see pin_lost) and later calls take the launch path.
  auto retire = [&]() {
    c->server_broken = true;
    mb->kind = ag::kJobQuit;
    __atomic_store_n(&mb->doorbell, ++c->server_seq, __ATOMIC_RELEASE);
    c->abandoned_pins.push_back(stage);
    stage = PinBuf{};
    return AG_RS_ERR_DEVICE;
  };
  if (c->fail_next_server_job) {
    c->fail_next_server_job = false;
    return retire();
  }
  mb->kind = kind;
  mb->mask = mask;
  // parameters only when their bytes changed (the server reuses its copy of the same version;
  // a fresh server launch holds no copy and reads them)
  if (dp) {
    if (std::memcmp(static_cast<const void*>(&mb->dp), dp, sizeof *dp) != 0 || c->server_dp_seq == 0) {
      std::memcpy(static_cast<void*>(&mb->dp), dp, sizeof *dp);
      mb->dp_seq = ++c->server_dp_seq;
    }
  } else if (std::memcmp(static_cast<const void*>(&mb->p), &p, sizeof p) != 0 || c->server_p_seq == 0) {
    std::memcpy(static_cast<void*>(&mb->p), &p, sizeof p);
    mb->p_seq = ++c->server_p_seq;
  }
  if (kind < 4) ++c->server_jobs[kind];
  const uint32_t seq = ++c->server_seq;
  __atomic_store_n(&mb->doorbell, seq, __ATOMIC_RELEASE);  // x86: the job's fields are visible first
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spins = 0;; ++spins) {
    if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) return AG_RS_OK;
    if (__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE) == 0) {
      // no server (first call, or it idled out -- possibly just after this doorbell)
      if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) return AG_RS_OK;
      __atomic_store_n(&mb->alive, 2u, __ATOMIC_RELEASE);
      if (ag::launch_latency_server(c->mb_dev, kServerIdleTicks, c->dtables().log, c->server_stream) != hipSuccess) {
        __atomic_store_n(&mb->alive, 0u, __ATOMIC_RELEASE);
        return AG_RS_ERR_DEVICE;
      }
    }
    if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
      return retire();
    __builtin_ia32_pause();
  }
}

// One codeword staged in `pin` (originals at 0, recovery shards at k * S): the recovery shards
// are computed in place.
int run_one_encode(ag_rs_ctx* c, size_t k, size_t m, size_t S, PinBuf& pin) {
  int st;
  if ((st = c->enter())) return st;
  const size_t ob = k * S, rb = m * S;
  uint8_t* pd = pin.dev<uint8_t>();
  if (server_fits(c, k, m, S)) return server_job(c, ag::kJobEncode32, one_tile(pd, ob, pd + ob, rb, S), 0, pin);
  if ((st = encode_device(c, k, m, S, 1, pd, ob, pd + ob, rb))) return st;
  return spin_sync(c);
}

// One codeword decoded on the device, zero-copy like run_one_encode: originals and recovery
// shards staged in `pin` (originals at 0, recovery at k * S), restored originals written in
// place, and with `coding` the re-encode of every recovery shard from the completed originals
// (ReedSolomonCoder::deshred's encode_coding_from_data, reed_solomon.rs:206) at (k + m) * S
// -- or, when the received shards are exactly the m recovery shards, *coding_src points at
// those (the re-encode reproduces them bit for bit).  EXACT runs as ANY_K when exactly k
// shards are present: k shards fix the codeword, so both decoders return its originals for
// any input bytes.
int run_one_decode(ag_rs_ctx* c, size_t k, size_t m, size_t S, PinBuf& pin, const uint8_t* opres,
                   const uint8_t* rpres, int mode, bool coding, const uint8_t** coding_src) {
  int st;
  if ((st = c->enter())) return st;
  const size_t ob = k * S, rb = m * S;
  size_t present = 0;
  for (size_t i = 0; i < k; ++i) present += opres[i] != 0;
  for (size_t i = 0; i < m; ++i) present += rpres[i] != 0;
  if (present < k) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  if (present == k) mode = AG_RS_DECODE_ANY_K;
  uint8_t* pd = pin.dev<uint8_t>();
  // exactly k shards, all of them recovery shards: the completed codeword passes through
  // them, so its re-encoded recovery shards are the received ones (bit for bit)
  size_t nr = 0;
  for (size_t i = 0; i < m; ++i) nr += rpres[i] != 0;
  const bool reuse = coding && present == k && nr == m;
  if (coding_src) *coding_src = pin.as<uint8_t>() + (reuse ? ob : ob + rb);
  if (nr == m && (present == k || mode == AG_RS_DECODE_ANY_K) && server_fits(c, k, m, S)) {
    // the whole recovery set: the erased originals are one transform of it (the decode class
    // "none" route of decode_cols), run by the per-call server
    uint64_t mask = 0;
    for (size_t i = 0; i < k; ++i)
      if (!opres[i]) mask |= uint64_t{1} << i;
    std::fill(std::begin(c->last_classes), std::end(c->last_classes), uint64_t{0});
    ++c->last_classes[mask ? 1 : 0];  // "transform" (or "none")
    if (mask && (st = server_job(c, (mask >> 16) ? ag::kJobDecode32 : ag::kJobDecode32Half,
                                 one_tile(pd + ob, rb, pd, ob, S), mask, pin)))
      return st;
    if (coding && !reuse &&
        (st = server_job(c, ag::kJobEncode32, one_tile(pd, ob, pd + ob + rb, rb, S), 0, pin)))
      return st;
    return AG_RS_OK;
  }
  const bool pk_size = S == 1024 || (S > 960 && S < 1024 && S % 2 == 0);  // 16 columns, tail included
  if (present == k && pk_size && k == 32 && m == 32 && !c->server_broken) {
    // exactly k = 32 of the 64 shreds of a 32:32 slice of 1 KiB shreds, or of 960 + T bytes
    // with a T >= 16-byte tail (the follower's deshred at its 32nd arriving shred):
    // decode_pk<-1>'s one-slice window decode on the server restores every absent data and
    // coding shred in place -- the codeword through the 32 survivors is unique, so the restored
    // coding shreds are the re-encode, bit for bit
    uint64_t pres = 0;
    for (size_t j = 0; j < m; ++j)
      if (rpres[j]) pres |= uint64_t{1} << j;
    for (size_t i = 0; i < k; ++i)
      if (opres[i]) pres |= uint64_t{1} << (32 + i);
    ag::DecodeXParams dp{};
    dp.rec = pd + ob;
    dp.rec_block_stride = (k + m) * S;
    dp.rec_shard_stride = S;
    dp.orig = pd;
    dp.orig_block_stride = (k + m) * S;
    dp.orig_shard_stride = S;
    dp.k = 32;
    dp.m = 32;
    dp.chunk = 32;
    dp.low_rate = 0;
    dp.chunks_per_shard = 16;
    dp.total_columns = 16;
    dp.per_lane = 1;
    dp.rows_w = 64;
    dp.any_k = 1;
    dp.fuse = 1;
    dp.tail_bytes = static_cast<uint32_t>(S % 64);
    std::fill(std::begin(c->last_classes), std::end(c->last_classes), uint64_t{0});
    ++c->last_classes[9];  // "server_window64"
    if ((st = server_job(c, ag::kJobDecodePk, ag::XformParams{}, pres, pin, &dp))) return st;
    if (coding_src) *coding_src = pin.as<uint8_t>() + ob;  // the whole coding set, in place
    return AG_RS_OK;
  }
  if ((st = decode_device(c, k, m, S, 1, pd, ob, pd + ob, rb, opres, rpres, 1, mode))) return st;
  if (coding && !reuse && (st = encode_device(c, k, m, S, 1, pd, ob, pd + ob + rb, rb))) return st;
  return spin_sync(c);
}
}  // namespace

extern "C" {

int ag_rs_encoder_reset(ag_rs_encoder* e, size_t k, size_t m, size_t S) {
  if (!e) return AG_RS_ERR_INVALID_ARGUMENT;
  int st = check_geometry(k, m, S);
  if (st) return st;
  // the staging only grows; its bytes need no clearing (encode reads the k added originals)
  if ((k + m) * S > e->pin.size && ((st = e->ctx->enter()) || (st = e->pin.ensure((k + m) * S)))) return st;
  e->k = k;
  e->m = m;
  e->S = S;
  e->received = 0;
  e->encoded = false;
  return AG_RS_OK;
}

int ag_rs_encoder_new(ag_rs_ctx* c, size_t k, size_t m, size_t S, ag_rs_encoder** out) {
  if (!c || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  auto* e = new (std::nothrow) ag_rs_encoder();
  if (!e) return AG_RS_ERR_OUT_OF_MEMORY;
  e->ctx = c;
  const int st = ag_rs_encoder_reset(e, k, m, S);
  if (st) {
    delete e;
    return st;
  }
  *out = e;
  return AG_RS_OK;
}

int ag_rs_encoder_new_on_device(int device, size_t k, size_t m, size_t S, ag_rs_encoder** out) {
  if (!out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  ag_rs_ctx* c = nullptr;
  int st = ag_rs_ctx_create(device, &c);
  if (st) return st;
  if ((st = ag_rs_encoder_new(c, k, m, S, out))) {
    ag_rs_ctx_destroy(c);
    return st;
  }
  (*out)->owned = c;
  return AG_RS_OK;
}

// A server job that timed out abandoned the object's staging (server_job: `stage` left
// empty): the shards it held are gone, so the object starts a new round in a fresh buffer.
static int encoder_pin_lost(ag_rs_encoder* e) {
  e->received = 0;
  e->encoded = false;
  int st = e->ctx->enter();
  return st ? st : e->pin.ensure((e->k + e->m) * e->S);
}

int ag_rs_encoder_add_original_shard(ag_rs_encoder* e, const uint8_t* shard, size_t len) {
  if (!e || (!shard && len)) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!e->pin.ptr) {
    const int st = encoder_pin_lost(e);
    if (st) return st;
  }
  if (e->encoded) {  // the crate resets the received set once a result is dropped
    e->received = 0;
    e->encoded = false;
  }
  if (e->received == e->k) return AG_RS_ERR_TOO_MANY_ORIGINAL_SHARDS;
  if (len != e->S) return AG_RS_ERR_DIFFERENT_SHARD_SIZE;
  std::memcpy(e->orig() + e->received * e->S, shard, len);
  ++e->received;
  return AG_RS_OK;
}

int ag_rs_encoder_encode(ag_rs_encoder* e) {
  if (!e) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!e->pin.ptr) e->received = 0;  // staging abandoned by a timed-out job: nothing received
  if (e->received != e->k) return AG_RS_ERR_TOO_FEW_ORIGINAL_SHARDS;
  const int st = run_one_encode(e->ctx, e->k, e->m, e->S, e->pin);
  if (st) {
    if (!e->pin.ptr) e->received = 0;
    e->encoded = false;
    return st;
  }
  e->encoded = true;
  return AG_RS_OK;
}

int ag_rs_encoder_recovery(const ag_rs_encoder* e, size_t index, const uint8_t** shard, size_t* len) {
  if (!e || !shard || !len) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!e->encoded || index >= e->m) return AG_RS_ERR_INVALID_ARGUMENT;
  *shard = e->rec() + index * e->S;
  *len = e->S;
  return AG_RS_OK;
}

void ag_rs_encoder_free(ag_rs_encoder* e) { delete e; }

int ag_rs_decoder_reset(ag_rs_decoder* d, size_t k, size_t m, size_t S) {
  if (!d) return AG_RS_ERR_INVALID_ARGUMENT;
  int st = check_geometry(k, m, S);
  if (st) return st;
  if ((k + 2 * m) * S > d->pin.size && ((st = d->ctx->enter()) || (st = d->pin.ensure((k + 2 * m) * S))))
    return st;
  d->k = k;
  d->m = m;
  d->S = S;
  d->opres.assign(k, 0);
  d->rpres.assign(m, 0);
  d->restored.assign(k, 0);
  d->no = d->nr = 0;
  d->decoded = false;
  return AG_RS_OK;
}

int ag_rs_decoder_new(ag_rs_ctx* c, size_t k, size_t m, size_t S, ag_rs_decoder** out) {
  if (!c || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  auto* d = new (std::nothrow) ag_rs_decoder();
  if (!d) return AG_RS_ERR_OUT_OF_MEMORY;
  d->ctx = c;
  const int st = ag_rs_decoder_reset(d, k, m, S);
  if (st) {
    delete d;
    return st;
  }
  *out = d;
  return AG_RS_OK;
}

int ag_rs_decoder_new_on_device(int device, size_t k, size_t m, size_t S, ag_rs_decoder** out) {
  if (!out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  ag_rs_ctx* c = nullptr;
  int st = ag_rs_ctx_create(device, &c);
  if (st) return st;
  if ((st = ag_rs_decoder_new(c, k, m, S, out))) {
    ag_rs_ctx_destroy(c);
    return st;
  }
  (*out)->owned = c;
  return AG_RS_OK;
}

// The decoder's counterpart of encoder_pin_lost: every received shard is dropped.
static int decoder_pin_lost(ag_rs_decoder* d) {
  std::fill(d->opres.begin(), d->opres.end(), 0);
  std::fill(d->rpres.begin(), d->rpres.end(), 0);
  std::fill(d->restored.begin(), d->restored.end(), 0);
  d->no = d->nr = 0;
  d->decoded = false;
  int st = d->ctx->enter();
  return st ? st : d->pin.ensure((d->k + 2 * d->m) * d->S);
}

static void decoder_begin_round(ag_rs_decoder* d) {
  if (!d->decoded) return;
  std::fill(d->opres.begin(), d->opres.end(), 0);
  std::fill(d->rpres.begin(), d->rpres.end(), 0);
  std::fill(d->restored.begin(), d->restored.end(), 0);
  d->no = d->nr = 0;
  d->decoded = false;
}

int ag_rs_decoder_add_original_shard(ag_rs_decoder* d, size_t index, const uint8_t* shard, size_t len) {
  if (!d || (!shard && len)) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!d->pin.ptr) {
    const int st = decoder_pin_lost(d);
    if (st) return st;
  }
  decoder_begin_round(d);
  if (index >= d->k) return AG_RS_ERR_INVALID_ORIGINAL_SHARD_INDEX;
  if (d->opres[index]) return AG_RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX;
  if (len != d->S) return AG_RS_ERR_DIFFERENT_SHARD_SIZE;
  std::memcpy(d->orig() + index * d->S, shard, len);
  d->opres[index] = 1;
  ++d->no;
  return AG_RS_OK;
}

int ag_rs_decoder_add_recovery_shard(ag_rs_decoder* d, size_t index, const uint8_t* shard, size_t len) {
  if (!d || (!shard && len)) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!d->pin.ptr) {
    const int st = decoder_pin_lost(d);
    if (st) return st;
  }
  decoder_begin_round(d);
  if (index >= d->m) return AG_RS_ERR_INVALID_RECOVERY_SHARD_INDEX;
  if (d->rpres[index]) return AG_RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX;
  if (len != d->S) return AG_RS_ERR_DIFFERENT_SHARD_SIZE;
  std::memcpy(d->rec() + index * d->S, shard, len);
  d->rpres[index] = 1;
  ++d->nr;
  return AG_RS_OK;
}

int ag_rs_decoder_decode(ag_rs_decoder* d) {
  if (!d) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!d->pin.ptr) {  // staging abandoned by a timed-out job: nothing received
    const int st = decoder_pin_lost(d);
    if (st) return st;
  }
  if (d->no + d->nr < d->k) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  std::fill(d->restored.begin(), d->restored.end(), 0);
  if (d->no < d->k) {
    // exact crate semantics: decode from every present shard
    const int st = run_one_decode(d->ctx, d->k, d->m, d->S, d->pin, d->opres.data(), d->rpres.data(),
                                  AG_RS_DECODE_EXACT, false, nullptr);
    if (st) {
      if (!d->pin.ptr) (void)decoder_pin_lost(d);
      return st;
    }
    for (size_t i = 0; i < d->k; ++i) d->restored[i] = d->opres[i] ? 0 : 1;
  }
  d->decoded = true;
  return AG_RS_OK;
}

int ag_rs_decoder_restored_original(const ag_rs_decoder* d, size_t index, const uint8_t** shard, size_t* len) {
  if (!d || !shard || !len) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!d->decoded || index >= d->k || !d->restored[index]) return AG_RS_ERR_NOT_RESTORED;
  *shard = d->orig() + index * d->S;
  *len = d->S;
  return AG_RS_OK;
}

void ag_rs_decoder_free(ag_rs_decoder* d) { delete d; }

}  // extern "C"

// =====================================================================================
// ReedSolomonCoder mirror (reed_solomon.rs:47-232)
// =====================================================================================
struct ag_rs_coder {
  ag_rs_ctx* ctx = nullptr;
  ag_rs_ctx* owned = nullptr;  // ag_rs_coder_new_on_device: shared by its encoder and decoder
  size_t num_coding = 0;
  ag_rs_encoder* enc = nullptr;
  ag_rs_decoder* dec = nullptr;
  ~ag_rs_coder() {
    ag_rs_encoder_free(enc);
    ag_rs_decoder_free(dec);
    ag_rs_ctx_destroy(owned);
  }
};

int ag_rs_internal_coder_last_job_ns(ag_rs_coder* coder, uint64_t* ns) {
  if (!coder || !coder->ctx || !ns) return AG_RS_ERR_INVALID_ARGUMENT;
  const ag::LatencyMailbox* mb = coder->ctx->mb;
  ns[0] = mb ? __atomic_load_n(&mb->job_ticks, __ATOMIC_ACQUIRE) * 10 : 0;  // 100 MHz wall clock
  for (int i = 0; i < 4; ++i) ns[1 + i] = mb ? uint64_t{__atomic_load_n(&mb->phase_ticks[i], __ATOMIC_ACQUIRE)} * 10 : 0;
  return AG_RS_OK;
}

namespace {
constexpr size_t kDataShreds = AG_RS_DATA_SHREDS;
constexpr size_t kTotalShreds = AG_RS_TOTAL_SHREDS;
constexpr size_t kMaxAfterPadding = kDataShreds * AG_RS_MAX_DATA_PER_SHRED;
constexpr size_t kMaxPayload = kMaxAfterPadding - 1;

// encode_coding_from_data (reed_solomon.rs:211-231) of the 32 data shards already staged in
// the encoder's originals (S bytes each): the coding shards land in c->enc->rec()
// (the caller reset the encoder to (32, num_coding, S) before staging them)
int coder_encode_staged(ag_rs_coder* c) {
  c->enc->received = kDataShreds;
  c->enc->encoded = false;
  return ag_rs_encoder_encode(c->enc);
}
}  // namespace

extern "C" {

int ag_rs_coder_new(ag_rs_ctx* ctx, size_t num_coding, ag_rs_coder** out) {
  if (!ctx || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  if (num_coding == 0 || num_coding > kTotalShreds) return AG_RS_ERR_UNSUPPORTED_SHARD_COUNT;
  auto* c = new (std::nothrow) ag_rs_coder();
  if (!c) return AG_RS_ERR_OUT_OF_MEMORY;
  c->ctx = ctx;
  c->num_coding = num_coding;
  int st = ag_rs_encoder_new(ctx, kDataShreds, num_coding, AG_RS_MAX_DATA_PER_SHRED, &c->enc);
  if (!st) st = ag_rs_decoder_new(ctx, kDataShreds, num_coding, AG_RS_MAX_DATA_PER_SHRED, &c->dec);
  if (st) {
    delete c;
    return st;
  }
  *out = c;
  return AG_RS_OK;
}

int ag_rs_coder_new_on_device(int device, size_t num_coding, ag_rs_coder** out) {
  if (!out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  ag_rs_ctx* c = nullptr;
  int st = ag_rs_ctx_create(device, &c);
  if (st) return st;
  if ((st = ag_rs_coder_new(c, num_coding, out))) {
    ag_rs_ctx_destroy(c);
    return st;
  }
  (*out)->owned = c;
  return AG_RS_OK;
}

void ag_rs_coder_free(ag_rs_coder* c) { delete c; }

int ag_rs_coder_num_coding(const ag_rs_coder* c, size_t* out) {
  if (!c || !out) return AG_RS_ERR_INVALID_ARGUMENT;
  *out = c->num_coding;
  return AG_RS_OK;
}

int ag_rs_coder_shred(ag_rs_coder* c, const uint8_t* payload, size_t len, uint8_t* data_out, uint8_t* coding_out,
                      size_t* shred_bytes) {
  if (!c || (!payload && len) || !data_out || !coding_out || !shred_bytes) return AG_RS_ERR_INVALID_ARGUMENT;
  if (len > kMaxPayload) return AG_RS_ERR_TOO_MUCH_DATA;
  // padding 0x80 00.. to a multiple of 2 * DATA_SHREDS (reed_solomon.rs:94-106)
  const size_t padding = 2 * kDataShreds - len % (2 * kDataShreds);
  const size_t S = (len + padding) / kDataShreds;
  // padded payload straight into the encoder's pinned originals
  int st = ag_rs_encoder_reset(c->enc, kDataShreds, c->num_coding, S);
  if (st) return st;
  uint8_t* padded = c->enc->orig();
  if (len) std::memcpy(padded, payload, len);
  padded[len] = 0x80;
  std::memset(padded + len + 1, 0, padding - 1);
  if ((st = coder_encode_staged(c))) return st;
  std::memcpy(data_out, padded, len + padding);
  std::memcpy(coding_out, c->enc->rec(), c->num_coding * S);
  *shred_bytes = S;
  return AG_RS_OK;
}

int ag_rs_coder_deshred(ag_rs_coder* c, size_t data_shreds, const uint8_t* const* shreds, const size_t* lens,
                        const uint8_t* is_data, uint8_t* payload_out, size_t* payload_len, uint8_t* data_out,
                        uint8_t* coding_out, size_t* shred_bytes) {
  if (!c || !shreds || !lens || !payload_out || !payload_len || !data_out || !coding_out || !shred_bytes)
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (data_shreds + c->num_coding != kTotalShreds) return AG_RS_ERR_INVALID_ARGUMENT;
  // Shredder::deshred: an empty set is too few shreds (shredder.rs:283-285)
  size_t present = 0, S = 0;
  for (size_t i = 0; i < kTotalShreds; ++i)
    if (shreds[i]) {
      if (!present) S = lens[i];
      ++present;
    }
  if (!present) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  // ValidatedShreds::try_new (validated_shreds.rs:34-70)
  if (S == 0 || S % 2) return AG_RS_ERR_INVALID_LAYOUT;
  for (size_t i = 0; i < kTotalShreds; ++i) {
    if (!shreds[i]) continue;
    if (lens[i] != S) return AG_RS_ERR_INVALID_LAYOUT;
    if (is_data && ((i < data_shreds) != (is_data[i] != 0))) return AG_RS_ERR_INVALID_LAYOUT;
  }
  // ReedSolomonCoder::deshred (reed_solomon.rs:140-208)
  if (present < kDataShreds) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  int st = ag_rs_decoder_reset(c->dec, kDataShreds, c->num_coding, S);
  if (st) return st;
  for (size_t i = 0; i < data_shreds; ++i)
    if (shreds[i] && (st = ag_rs_decoder_add_original_shard(c->dec, i, shreds[i], S))) return st;
  for (size_t j = data_shreds; j < kTotalShreds; ++j)
    if (shreds[j] && (st = ag_rs_decoder_add_recovery_shard(c->dec, j - data_shreds, shreds[j], S))) return st;
  ag_rs_decoder* dec = c->dec;
  if (dec->no + dec->nr < kDataShreds) return AG_RS_ERR_NOT_ENOUGH_SHARDS;
  // decode and the re-encode of every coding shard (:206) in one device round trip; the
  // completed originals (present ones as added, restored ones written back) are dec->orig()
  const uint8_t* coding = nullptr;
  const bool coded = dec->no < kDataShreds;
  if (coded && (st = run_one_decode(c->ctx, kDataShreds, c->num_coding, S, dec->pin, dec->opres.data(),
                                    dec->rpres.data(), AG_RS_DECODE_EXACT, true, &coding)))
    return st;
  // concatenation with the TooMuchData bound of :169-188 (exceeded iff 32 S > 32 768)
  if (kDataShreds * S > kMaxAfterPadding) return AG_RS_ERR_TOO_MUCH_DATA;
  const uint8_t* data = dec->orig();
  const size_t total = kDataShreds * S;
  // strip padding: trailing zeros then the 0x80 marker
  size_t zeros = 0;
  while (zeros < total && data[total - 1 - zeros] == 0) ++zeros;
  const size_t padding = zeros + 1;
  if (padding > total || data[total - padding] != 0x80) return AG_RS_ERR_INVALID_PADDING;
  const size_t plen = total - padding;
  if (!coded) {  // every data shred present: encode them (staged in the encoder)
    if ((st = ag_rs_encoder_reset(c->enc, kDataShreds, c->num_coding, S))) return st;
    std::memcpy(c->enc->orig(), data, total);
    if ((st = coder_encode_staged(c))) return st;
    coding = c->enc->rec();
  }
  std::memcpy(payload_out, data, plen);
  *payload_len = plen;
  std::memcpy(data_out, data, total);
  std::memcpy(coding_out, coding, c->num_coding * S);
  *shred_bytes = S;
  return AG_RS_OK;
}

int ag_rs_coder_shred_batch(ag_rs_ctx* c, size_t m, size_t n, size_t S, const uint8_t* payloads,
                            size_t payload_stride, const uint32_t* lens, uint8_t* cw, size_t cw_stride) {
  if (!c || (n && (!lens || !cw))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (m == 0 || m > kTotalShreds) return AG_RS_ERR_UNSUPPORTED_SHARD_COUNT;
  if (S == 0 || S % 2 || S > AG_RS_MAX_DATA_PER_SHRED) return AG_RS_ERR_INVALID_SHARD_SIZE;
  if (cw_stride < (kDataShreds + m) * S) return AG_RS_ERR_INVALID_ARGUMENT;
  for (size_t b = 0; b < n; ++b) {
    if (lens[b] > kMaxPayload) return AG_RS_ERR_TOO_MUCH_DATA;
    const size_t padded = lens[b] + 2 * kDataShreds - lens[b] % (2 * kDataShreds);  // reed_solomon.rs:94-95
    if (padded / kDataShreds != S) return AG_RS_ERR_INVALID_ARGUMENT;
  }
  if (n == 0) return AG_RS_OK;
  int st = c->enter();
  if (st) return st;
  // the lengths go up through pinned staging on the context stream (ordered after a previous
  // call's pad kernel, which may still read d_lens); the staging is rewritten once its last
  // upload has completed -- no stream synchronisation before the call's work is enqueued
  if (c->lens_ev) AG_HIP(hipEventSynchronize(c->lens_ev));
  else AG_HIP(hipEventCreateWithFlags(&c->lens_ev, hipEventDisableTiming));
  if ((st = c->h_lens.ensure(n * 4))) return st;
  std::memcpy(c->h_lens.ptr, lens, n * 4);
  if ((st = c->d_lens.ensure(n * 4, c->stream))) return st;
  AG_HIP(hipMemcpyAsync(c->d_lens.ptr, c->h_lens.ptr, n * 4, hipMemcpyHostToDevice, c->stream));
  AG_HIP(hipEventRecord(c->lens_ev, c->stream));
  if (ag::launch_coder_pad(payloads, payload_stride, c->d_lens.as<uint32_t>(), cw, cw_stride,
                           static_cast<uint32_t>(kDataShreds * S), n, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  return encode_device(c, kDataShreds, m, S, n, cw, cw_stride, cw + kDataShreds * S, cw_stride);
}

namespace {
int pipe_coder_deshred(ag_rs_ctx* c, size_t n, size_t S, uint8_t* cw, size_t cw_stride, const uint64_t* d_present,
                       int64_t* plen, size_t m, bool no_surplus = false);
// shred sizes pipe_coder_deshred decodes on the device: whole 64-byte chunks (any m of the
// device-pattern path), or for 32:32 a last chunk of T = S mod 64 bytes -- T >= 16 always, a
// shorter T when no slice needs the re-encode (no_reencode: no surplus shreds, no slice with
// every data shred; the TAIL encode takes T >= 16 only)
bool pipe_tail_ok(size_t S, size_t m, bool no_reencode = false) {
  const size_t T = S % 64;
  return T == 0 || (m == kDataShreds && S % 2 == 0 && (T >= 16 || no_reencode));
}
}  // namespace

namespace {
// Per-slice present words of ag_rs_coder_deshred_batch's device-pattern path: word 0 = data
// flags | coding 0..31 << 32 (and word 1 = coding 32..63 when m = 64).  Returns whether any
// slice keeps more than 32 shreds.  The flag bytes are 4 MiB per 65 536 slices: compared 32
// at a time with AVX2 where the host has it (the 8-byte multiply trick of pack_flags took
// ~0.5 ms of the call).
__attribute__((target("avx2"))) uint32_t nonzero_mask32_avx2(const uint8_t* f) {
  const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(f));
  return ~static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x, _mm256_setzero_si256())));
}
// (a macro body, not a template: this part of the file has C linkage)
#define AG_PACK_PRESENT(MASK32)                                                   \
  const size_t wps = m == kDataShreds ? 1 : 2;                                    \
  bool surplus = false, full_data = false;                                        \
  for (size_t b = 0; b < n; ++b) {                                                \
    uint64_t* q = pres + wps * b;                                                 \
    q[0] = uint64_t{MASK32(dpres + b * kDataShreds)} | (uint64_t{MASK32(cpres + b * m)} << 32); \
    int cnt = __builtin_popcountll(q[0]);                                         \
    if (wps == 2) {                                                               \
      q[1] = m == 2 * kDataShreds ? MASK32(cpres + b * m + 32)                    \
                                  : pack_flags(cpres + b * m + 32, m - 32);       \
      cnt += __builtin_popcountll(q[1]);                                          \
    }                                                                             \
    surplus |= cnt > static_cast<int>(kDataShreds);                               \
    full_data |= (q[0] & 0xFFFFFFFFull) == 0xFFFFFFFFull;                         \
  }                                                                               \
  *any_full_data = full_data;                                                     \
  return surplus;
__attribute__((target("avx2"))) bool pack_present_avx2(const uint8_t* dpres, const uint8_t* cpres, size_t m, size_t n,
                                                       uint64_t* pres, bool* any_full_data) {
  AG_PACK_PRESENT(nonzero_mask32_avx2)
}
uint32_t nonzero_mask32(const uint8_t* f) { return static_cast<uint32_t>(pack_flags(f, 32)); }
bool pack_present_scalar(const uint8_t* dpres, const uint8_t* cpres, size_t m, size_t n, uint64_t* pres,
                         bool* any_full_data) {
  AG_PACK_PRESENT(nonzero_mask32)
}
#undef AG_PACK_PRESENT
// *any_full_data: some slice holds every data shred (its decode is skipped, so its absent
// coding shreds come from the re-encode)
bool pack_present_words(const uint8_t* dpres, const uint8_t* cpres, size_t m, size_t n, uint64_t* pres,
                        bool* any_full_data) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  return avx2 ? pack_present_avx2(dpres, cpres, m, n, pres, any_full_data)
              : pack_present_scalar(dpres, cpres, m, n, pres, any_full_data);
}

// ag_rs_coder_deshred_batch when every slice has the same present shreds (pattern = slice 0's).
int coder_deshred_uniform(ag_rs_ctx* c, size_t m, size_t n, size_t S, uint8_t* cw, size_t cw_stride,
                          const uint8_t* dpres, const uint8_t* cpres, int mode, int64_t* out) {
  const size_t nd = count_flags(dpres, kDataShreds), nc = count_flags(cpres, m);
  if (nd + nc < kDataShreds) {  // reed_solomon.rs:144: nothing decoded, coding untouched
    for (size_t b = 0; b < n; ++b) out[b] = -AG_RS_ERR_NOT_ENOUGH_SHARDS;
    return AG_RS_OK;
  }
  uint8_t* rec = cw + kDataShreds * S;
  int st = decode_device(c, kDataShreds, m, S, n, cw, cw_stride, rec, cw_stride, dpres, cpres, 1, mode);
  if (st) return st;
  if ((st = c->d_strip.ensure(n * 8, c->stream))) return st;
  if (ag::launch_coder_strip(cw, cw_stride, static_cast<uint32_t>(kDataShreds * S), n, c->d_strip.as<int64_t>(),
                             c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  AG_HIP(hipMemcpyAsync(out, c->d_strip.ptr, n * 8, hipMemcpyDeviceToHost, c->stream));
  AG_HIP(hipStreamSynchronize(c->stream));
  for (size_t b = 0; b < n; ++b)
    if (out[b] < 0) out[b] = -AG_RS_ERR_INVALID_PADDING;
  // re-encode (encode_coding_from_data) the runs of slices that stripped; skipped when the
  // present shreds are exactly the 32 coding shreds (the re-encode reproduces them)
  if (m == kDataShreds && nd == 0 && nc == m) return AG_RS_OK;
  // LowRate 32:64 (CodingOnly) with exactly 32 kept shreds: the codeword is unique, so the
  // re-encode reproduces every kept coding shred.  When the absent ones all lie in one 32-shard
  // recovery chunk (the reference bench's shape: coding 32..63 kept), only that chunk is
  // encoded -- one 32-point transform under a store mask of its absent shreds instead of the
  // two-chunk 64-point one
  int lone = -1;
  if (m == 2 * kDataShreds && nd + nc == kDataShreds && S % 64 == 0 && !odd_layout(cw, cw, cw_stride, cw_stride)) {
    const uint64_t absent = ~pack_flags(cpres, m);
    const uint64_t lo = absent & 0xFFFFFFFFull, hi = absent >> 32;
    if (lo == 0 || hi == 0) {
      lone = lo == 0 ? 1 : 0;
      const uint64_t w = lo == 0 ? hi : lo;
      if ((st = c->d_reenc_mask.ensure(8, c->stream))) return st;
      AG_HIP(hipMemsetD32Async(c->d_reenc_mask.ptr, static_cast<int>(static_cast<uint32_t>(w)), 1, c->stream));
      AG_HIP(hipMemsetD32Async(c->d_reenc_mask.as<uint32_t>() + 1, 0, 1, c->stream));
    }
  }
  for (size_t b = 0; b < n;) {
    if (out[b] < 0) {
      ++b;
      continue;
    }
    size_t e = b;
    while (e < n && out[e] >= 0) ++e;
    if (lone >= 0) {
      ag::XformParams p{};
      p.in = cw + b * cw_stride;
      p.in_block_stride = cw_stride;
      p.in_shard_stride = S;
      p.out = rec + b * cw_stride + static_cast<size_t>(lone) * 32 * S;
      p.out_block_stride = cw_stride;
      p.out_shard_stride = S;
      p.out_mask = c->d_reenc_mask.as<uint64_t>();
      p.n_in = static_cast<uint32_t>(kDataShreds);
      p.n_out = 32;
      p.chunks_per_shard = static_cast<uint32_t>(S / 64);
      p.total_columns = static_cast<uint64_t>(e - b) * (S / 64);
      c->last_encode_kernels |= ag::kEkLowRate;
      if (ag::launch_xform_lowrate(32, static_cast<unsigned>(lone), p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    } else if ((st = encode_device(c, kDataShreds, m, S, e - b, cw + b * cw_stride, cw_stride, rec + b * cw_stride,
                                   cw_stride))) {
      return st;
    }
    b = e;
  }
  AG_HIP(hipStreamSynchronize(c->stream));
  return AG_RS_OK;
}
}  // namespace

int ag_rs_coder_deshred_batch(ag_rs_ctx* c, size_t m, size_t n, size_t S, uint8_t* cw, size_t cw_stride,
                              const uint8_t* dpres, const uint8_t* cpres, int mode, int64_t* out) {
  if (!c || (n && (!cw || !dpres || !cpres || !out))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (m == 0 || m > kTotalShreds) return AG_RS_ERR_UNSUPPORTED_SHARD_COUNT;
  if (mode != AG_RS_DECODE_EXACT && mode != AG_RS_DECODE_ANY_K) return AG_RS_ERR_INVALID_ARGUMENT;
  if (S == 0 || S % 2) return AG_RS_ERR_INVALID_SHARD_SIZE;
  if (kDataShreds * S > kMaxAfterPadding) return AG_RS_ERR_TOO_MUCH_DATA;  // reed_solomon.rs:183
  if (cw_stride < (kDataShreds + m) * S) return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  int st = c->enter();
  if (st) return st;
  c->last_encode_kernels = 0;  // the re-encode's kernels (test aid)
  c->last_window_kernels = 0;  // the window decode's kernels (test aid)
  // One pattern for the whole batch (a repair batch; the reference bench's shape): one
  // pattern word on the host, no per-slice bookkeeping past the strip results.
  bool uniform = true;
  for (size_t b = 1; b < n && uniform; ++b)
    uniform = std::memcmp(dpres, dpres + b * kDataShreds, kDataShreds) == 0 && std::memcmp(cpres, cpres + b * m, m) == 0;
  if (uniform) return coder_deshred_uniform(c, m, n, S, cw, cw_stride, dpres, cpres, mode, out);
  // Per-slice patterns of RegularShredder's 32:32 on whole-chunk shreds (the follower's
  // random arrival): one 64-bit present mask per slice goes to the device, and the window
  // patterns, locator constants, per-lane decode, padding strip and re-encode run there
  // (pipe_coder_deshred, the composed deshred's coder stage) -- no per-slice host work past
  // the packing.  ANY_K, or EXACT where no slice holds more than 32 shreds (k shreds fix the
  // codeword, so both decoders agree).  One pattern for the whole batch stays on the host
  // path below (a single transform launch).
  // CodingOnlyShredder's 32:64 and PetsShredder's 32:33 (LowRate, 32 < m <= 64) take the same
  // path with the W = 128 window (positions of coding shreds past m are simply never present).
  if (m >= kDataShreds && m <= 2 * kDataShreds && pipe_tail_ok(S, m, true) && n > 1 &&
      !odd_layout(cw, cw, cw_stride, cw_stride)) {
    const size_t wps = m == kDataShreds ? 1 : 2;  // present words per slice
    // packed straight into pinned staging, so the upload is one DMA with no pageable bounce
    // (once the previous call's upload of it has completed)
    if (c->present_ev) AG_HIP(hipEventSynchronize(c->present_ev));
    else AG_HIP(hipEventCreateWithFlags(&c->present_ev, hipEventDisableTiming));
    if ((st = c->h_present.ensure(wps * n * 8))) return st;
    uint64_t* pres = c->h_present.as<uint64_t>();
    // (uniform batches returned above)
    // ANY_K always takes the device path; EXACT when no slice keeps more than 32 shreds (both
    // decoders agree then).  (Packing a first ~1/8 range and the rest behind its decode
    // measured even with one whole-batch range, profiles/r05_ab_coder_ranges.jsonl.)
    bool full_data = false;
    const bool surplus = pack_present_words(dpres, cpres, m, n, pres, &full_data);
    if ((mode == AG_RS_DECODE_ANY_K || !surplus) && pipe_tail_ok(S, m, !surplus && !full_data)) {
      if ((st = c->d_present.ensure(wps * n * 8, c->stream))) return st;
      AG_HIP(hipMemcpyAsync(c->d_present.ptr, pres, wps * n * 8, hipMemcpyHostToDevice, c->stream));
      AG_HIP(hipEventRecord(c->present_ev, c->stream));
      // no surplus and no slice with every data shred: no store mask of the re-encode is set
      return pipe_coder_deshred(c, n, S, cw, cw_stride, c->d_present.as<uint64_t>(), out, m,
                                !surplus && !full_data);  // synchronous
    }
  }
  // slices with fewer than 32 shreds: reported, and decoded as "nothing missing" (untouched)
  std::vector<uint8_t> op(dpres, dpres + n * kDataShreds);
  std::vector<uint8_t> ok(n, 1);
  for (size_t b = 0; b < n; ++b) {
    const size_t cnt = count_flags(dpres + b * kDataShreds, kDataShreds) + count_flags(cpres + b * m, m);
    if (cnt < kDataShreds) {
      ok[b] = 0;
      out[b] = -AG_RS_ERR_NOT_ENOUGH_SHARDS;
      std::fill(op.begin() + b * kDataShreds, op.begin() + (b + 1) * kDataShreds, uint8_t{1});
    }
  }
  uint8_t* rec = cw + kDataShreds * S;
  if ((st = decode_device(c, kDataShreds, m, S, n, cw, cw_stride, rec, cw_stride, op.data(), cpres, n, mode)))
    return st;
  if ((st = c->d_strip.ensure(n * 8, c->stream))) return st;
  if (ag::launch_coder_strip(cw, cw_stride, static_cast<uint32_t>(kDataShreds * S), n, c->d_strip.as<int64_t>(),
                             c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  std::vector<int64_t> lens(n);
  AG_HIP(hipMemcpyAsync(lens.data(), c->d_strip.ptr, n * 8, hipMemcpyDeviceToHost, c->stream));
  AG_HIP(hipStreamSynchronize(c->stream));
  for (size_t b = 0; b < n; ++b) {
    if (!ok[b]) continue;
    if (lens[b] < 0) {
      ok[b] = 0;
      out[b] = -AG_RS_ERR_INVALID_PADDING;
    } else {
      out[b] = lens[b];
    }
  }
  // re-encode all coding shards (encode_coding_from_data) of each run of good slices.  A
  // slice whose present shards are exactly its k = 32 coding shards (every data shred lost,
  // the reference bench's shape) is skipped: its re-encoded coding shards are the received
  // ones already in place, bit for bit.
  for (size_t b = 0; b < n; ++b)
    if (ok[b] && m == kDataShreds && count_flags(dpres + b * kDataShreds, kDataShreds) == 0 &&
        count_flags(cpres + b * m, m) == m)
      ok[b] = 0;
  for (size_t b = 0; b < n;) {
    if (!ok[b]) {
      ++b;
      continue;
    }
    size_t e = b;
    while (e < n && ok[e]) ++e;
    if ((st = encode_device(c, kDataShreds, m, S, e - b, cw + b * cw_stride, cw_stride, rec + b * cw_stride,
                            cw_stride)))
      return st;
    b = e;
  }
  AG_HIP(hipStreamSynchronize(c->stream));
  return AG_RS_OK;
}

// ---- Ed25519 shred signatures ------------------------------------------------------------

namespace {
int ensure_ed_base(ag_rs_ctx* c) {
  if (c->d_ed_base.ptr) return AG_RS_OK;
  int st = c->d_ed_base.ensure(ag::kEdBaseTableBytes, c->stream);
  if (st) return st;
  return ag::launch_ed25519_init(c->d_ed_base.as<int32_t>(), c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}
constexpr size_t kMaxSigBatch = size_t{1} << 31;
int shred_validate_impl(ag_rs_ctx* c, size_t n, const uint8_t* data, size_t data_stride, size_t data_bytes,
                        const uint32_t* shred_index, const uint8_t* proofs, size_t proofs_stride, size_t height,
                        const uint64_t* slots, const uint64_t* slice_indices, const uint8_t* is_last,
                        const uint8_t* sigs, size_t sig_stride, const uint8_t* pk, const uint8_t* cached,
                        const uint8_t* has_cached, uint32_t cached_group, const uint8_t* active, uint8_t* status,
                        uint8_t* roots_out, uint8_t* commitments_out, uint8_t* leaf_nodes = nullptr,
                        size_t leaf_nodes_stride = 0, uint32_t leaves_per_tree = 0, size_t group_stride = 0,
                        uint32_t skip_row = 0, bool roots_ready = false);
}  // namespace

int ag_ed25519_public_key_batch(ag_rs_ctx* c, size_t n, const uint8_t* seeds, uint8_t* pks) {
  if (!c || n >= kMaxSigBatch || (n && (!seeds || !pks))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_ed_base(c);
  if (st) return st;
  return ag::launch_ed25519_public_key(seeds, pks, n, c->d_ed_base.as<int32_t>(), c->stream) == hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}

int ag_ed25519_sign_batch(ag_rs_ctx* c, size_t n, const uint8_t* seeds, size_t seed_stride, const uint8_t* pks,
                          size_t pk_stride, const uint8_t* msgs, size_t msg_stride, size_t msg_len, uint8_t* sigs) {
  if (!c || n >= kMaxSigBatch || msg_len >= (size_t{1} << 28) ||
      (n && (!seeds || !pks || !sigs || (msg_len && !msgs))))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_ed_base(c);
  if (st) return st;
  ag::EdSignParams p{};
  p.seeds = seeds;
  p.seed_stride = seed_stride;
  p.pks = pks;
  p.pk_stride = pk_stride;
  p.msgs = msgs;
  p.msg_stride = msg_stride;
  p.msg_len = static_cast<uint32_t>(msg_len);
  p.sigs = sigs;
  p.n = n;
  p.base_table = c->d_ed_base.as<int32_t>();
  return ag::launch_ed25519_sign(p, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_ed25519_verify_batch(ag_rs_ctx* c, size_t n, const uint8_t* pks, size_t pk_stride, const uint8_t* msgs,
                            size_t msg_stride, const uint32_t* msg_lens, size_t msg_len, const uint8_t* sigs,
                            size_t sig_stride, uint8_t* ok) {
  if (!c || n >= kMaxSigBatch || msg_len >= (size_t{1} << 28) || (n && (!pks || !sigs || !ok)) ||
      (n && !msgs && (msg_lens || msg_len)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_ed_base(c);
  if (st) return st;
  ag::EdVerifyParams p{};
  p.pks = pks;
  p.pk_stride = pk_stride;
  p.msgs = msgs;
  p.msg_stride = msg_stride;
  p.msg_lens = msg_lens;
  p.msg_len = static_cast<uint32_t>(msg_len);
  p.sigs = sigs;
  p.sig_stride = sig_stride;
  p.n = n;
  p.ok = ok;
  p.base_table = c->d_ed_base.as<int32_t>();
  return ag::launch_ed25519_verify(p, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

int ag_shred_validate_batch(ag_rs_ctx* c, size_t n, const uint8_t* data, size_t data_stride, size_t data_bytes,
                            const uint32_t* shred_index, const uint8_t* proofs, size_t proofs_stride, size_t height,
                            const uint64_t* slots, const uint64_t* slice_indices, const uint8_t* is_last,
                            const uint8_t* sigs, size_t sig_stride, const uint8_t* pk, const uint8_t* cached,
                            const uint8_t* has_cached, uint8_t* status, uint8_t* roots_out, uint8_t* commitments_out) {
  return shred_validate_impl(c, n, data, data_stride, data_bytes, shred_index, proofs, proofs_stride, height, slots,
                             slice_indices, is_last, sigs, sig_stride, pk, cached, has_cached, 1, nullptr, status,
                             roots_out, commitments_out);
}

}  // extern "C"

namespace {

// ag_shred_validate_batch with the cache entries shared by cached_group consecutive shreds
// (the composed deshred: one cached commitment per slice).
int shred_validate_impl(ag_rs_ctx* c, size_t n, const uint8_t* data, size_t data_stride, size_t data_bytes,
                        const uint32_t* shred_index, const uint8_t* proofs, size_t proofs_stride, size_t height,
                        const uint64_t* slots, const uint64_t* slice_indices, const uint8_t* is_last,
                        const uint8_t* sigs, size_t sig_stride, const uint8_t* pk, const uint8_t* cached,
                        const uint8_t* has_cached, uint32_t cached_group, const uint8_t* active, uint8_t* status,
                        uint8_t* roots_out, uint8_t* commitments_out, uint8_t* leaf_nodes, size_t leaf_nodes_stride,
                        uint32_t leaves_per_tree, size_t group_stride, uint32_t skip_row, bool roots_ready) {
  // roots_ready: step 1 already ran (launch_derive_roots, e.g. on another stream): roots_out holds
  // every active shred's derived root
  if (roots_ready && !roots_out) return AG_RS_ERR_INVALID_ARGUMENT;
  if (!c || n >= kMaxSigBatch || data_bytes >= (size_t{1} << 28) ||
      height > static_cast<size_t>(ag::kMerkleMaxHeight) ||
      (n && (!shred_index || !slots || !slice_indices || !is_last || !sigs || !pk || !status ||
             (data_bytes && !data) || (height && !proofs))) ||
      (cached == nullptr) != (has_cached == nullptr) || proofs_stride % 16 ||
      reinterpret_cast<uintptr_t>(proofs) % 16 || (n > 1 && data_stride < data_bytes))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_ed_base(c);
  if (st) return st;
  uint8_t* roots = roots_out;
  if (!roots) {
    if ((st = c->d_sh_roots.ensure(32 * n, c->stream))) return st;
    roots = c->d_sh_roots.as<uint8_t>();
  }
  uint8_t* commits = commitments_out;
  if (!commits) {
    if ((st = c->d_sh_commit.ensure(ag::kSliceCommitmentLen * n, c->stream))) return st;
    commits = c->d_sh_commit.as<uint8_t>();
  }
  if ((st = c->d_sh_onvalid.ensure(n, c->stream)) || (st = c->d_sh_list.ensure(4 * (n + 1), c->stream))) return st;
  uint32_t* list = c->d_sh_list.as<uint32_t>();
  uint32_t* count = list + n;
  // 1. Shred::slice_root (shredder.rs:168-175): derive_root from the Merkle path
  ag::MerkleVerifyParams mp{};
  mp.leaves = data;
  mp.leaf_stride = data_stride;
  mp.leaf_bytes = static_cast<uint32_t>(data_bytes);
  mp.height = static_cast<uint32_t>(height);
  mp.index = shred_index;
  mp.proofs = proofs;
  mp.proofs_stride = proofs_stride;
  mp.n = n;
  mp.roots_out = roots;
  mp.active = active;
  mp.list = list;  // scratch until the signature list below reuses it (stream order)
  mp.leaf_nodes = leaf_nodes;  // the leaf digests for a later Merkle rebuild over the same rows
  mp.leaf_nodes_stride = leaf_nodes_stride;
  mp.leaves_per_tree = leaves_per_tree;
  mp.group_stride = group_stride;
  mp.skip_row = skip_row;
  if (!roots_ready && ag::launch_merkle_verify(mp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // 2. SliceCommitment + cached-commitment rule (validated_shred.rs:57-64)
  AG_HIP(hipMemsetAsync(count, 0, 4, c->stream));
  ag::ShredCommitParams cp{};
  cp.slots = slots;
  cp.slice_indices = slice_indices;
  cp.is_last = is_last;
  cp.roots = roots;
  cp.cached = cached;
  cp.has_cached = has_cached;
  cp.cached_group = cached_group;
  cp.active = active;
  cp.n = n;
  cp.commitments = commits;
  cp.status = status;
  cp.on_valid = c->d_sh_onvalid.as<uint8_t>();
  cp.list = list;
  cp.list_count = count;
  if (ag::launch_shred_commit(cp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // 3. signature checks for the listed shreds (validated_shred.rs:65-77)
  ag::EdVerifyParams vp{};
  vp.pks = pk;
  vp.pk_stride = 0;
  vp.msgs = commits;
  vp.msg_stride = ag::kSliceCommitmentLen;
  vp.msg_len = ag::kSliceCommitmentLen;
  vp.sigs = sigs;
  vp.sig_stride = sig_stride;
  vp.n = n;
  vp.list = list;
  vp.list_count = count;
  vp.status = status;
  vp.on_valid = c->d_sh_onvalid.as<uint8_t>();
  vp.base_table = c->d_ed_base.as<int32_t>();
  return ag::launch_ed25519_verify(vp, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

}  // namespace

extern "C" {

int ag_slice_sign_batch(ag_rs_ctx* c, size_t nslices, const uint8_t* seed, const uint8_t* pk, const uint64_t* slots,
                        const uint64_t* slice_indices, const uint8_t* is_last, const uint8_t* roots, uint8_t* sigs,
                        uint8_t* commitments_out) {
  if (!c || nslices >= kMaxSigBatch ||
      (nslices && (!seed || !pk || !slots || !slice_indices || !is_last || !roots || !sigs)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  int st = ensure_ed_base(c);
  if (st) return st;
  uint8_t* commits = commitments_out;
  if (!commits) {
    if ((st = c->d_sh_commit.ensure(ag::kSliceCommitmentLen * nslices, c->stream))) return st;
    commits = c->d_sh_commit.as<uint8_t>();
  }
  const size_t n = nslices;
  if ((st = c->d_sh_onvalid.ensure(2 * n, c->stream)) || (st = c->d_sh_list.ensure(4 * (n + 1), c->stream)))
    return st;
  uint32_t* list = c->d_sh_list.as<uint32_t>();
  AG_HIP(hipMemsetAsync(list + n, 0, 4, c->stream));
  // SliceCommitment::new (shredder.rs:206-215); no cache, so every slice is listed
  ag::ShredCommitParams cp{};
  cp.slots = slots;
  cp.slice_indices = slice_indices;
  cp.is_last = is_last;
  cp.roots = roots;
  cp.n = n;
  cp.commitments = commits;
  cp.status = c->d_sh_onvalid.as<uint8_t>() + n;
  cp.on_valid = c->d_sh_onvalid.as<uint8_t>();
  cp.list = list;
  cp.list_count = list + n;
  if (ag::launch_shred_commit(cp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // sk.sign_bytes(commitment) (shredder.rs:540)
  ag::EdSignParams p{};
  p.seeds = seed;
  p.seed_stride = 0;
  p.pks = pk;
  p.pk_stride = 0;
  p.msgs = commits;
  p.msg_stride = ag::kSliceCommitmentLen;
  p.msg_len = ag::kSliceCommitmentLen;
  p.sigs = sigs;
  p.n = n;
  p.base_table = c->d_ed_base.as<int32_t>();
  return ag::launch_ed25519_sign(p, c->stream) == hipSuccess ? AG_RS_OK : AG_RS_ERR_DEVICE;
}

// ---- shred wire format ----------------------------------------------------------------

namespace {
bool columns_ok(const ag_shred_columns* c) {
  return c && c->kind && c->slot && c->slice_index && c->is_last && c->shred_index && c->data_len && c->sig &&
         c->height && (c->data || c->data_stride == 0) && (c->proof || c->proof_stride == 0);
}
ag::ShredColumns to_columns(const ag_shred_columns* c) {
  ag::ShredColumns r{};
  r.kind = c->kind;
  r.slot = c->slot;
  r.slice_index = c->slice_index;
  r.is_last = c->is_last;
  r.shred_index = c->shred_index;
  r.data = c->data;
  r.data_stride = c->data_stride;
  r.data_len = c->data_len;
  r.sig = c->sig;
  r.proof = c->proof;
  r.proof_stride = c->proof_stride;
  r.height = c->height;
  return r;
}
}  // namespace

int ag_shred_deserialize_batch(ag_rs_ctx* c, size_t n, const uint8_t* packets, size_t packet_stride,
                               const uint32_t* packet_lens, const ag_shred_columns* cols, uint8_t* status) {
  if (!c || n >= kMaxSigBatch || (n && (!packets || !packet_lens || !status || !columns_ok(cols))))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  return ag::launch_shred_deserialize(packets, packet_stride, packet_lens, n, to_columns(cols), status, c->stream) ==
                 hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}

int ag_shred_serialize_batch(ag_rs_ctx* c, size_t n, const ag_shred_columns* cols, uint8_t* packets,
                             size_t packet_stride, uint32_t* packet_lens) {
  if (!c || n >= kMaxSigBatch || (n && (!packets || !packet_lens || !columns_ok(cols))))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (n == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  return ag::launch_shred_serialize(to_columns(cols), n, packets, packet_stride, packet_lens, c->stream) ==
                 hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}

int ag_slice_frame_batch(ag_rs_ctx* c, size_t nslices, size_t shred_bytes, const uint8_t* parent_flags,
                         const uint8_t* parent_ids, const uint8_t* data, size_t data_stride, const uint32_t* data_lens,
                         uint8_t* codewords, size_t codeword_stride, uint32_t* payload_lens_out) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (!parent_flags || !parent_ids || !data_lens || !codewords || !payload_lens_out || nslices > 0x7FFFFFFFull ||
      shred_bytes == 0 || reinterpret_cast<uintptr_t>(codewords) % 4 || codeword_stride % 4 ||
      (nslices > 1 && codeword_stride < 32 * shred_bytes))
    return AG_RS_ERR_INVALID_ARGUMENT;
  size_t max_len = 0;
  for (size_t b = 0; b < nslices; ++b) {
    if (parent_flags[b] > 1) return AG_RS_ERR_INVALID_ARGUMENT;
    const size_t framed = 1 + (parent_flags[b] ? AG_SLICE_BLOCK_ID_BYTES : 0) + 8 + size_t{data_lens[b]};
    if (framed > AG_SLICE_MAX_DATA || framed >= 32 * shred_bytes) return AG_RS_ERR_TOO_MUCH_DATA;
    max_len = std::max<size_t>(max_len, data_lens[b]);
  }
  if (max_len && (!data || (nslices > 1 && data_stride < max_len))) return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  // metadata: flags | ids | lens, one upload
  const size_t off_ids = (nslices + 15) / 16 * 16, off_lens = off_ids + (nslices * AG_SLICE_BLOCK_ID_BYTES + 15) / 16 * 16;
  const size_t bytes = off_lens + 4 * nslices;
  int st = c->d_slice_meta.ensure(bytes, c->stream);
  if (st) return st;
  std::vector<uint8_t> meta(bytes, 0);
  std::memcpy(meta.data(), parent_flags, nslices);
  std::memcpy(meta.data() + off_ids, parent_ids, nslices * AG_SLICE_BLOCK_ID_BYTES);
  std::memcpy(meta.data() + off_lens, data_lens, 4 * nslices);
  AG_HIP(hipMemcpyAsync(c->d_slice_meta.ptr, meta.data(), bytes, hipMemcpyHostToDevice, c->stream));
  ag::SliceFrameParams p{};
  uint8_t* d = c->d_slice_meta.as<uint8_t>();
  p.parent_flags = d;
  p.parent_ids = d + off_ids;
  p.data_lens = reinterpret_cast<const uint32_t*>(d + off_lens);
  p.data = data;
  p.data_stride = data_stride;
  p.cw = codewords;
  p.cw_stride = codeword_stride;
  p.n = nslices;
  if (ag::launch_slice_frame(p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  AG_HIP(hipStreamSynchronize(c->stream));  // the host metadata buffer goes out of scope
  for (size_t b = 0; b < nslices; ++b)
    payload_lens_out[b] = static_cast<uint32_t>(1 + (parent_flags[b] ? AG_SLICE_BLOCK_ID_BYTES : 0) + 8 + data_lens[b]);
  return AG_RS_OK;
}

int ag_slice_parse_batch(ag_rs_ctx* c, size_t nslices, const uint8_t* codewords, size_t codeword_stride,
                         const int64_t* payload_lens, uint8_t* status, uint8_t* parent_flags, uint8_t* parent_ids,
                         uint32_t* data_offsets, uint32_t* data_lens) {
  if (!c) return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (!codewords || !payload_lens || !status || !parent_flags || !parent_ids || !data_offsets || !data_lens ||
      nslices > 0x7FFFFFFFull)
    return AG_RS_ERR_INVALID_ARGUMENT;
  for (size_t b = 0; b < nslices; ++b)  // the bytes parsed must lie inside the codeword
    if (nslices > 1 && payload_lens[b] > 0 && static_cast<uint64_t>(payload_lens[b]) > codeword_stride)
      return AG_RS_ERR_INVALID_ARGUMENT;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  // device layout: lens (8n) | status (n) | flags (n) | ids (40n) | offsets (4n) | data lens (4n)
  const size_t o_st = 8 * nslices, o_fl = o_st + nslices, o_id = o_fl + nslices,
               o_off = (o_id + AG_SLICE_BLOCK_ID_BYTES * nslices + 3) / 4 * 4, o_len = o_off + 4 * nslices;
  const size_t bytes = o_len + 4 * nslices;
  int st = c->d_slice_meta.ensure(bytes, c->stream);
  if (st) return st;
  uint8_t* d = c->d_slice_meta.as<uint8_t>();
  AG_HIP(hipMemcpyAsync(d, payload_lens, 8 * nslices, hipMemcpyHostToDevice, c->stream));
  ag::SliceParseParams p{};
  p.cw = codewords;
  p.cw_stride = codeword_stride;
  p.payload_lens = reinterpret_cast<const int64_t*>(d);
  p.status = d + o_st;
  p.parent_flags = d + o_fl;
  p.parent_ids = d + o_id;
  p.data_offsets = reinterpret_cast<uint32_t*>(d + o_off);
  p.data_lens = reinterpret_cast<uint32_t*>(d + o_len);
  p.n = nslices;
  if (ag::launch_slice_parse(p, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // read back through pinned staging (a pageable destination costs a staged copy: ~0.3 ms more
  // for a 65 536-slice batch)
  if ((st = c->h_slice_meta.ensure(bytes - o_st))) return st;
  const uint8_t* out = c->h_slice_meta.as<uint8_t>();
  AG_HIP(hipMemcpyAsync(c->h_slice_meta.ptr, d + o_st, bytes - o_st, hipMemcpyDeviceToHost, c->stream));
  AG_HIP(hipStreamSynchronize(c->stream));
  std::memcpy(status, out, nslices);
  std::memcpy(parent_flags, out + (o_fl - o_st), nslices);
  std::memcpy(parent_ids, out + (o_id - o_st), AG_SLICE_BLOCK_ID_BYTES * nslices);
  std::memcpy(data_offsets, out + (o_off - o_st), 4 * nslices);
  std::memcpy(data_lens, out + (o_len - o_st), 4 * nslices);
  return AG_RS_OK;
}

}  // extern "C"

// =====================================================================================
// Composed Shredder (RegularShredder): ag_shredder_shred_batch / ag_shredder_deshred_batch
// =====================================================================================
namespace {

constexpr size_t kPipeProofBytes = 32 * ag::kPipeHeight;  // one Merkle path of a slice tree

int pipe_buf(ag_rs_ctx* c, int i, size_t bytes, uint8_t** out) {
  const int st = c->pipe[i].ensure(std::max<size_t>(bytes, 64), c->stream);
  if (st) return st;
  *out = c->pipe[i].as<uint8_t>();
  return AG_RS_OK;
}

// The per-slice columns pipe_check writes (present | slot | slice index | is_last, contiguous
// from `present`) read back in one copy into pinned staging: views valid until the next call
// on the context
struct PipeMeta {
  const uint64_t *present, *slot, *sidx;
  const uint8_t* last;
};
int read_pipe_meta(ag_rs_ctx* c, const uint64_t* d_present, size_t n, PipeMeta* m) {
  const int st = c->h_pipe_meta.ensure(25 * n);
  if (st) return st;
  uint8_t* h = c->h_pipe_meta.as<uint8_t>();
  AG_HIP(hipMemcpyAsync(h, d_present, 25 * n, hipMemcpyDeviceToHost, c->stream));
  AG_HIP(hipStreamSynchronize(c->stream));
  m->present = reinterpret_cast<const uint64_t*>(h);
  m->slot = m->present + n;
  m->sidx = m->slot + n;
  m->last = h + 24 * n;
  return AG_RS_OK;
}

bool pipe_args_ok(size_t nslices, size_t S, const uint8_t* codewords, const uint8_t* packets,
                  const uint32_t* packet_lens) {
  return S != 0 && S % 2 == 0 && S <= 1024 && nslices < (size_t{1} << 24) &&
         (nslices == 0 || (codewords && packets && packet_lens)) && reinterpret_cast<uintptr_t>(codewords) % 16 == 0;
}

}  // namespace

namespace {
// ReedSolomonCoder::deshred (reed_solomon.rs:140-208, ANY_K) over the kept shreds of every
// slice without a host round trip, for whole-chunk shreds (S % 64 == 0): the per-slice
// patterns come from the kept-shred masks on the device (launch_pipe_patterns), the per-lane
// window decoder restores the data shreds, coder_strip finds each payload's padding, and the
// 32-point encode rewrites the coding shreds of the slices that decoded and stripped (store
// masks per slice; the others keep theirs).  HighRate 32:32 also takes shreds with a tail of
// T = S mod 64 >= 16 bytes (pipe_tail_ok): the tail is the last column (decode_h8's TAIL
// variant, the TAIL encode).  plen[s] as ag_rs_coder_deshred_batch: the
// payload length, or -NotEnoughShreds / -InvalidPadding.
//
// pipe_coder_enqueue runs slices s0 .. s0 + n of a batch whose scratch pipe_coder_reserve
// sized (cw / d_present already at slice s0); pipe_coder_finish reads the results back.  The
// store-mask kernel writes each slice's final result (length or error) into the strip words.
int pipe_coder_reserve(ag_rs_ctx* c, size_t ntot, size_t m) {
  int st;
  if ((st = c->ensure_tables()) || (st = c->d_pipe_few.ensure(ntot, c->stream)) ||
      (st = c->d_pipe_mask.ensure(8 * ntot, c->stream)) || (st = c->d_strip.ensure(8 * ntot, c->stream)))
    return st;
  if (m > kDataShreds)
    return (st = c->d_x128.ensure(10 * ntot * 8, c->stream)) ? st : c->d_rows128.ensure(ntot * 128 * 4, c->stream);
  if ((st = c->d_xmask.ensure(3 * ntot * 8, c->stream)) || (st = c->d_rows.ensure(ntot * 64 * 4, c->stream))) return st;
  c->xmask_host.clear();  // d_xmask / d_rows no longer hold decode_device's cached patterns
  c->xmask_w = 0;
  return AG_RS_OK;
}
int pipe_coder_finish(ag_rs_ctx* c, size_t n, int64_t* plen);
int pipe_coder_enqueue(ag_rs_ctx* c, size_t s0, size_t n, size_t S, uint8_t* cw, size_t cw_stride,
                       const uint64_t* d_present, size_t m, bool no_surplus);
// The whole batch in one range (the composed deshred's coder stage).  no_surplus: the caller
// knows that no slice keeps more than 32 shreds and none keeps all 32 data shreds.
int pipe_coder_deshred(ag_rs_ctx* c, size_t n, size_t S, uint8_t* cw, size_t cw_stride, const uint64_t* d_present,
                       int64_t* plen, size_t m, bool no_surplus) {
  int st;
  if ((st = pipe_coder_reserve(c, n, m)) ||
      (st = pipe_coder_enqueue(c, 0, n, S, cw, cw_stride, d_present, m, no_surplus)))
    return st;
  return pipe_coder_finish(c, n, plen);
}
// The same for CodingOnlyShredder's coder (LowRate 32:64, shredder.rs:362-395) and
// PetsShredder's (32:33, :403-444; its recovery shards are the first 33 of 32:64's): every slice
// decodes in the W = 128 window as the two per-lane decode_x16 passes (the class-8 patterns of
// decode_device, built on the device by launch_pipe_patterns128), then the strip, and the
// LowRate re-encode of both 32-shard recovery chunks under the per-slice store masks.
// present: two words per slice (launch_pipe_patterns128).
int pipe_coder_enqueue_lowrate(ag_rs_ctx* c, size_t s0, size_t n, size_t S, uint8_t* cw, size_t cw_stride,
                               const uint64_t* d_present, size_t m) {
  constexpr size_t k = kDataShreds;
  const size_t cps = S / 64;
  uint64_t* xm = c->d_x128.as<uint64_t>() + 10 * s0;
  uint32_t* rows = c->d_rows128.as<uint32_t>() + 128 * s0;
  uint8_t* few = c->d_pipe_few.as<uint8_t>() + s0;
  uint64_t* mask = c->d_pipe_mask.as<uint64_t>() + s0;
  int64_t* strip = c->d_strip.as<int64_t>() + s0;
  if (ag::launch_pipe_patterns128(d_present, n, xm, few, c->stream) != hipSuccess ||
      ag::launch_decode_rows128(xm, static_cast<uint32_t>(n), c->dtables(), rows, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  ag::DecodeXParams p{};
  p.rec = cw + k * S;
  p.rec_block_stride = cw_stride;
  p.rec_shard_stride = S;
  p.orig = cw;
  p.orig_block_stride = cw_stride;
  p.orig_shard_stride = S;
  p.rows = rows;
  p.rows_w = 128;
  p.k = static_cast<uint32_t>(k);
  p.m = 32;  // recovery shards per window half (the kernel addresses the rest from p.rec)
  p.chunk = 32;
  p.low_rate = 1;
  p.chunks_per_shard = static_cast<uint32_t>(cps);
  p.total_columns = static_cast<uint64_t>(n) * cps;
  p.per_lane = 1;
  for (int pass = 1; pass <= 2; ++pass) {
    p.pmask = xm + (pass == 1 ? 6 : 8) * n;
    if (ag::launch_decode_x(128, pass, p, (p.total_columns + 63) / 64, c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
  }
  if (ag::launch_coder_strip(cw, cw_stride, static_cast<uint32_t>(k * S), n, strip, c->stream) != hipSuccess ||
      ag::launch_pipe_store_masks(few, strip, d_present, 2, n, mask, -AG_RS_ERR_NOT_ENOUGH_SHARDS,
                                  -AG_RS_ERR_INVALID_PADDING, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  for (unsigned j = 0; j * 32 < m;) {  // the recovery chunks, two per launch (encode_cols' LowRate loop)
    ag::XformParams xp{};
    xp.in = cw;
    xp.in_block_stride = cw_stride;
    xp.in_shard_stride = S;
    xp.out = cw + (k + 32 * j) * S;
    xp.out_block_stride = cw_stride;
    xp.out_shard_stride = S;
    xp.out_mask = mask;  // the slice's absent coding shreds, all, or none
    xp.pattern_per_block = 1;
    xp.n_in = static_cast<uint32_t>(k);
    xp.chunks_per_shard = static_cast<uint32_t>(cps);
    xp.total_columns = static_cast<uint64_t>(n) * cps;
    const bool pair = j % 2 == 0 && (j + 1) * 32 < m && j < 4;
    xp.n_out = static_cast<uint32_t>(std::min<size_t>(pair ? 64 : 32, m - 32 * j));
    if ((pair ? ag::launch_xform_lowrate2(j / 2, xp, c->stream) : ag::launch_xform_lowrate(32, j, xp, c->stream)) !=
        hipSuccess)
      return AG_RS_ERR_DEVICE;
    j += pair ? 2 : 1;
  }
  return AG_RS_OK;
}

int pipe_coder_enqueue(ag_rs_ctx* c, size_t s0, size_t n, size_t S, uint8_t* cw, size_t cw_stride,
                       const uint64_t* d_present, size_t m, bool no_surplus) {
  constexpr size_t k = kDataShreds;
  // whole 64-byte chunks, then (S mod 64 = T >= 16) the shard's T-byte tail as one more column
  const size_t cps = (S + 63) / 64;
  const uint32_t tail = static_cast<uint32_t>(S % 64);
  if (n == 0) return AG_RS_OK;
  if (m > kDataShreds) return pipe_coder_enqueue_lowrate(c, s0, n, S, cw, cw_stride, d_present, m);
  constexpr size_t W = 64;
  uint64_t* xm = c->d_xmask.as<uint64_t>() + 3 * s0;
  uint32_t* rows = c->d_rows.as<uint32_t>() + W * s0;
  uint8_t* few = c->d_pipe_few.as<uint8_t>() + s0;
  uint64_t* mask = c->d_pipe_mask.as<uint64_t>() + s0;
  int64_t* strip = c->d_strip.as<int64_t>() + s0;
  // The window decode also restores the absent coding shreds of exactly-k slices (few 2): the
  // re-encode below skips those.  1 KiB shreds (every maximum slice) run the packed decoder
  // (decode_pk<-1>), the other whole-chunk sizes decode_h8<-1> (the full 64-point FFT).
  const bool fuse = true;
  if (ag::launch_pipe_patterns(d_present, n, xm, few, fuse, c->stream) != hipSuccess ||
      ag::launch_decode_rows(xm, xm + n, static_cast<uint32_t>(n), static_cast<uint32_t>(W), c->dtables(), rows, true,
                             c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  ag::DecodeXParams p{};
  p.rec = cw + k * S;
  p.rec_block_stride = cw_stride;
  p.rec_shard_stride = S;
  p.orig = cw;
  p.orig_block_stride = cw_stride;
  p.orig_shard_stride = S;
  p.pmask = xm + n;
  p.rows = rows;
  p.k = static_cast<uint32_t>(k);
  p.m = 32;
  p.chunk = 32;
  p.low_rate = 0;
  p.chunks_per_shard = static_cast<uint32_t>(cps);
  p.total_columns = static_cast<uint64_t>(n) * cps;
  p.per_lane = 1;
  p.rows_w = static_cast<uint32_t>(W);
  p.any_k = 1;  // launch_pipe_patterns keeps exactly k survivors
  p.fuse = fuse ? 1u : 0u;
  p.tail_bytes = tail;
  if (ag::launch_decode_x(static_cast<unsigned>(W), 0, p, (p.total_columns + 63) / 64, c->stream,
                          &c->last_window_kernels) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  if (ag::launch_coder_strip(cw, cw_stride, static_cast<uint32_t>(k * S), n, strip, c->stream) != hipSuccess ||
      ag::launch_pipe_store_masks(few, strip, d_present, 1, n, mask, -AG_RS_ERR_NOT_ENOUGH_SHARDS,
                                  -AG_RS_ERR_INVALID_PADDING, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  ag::XformParams xp{};
  xp.in = cw;
  xp.in_block_stride = cw_stride;
  xp.in_shard_stride = S;
  xp.out = cw + k * S;
  xp.out_block_stride = cw_stride;
  xp.out_shard_stride = S;
  xp.out_mask = mask;
  xp.pattern_per_block = 1;
  xp.n_in = static_cast<uint32_t>(k);
  xp.n_out = 32;
  xp.chunks_per_shard = static_cast<uint32_t>(cps);
  xp.total_columns = static_cast<uint64_t>(n) * cps;
  xp.skip_idle = fuse ? 1u : 0u;  // tiles of fused slices only: nothing to re-encode
  xp.tail_bytes = tail;
  // fused, no slice with surplus shreds and none with every data shred: every store mask is
  // zero (exactly 32 kept: restored by the decode; fewer, or a failed strip: untouched)
  if (fuse && no_surplus) return AG_RS_OK;
  if (ag::launch_xform(ag::XformKind::kEncode32, xp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  return AG_RS_OK;
}
// plen[0 .. n) from the store-mask kernels' results (synchronous): read back through pinned
// staging (a pageable destination would take the runtime's bounce path)
int pipe_coder_finish(ag_rs_ctx* c, size_t n, int64_t* plen) {
  int st;
  if ((st = c->h_strip.ensure(8 * n))) return st;
  AG_HIP(hipMemcpyAsync(c->h_strip.ptr, c->d_strip.ptr, 8 * n, hipMemcpyDeviceToHost, c->stream));
  AG_HIP(hipStreamSynchronize(c->stream));
  std::memcpy(plen, c->h_strip.ptr, 8 * n);
  return AG_RS_OK;
}
// Step 6b of ag_shredder_deshred_batch for slice s: its datagram rows are parsed again into
// the codeword (the pass before rewrote the restored and re-encoded rows), the kept shreds
// (present bit mask) go through ReedSolomonCoder::deshred with the crate's EXACT decoder,
// and the Merkle rebuild (roots2 row s, the slice's proof rows), root comparison and
// SlicePayload parse are redone for this slice.  Outputs replace slice s's entries.
int pipe_rerun_exact(ag_rs_ctx* c, size_t s, size_t S, const uint8_t* packets, size_t packet_stride,
                     const uint32_t* packet_lens, const ag::ShredColumns& cols, uint8_t* wire, uint8_t* codewords,
                     uint8_t* proof, uint8_t* roots2, const uint8_t* sroot, uint8_t* same, int64_t* plen,
                     uint8_t* h_same, uint8_t* sstat, uint8_t* parent_flag, uint8_t* parent_id, uint32_t* data_offset,
                     uint32_t* data_len, uint64_t present) {
  constexpr size_t kRows = ag::kPipeShreds;
  const size_t r0 = s * kRows, cw_stride = kRows * S;
  uint8_t* cw = codewords + s * cw_stride;
  ag::ShredColumns rc = cols;
  rc.kind += r0;
  rc.slot += r0;
  rc.slice_index += r0;
  rc.is_last += r0;
  rc.shred_index += r0;
  rc.data = cw;
  rc.data_len += r0;
  rc.sig += 64 * r0;
  rc.proof += r0 * cols.proof_stride;
  rc.height += r0;
  if (ag::launch_shred_deserialize(packets + r0 * packet_stride, packet_stride, packet_lens + r0, kRows, rc, wire + r0,
                                   c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  uint8_t dp[ag::kPipeData], cp[kRows - ag::kPipeData];
  for (uint32_t j = 0; j < kRows; ++j) {
    const uint8_t bit = static_cast<uint8_t>((present >> j) & 1);
    if (j < ag::kPipeData) dp[j] = bit;
    else cp[j - ag::kPipeData] = bit;
  }
  int st = ag_rs_coder_deshred_batch(c, kRows - ag::kPipeData, 1, S, cw, cw_stride, dp, cp, AG_RS_DECODE_EXACT, plen);
  if (st) return st;
  *h_same = 0;
  if (*plen < 0) return AG_RS_OK;
  if ((st = ag_merkle_build_batch(c, kRows, S, 1, cw, S, cw_stride, roots2 + 32 * s, nullptr, 0,
                                  proof + r0 * cols.proof_stride, kRows * cols.proof_stride)))
    return st;
  if (ag::launch_pipe_root_cmp(roots2 + 32 * s, sroot + 32 * s, 1, same + s, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  AG_HIP(hipMemcpyAsync(h_same, same + s, 1, hipMemcpyDeviceToHost, c->stream));
  // synchronous: h_same has landed when it returns
  return ag_slice_parse_batch(c, 1, cw, cw_stride, plen, sstat, parent_flag, parent_id, data_offset, data_len);
}

}  // namespace

namespace {
// ag_slice_sign_batch on the context's side stream, forked from the main stream's current point
// (the roots): the signing (one signature per lane, latency-bound) overlaps the serialization of
// everything else in the datagrams; the caller waits on side_join before launch_shred_sig_patch.
int sign_on_side(ag_rs_ctx* c, size_t n, const uint8_t* seed, const uint8_t* pk, const uint64_t* slots,
                 const uint64_t* slice_indices, const uint8_t* is_last, const uint8_t* roots, uint8_t* sigs) {
  int st;
  if ((st = c->ensure_side_stream())) return st;
  AG_HIP(hipEventRecord(c->side_fork, c->stream));
  AG_HIP(hipStreamWaitEvent(c->side, c->side_fork, 0));
  std::swap(c->stream, c->side);
  st = ag_slice_sign_batch(c, n, seed, pk, slots, slice_indices, is_last, roots, sigs, nullptr);
  std::swap(c->stream, c->side);
  if (st) {
    (void)hipStreamSynchronize(c->side);
    return st;
  }
  AG_HIP(hipEventRecord(c->side_join, c->side));
  return AG_RS_OK;
}
}  // namespace

extern "C" {

int ag_shredder_shred_batch(ag_rs_ctx* c, size_t nslices, size_t S, const uint8_t* parent_flags,
                            const uint8_t* parent_ids, const uint8_t* data, size_t data_stride,
                            const uint32_t* data_lens, const uint64_t* slots, const uint64_t* slice_indices,
                            const uint8_t* is_last, const uint8_t* seed, const uint8_t* pk, uint8_t* codewords,
                            uint8_t* roots_out, uint8_t* sigs_out, uint8_t* packets, size_t packet_stride,
                            uint32_t* packet_lens) {
  if (!c || !pipe_args_ok(nslices, S, codewords, packets, packet_lens) ||
      (nslices && (!parent_flags || !parent_ids || !data_lens || !slots || !slice_indices || !is_last || !seed ||
                   !pk)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  const size_t n = nslices, N = n * ag::kPipeShreds, cw_stride = ag::kPipeShreds * S;
  // 1. Slice::payload_bytes into the data regions, 2. ReedSolomonCoder::shred in place
  std::vector<uint32_t> lens(n);
  int st = ag_slice_frame_batch(c, n, S, parent_flags, parent_ids, data, data_stride, data_lens, codewords, cw_stride,
                                lens.data());
  if (st) return st;
  if ((st = ag_rs_coder_shred_batch(c, ag::kPipeShreds - ag::kPipeData, n, S, nullptr, 0, lens.data(), codewords,
                                    cw_stride)))
    return st;
  // 3. slice Merkle trees: roots and every shred's path
  uint8_t *roots = roots_out, *sigs = sigs_out, *proofs, *kind, *sidx, *dlen, *height;
  if (!roots && (st = pipe_buf(c, 0, 32 * n, &roots))) return st;
  if (!sigs && (st = pipe_buf(c, 1, 64 * n, &sigs))) return st;
  if ((st = pipe_buf(c, 2, kPipeProofBytes * N, &proofs)) || (st = pipe_buf(c, 3, N, &kind)) ||
      (st = pipe_buf(c, 4, 4 * N, &sidx)) || (st = pipe_buf(c, 5, 4 * N, &dlen)) ||
      (st = pipe_buf(c, 6, 4 * N, &height)))
    return st;
  if ((st = ag_merkle_build_batch(c, ag::kPipeShreds, S, n, codewords, S, cw_stride, roots, nullptr, 0, proofs,
                                  ag::kPipeShreds * kPipeProofBytes)))
    return st;
  // 4. slice_sig = sign(SliceCommitment(header, root))
  // 4b. signed on the side stream while 5 serializes the rest of the datagrams
  if ((st = sign_on_side(c, n, seed, pk, slots, slice_indices, is_last, roots, sigs))) return st;
  // 5. the 64 datagrams per slice (header and signature shared by the slice's rows)
  ag::PipeExpandParams ep{};
  ep.nslices = n;
  ep.shred_bytes = static_cast<uint32_t>(S);
  ep.num_data = ag::kPipeData;
  ep.kind = kind;
  ep.shred_index = reinterpret_cast<uint32_t*>(sidx);
  ep.data_len = reinterpret_cast<uint32_t*>(dlen);
  ep.height = reinterpret_cast<uint32_t*>(height);
  if (ag::launch_pipe_expand(ep, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  ag::ShredColumns cols{};
  cols.kind = kind;
  cols.slot = const_cast<uint64_t*>(slots);
  cols.slice_index = const_cast<uint64_t*>(slice_indices);
  cols.is_last = const_cast<uint8_t*>(is_last);
  cols.shred_index = ep.shred_index;
  cols.data = codewords;
  cols.data_stride = S;
  cols.data_len = ep.data_len;
  cols.sig = sigs;
  cols.proof = proofs;
  cols.proof_stride = kPipeProofBytes;
  cols.height = ep.height;
  cols.hdr_group = ag::kPipeShreds;
  cols.skip_sig = 1;
  if (ag::launch_shred_serialize(cols, N, packets, packet_stride, packet_lens, c->stream) != hipSuccess) {
    (void)hipStreamSynchronize(c->side);
    return AG_RS_ERR_DEVICE;
  }
  AG_HIP(hipStreamWaitEvent(c->stream, c->side_join, 0));
  if (ag::launch_shred_sig_patch(cols, N, packets, packet_stride, packet_lens, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  return AG_RS_OK;
}

int ag_shredder_deshred_batch(ag_rs_ctx* c, size_t nslices, size_t S, uint8_t* packets, size_t packet_stride,
                              uint32_t* packet_lens, const uint8_t* pk, uint8_t* codewords, int32_t* status,
                              uint64_t* slots_out, uint64_t* slice_indices_out, uint8_t* is_last_out,
                              uint8_t* parent_flags_out, uint8_t* parent_ids_out, uint32_t* data_offsets_out,
                              uint32_t* data_lens_out) {
  if (!c || !pipe_args_ok(nslices, S, codewords, packets, packet_lens) ||
      (nslices && (!pk || !status || !slots_out || !slice_indices_out || !is_last_out || !parent_flags_out ||
                   !parent_ids_out || !data_offsets_out || !data_lens_out)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  const size_t n = nslices, N = n * ag::kPipeShreds, cw_stride = ag::kPipeShreds * S;
  int st;
  // per-shred columns (payload rows straight into the codewords: row 64 s + j is shard j of slice s)
  uint8_t *kind, *slot, *sidx, *last, *shidx, *dlen, *sig, *proof, *height, *wire, *vstat, *roots;
  if ((st = pipe_buf(c, 0, N, &kind)) || (st = pipe_buf(c, 1, 8 * N, &slot)) || (st = pipe_buf(c, 2, 8 * N, &sidx)) ||
      (st = pipe_buf(c, 3, N, &last)) || (st = pipe_buf(c, 4, 4 * N, &shidx)) || (st = pipe_buf(c, 5, 4 * N, &dlen)) ||
      (st = pipe_buf(c, 6, 64 * N, &sig)) || (st = pipe_buf(c, 7, kPipeProofBytes * N, &proof)) ||
      (st = pipe_buf(c, 8, 4 * N, &height)) || (st = pipe_buf(c, 9, N, &wire)) || (st = pipe_buf(c, 10, N, &vstat)) ||
      (st = pipe_buf(c, 11, 32 * N, &roots)))
    return st;
  ag::ShredColumns cols{};
  cols.kind = kind;
  cols.slot = reinterpret_cast<uint64_t*>(slot);
  cols.slice_index = reinterpret_cast<uint64_t*>(sidx);
  cols.is_last = last;
  cols.shred_index = reinterpret_cast<uint32_t*>(shidx);
  cols.data = codewords;
  cols.data_stride = S;
  cols.data_len = reinterpret_cast<uint32_t*>(dlen);
  cols.sig = sig;
  cols.proof = proof;
  cols.proof_stride = kPipeProofBytes;
  cols.height = reinterpret_cast<uint32_t*>(height);
  // 1. network::deserialize (absent slots have length 0: malformed, never written)
  if (ag::launch_shred_deserialize(packets, packet_stride, packet_lens, N, cols, wire, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  // 2. ValidatedShred::try_new: one signature per slice (its first plausible shred) ...
  uint8_t *pick, *gdata, *gproof, *gslot, *gsidx, *glast, *gidx, *gsig, *pstat, *commits, *hasc;
  if ((st = pipe_buf(c, 12, n, &pick)) || (st = pipe_buf(c, 13, n * S, &gdata)) ||
      (st = pipe_buf(c, 14, kPipeProofBytes * n, &gproof)) || (st = pipe_buf(c, 15, 8 * n, &gslot)) ||
      (st = pipe_buf(c, 16, 8 * n, &gsidx)) || (st = pipe_buf(c, 17, n, &glast)) || (st = pipe_buf(c, 18, 4 * n, &gidx)) ||
      (st = pipe_buf(c, 19, 64 * n, &gsig)) || (st = pipe_buf(c, 20, n, &pstat)) ||
      (st = pipe_buf(c, 21, ag::kSliceCommitmentLen * n, &commits)) || (st = pipe_buf(c, 22, n, &hasc)))
    return st;
  uint8_t* plaus;  // per shred: the datagram parsed and fits its slot
  if ((st = pipe_buf(c, 24, N, &plaus))) return st;
  ag::PipePickParams pp{};
  pp.nslices = n;
  pp.shred_bytes = static_cast<uint32_t>(S);
  pp.num_data = ag::kPipeData;
  pp.wire_status = wire;
  pp.cols = cols;
  pp.pick = pick;
  pp.g_data = gdata;
  pp.g_proof = gproof;
  pp.g_slot = reinterpret_cast<uint64_t*>(gslot);
  pp.g_slice_index = reinterpret_cast<uint64_t*>(gsidx);
  pp.g_is_last = glast;
  pp.g_shred_index = reinterpret_cast<uint32_t*>(gidx);
  pp.g_sig = gsig;
  pp.plausible = plaus;
  AG_HIP(hipMemsetAsync(gdata, 0, n * S, c->stream));  // slices without a pick: defined bytes
  AG_HIP(hipMemsetAsync(gidx, 0, 4 * n, c->stream));
  if (ag::launch_pipe_pick(pp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // every plausible shred's root (derive_root, with its leaf digest for the Merkle rebuild's level
  // 0: step 5 hashes only the rows the coder restores or may rewrite) on the side stream: it needs
  // only the parse and the pick's plausibility flags, so it overlaps the picked shreds'
  // signature checks below (one signature per lane: a latency-bound kernel)
  const size_t nodes_stride = (32 * ag_merkle_node_count(ag::kPipeShreds) + 255) / 256 * 256;
  uint8_t* dlist;
  if ((st = c->d_merkle_nodes.ensure(n * nodes_stride, c->stream)) || (st = c->ensure_side_stream()) ||
      (st = pipe_buf(c, 26, 4 * (N + 1), &dlist)))
    return st;
  uint8_t* nodes = c->d_merkle_nodes.as<uint8_t>();
  {
    ag::MerkleVerifyParams mp{};
    mp.leaves = codewords;
    mp.leaf_stride = S;
    mp.leaf_bytes = static_cast<uint32_t>(S);
    mp.height = ag::kPipeHeight;
    mp.index = cols.shred_index;
    mp.proofs = proof;
    mp.proofs_stride = kPipeProofBytes;
    mp.n = N;
    mp.roots_out = roots;
    mp.active = plaus;
    mp.list = reinterpret_cast<uint32_t*>(dlist);
    mp.leaf_nodes = nodes;
    mp.leaf_nodes_stride = nodes_stride;
    mp.leaves_per_tree = ag::kPipeShreds;
    AG_HIP(hipEventRecord(c->side_fork, c->stream));
    AG_HIP(hipStreamWaitEvent(c->side, c->side_fork, 0));
    if (ag::launch_merkle_verify(mp, c->side) != hipSuccess) return AG_RS_ERR_DEVICE;
    AG_HIP(hipEventRecord(c->side_join, c->side));
  }
  if ((st = shred_validate_impl(c, n, gdata, S, S, pp.g_shred_index, gproof, kPipeProofBytes, ag::kPipeHeight,
                                pp.g_slot, pp.g_slice_index, glast, gsig, 64, pk, nullptr, nullptr, 1, nullptr, pstat,
                                nullptr, commits))) {
    (void)hipStreamSynchronize(c->side);
    return st;
  }
  if (ag::launch_pipe_cache_flags(pick, pstat, n, hasc, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  // ... then every shred against its slice's commitment (signature only without a cache)
  AG_HIP(hipStreamWaitEvent(c->stream, c->side_join, 0));
  if ((st = shred_validate_impl(c, N, codewords, S, S, cols.shred_index, proof, kPipeProofBytes, ag::kPipeHeight,
                                cols.slot, cols.slice_index, last, sig, 64, pk, commits, hasc, ag::kPipeShreds, plaus,
                                vstat, roots, nullptr, nodes, nodes_stride, ag::kPipeShreds, 0, 0, true)))
    return st;
  // 3. per slice: the shreds kept, the root, header and signature
  uint8_t* per_slice;
  if ((st = pipe_buf(c, 23, (8 + 8 + 8 + 32 + 32 + 64 + 8) * n, &per_slice))) return st;
  // 32-byte rows first: the Merkle build wants 16-byte aligned roots
  uint8_t* sroot = per_slice;
  uint8_t* roots2 = sroot + 32 * n;
  uint8_t* ssig = roots2 + 32 * n;
  uint64_t* d_present = reinterpret_cast<uint64_t*>(ssig + 64 * n);
  uint64_t* d_slot = d_present + n;
  uint8_t* ssidx = reinterpret_cast<uint8_t*>(d_slot + n);
  uint8_t* slast = ssidx + 8 * n;
  ag::PipeCheckParams kp{};
  kp.nslices = n;
  kp.shred_bytes = static_cast<uint32_t>(S);
  kp.num_data = ag::kPipeData;
  kp.wire_status = wire;
  kp.val_status = vstat;
  kp.roots = roots;
  kp.cols = cols;
  kp.present = d_present;
  kp.root = sroot;
  kp.slot = d_slot;
  kp.slice_index = reinterpret_cast<uint64_t*>(ssidx);
  kp.is_last = slast;
  kp.sig = ssig;
  if (ag::launch_pipe_check(kp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  PipeMeta hm;
  if ((st = read_pipe_meta(c, d_present, n, &hm))) return st;
  const uint64_t *h_present = hm.present, *h_slot = hm.slot, *h_sidx = hm.sidx;
  const uint8_t* h_last = hm.last;
  // 4. ReedSolomonCoder::deshred over the kept shreds (restores the data shreds, re-encodes
  //    all coding shreds, strips the padding); on the device for whole-chunk shreds
  std::vector<int64_t> plen(n);
  bool no_reencode = true;  // no surplus shreds and no slice with every data shred
  for (size_t s = 0; s < n && no_reencode; ++s)
    no_reencode = __builtin_popcountll(h_present[s]) <= static_cast<int>(ag::kPipeData) &&
                  (h_present[s] & 0xFFFFFFFFull) != 0xFFFFFFFFull;
  const bool device_coder = pipe_tail_ok(S, kDataShreds, no_reencode);
  if (device_coder) {
    if ((st = pipe_coder_deshred(c, n, S, codewords, cw_stride, d_present, plen.data(), kDataShreds, no_reencode)))
      return st;
  } else {
    std::vector<uint8_t> dp(n * ag::kPipeData), cp(n * (ag::kPipeShreds - ag::kPipeData));
    for (size_t s = 0; s < n; ++s)
      for (uint32_t j = 0; j < ag::kPipeShreds; ++j) {
        const uint8_t bit = static_cast<uint8_t>((h_present[s] >> j) & 1);
        if (j < ag::kPipeData) dp[s * ag::kPipeData + j] = bit;
        else cp[s * (ag::kPipeShreds - ag::kPipeData) + j - ag::kPipeData] = bit;
      }
    if ((st = ag_rs_coder_deshred_batch(c, ag::kPipeShreds - ag::kPipeData, n, S, codewords, cw_stride, dp.data(),
                                        cp.data(), AG_RS_DECODE_ANY_K, plen.data())))
      return st;
  }
  // 5. check_merkle_tree: the rebuilt tree's root must be the signed one; its paths serve
  //    the reconstructed datagrams.  Kept shreds the coder left as received reuse the digests
  //    their proof check computed (same bytes); restored rows, and coding rows the re-encode
  //    may have rewritten, are hashed again.
  //    Invariant the reuse depends on: present ⊆ active ∧ proof-ok.  Every kept
  //    shred (a bit of d_present, set by pipe_check only for shreds that were active in the
  //    step-3 verify and whose derived root matched) had its leaf digest written to
  //    d_merkle_nodes at (slice, index) by that verify; nothing between step 3 and here writes
  //    those rows of the codeword or those nodes (the coder stage touches only absent rows
  //    and, per the store masks, coding rows the leaf flags mark for re-hashing).  The verify
  //    also stores digests of rows it then rejects: those rows are not in d_present, so the
  //    flags below re-hash or ignore them.  A new step in between that writes kept rows or
  //    d_merkle_nodes must clear the matching present bits or re-hash.
  {
    uint8_t *lflags, *llist;
    if ((st = pipe_buf(c, 25, N, &lflags)) || (st = pipe_buf(c, 26, 4 * (N + 1), &llist)) ||
        (st = ensure_empty_roots(c)))
      return st;
    // the host coder path (shreds not whole 64-byte chunks) re-encodes every coding shred
    if (ag::launch_pipe_leaf_flags(d_present, n, !device_coder, lflags, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    ag::MerkleBuildParams mb{};
    mb.leaves = codewords;
    mb.leaf_stride = S;
    mb.slice_stride = cw_stride;
    mb.leaf_bytes = static_cast<uint32_t>(S);
    mb.n_leaves = ag::kPipeShreds;
    mb.nslices = n;
    mb.empty_roots = c->d_empty_roots.as<uint32_t>();
    mb.roots = roots2;
    mb.proofs = proof;
    mb.proofs_stride = ag::kPipeShreds * kPipeProofBytes;
    mb.hash_leaf = lflags;
    mb.list = reinterpret_cast<uint32_t*>(llist);
    if (ag::launch_merkle_build(mb, nodes, nodes_stride, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  }
  uint8_t* same = pstat;  // first validation's statuses are dead
  if (ag::launch_pipe_root_cmp(roots2, sroot, n, same, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  std::vector<uint8_t> h_same(n);
  AG_HIP(hipMemcpyAsync(h_same.data(), same, n, hipMemcpyDeviceToHost, c->stream));
  // 6. SlicePayload::try_from
  std::vector<uint8_t> sstat(n);
  if ((st = ag_slice_parse_batch(c, n, codewords, cw_stride, plen.data(), sstat.data(), parent_flags_out,
                                 parent_ids_out, data_offsets_out, data_lens_out)))
    return st;  // synchronous: h_same has landed
  // 6b. The crate's decoder reads every kept shred (reed_solomon.rs:154-166); the pass above
  //     reads 32 of them (ANY_K).  On a consistent slice both restore the same bytes (MDS), and
  //     a slice that passed check_merkle_tree is consistent: the rebuilt codeword matches the
  //     signed root that commits every kept shred.  A slice that failed the padding or the
  //     Merkle check with more than 32 kept shreds may hold an inconsistent shred the ANY_K
  //     pass did not read (a leader signing a non-codeword), and the crate's bytes -- hence
  //     the error, BadEncoding vs InvalidMerkleTree -- can differ.  Such slices are decoded
  //     again from their received bytes with EXACT and re-checked, one by one (honest
  //     leaders never produce them).
  for (size_t s = 0; s < n; ++s) {
    const bool failed = plen[s] == -AG_RS_ERR_INVALID_PADDING || (plen[s] >= 0 && !h_same[s]);
    if (!failed || __builtin_popcountll(h_present[s]) <= static_cast<int>(ag::kPipeData)) continue;
    if ((st = pipe_rerun_exact(c, s, S, packets, packet_stride, packet_lens, cols, wire, codewords, proof, roots2,
                               sroot, same, &plen[s], &h_same[s], &sstat[s], parent_flags_out + s,
                               parent_ids_out + AG_SLICE_BLOCK_ID_BYTES * s, data_offsets_out + s,
                               data_lens_out + s, h_present[s])))
      return st;
  }
  std::vector<uint8_t> ok(n);
  for (size_t s = 0; s < n; ++s) {
    int32_t r = AG_RS_OK;
    if (plen[s] < 0) {
      r = -plen[s] == AG_RS_ERR_INVALID_PADDING ? AG_RS_ERR_BAD_ENCODING : static_cast<int32_t>(-plen[s]);
    } else if (!h_same[s]) {
      r = AG_RS_ERR_INVALID_MERKLE_TREE;
    } else if (sstat[s] == AG_SLICE_TOO_LARGE) {
      r = AG_RS_ERR_TOO_MUCH_DATA;
    } else if (sstat[s] != AG_SLICE_OK) {
      r = AG_RS_ERR_BAD_ENCODING;
    }
    status[s] = r;
    ok[s] = r == AG_RS_OK;
    slots_out[s] = ok[s] ? h_slot[s] : 0;
    slice_indices_out[s] = ok[s] ? h_sidx[s] : 0;
    is_last_out[s] = ok[s] ? h_last[s] : 0;
  }
  // 7. fill_missing_shreds: datagrams for the absent slots of the slices that succeeded
  uint8_t *d_ok, *fresh;
  if ((st = pipe_buf(c, 20, n, &d_ok)) || (st = pipe_buf(c, 10, 4 * N, &fresh))) return st;
  AG_HIP(hipMemcpyAsync(d_ok, ok.data(), n, hipMemcpyHostToDevice, c->stream));
  ag::PipeExpandParams ep{};
  ep.nslices = n;
  ep.shred_bytes = static_cast<uint32_t>(S);
  ep.num_data = ag::kPipeData;
  ep.skip = d_present;
  ep.slice_ok = d_ok;
  ep.kind = kind;
  ep.shred_index = cols.shred_index;
  ep.data_len = cols.data_len;
  ep.height = cols.height;
  if (ag::launch_pipe_expand(ep, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  ag::ShredColumns fc = cols;
  fc.slot = d_slot;
  fc.slice_index = reinterpret_cast<uint64_t*>(ssidx);
  fc.is_last = slast;
  fc.sig = ssig;
  fc.hdr_group = ag::kPipeShreds;
  if (ag::launch_shred_serialize(fc, N, packets, packet_stride, reinterpret_cast<uint32_t*>(fresh), c->stream) !=
          hipSuccess ||
      ag::launch_pipe_merge_lens(reinterpret_cast<uint32_t*>(fresh), d_present, d_ok, n, packet_lens, c->stream) !=
          hipSuccess)
    return AG_RS_ERR_DEVICE;
  AG_HIP(hipStreamSynchronize(c->stream));  // host vectors read by async copies
  return AG_RS_OK;
}


// ---- the other three shredders of shredder.rs composed (CodingOnly, PETS, AONT) -------------
// (outside extern "C": helpers)
}  // extern "C"

namespace {
// Output shred j of a slice <-> codeword row (data rows 0..31, coding rows 32..32+m-1):
// Regular / AONT: j; CodingOnly: 32 + j (the 64 coding shreds, no data shreds: shredder.rs:
// 367-376); PETS: j for j < 31, j + 1 after (the data shred holding the key withheld,
// :414-422).  The pipeline addresses the output rows in the caller's codeword buffer itself
// (grouped_row_offset: base row row0, slice stride cw_stride, row `skip` and later one shard
// further), so no row is copied between the coder's layout and the datagrams'.
struct ShredderKind {
  uint32_t m;         // coding shreds of the coder (ReedSolomonCoder::new(CODING_OUTPUT_SHREDS))
  uint32_t num_data;  // DATA_OUTPUT_SHREDS
  int aon;            // AG_AON_* or -1
  uint32_t row0;      // codeword row of output shred 0
  uint32_t skip;      // output shreds >= skip sit one row further (0: none)
};
bool shredder_kind(int kind, ShredderKind* k) {
  switch (kind) {
    case AG_SHREDDER_CODING_ONLY: *k = {64, 0, -1, kDataShreds, 0}; return true;
    case AG_SHREDDER_PETS: *k = {33, 31, AG_AON_PETS, 0, 31}; return true;
    case AG_SHREDDER_AONT: *k = {32, 32, AG_AON_AONT, 0, 0}; return true;
    default: return false;
  }
}
uint32_t kind_row(const ShredderKind& k, uint32_t j) { return k.row0 + j + (k.skip && j >= k.skip ? 1u : 0u); }
// the Merkle tree over the 64 output rows of each slice: roots, proofs (nodes in context scratch)
int kind_merkle(ag_rs_ctx* c, const ShredderKind& k, size_t n, size_t S, const uint8_t* codewords, size_t cw_stride,
                uint8_t* roots, uint8_t* proofs) {
  const size_t nodes_stride = (32 * ag_merkle_node_count(ag::kPipeShreds) + 255) / 256 * 256;
  int st;
  if ((st = c->d_merkle_nodes.ensure(n * nodes_stride, c->stream)) || (st = ensure_empty_roots(c))) return st;
  ag::MerkleBuildParams mb{};
  mb.leaves = codewords + k.row0 * S;
  mb.leaf_stride = S;
  mb.slice_stride = cw_stride;
  mb.skip_leaf = k.skip;
  mb.leaf_bytes = static_cast<uint32_t>(S);
  mb.n_leaves = ag::kPipeShreds;
  mb.nslices = n;
  mb.empty_roots = c->d_empty_roots.as<uint32_t>();
  mb.roots = roots;
  mb.proofs = proofs;
  mb.proofs_stride = ag::kPipeShreds * kPipeProofBytes;
  return ag::launch_merkle_build(mb, c->d_merkle_nodes.as<uint8_t>(), nodes_stride, c->stream) == hipSuccess
             ? AG_RS_OK
             : AG_RS_ERR_DEVICE;
}
void kind_rows(const ShredderKind& k, uint8_t* codewords, size_t S, size_t cw_stride, ag::ShredColumns* cols) {
  cols->data = codewords + k.row0 * S;
  cols->data_stride = S;
  cols->group_stride = cw_stride;
  cols->skip_row = k.skip;
}
}  // namespace

extern "C" {

int ag_shredder_shred_batch_kind(ag_rs_ctx* c, int kind, size_t nslices, size_t S, const uint8_t* parent_flags,
                                 const uint8_t* parent_ids, const uint8_t* data, size_t data_stride,
                                 const uint32_t* data_lens, const uint64_t* slots, const uint64_t* slice_indices,
                                 const uint8_t* is_last, const uint8_t* seed, const uint8_t* pk, const uint8_t* keys,
                                 uint8_t* codewords, size_t cw_stride, uint8_t* roots_out, uint8_t* sigs_out,
                                 uint8_t* packets, size_t packet_stride, uint32_t* packet_lens) {
  if (kind == AG_SHREDDER_REGULAR) {
    if (cw_stride != ag::kPipeShreds * S) return AG_RS_ERR_INVALID_ARGUMENT;
    return ag_shredder_shred_batch(c, nslices, S, parent_flags, parent_ids, data, data_stride, data_lens, slots,
                                   slice_indices, is_last, seed, pk, codewords, roots_out, sigs_out, packets,
                                   packet_stride, packet_lens);
  }
  ShredderKind k;
  if (!c || !shredder_kind(kind, &k) || !pipe_args_ok(nslices, S, codewords, packets, packet_lens) ||
      cw_stride < (kDataShreds + k.m) * S || cw_stride % 4 ||
      (nslices && (!parent_flags || !parent_ids || !data_lens || !slots || !slice_indices || !is_last || !seed ||
                   !pk || (k.aon >= 0 && !keys))))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  const size_t n = nslices, N = n * ag::kPipeShreds;
  // MAX_DATA_SIZE: the key tail of PETS / AONT must fit the slice as well (shredder.rs:409, 457)
  const size_t extra = k.aon >= 0 ? ag::kCipherKeyBytes : 0;
  for (size_t b = 0; b < n; ++b) {
    const size_t framed = 1 + (parent_flags[b] ? AG_SLICE_BLOCK_ID_BYTES : 0) + 8 + size_t{data_lens[b]};
    if (framed + extra > kMaxPayload) return AG_RS_ERR_TOO_MUCH_DATA;
  }
  // 1. Slice::payload_bytes into the data regions; 2. PETS / AONT: encrypt_with_random_key with
  //    the caller's key + the key tail; 3. ReedSolomonCoder::shred in place
  std::vector<uint32_t> lens(n);
  int st = ag_slice_frame_batch(c, n, S, parent_flags, parent_ids, data, data_stride, data_lens, codewords, cw_stride,
                                lens.data());
  if (st) return st;
  if (k.aon >= 0) {
    if ((st = ag_aon_encrypt_batch(c, k.aon, n, keys, codewords, cw_stride, lens.data()))) return st;
    for (uint32_t& l : lens) l += static_cast<uint32_t>(ag::kCipherKeyBytes);
  }
  if ((st = ag_rs_coder_shred_batch(c, k.m, n, S, nullptr, 0, lens.data(), codewords, cw_stride))) return st;
  // 4. the 64 output shreds (data first) in place: Merkle tree, signature, datagrams over them
  uint8_t *roots = roots_out, *sigs = sigs_out, *proofs, *kcol, *sidx, *dlen, *height;
  if (!roots && (st = pipe_buf(c, 0, 32 * n, &roots))) return st;
  if (!sigs && (st = pipe_buf(c, 1, 64 * n, &sigs))) return st;
  if ((st = pipe_buf(c, 2, kPipeProofBytes * N, &proofs)) || (st = pipe_buf(c, 3, N, &kcol)) ||
      (st = pipe_buf(c, 4, 4 * N, &sidx)) || (st = pipe_buf(c, 5, 4 * N, &dlen)) ||
      (st = pipe_buf(c, 6, 4 * N, &height)))
    return st;
  if ((st = kind_merkle(c, k, n, S, codewords, cw_stride, roots, proofs))) return st;
  // 4b. signed on the side stream while 5 serializes the rest of the datagrams
  if ((st = sign_on_side(c, n, seed, pk, slots, slice_indices, is_last, roots, sigs))) return st;
  ag::PipeExpandParams ep{};
  ep.nslices = n;
  ep.shred_bytes = static_cast<uint32_t>(S);
  ep.num_data = k.num_data;
  ep.kind = kcol;
  ep.shred_index = reinterpret_cast<uint32_t*>(sidx);
  ep.data_len = reinterpret_cast<uint32_t*>(dlen);
  ep.height = reinterpret_cast<uint32_t*>(height);
  if (ag::launch_pipe_expand(ep, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
  ag::ShredColumns cols{};
  cols.kind = kcol;
  cols.slot = const_cast<uint64_t*>(slots);
  cols.slice_index = const_cast<uint64_t*>(slice_indices);
  cols.is_last = const_cast<uint8_t*>(is_last);
  cols.shred_index = ep.shred_index;
  kind_rows(k, codewords, S, cw_stride, &cols);
  cols.data_len = ep.data_len;
  cols.sig = sigs;
  cols.proof = proofs;
  cols.proof_stride = kPipeProofBytes;
  cols.height = ep.height;
  cols.hdr_group = ag::kPipeShreds;
  cols.skip_sig = 1;
  if (ag::launch_shred_serialize(cols, N, packets, packet_stride, packet_lens, c->stream) != hipSuccess) {
    (void)hipStreamSynchronize(c->side);
    return AG_RS_ERR_DEVICE;
  }
  AG_HIP(hipStreamWaitEvent(c->stream, c->side_join, 0));
  if (ag::launch_shred_sig_patch(cols, N, packets, packet_stride, packet_lens, c->stream) != hipSuccess)
    return AG_RS_ERR_DEVICE;
  return AG_RS_OK;
}

int ag_shredder_deshred_batch_kind(ag_rs_ctx* c, int kind, size_t nslices, size_t S, uint8_t* packets,
                                   size_t packet_stride, uint32_t* packet_lens, const uint8_t* pk, uint8_t* codewords,
                                   size_t cw_stride, int32_t* status, uint64_t* slots_out, uint64_t* slice_indices_out,
                                   uint8_t* is_last_out, uint8_t* parent_flags_out, uint8_t* parent_ids_out,
                                   uint32_t* data_offsets_out, uint32_t* data_lens_out) {
  if (kind == AG_SHREDDER_REGULAR) {
    if (cw_stride != ag::kPipeShreds * S) return AG_RS_ERR_INVALID_ARGUMENT;
    return ag_shredder_deshred_batch(c, nslices, S, packets, packet_stride, packet_lens, pk, codewords, status,
                                     slots_out, slice_indices_out, is_last_out, parent_flags_out, parent_ids_out,
                                     data_offsets_out, data_lens_out);
  }
  ShredderKind k;
  if (!c || !shredder_kind(kind, &k) || !pipe_args_ok(nslices, S, codewords, packets, packet_lens) ||
      cw_stride < (kDataShreds + k.m) * S || cw_stride % 4 ||
      (nslices && (!pk || !status || !slots_out || !slice_indices_out || !is_last_out || !parent_flags_out ||
                   !parent_ids_out || !data_offsets_out || !data_lens_out)))
    return AG_RS_ERR_INVALID_ARGUMENT;
  if (nslices == 0) return AG_RS_OK;
  if (c->enter()) return AG_RS_ERR_DEVICE;
  const size_t n = nslices, N = n * ag::kPipeShreds;
  int st;
  // per-shred columns; payloads parsed straight into their codeword rows
  uint8_t *kcol, *slot, *sidx, *last, *shidx, *dlen, *sig, *proof, *height, *wire, *vstat, *roots;
  if ((st = pipe_buf(c, 0, N, &kcol)) || (st = pipe_buf(c, 1, 8 * N, &slot)) ||
      (st = pipe_buf(c, 2, 8 * N, &sidx)) || (st = pipe_buf(c, 3, N, &last)) || (st = pipe_buf(c, 4, 4 * N, &shidx)) ||
      (st = pipe_buf(c, 5, 4 * N, &dlen)) || (st = pipe_buf(c, 6, 64 * N, &sig)) ||
      (st = pipe_buf(c, 7, kPipeProofBytes * N, &proof)) || (st = pipe_buf(c, 8, 4 * N, &height)) ||
      (st = pipe_buf(c, 9, N, &wire)) || (st = pipe_buf(c, 10, N, &vstat)) || (st = pipe_buf(c, 11, 32 * N, &roots)))
    return st;
  ag::ShredColumns cols{};
  cols.kind = kcol;
  cols.slot = reinterpret_cast<uint64_t*>(slot);
  cols.slice_index = reinterpret_cast<uint64_t*>(sidx);
  cols.is_last = last;
  cols.shred_index = reinterpret_cast<uint32_t*>(shidx);
  kind_rows(k, codewords, S, cw_stride, &cols);
  cols.data_len = reinterpret_cast<uint32_t*>(dlen);
  cols.sig = sig;
  cols.proof = proof;
  cols.proof_stride = kPipeProofBytes;
  cols.height = reinterpret_cast<uint32_t*>(height);
  // Pass 0 decodes with ANY_K on the device (per-slice window patterns, no host per-slice work);
  // a slice with surplus kept shreds that then fails some check could decode differently under
  // the crate's decoder over every kept shred, so the batch is redone with EXACT (pass 1).  A
  // slice that passes every check decoded the codeword its signed root commits, which every
  // kept shred matches: EXACT agrees there.  The packets' lengths change only
  // in step 7 (PETS / AONT serialize the absent datagrams before decrypting, into length-0 slots
  // that a redo parses as absent), so the redo starts from the same datagrams.
  const uint64_t *h_present = nullptr, *h_slot = nullptr, *h_sidx = nullptr;
  const uint8_t* h_last = nullptr;
  std::vector<uint8_t> ok(n), pre_ok(n);
  uint64_t* d_present = nullptr;
  uint8_t *sroot = nullptr, *ssig = nullptr, *ssidx = nullptr, *slast = nullptr, *fresh = nullptr;
  uint64_t* d_slot = nullptr;
  const bool fast_ok = pipe_tail_ok(S, k.m, true) && n > 1 && k.m >= kDataShreds && k.m <= 2 * kDataShreds;
  // 7. fill_missing_shreds (part 1): the absent datagrams of the slices in `okv`, lengths into
  // `fresh` (pipe_merge_lens moves the final slices' lengths into packet_lens)
  auto serialize_absent = [&](const std::vector<uint8_t>& okv) -> int {
    uint8_t* d_ok;
    int e;
    if ((e = pipe_buf(c, 20, n, &d_ok)) || (e = pipe_buf(c, 26, 4 * N, &fresh))) return e;
    AG_HIP(hipMemcpyAsync(d_ok, okv.data(), n, hipMemcpyHostToDevice, c->stream));
    ag::PipeExpandParams ep{};
    ep.nslices = n;
    ep.shred_bytes = static_cast<uint32_t>(S);
    ep.num_data = k.num_data;
    ep.skip = d_present;
    ep.slice_ok = d_ok;
    ep.kind = kcol;
    ep.shred_index = cols.shred_index;
    ep.data_len = cols.data_len;
    ep.height = cols.height;
    if (ag::launch_pipe_expand(ep, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    ag::ShredColumns fc = cols;
    fc.slot = d_slot;
    fc.slice_index = reinterpret_cast<uint64_t*>(ssidx);
    fc.is_last = slast;
    fc.sig = ssig;
    fc.hdr_group = ag::kPipeShreds;
    if (ag::launch_shred_serialize(fc, N, packets, packet_stride, reinterpret_cast<uint32_t*>(fresh), c->stream) !=
        hipSuccess)
      return AG_RS_ERR_DEVICE;
    // (okv is host memory the upload reads: the caller synchronizes before it changes)
    AG_HIP(hipStreamSynchronize(c->stream));
    return AG_RS_OK;
  };
  for (int pass = fast_ok ? 0 : 1; pass < 2; ++pass) {
    // 1. network::deserialize
    if (ag::launch_shred_deserialize(packets, packet_stride, packet_lens, N, cols, wire, c->stream) != hipSuccess)
      return AG_RS_ERR_DEVICE;
    // 2. ValidatedShred::try_new with the blockstore's cached commitment (the Regular pipeline's
    //    steps 2-3 with this shredder's data / coding layout)
    uint8_t *pick, *gdata, *gproof, *gslot, *gsidx, *glast, *gidx, *gsig, *pstat, *commits, *hasc, *plaus;
    if ((st = pipe_buf(c, 12, n, &pick)) || (st = pipe_buf(c, 13, n * S, &gdata)) ||
        (st = pipe_buf(c, 14, kPipeProofBytes * n, &gproof)) || (st = pipe_buf(c, 15, 8 * n, &gslot)) ||
        (st = pipe_buf(c, 16, 8 * n, &gsidx)) || (st = pipe_buf(c, 17, n, &glast)) || (st = pipe_buf(c, 18, 4 * n, &gidx)) ||
        (st = pipe_buf(c, 19, 64 * n, &gsig)) || (st = pipe_buf(c, 21, ag::kSliceCommitmentLen * n, &commits)) ||
        (st = pipe_buf(c, 22, n, &hasc)) || (st = pipe_buf(c, 24, N, &plaus)) || (st = pipe_buf(c, 27, n, &pstat)))
      return st;
    ag::PipePickParams pp{};
    pp.nslices = n;
    pp.shred_bytes = static_cast<uint32_t>(S);
    pp.num_data = k.num_data;
    pp.wire_status = wire;
    pp.cols = cols;
    pp.pick = pick;
    pp.g_data = gdata;
    pp.g_proof = gproof;
    pp.g_slot = reinterpret_cast<uint64_t*>(gslot);
    pp.g_slice_index = reinterpret_cast<uint64_t*>(gsidx);
    pp.g_is_last = glast;
    pp.g_shred_index = reinterpret_cast<uint32_t*>(gidx);
    pp.g_sig = gsig;
    pp.plausible = plaus;
    AG_HIP(hipMemsetAsync(gdata, 0, n * S, c->stream));
    AG_HIP(hipMemsetAsync(gidx, 0, 4 * n, c->stream));
    if (ag::launch_pipe_pick(pp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    // every plausible shred's root on the side stream, overlapping the picked shreds' signature
    // checks (as the Regular pipeline)
    uint8_t* dlist;
    if ((st = c->ensure_side_stream()) || (st = pipe_buf(c, 25, 4 * (N + 1), &dlist))) return st;
    {
      ag::MerkleVerifyParams mp{};
      mp.leaves = cols.data;
      mp.leaf_stride = S;
      mp.leaf_bytes = static_cast<uint32_t>(S);
      mp.height = ag::kPipeHeight;
      mp.index = cols.shred_index;
      mp.proofs = proof;
      mp.proofs_stride = kPipeProofBytes;
      mp.n = N;
      mp.roots_out = roots;
      mp.active = plaus;
      mp.list = reinterpret_cast<uint32_t*>(dlist);
      mp.group_stride = cw_stride;
      mp.skip_row = k.skip;
      AG_HIP(hipEventRecord(c->side_fork, c->stream));
      AG_HIP(hipStreamWaitEvent(c->side, c->side_fork, 0));
      if (ag::launch_merkle_verify(mp, c->side) != hipSuccess) return AG_RS_ERR_DEVICE;
      AG_HIP(hipEventRecord(c->side_join, c->side));
    }
    if ((st = shred_validate_impl(c, n, gdata, S, S, pp.g_shred_index, gproof, kPipeProofBytes, ag::kPipeHeight,
                                  pp.g_slot, pp.g_slice_index, glast, gsig, 64, pk, nullptr, nullptr, 1, nullptr, pstat,
                                  nullptr, commits))) {
      (void)hipStreamSynchronize(c->side);
      return st;
    }
    if (ag::launch_pipe_cache_flags(pick, pstat, n, hasc, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    AG_HIP(hipStreamWaitEvent(c->stream, c->side_join, 0));
    if ((st = shred_validate_impl(c, N, cols.data, S, S, cols.shred_index, proof, kPipeProofBytes, ag::kPipeHeight,
                                  cols.slot, cols.slice_index, last, sig, 64, pk, commits, hasc, ag::kPipeShreds, plaus,
                                  vstat, roots, nullptr, nullptr, 0, 0, cw_stride, k.skip, true)))
      return st;
    // 3. per slice: the shreds kept, the root, header and signature
    uint8_t* per_slice;
    if ((st = pipe_buf(c, 23, (8 + 8 + 8 + 32 + 32 + 64 + 8) * n, &per_slice))) return st;
    sroot = per_slice;
    uint8_t* roots2 = sroot + 32 * n;
    ssig = roots2 + 32 * n;
    d_present = reinterpret_cast<uint64_t*>(ssig + 64 * n);
    d_slot = d_present + n;
    ssidx = reinterpret_cast<uint8_t*>(d_slot + n);
    slast = ssidx + 8 * n;
    ag::PipeCheckParams kp{};
    kp.nslices = n;
    kp.shred_bytes = static_cast<uint32_t>(S);
    kp.num_data = k.num_data;
    kp.wire_status = wire;
    kp.val_status = vstat;
    kp.roots = roots;
    kp.cols = cols;
    kp.present = d_present;
    kp.root = sroot;
    kp.slot = d_slot;
    kp.slice_index = reinterpret_cast<uint64_t*>(ssidx);
    kp.is_last = slast;
    kp.sig = ssig;
    if (ag::launch_pipe_check(kp, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    PipeMeta hm;
    if ((st = read_pipe_meta(c, d_present, n, &hm))) return st;
    h_present = hm.present;
    h_slot = hm.slot;
    h_sidx = hm.sidx;
    h_last = hm.last;
    // 4. deshred_validated_shreds: ReedSolomonCoder::deshred over the kept shreds (in their
    //    codeword rows already), then decrypt_payload (PETS / AONT) after the raw shreds are
    //    taken.  Pass 0: ANY_K with the window patterns built on the device from the kept
    //    shreds' codeword-row words; pass 1: the crate's decoder over every kept shred (EXACT)
    std::vector<int64_t> plen(n);
    bool surplus = false;
    for (size_t s = 0; s < n; ++s) surplus |= __builtin_popcountll(h_present[s]) > static_cast<int>(kDataShreds);
    bool full_data = false;
    if (kind == AG_SHREDDER_AONT)
      for (size_t s = 0; s < n; ++s) full_data |= (h_present[s] & 0xFFFFFFFFull) == 0xFFFFFFFFull;
    if (pass == 0 && pipe_tail_ok(S, k.m, !surplus && !full_data)) {
      // codeword-row present words (pipe_coder_deshred: data | coding 0..31 << 32, coding
      // 32..63 in word 1 when m > 32); AONT's rows are the codeword rows
      const size_t wps = k.m > kDataShreds ? 2 : 1;
      const uint64_t* words = d_present;
      if (kind != AG_SHREDDER_AONT) {
        uint8_t* dw;
        if ((st = pipe_buf(c, 25, 8 * wps * n, &dw)) || (st = c->h_strip.ensure(8 * wps * n))) return st;
        uint64_t* hw = c->h_strip.as<uint64_t>();
        for (size_t s = 0; s < n; ++s) {
          const uint64_t o = h_present[s];
          if (kind == AG_SHREDDER_CODING_ONLY) {  // output j = coding j
            hw[2 * s] = (o & 0xFFFFFFFFull) << 32;
            hw[2 * s + 1] = o >> 32;
          } else {  // PETS: output j < 31 = data j, output 31 + i = coding i
            hw[2 * s] = (o & 0x7FFFFFFFull) | (((o >> 31) & 0xFFFFFFFFull) << 32);
            hw[2 * s + 1] = o >> 63;
          }
        }
        AG_HIP(hipMemcpyAsync(dw, hw, 8 * wps * n, hipMemcpyHostToDevice, c->stream));
        words = reinterpret_cast<const uint64_t*>(dw);
      }
      // (pipe_coder_deshred reads its results back through h_strip after the upload completed)
      if ((st = pipe_coder_deshred(c, n, S, codewords, cw_stride, words, plen.data(), k.m, !surplus && !full_data)))
        return st;
    } else {
      std::vector<uint8_t> dp(n * kDataShreds, 0), cp(n * k.m, 0);
      for (size_t s = 0; s < n; ++s)
        for (uint32_t j = 0; j < ag::kPipeShreds; ++j) {
          const uint32_t r = kind_row(k, j);
          const uint8_t bit = static_cast<uint8_t>((h_present[s] >> j) & 1);
          if (r < kDataShreds) dp[s * kDataShreds + r] = bit;
          else cp[s * k.m + (r - kDataShreds)] = bit;
        }
      if ((st = ag_rs_coder_deshred_batch(c, k.m, n, S, codewords, cw_stride, dp.data(), cp.data(), AG_RS_DECODE_EXACT,
                                          plen.data())))
        return st;
    }
    // AONT: the SHA-256 of every decoded ciphertext (decrypt_payload's key mask) runs on the side
    // stream, overlapping the Merkle rebuild, the root comparison and the absent datagrams'
    // serialization below (all of them only read the rows); one SHA-256 chain per slice leaves
    // most of the chip's issue slots to them
    bool sha_side = false;
    if (k.aon == AG_AON_AONT) {
      std::vector<uint32_t> shl(n);
      uint32_t mx = ag::kCipherKeyBytes;
      for (size_t s = 0; s < n; ++s) {
        shl[s] = plen[s] >= static_cast<int64_t>(ag::kCipherKeyBytes) ? static_cast<uint32_t>(plen[s])
                                                                      : static_cast<uint32_t>(ag::kCipherKeyBytes);
        mx = std::max(mx, shl[s]);
      }
      if ((st = c->ensure_side_stream()) || (st = c->d_aon_lens2.ensure(n * 4, c->stream)) ||
          (st = c->d_aon_digests.ensure(n * 32, c->stream)))
        return st;
      AG_HIP(hipStreamSynchronize(c->stream));
      AG_HIP(hipMemcpy(c->d_aon_lens2.ptr, shl.data(), n * 4, hipMemcpyHostToDevice));
      ag::BufferBatch sb;
      sb.base = codewords;
      sb.stride = cw_stride;
      sb.lens = c->d_aon_lens2.as<uint32_t>();
      sb.n = n;
      sb.max_len = mx;
      AG_HIP(hipEventRecord(c->side_fork, c->stream));
      AG_HIP(hipStreamWaitEvent(c->side, c->side_fork, 0));
      if (ag::launch_sha256(sb, ag::kCipherKeyBytes, c->d_aon_digests.as<uint8_t>(), c->side) != hipSuccess)
        return AG_RS_ERR_DEVICE;
      AG_HIP(hipEventRecord(c->side_join, c->side));
      sha_side = true;
    }
    // 5. check_merkle_tree over the raw output shreds (before any decryption: they are the
    //    codeword rows)
    if ((st = kind_merkle(c, k, n, S, codewords, cw_stride, roots2, proof))) return st;
    uint8_t* same = pstat;
    if (ag::launch_pipe_root_cmp(roots2, sroot, n, same, c->stream) != hipSuccess) return AG_RS_ERR_DEVICE;
    std::vector<uint8_t> h_same(n);
    AG_HIP(hipMemcpyAsync(h_same.data(), same, n, hipMemcpyDeviceToHost, c->stream));
    AG_HIP(hipStreamSynchronize(c->stream));
    if (k.aon >= 0) {
      // the absent datagrams of the slices that decoded and match their root, serialized from
      // the encrypted rows; then decrypt_payload (BadEncoding for a failed key check)
      for (size_t s = 0; s < n; ++s) pre_ok[s] = plen[s] >= 0 && h_same[s];
      if ((st = serialize_absent(pre_ok))) return st;
      std::vector<uint32_t> cl(n);
      for (size_t s = 0; s < n; ++s) cl[s] = pre_ok[s] ? static_cast<uint32_t>(plen[s]) : 0;
      std::vector<int64_t> pl(n);
      if (sha_side) {
        // decrypt_payload with the side stream's digests (ag_aon_decrypt_batch's key and
        // length rules; the digests of the slices decrypted here hash the same lengths)
        for (size_t s = 0; s < n; ++s) {
          pl[s] = cl[s] < ag::kCipherKeyBytes ? -AG_RS_ERR_BAD_ENCODING
                                              : static_cast<int64_t>(cl[s]) - ag::kCipherKeyBytes;
          if (cl[s] < ag::kCipherKeyBytes) cl[s] = ag::kCipherKeyBytes;  // no-op
        }
        ag::BufferBatch bb;
        if ((st = aon_batch(c, n, codewords, cw_stride, cl.data(), 0, &bb)) ||
            (st = c->d_aon_keys.ensure(n * 16, c->stream)))
          return st;
        AG_HIP(hipStreamWaitEvent(c->stream, c->side_join, 0));
        if (ag::launch_derive_keys(bb, 1, c->d_aon_digests.as<uint8_t>(), c->d_aon_keys.as<uint8_t>(), c->stream) !=
                hipSuccess ||
            ag::launch_apply_keystream(bb, c->d_aon_keys.as<uint8_t>(), ag::kCipherKeyBytes, c->stream) != hipSuccess)
          return AG_RS_ERR_DEVICE;
        AG_HIP(hipStreamSynchronize(c->stream));
      } else if ((st = ag_aon_decrypt_batch(c, k.aon, n, codewords, cw_stride, cl.data(), pl.data()))) {
        return st;
      }
      for (size_t s = 0; s < n; ++s)
        if (pre_ok[s]) plen[s] = pl[s];
    }
    // 6. SlicePayload::try_from on the (decrypted) payload
    std::vector<uint8_t> sstat(n);
    if ((st = ag_slice_parse_batch(c, n, codewords, cw_stride, plen.data(), sstat.data(), parent_flags_out,
                                   parent_ids_out, data_offsets_out, data_lens_out)))
      return st;
    bool redo = false;
    for (size_t s = 0; s < n; ++s) {
      int32_t r = AG_RS_OK;
      if (plen[s] < 0) {
        r = -plen[s] == AG_RS_ERR_INVALID_PADDING ? AG_RS_ERR_BAD_ENCODING : static_cast<int32_t>(-plen[s]);
      } else if (!h_same[s]) {
        r = AG_RS_ERR_INVALID_MERKLE_TREE;
      } else if (sstat[s] == AG_SLICE_TOO_LARGE) {
        r = AG_RS_ERR_TOO_MUCH_DATA;
      } else if (sstat[s] != AG_SLICE_OK) {
        r = AG_RS_ERR_BAD_ENCODING;
      }
      status[s] = r;
      ok[s] = r == AG_RS_OK;
      slots_out[s] = ok[s] ? h_slot[s] : 0;
      slice_indices_out[s] = ok[s] ? h_sidx[s] : 0;
      is_last_out[s] = ok[s] ? h_last[s] : 0;
      redo |= !ok[s] && __builtin_popcountll(h_present[s]) > static_cast<int>(kDataShreds);
    }
    if (!redo) break;
  }
  // 7. fill_missing_shreds: every absent slot of a successful slice gets its datagram
  if (k.aon < 0 && (st = serialize_absent(ok))) return st;
  uint8_t* d_ok;
  if ((st = pipe_buf(c, 20, n, &d_ok))) return st;
  AG_HIP(hipMemcpyAsync(d_ok, ok.data(), n, hipMemcpyHostToDevice, c->stream));
  if (ag::launch_pipe_merge_lens(reinterpret_cast<uint32_t*>(fresh), d_present, d_ok, n, packet_lens, c->stream) !=
      hipSuccess)
    return AG_RS_ERR_DEVICE;
  AG_HIP(hipStreamSynchronize(c->stream));
  return AG_RS_OK;
}

}  // extern "C"
