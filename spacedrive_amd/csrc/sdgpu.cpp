// libsdgpu.so -- C ABI (include/sdgpu.h) over the gfx950 kernels.
//
// Host side of the MI355X content-identification path.  The reference host is
// Rust (sd-core); its toolchain is absent here, so the host logic that would sit
// in core/src/object/{cas.rs, validation/hash.rs, file_identifier/mod.rs} is
// written in C++ below the C ABI, and the Rust binding a maintainer adds is in
// INTEGRATION.md.
//
// Nothing here computes a hash on the CPU: every BLAKE3 compression runs in the
// HIP kernels (b3_batch.hip, b3_tree.hip).  The host only reads files, packs the
// cas messages into pinned memory and moves bytes.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <new>
#include <thread>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/sdgpu.h"
#include "ctx.hpp"
#include "host_io.hpp"
#include "uring.hpp"
#include "internal.hpp"
#include "scan_device.hpp"

using namespace sdgpu;
using sdgpu::hostio::parallel_for;
using sdgpu::hostio::pread_exact;
using sdgpu::hostio::read_cas_message;
using sdgpu::hostio::read_cas_message_bounce;
using sdgpu::hostio::read_whole;
using sdgpu::hostio::read_whole_fd;
using sdgpu::hostio::slab_layout;
using sdgpu::hostio::SlabLayout;
using sdgpu::hostio::to_hex;

namespace {

// Carves the K1 workspace for n messages / max_chunks chunks out of ctx->batch_ws.
int batch_work(sdgpu_ctx* c, uint32_t n, uint64_t max_chunks, BatchWork& w) {
  const size_t o_nch = 0;
  const size_t o_base = align_up(o_nch + 4ull * n, 256);
  const size_t o_sums = align_up(o_base + 4ull * (n + 1), 256);
  const size_t o_tot = align_up(o_sums + 4ull * (scan::tiles_for(n) + 1), 256);
  const size_t o_order = align_up(o_tot + 4, 256);
  const size_t n_hist = 2ull * 128 * 256;
  const size_t o_hist = align_up(o_order + 8ull * n, 256);
  const size_t o_hsum = align_up(o_hist + 4ull * (n_hist + 1), 256);
  const size_t o_grab = align_up(o_hsum + 4ull * (scan::tiles_for(n_hist) + 1), 256);
  const size_t o_map = align_up(o_grab + 4, 256);
  const size_t o_cvs = align_up(o_map + 4ull * max_chunks, 256);
  const size_t total = align_up(o_cvs + 32ull * max_chunks, 256);
  SD_TRY_RC(ensure_dev(c, c->batch_ws, total));
  uint8_t* b = static_cast<uint8_t*>(c->batch_ws.p);
  w.n_chunks = reinterpret_cast<uint32_t*>(b + o_nch);
  w.chunk_base = reinterpret_cast<uint32_t*>(b + o_base);
  w.block_sums = reinterpret_cast<uint32_t*>(b + o_sums);
  w.total = reinterpret_cast<uint32_t*>(b + o_tot);
  w.order = reinterpret_cast<uint32_t*>(b + o_order);
  w.hist = reinterpret_cast<uint32_t*>(b + o_hist);
  w.hist_sums = reinterpret_cast<uint32_t*>(b + o_hsum);
  w.grab = reinterpret_cast<uint32_t*>(b + o_grab);
  w.chunk_msg = reinterpret_cast<uint32_t*>(b + o_map);
  w.cvs = reinterpret_cast<uint32_t*>(b + o_cvs);
  w.max_chunks = max_chunks;
  return 0;
}

// Tree launch with the context's pinned plan scratch (waits for the previous
// plan copy before rewriting the scratch).
int tree_launch(sdgpu_ctx* c, const TreeSeg* segs, uint32_t nseg, bool cv_input, uint8_t* d_out,
                hipStream_t s) {
  SD_TRY_RC(ensure_dev(c, c->tree_ws, tree_workspace_bytes(segs, nseg, cv_input)));
  if (c->plan_pending) {
    SD_TRY(hipEventSynchronize(c->plan_evt));
    c->plan_pending = false;
  }
  SD_TRY_RC(ensure_pin(c->plan_pin, tree_plan_bytes(nseg)));
  SD_TRY(tree_hash_launch(segs, nseg, cv_input, d_out, c->tree_ws.p, c->plan_pin.p, s, c->kt()));
  SD_TRY(hipEventRecord(c->plan_evt, s));
  c->plan_pending = true;
  return 0;
}

int cas_grown_locked(sdgpu_ctx* c, const char* path, uint64_t size, uint8_t out8[8]);

// ---------------------------------------------------------------------------
// K1 staging pipeline: slabs of messages packed into pinned memory by a
// producer (the file reads, on the pool threads), H2D + K1 + D2H on the
// context stream, three slabs in rotation so the host fills slab k+1 while the
// GPU works on slab k.  The reads are the bound, so slabs are sized to about a
// sixth of the call's bytes (16-256 MiB): the device work left after the last
// read is one small slab, not half the input.
// ---------------------------------------------------------------------------

struct Slab {
  uint8_t* h = nullptr;  // pinned [arena | off | len | out | status]
  uint8_t* d = nullptr;  // same layout on the device
  hipEvent_t done = nullptr;
  bool busy = false;
  uint32_t first = 0, count = 0;
};

// Pinned + device staging slot k of the context (grown on demand, kept).  Only
// called when no work of the context is in flight.
int pipe_slot(sdgpu_ctx* c, int k, size_t bytes) {
  SD_TRY_RC(ensure_pin(c->pipe_h[k], bytes));
  SD_TRY_RC(ensure_dev(c, c->pipe_d[k], bytes));
  if (!c->pipe_evt[k]) SD_TRY(hipEventCreateWithFlags(&c->pipe_evt[k], hipEventDisableTiming));
  return 0;
}

// producer(i, dst, cap) -> message length (>= 0), or -errno, or 0x7fffffff
// meaning "no message for this file" (size 0).  est(i) = bytes to reserve.
// Slabs are sized for this call (at most kSlabBytes / kSlabFiles): a single
// file costs one ~60 KiB slab, not 256 MiB.
// fill_batch (optional): fill_batch(first, cnt, off, cap_end, hb, len, pst) fills
// a whole slab's messages at once (the io_uring reader) instead of produce().
template <typename Est, typename Produce, typename Finish, typename FillBatch = std::nullptr_t>
int run_pipeline(sdgpu_ctx* c, uint32_t n, Est&& est, Produce&& produce, Finish&& finish,
                 FillBatch&& fill_batch = nullptr) {
  (void)pick(c, nullptr);  // runs on the context stream, after earlier work on others
  constexpr int S = sdgpu_ctx::kPipeSlabs;
  uint64_t want = 0, biggest = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t e = align_up(est(i), 16);
    want += e;
    biggest = std::max(biggest, e);
  }
  // slab = a sixth of the call; SDGPU_SLAB_DIV / SDGPU_SLAB_TAPER (A/B of
  // config-1 staging, scripts/gpu_r4_slab_ab.sh) override the division and
  // switch the tail taper below on
  static const uint64_t div = [] {
    const char* e = getenv("SDGPU_SLAB_DIV");
    const unsigned long v = e ? strtoul(e, nullptr, 10) : 0;
    return v >= 2 && v <= 64 ? static_cast<uint64_t>(v) : uint64_t(6);
  }();
  static const bool taper = [] {
    const char* e = getenv("SDGPU_SLAB_TAPER");
    return e && e[0] == '1';
  }();
  const uint64_t target = want <= (kSlabMinBytes << 1) ? want : std::max(want / div, kSlabMinBytes);
  const SlabLayout L = slab_layout(
      static_cast<size_t>(std::clamp<uint64_t>(std::max(target, biggest), 4096, kSlabBytes)),
      std::clamp<uint32_t>(n, 1, kSlabFiles));
  Slab slabs[S];
  int rc = 0;
  for (int k = 0; k < S && rc == 0; ++k) {
    if ((rc = pipe_slot(c, k, L.total)) != 0) break;
    slabs[k].h = static_cast<uint8_t*>(c->pipe_h[k].p);
    slabs[k].d = static_cast<uint8_t*>(c->pipe_d[k].p);
    slabs[k].done = c->pipe_evt[k];
  }
  BatchWork w;
  if (rc == 0) rc = batch_work(c, L.files_cap, L.arena_cap / kChunkLen + L.files_cap, w);
  EventTimer* ht = c->timing ? &c->timer : nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms_since = [&](std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(now() - t0).count();
  };
  auto drain = [&](Slab& sl) -> int {
    if (!sl.busy) return 0;
    const auto t0 = now();
    if (hipEventSynchronize(sl.done) != hipSuccess) return -EIO;
    if (ht) ht->host("stage_wait", ms_since(t0));
    sl.busy = false;
    finish(sl.first, sl.count, reinterpret_cast<const uint8_t(*)[8]>(sl.h + L.out),
           reinterpret_cast<const int32_t*>(sl.h + L.status));
    return 0;
  };
  // Taper (off by default): the device work left after the last read is the
  // last slab's copy + hash, so the final slabs may shrink geometrically (half
  // of what is left, down to kTailBytes).  Round 3 measured a taper as a loss
  // (651 k -> 516 k files/s: per-slab planning and pool barriers); round 4's
  // guided pool grains reopened the question (A/B: DESIGN.md §8).
  constexpr uint64_t kTailBytes = 4ull << 20;
  uint64_t left = want;
  uint32_t i = 0, k = 0;
  while (rc == 0 && i < n) {
    Slab& sl = slabs[k % S];
    if ((rc = drain(sl)) != 0) break;
    const uint64_t cap_now =
        !taper || left >= 2 * L.arena_cap
            ? L.arena_cap
            : std::min<uint64_t>(L.arena_cap, std::max<uint64_t>(left / 2, kTailBytes));
    // assign files to this slab
    uint8_t* hb = sl.h;
    uint64_t* off = reinterpret_cast<uint64_t*>(hb + L.off);
    uint32_t* len = reinterpret_cast<uint32_t*>(hb + L.len);
    int32_t* pst = reinterpret_cast<int32_t*>(hb + L.status);
    sl.first = i;
    uint64_t pos = 0;
    uint32_t cnt = 0;
    while (i + cnt < n && cnt < L.files_cap) {
      const uint64_t need = align_up(est(i + cnt), 16);
      if (pos + need > cap_now && cnt > 0) break;
      off[cnt] = pos;
      pos += std::min<uint64_t>(need, L.arena_cap);
      left -= std::min<uint64_t>(need, left);
      ++cnt;
    }
    sl.count = cnt;
    // fill (pool threads): message bytes + per-file pre-status
    const auto t_fill = now();
    auto settle = [&](uint32_t j, int64_t r) {
      if (r >= 0 && r != 0x7fffffff) {
        len[j] = static_cast<uint32_t>(r);
        pst[j] = 0;
      } else {
        len[j] = 0;  // hashed as an empty message; status says why it is void
        pst[j] = r == 0x7fffffff ? 1 : static_cast<int32_t>(r);
      }
    };
    bool filled = false;
    if constexpr (!std::is_same_v<std::decay_t<FillBatch>, std::nullptr_t>)
      filled = fill_batch(sl.first, cnt, off, std::min<uint64_t>(pos, L.arena_cap), hb, settle);
    if (!filled)
      parallel_for(cnt, [&](uint32_t j) {
        const uint64_t cap =
            (j + 1 < cnt ? off[j + 1] : std::min<uint64_t>(pos, L.arena_cap)) - off[j];
        settle(j, produce(sl.first + j, hb + off[j], static_cast<size_t>(cap)));
      });
    if (ht) ht->host("stage_fill", ms_since(t_fill));
    // device: copy, hash, copy back.  A few messages of <= 1 MiB take the
    // one-launch latency kernel and one H2D copy of the whole slab prefix.
    hipStream_t s = c->stream;
    uint8_t* db = sl.d;
    uint32_t max_msg = 0;
    for (uint32_t j = 0; j < cnt; ++j) max_msg = std::max(max_msg, len[j]);
    const bool small = cnt <= kSmallBatch && max_msg <= SMALL_MAX_BYTES;
    const size_t prefix = L.len + 4ull * cnt;
    // a few cas messages (the single-file and small-batch callers): read from
    // the pinned slab and the ids written back into it by the kernel itself,
    // no copy commands
    const bool host1 = small && max_msg <= kHostStageMax;
    bool ok;
    if (host1) {
      ok = small_host_launch(hb, off, len, cnt, max_msg, 2, hb + L.out, s, c->kt()) == hipSuccess;
    } else if (small && prefix <= (size_t(8) << 20)) {
      ok = hipMemcpyAsync(db, hb, prefix, hipMemcpyHostToDevice, s) == hipSuccess;
    } else {
      ok = hipMemcpyAsync(db, hb, pos, hipMemcpyHostToDevice, s) == hipSuccess &&
           hipMemcpyAsync(db + L.off, hb + L.off, 8ull * cnt, hipMemcpyHostToDevice, s) ==
               hipSuccess &&
           hipMemcpyAsync(db + L.len, hb + L.len, 4ull * cnt, hipMemcpyHostToDevice, s) ==
               hipSuccess;
    }
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(db + L.off);
    const uint32_t* d_len = reinterpret_cast<const uint32_t*>(db + L.len);
    if (ok && !host1)
      ok = (small ? small_split_launch(db, d_off, d_len, cnt, kStageMaxMsg,
                                       max_msg <= kChunkLen ? 1u : (max_msg + kChunkLen - 1) / kChunkLen,
                                       2, db + L.out, nullptr, small_scratch(c, s), s, c->kt())
                  : batch_hash_launch(db, L.arena_cap, d_off, d_len, cnt, kStageMaxMsg, 2,
                                      db + L.out, nullptr, w, s, c->kt())) == hipSuccess;
    if (!ok ||
        (!host1 &&
         hipMemcpyAsync(hb + L.out, db + L.out, 8ull * cnt, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipEventRecord(sl.done, s) != hipSuccess) {
      rc = -EIO;
      break;
    }
    sl.busy = true;
    i += cnt;
    ++k;
  }
  for (auto& sl : slabs) {
    const int r2 = drain(sl);
    if (rc == 0) rc = r2;
  }
  (void)hipStreamSynchronize(c->stream);
  return rc;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================

extern "C" {

int sdgpu_abi_version(void) { return SDGPU_ABI_VERSION; }

const char* sdgpu_strerror(int rc) {
  if (rc == 0) return "success";
  if (rc == -EIO) return "HIP runtime error";
  if (rc == -ENODEV) return "no usable gfx950 device";
  return strerror(-rc);
}

int sdgpu_device_count(int* count) {
  if (!count) return -EINVAL;
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  *count = e == hipSuccess ? n : 0;
  return e == hipSuccess ? 0 : -ENODEV;
}

int sdgpu_open(int device, sdgpu_ctx** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -ENODEV;
  if (device < 0 || device >= n) return -ENODEV;
  hipDeviceProp_t prop;
  SD_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return -ENODEV;
  SD_TRY(hipSetDevice(device));
  sdgpu_ctx* c = new (std::nothrow) sdgpu_ctx;
  if (!c) return -ENOMEM;
  c->device = device;
  {  // staging reads of sdgpu_identify_files: pread into a per-thread buffer
     // streamed into the slab (default), pread straight into the slab
     // (SDGPU_IO=pread), or io_uring (SDGPU_IO=uring).  Config 1, one box,
     // 16 threads (scripts/exp/diag_config1.sh): fill 10.7-10.8 ms against
     // 12.9-14.8 ms for pread and 17.8 ms for io_uring.
    const char* io = getenv("SDGPU_IO");
    c->io_uring = io && strcmp(io, "uring") == 0;
    c->io_bounce = !io || (strcmp(io, "uring") != 0 && strcmp(io, "pread") != 0);
  }
  // A BLOCKING stream: callers that pass NULL (e.g. torch's legacy default
  // stream, whose handle is 0) get work ordered with the null stream both ways.
  if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess ||
      hipEventCreateWithFlags(&c->plan_evt, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return -EIO;
  }
  c->last = c->stream;
  *out = c;
  return 0;
}

int sdgpu_close(sdgpu_ctx* c) {
  if (!c) return -EINVAL;
  (void)hipSetDevice(c->device);
  service_stop(c);
  if (c->svc_stream) (void)hipStreamDestroy(c->svc_stream);
  if (c->svc_mb) (void)hipHostFree(c->svc_mb);
  (void)hipStreamSynchronize(c->stream);
  if (c->last && c->last != c->stream) (void)hipStreamSynchronize(c->last);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  for (DevBuf* b : {&c->batch_ws, &c->tree_ws, &c->dedup_ws, &c->shard_ws, &c->io_a, &c->io_b,
                    &c->link_ws, &c->stage_meta, &c->stage_slab[0], &c->stage_slab[1],
                    &c->stage_slab[2]})
    if (b->p) (void)hipFree(b->p);
  for (int k = 0; k < sdgpu_ctx::kPipeSlabs; ++k) {
    if (c->pipe_d[k].p) (void)hipFree(c->pipe_d[k].p);
    if (c->pipe_h[k].p) (void)hipHostFree(c->pipe_h[k].p);
    if (c->pipe_evt[k]) (void)hipEventDestroy(c->pipe_evt[k]);
  }
  for (int k = 0; k < 3; ++k) {
    if (c->stage_copied[k]) (void)hipEventDestroy(c->stage_copied[k]);
    if (c->stage_freed[k]) (void)hipEventDestroy(c->stage_freed[k]);
  }
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->plan_pin.p) (void)hipHostFree(c->plan_pin.p);
  for (DevBuf* b : {&c->xs_send, &c->xs_recv, &c->xs_back, &c->xs_ret, &c->xs_rback,
                    &c->xs_cursor, &c->xs_sink, &c->xs_agree})
    if (b->p) (void)hipFree(b->p);
  if (c->xs_counts.p) (void)hipHostFree(c->xs_counts.p);
  if (c->handover) (void)hipEventDestroy(c->handover);
  (void)hipEventDestroy(c->plan_evt);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int sdgpu_sync(sdgpu_ctx* c) {
  if (!c) return -EINVAL;
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(hipStreamSynchronize(c->stream));
  if (c->last && c->last != c->stream) SD_TRY(hipStreamSynchronize(c->last));
  return 0;
}

void* sdgpu_stream(sdgpu_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int sdgpu_alloc_pinned(sdgpu_ctx* c, size_t bytes, void** out) {
  if (!c || !out) return -EINVAL;
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
  return 0;
}

int sdgpu_free_pinned(sdgpu_ctx* c, void* p) {
  if (!c) return -EINVAL;
  SD_TRY(hipHostFree(p));
  return 0;
}

int sdgpu_alloc_device(sdgpu_ctx* c, size_t bytes, void** out) {
  if (!c || !out) return -EINVAL;
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(hipMalloc(out, std::max<size_t>(bytes, 1)));
  return 0;
}

int sdgpu_free_device(sdgpu_ctx* c, void* p) {
  if (!c) return -EINVAL;
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(hipFree(p));
  return 0;
}

int sdgpu_memcpy_async(sdgpu_ctx* c, void* dst, const void* src, size_t bytes, void* stream) {
  if (!c) return -EINVAL;
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, pick(c, stream)));
  return 0;
}

// ---- K1 ---------------------------------------------------------------------

int sdgpu_cas_batch_device(sdgpu_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes,
                           const uint64_t* d_off, const uint32_t* d_len, uint32_t n,
                           uint8_t* d_out8, int32_t* d_status, void* stream) {
  if (!c || (n && (!d_arena || !d_off || !d_len || !d_out8))) return -EINVAL;
  if (reinterpret_cast<uintptr_t>(d_arena) % 16 || reinterpret_cast<uintptr_t>(d_out8) % 4)
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  BatchWork w;
  SD_TRY_RC(batch_work(c, n, arena_bytes / kChunkLen + n, w));
  SD_TRY(batch_hash_launch(d_arena, arena_bytes, d_off, d_len, n, CAS_MAX_MSG_LEN, 2, d_out8,
                           d_status, w, s, c->kt()));
  return 0;
}

// Pinned-host staged K1 (config 5): slabs of the caller's pinned arena are
// copied H2D on the context's copy stream (SDMA) into a ring of three device
// slabs while K1 hashes the previous slab on the compute stream; events order
// copy k after the hash of slab k-3 and hash k after copy k.  No host packing:
// the arena is the pinned buffer the file reads landed in.
int sdgpu_cas_stage_pinned(sdgpu_ctx* c, const uint8_t* h_arena, const uint64_t* h_off,
                           const uint32_t* h_len, uint32_t n, uint8_t* d_out8, int32_t* d_status,
                           void* stream) {
  if (!c || (n && (!h_arena || !h_off || !h_len || !d_out8))) return -EINVAL;
  if (reinterpret_cast<uintptr_t>(h_arena) % 16 || reinterpret_cast<uintptr_t>(d_out8) % 4)
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  if (n == 0) return 0;
  // slab plan: consecutive files whose byte extent fits one slab
  struct Piece {
    uint32_t first, count;
    uint64_t base, bytes;
  };
  std::vector<Piece> pieces;
  uint64_t max_chunks = 0;
  uint32_t max_count = 0;
  {
    uint32_t i = 0;
    while (i < n) {
      if (i && h_off[i] < h_off[i - 1]) return -EINVAL;  // arena must be in file order
      const uint64_t base = h_off[i];
      uint64_t end = base;
      uint32_t j = i;
      while (j < n && j - i < kSlabFiles) {
        if (j > i && h_off[j] < h_off[j - 1]) return -EINVAL;
        const uint64_t ext = h_len[j] <= CAS_MAX_MSG_LEN ? h_len[j] : 0;  // invalid: not read
        const uint64_t e = std::max(end, h_off[j] + ext);
        if (e - base > kStageSlabBytes && j > i) break;
        end = e;
        ++j;
      }
      pieces.push_back(Piece{i, j - i, base, end - base});
      max_chunks = std::max<uint64_t>(max_chunks, (end - base) / kChunkLen + (j - i));
      max_count = std::max(max_count, j - i);
      i = j;
    }
  }
  // device copies of the file table, slabs, events, copy stream
  const size_t meta_off = align_up(8ull * n, 256);
  SD_TRY_RC(ensure_dev(c, c->stage_meta, meta_off + 4ull * n));
  uint64_t* d_off = static_cast<uint64_t*>(c->stage_meta.p);
  uint32_t* d_len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(c->stage_meta.p) + meta_off);
  SD_TRY(hipMemcpyAsync(d_off, h_off, 8ull * n, hipMemcpyHostToDevice, s));
  SD_TRY(hipMemcpyAsync(d_len, h_len, 4ull * n, hipMemcpyHostToDevice, s));
  if (!c->copy_stream) {
    SD_TRY(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int k = 0; k < 3; ++k) {
      SD_TRY(hipEventCreateWithFlags(&c->stage_copied[k], hipEventDisableTiming));
      SD_TRY(hipEventCreateWithFlags(&c->stage_freed[k], hipEventDisableTiming));
    }
  }
  for (int k = 0; k < 3; ++k) SD_TRY_RC(ensure_dev(c, c->stage_slab[k], kStageSlabBytes + 256));
  BatchWork w;
  SD_TRY_RC(batch_work(c, max_count, max_chunks, w));
  // the copy stream starts after everything issued on s so far (slab reuse
  // across calls, the file table copies above)
  SD_TRY(hipEventRecord(c->stage_freed[0], s));
  SD_TRY(hipStreamWaitEvent(c->copy_stream, c->stage_freed[0], 0));
  for (size_t k = 0; k < pieces.size(); ++k) {
    const Piece& pc = pieces[k];
    const int r = static_cast<int>(k % 3);
    uint8_t* slab = static_cast<uint8_t*>(c->stage_slab[r].p);
    if (k >= 3) SD_TRY(hipStreamWaitEvent(c->copy_stream, c->stage_freed[r], 0));
    SD_TRY(hipMemcpyAsync(slab, h_arena + pc.base, pc.bytes, hipMemcpyHostToDevice,
                          c->copy_stream));
    SD_TRY(hipEventRecord(c->stage_copied[r], c->copy_stream));
    SD_TRY(hipStreamWaitEvent(s, c->stage_copied[r], 0));
    // message i of the piece sits at slab + (off[i] - base): hand K1 an arena
    // origin of slab - base (16-B aligned: slab and off are)
    const uint8_t* origin = slab - pc.base;
    SD_TRY(batch_hash_launch(origin, pc.base + pc.bytes, d_off + pc.first, d_len + pc.first,
                             pc.count, CAS_MAX_MSG_LEN, 2, d_out8 + 8ull * pc.first,
                             d_status ? d_status + pc.first : nullptr, w, s, c->kt()));
    SD_TRY(hipEventRecord(c->stage_freed[r], s));
  }
  return 0;
}

int sdgpu_link_batch_device(sdgpu_ctx* c, const uint32_t* d_rep, const uint32_t* d_rank,
                            const uint8_t* d_valid, uint32_t first_rank, uint64_t n,
                            uint32_t* d_create, uint32_t* d_link_row, uint32_t* d_link_obj,
                            uint32_t* d_counts, void* stream) {
  if (!c || !d_counts || (n && (!d_rep || !d_create || !d_link_row || !d_link_obj)))
    return -EINVAL;
  if (n > 0xffffffffull) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY_RC(ensure_dev(c, c->link_ws, link_workspace_bytes(n)));
  SD_TRY(link_batch_launch(d_rep, d_rank, d_valid, first_rank, n, d_create, d_link_row,
                           d_link_obj, d_counts, c->link_ws.p, s, c->kt()));
  return 0;
}

int sdgpu_cas_batch(sdgpu_ctx* c, const uint8_t* msg_arena, const uint64_t* msg_off,
                    const uint32_t* msg_len, uint32_t n, uint8_t (*out8)[8], int32_t* status) {
  if (!c || (n && (!msg_arena || !msg_off || !msg_len || !out8))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  std::vector<uint8_t> bad(n, 0);
  for (uint32_t i = 0; i < n; ++i) bad[i] = msg_len[i] > CAS_MAX_MSG_LEN;
  const int rc = run_pipeline(
      c, n, [&](uint32_t i) -> uint64_t { return bad[i] ? 16 : msg_len[i]; },
      [&](uint32_t i, uint8_t* dst, size_t cap) -> int64_t {
        if (bad[i]) return -EINVAL;
        if (msg_len[i] > cap) return -ENOBUFS;
        memcpy(dst, msg_arena + msg_off[i], msg_len[i]);
        return msg_len[i];
      },
      [&](uint32_t first, uint32_t cnt, const uint8_t (*o)[8], const int32_t* st) {
        for (uint32_t j = 0; j < cnt; ++j) {
          const int32_t sj = st[j];
          if (sj == 0) memcpy(out8[first + j], o[j], 8);
          else memset(out8[first + j], 0, 8);
          if (status) status[first + j] = sj == 1 ? 0 : sj;
        }
      });
  return rc;
}

int sdgpu_identify_files(sdgpu_ctx* c, const char* const* paths, const uint64_t* size_in,
                         uint32_t n, uint8_t (*out8)[8], uint8_t* has_key, int32_t* status) {
  if (!c || (n && (!paths || !out8))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  // size NULL (ABI 6): the fresh fs::metadata(path).len() of the reference
  // (file_identifier/mod.rs:65,80-81), stat-ed here by the read pool; a path
  // whose stat fails gets status -errno and no key (the row is dropped,
  // mod.rs:113,127).  A directory gets -EISDIR (the reference asserts it is
  // not one, mod.rs:69-72), also when its st_size is 0 -- it is not an
  // empty file
  std::vector<uint64_t> fresh;
  std::vector<int32_t> stat_rc;
  if (!size_in && n) {
    fresh.assign(n, 0);
    stat_rc.assign(n, 0);
    parallel_for(n, [&](uint32_t i) {
      struct stat st;
      if (stat(paths[i], &st) != 0) stat_rc[i] = -errno;
      else if (S_ISDIR(st.st_mode)) stat_rc[i] = -EISDIR;
      else fresh[i] = static_cast<uint64_t>(st.st_size);
    });
  }
  const uint64_t* size = size_in ? size_in : fresh.data();
  auto failed = [&](uint32_t i) -> int32_t { return stat_rc.empty() ? 0 : stat_rc[i]; };
  std::vector<uint32_t> grown;  // <= 100 KiB at stat, longer than its room at read
  const int rc = run_pipeline(
      c, n,
      [&](uint32_t i) -> uint64_t {
        if (size[i] == 0 || failed(i)) return 16;
        return size[i] <= SDGPU_CAS_MINIMUM_FILE_SIZE ? 8 + size[i] + 4096  // room to grow
                                                      : SDGPU_CAS_SAMPLED_MSG_LEN;
      },
      [&](uint32_t i, uint8_t* dst, size_t cap) -> int64_t {
        if (failed(i)) return failed(i);
        if (size[i] == 0) return 0x7fffffff;  // cas_id None (file_identifier/mod.rs:80-88)
        if (c->io_bounce) return read_cas_message_bounce(paths[i], size[i], dst, cap);
        return read_cas_message(paths[i], size[i], dst, cap);
      },
      [&](uint32_t first, uint32_t cnt, const uint8_t (*o)[8], const int32_t* st) {
        for (uint32_t j = 0; j < cnt; ++j) {
          const int32_t sj = st[j];
          const bool ok = sj == 0;
          if (sj == -EFBIG) grown.push_back(first + j);
          if (ok) memcpy(out8[first + j], o[j], 8);
          else memset(out8[first + j], 0, 8);
          if (has_key) has_key[first + j] = ok ? 1 : 0;
          if (status) status[first + j] = sj == 1 ? 0 : sj;
        }
      },
      [&](uint32_t first, uint32_t cnt, const uint64_t* off, uint64_t end, uint8_t* hb,
          auto&& settle) -> bool {
        // batched io_uring chains (csrc/uring.hpp), one ring per pool thread:
        // the same bytes and statuses as read_cas_message
        if (!c->io_uring) return false;
        constexpr uint32_t kGrain = uring::kBatchFiles;
        parallel_for((cnt + kGrain - 1) / kGrain, [&](uint32_t g) {
          thread_local uring::Ring ring;
          thread_local int ring_ok = -1;
          if (ring_ok < 0) ring_ok = ring.open_ring() ? 1 : 0;
          const uint32_t j0 = g * kGrain, j1 = std::min(cnt, j0 + kGrain);
          uring::FileJob jobs[kGrain];
          uint32_t idx[kGrain], m = 0;
          for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t i = first + j;
            if (failed(i)) {
              settle(j, failed(i));
              continue;
            }
            if (size[i] == 0) {
              settle(j, 0x7fffffff);  // cas_id None (file_identifier/mod.rs:80-88)
              continue;
            }
            const uint64_t cap = (j + 1 < cnt ? off[j + 1] : end) - off[j];
            jobs[m] = uring::FileJob{paths[i], size[i], hb + off[j], static_cast<size_t>(cap), 0};
            idx[m++] = j;
          }
          if (ring_ok) {
            // false: the ring failed (the batch finished through pread or -EIO)
            // and was closed; this thread reads with pread from now on
            if (!uring::read_cas_batch(ring, jobs, m)) ring_ok = 0;
          } else
            for (uint32_t k = 0; k < m; ++k)
              jobs[k].result = read_cas_message(jobs[k].path, jobs[k].size, jobs[k].dst, jobs[k].cap);
          for (uint32_t k = 0; k < m; ++k) settle(idx[k], jobs[k].result);
        });
        return true;
      });
  if (rc) return rc;
  for (const uint32_t i : grown) {
    const int r = cas_grown_locked(c, paths[i], size[i], out8[i]);
    if (r) memset(out8[i], 0, 8);
    if (has_key) has_key[i] = r == 0 ? 1 : 0;
    if (status) status[i] = r;
  }
  return 0;
}

// ---- the resident latency service (f3) ----------------------------------------
//
// The single-file callers (watcher/utils.rs:236,411,467; non_indexed.rs:161)
// pay a launch and a stream synchronisation per call on the one-shot path.
// With the service enabled, a message of at most kHostStageMax bytes is read
// straight into the coherent message area and handed to a workgroup that
// stays resident (k_service), through a mailbox: the call is the file read, a
// few PCIe round trips and the hash itself.  The kernel ends itself after
// 20 ms without a request (and after 1 s in total); the next call relaunches
// it, and every other entry point stops it first (pick()).

namespace {

int service_open(sdgpu_ctx* c) {
  if (c->svc_mb) return 0;
  const size_t bytes = align_up(sizeof(SvcMailbox), 256) + kHostStageMax + 256;
  void* p = nullptr;
  SD_TRY(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped));
  memset(p, 0, bytes);
  if (hipStreamCreateWithFlags(&c->svc_stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipHostFree(p);
    return -EIO;
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess ||
      khz <= 0)
    khz = 100000;  // the 100 MHz constant clock of s_memrealtime
  c->svc_idle_ticks = 20ull * static_cast<uint64_t>(khz);     // 20 ms
  c->svc_life_ticks = 1000ull * static_cast<uint64_t>(khz);   // 1 s
  c->svc_mb = static_cast<SvcMailbox*>(p);
  c->svc_msg = static_cast<uint8_t*>(p) + align_up(sizeof(SvcMailbox), 256);
  c->svc_seq = 0;
  return 0;
}

int service_relaunch(sdgpu_ctx* c, uint32_t last_seq) {
  if (c->svc_launched) (void)hipStreamSynchronize(c->svc_stream);  // the old one has ended
  __atomic_store_n(&c->svc_mb->state, kSvcRunning, __ATOMIC_RELEASE);
  SD_TRY(service_launch(c->svc_mb, c->svc_msg, last_seq, c->svc_idle_ticks, c->svc_life_ticks,
                        c->svc_stream));
  c->svc_launched = true;
  return 0;
}

// Hashes the len-byte message at c->svc_msg; out_words digest words.  Context
// lock held.  -ETIMEDOUT (service disabled) if no answer within 2 s.
int service_hash(sdgpu_ctx* c, uint32_t len, uint32_t out_words, uint32_t* digest) {
  SvcMailbox* mb = c->svc_mb;
  if (!c->svc_launched || __atomic_load_n(&mb->state, __ATOMIC_ACQUIRE) == kSvcExited)
    SD_TRY_RC(service_relaunch(c, c->svc_seq));
  mb->op = kSvcHash;
  mb->len = len;
  mb->out_words = out_words;
  const uint32_t seq = ++c->svc_seq;
  __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(2);
  for (uint32_t spin = 0;; ++spin) {
    if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) break;
    if (__atomic_load_n(&mb->state, __ATOMIC_ACQUIRE) == kSvcExited) {
      // it timed out before it saw this request: a new one picks it up
      (void)hipStreamSynchronize(c->svc_stream);
      if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) break;
      SD_TRY_RC(service_relaunch(c, seq - 1));
      continue;
    }
    if ((spin & 1023u) == 0 && std::chrono::steady_clock::now() > deadline) {
      service_stop(c);
      c->svc_enabled = false;
      return -ETIMEDOUT;
    }
    __builtin_ia32_pause();
  }
  for (uint32_t w = 0; w < out_words; ++w) digest[w] = __atomic_load_n(&mb->digest[w], __ATOMIC_RELAXED);
  return 0;
}

}  // namespace

int sdgpu_latency_service_diag(sdgpu_ctx* c, double out_us[4]) {
  if (!c || !out_us) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->svc_mb) return -ENOENT;
  SvcMailbox* mb = c->svc_mb;
  const double tick_us = 1000.0 / static_cast<double>(c->svc_idle_ticks / 20);  // ticks per ms
  const uint64_t a = __atomic_load_n(&mb->t_seen, __ATOMIC_RELAXED);
  const uint64_t b = __atomic_load_n(&mb->t_loaded, __ATOMIC_RELAXED);
  const uint64_t d = __atomic_load_n(&mb->t_done, __ATOMIC_RELAXED);
  out_us[0] = static_cast<double>(b - a) * tick_us;  // message copied into LDS
  out_us[1] = static_cast<double>(d - b) * tick_us;  // hashed, digest written
  out_us[2] = c->svc_host_post_us;                   // host: read + post -> answer seen
  out_us[3] = c->svc_host_read_us;                   // host: the file read
  return 0;
}

int sdgpu_latency_service(sdgpu_ctx* c, int enable) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  if (!enable) {
    service_stop(c);
    c->svc_enabled = false;
    return 0;
  }
  SD_TRY_RC(service_open(c));
  c->svc_enabled = true;
  return 0;
}

int sdgpu_generate_cas_id(sdgpu_ctx* c, const char* path, uint64_t size, char out_hex[17]) {
  if (!c || !path || !out_hex) return -EINVAL;
  uint8_t out[8];
  int32_t st = 0;
  // the single-file call keeps the reference's semantics for size 0 too
  // (non_indexed.rs:161 hashes the 8 zero bytes of an empty file)
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  if (c->svc_enabled) {
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t r = read_cas_message(path, size, c->svc_msg, kHostStageMax);
    const auto t1 = std::chrono::steady_clock::now();
    if (r < 0 && r != -EFBIG) return static_cast<int>(r);
    if (r >= 0) {
      uint32_t d[2];
      const int rc = service_hash(c, static_cast<uint32_t>(r), 2, d);
      c->svc_host_read_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
      c->svc_host_post_us =
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
      if (rc == 0) {
        memcpy(out, d, 8);
        to_hex(out, 8, out_hex);
        return 0;
      }
      if (rc != -ETIMEDOUT) return rc;
    }
    // grew past the message area since stat, or the service timed out: the
    // one-shot path below (which re-reads the file)
  }
  const int rc = run_pipeline(
      c, 1,
      [&](uint32_t) -> uint64_t {
        return size <= SDGPU_CAS_MINIMUM_FILE_SIZE ? 8 + size + 4096 : SDGPU_CAS_SAMPLED_MSG_LEN;
      },
      [&](uint32_t, uint8_t* dst, size_t cap) -> int64_t {
        return read_cas_message(path, size, dst, cap);
      },
      [&](uint32_t, uint32_t, const uint8_t (*o)[8], const int32_t* s) {
        st = s[0];
        memcpy(out, o[0], 8);
      });
  if (rc) return rc;
  if (st == -EFBIG) st = cas_grown_locked(c, path, size, out);  // grew since stat
  if (st) return st;
  to_hex(out, 8, out_hex);
  return 0;
}

// ---- K2/K3 ------------------------------------------------------------------

int sdgpu_checksum_batch_device(sdgpu_ctx* c, const uint8_t* const* d_files, const uint64_t* lens,
                                uint32_t n, uint8_t* d_out32, void* stream) {
  if (!c || (n && (!d_files || !lens || !d_out32))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  std::vector<TreeSeg> segs(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (reinterpret_cast<uintptr_t>(d_files[i]) % 16) return -EINVAL;
    segs[i] = TreeSeg{d_files[i], lens[i], 0, 1, 0};
  }
  return tree_launch(c, segs.data(), n, false, d_out32, s);
}

int sdgpu_subtree_device(sdgpu_ctx* c, const uint8_t* d_bytes, uint64_t len, uint64_t chunk_offset,
                         int root, uint8_t* d_out32, void* stream) {
  if (!c || !d_bytes || !d_out32 || reinterpret_cast<uintptr_t>(d_bytes) % 16) return -EINVAL;
  if (root && chunk_offset != 0) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  const TreeSeg seg{d_bytes, len, chunk_offset, root ? 1u : 0u, 0};
  return tree_launch(c, &seg, 1, false, d_out32, s);
}

int sdgpu_combine_subtrees_device(sdgpu_ctx* c, const uint8_t* d_cvs, uint64_t n, uint8_t* d_out32,
                                  void* stream) {
  if (!c || !d_cvs || !d_out32 || n < 2 || reinterpret_cast<uintptr_t>(d_cvs) % 16) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  // the slices' CVs are the leaves of the tree's top levels (file_checksum's
  // slice fold, hash.rs:10-24 as one message)
  const TreeSeg seg{d_cvs, n, 0, 1u, 0};
  return tree_launch(c, &seg, 1, true, d_out32, s);
}

namespace {

// BLAKE3 of a host buffer through the tree kernels (context lock held).
int checksum_host_locked(sdgpu_ctx* c, const void* bytes, uint64_t len, uint8_t out32[32]) {
  hipStream_t s = pick(c, nullptr);
  SD_TRY_RC(ensure_dev(c, c->io_a, align_up(len, 256) + 256));
  uint8_t* d = static_cast<uint8_t*>(c->io_a.p);
  if (len) SD_TRY(hipMemcpyAsync(d, bytes, len, hipMemcpyHostToDevice, s));
  uint8_t* dout = d + align_up(len, 256);
  const TreeSeg seg{d, len, 0, 1, 0};
  SD_TRY_RC(tree_launch(c, &seg, 1, false, dout, s));
  SD_TRY(hipMemcpyAsync(out32, dout, 32, hipMemcpyDeviceToHost, s));
  SD_TRY(hipStreamSynchronize(s));
  return 0;
}

// cas_id of a file that was <= 100 KiB at stat time but longer than its slab
// reservation at read time: fs::read takes whatever the file holds then
// (cas.rs:27-29), so the message is u64 size LE || the whole current content,
// of any length; hashed by the tree kernels.  out8 = BLAKE3(M)[0..8).
int cas_grown_locked(sdgpu_ctx* c, const char* path, uint64_t size, uint8_t out8[8]) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  std::vector<uint8_t> msg(8);
  for (int i = 0; i < 8; ++i) msg[i] = static_cast<uint8_t>(size >> (8 * i));
  int rc = 0;
  for (;;) {
    const size_t at = msg.size();
    msg.resize(at + (size_t(1) << 20));
    const ssize_t r = read(fd, msg.data() + at, size_t(1) << 20);
    if (r < 0 && errno == EINTR) {
      msg.resize(at);
      continue;
    }
    msg.resize(at + (r > 0 ? static_cast<size_t>(r) : 0));
    if (r < 0) rc = -errno;
    if (r <= 0) break;
  }
  close(fd);
  if (rc) return rc;
  uint8_t d[32];
  SD_TRY_RC(checksum_host_locked(c, msg.data(), msg.size(), d));
  memcpy(out8, d, 8);
  return 0;
}

}  // namespace

int sdgpu_checksum(sdgpu_ctx* c, const void* bytes, uint64_t len, uint8_t out32[32]) {
  if (!c || (len && !bytes) || !out32) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  return checksum_host_locked(c, bytes, len, out32);
}

namespace {

// file_checksum of one file, streamed in slices (context lock held).
int file_checksum_locked(sdgpu_ctx* c, const char* path, uint8_t digest[32]) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  // the stream (pick: which also stops the resident service) only once the
  // service path is not taken
  hipStream_t s = c->svc_enabled ? nullptr : pick(c, nullptr);
  // two pinned + two device slices; slice k's subtree CV lands in cvs[k]
  PinBuf* hp = c->pipe_h;  // the context's two staging slots
  int rc = 0;
  uint64_t nslices = 0;
  uint64_t total = 0;
  hipEvent_t* ev = c->pipe_evt;
  bool inflight[2] = {false, false};
  bool root_done = false;  // the digest was launched directly (single slice)
  std::vector<uint8_t> out(32);
  do {
    struct stat st;
    if (c->svc_enabled && fstat(fd, &st) == 0 && static_cast<uint64_t>(st.st_size) <= kHostStageMax) {
      // resident service: the whole file read into the coherent message area
      const int64_t got = read_whole_fd(fd, c->svc_msg, kHostStageMax);
      if (got >= 0) {
        uint32_t d[8];
        rc = service_hash(c, static_cast<uint32_t>(got), 8, d);
        if (rc == 0) {
          memcpy(out.data(), d, 32);
          break;
        }
        if (rc != -ETIMEDOUT) break;
        rc = 0;
      } else if (got != -EFBIG) {
        rc = static_cast<int>(got);
        break;
      }
      if (lseek(fd, 0, SEEK_SET) < 0) {  // grew, or the service timed out: one-shot path
        rc = -errno;
        break;
      }
    }
    if (!s) s = pick(c, nullptr);
    if (fstat(fd, &st) == 0 && static_cast<uint64_t>(st.st_size) <= SMALL_MAX_BYTES) {
      // latency path: the whole file in one read and one launch (the
      // reference's 1 MiB read loop, hash.rs:14-20, ends on the short read)
      const size_t cap = SMALL_MAX_BYTES;  // room for growth up to 1 MiB
      if ((rc = pipe_slot(c, 0, cap + 256))) break;
      uint8_t* hb = static_cast<uint8_t*>(hp[0].p);
      const int64_t got = read_whole_fd(fd, hb, cap);
      if (got >= 0) {
        const uint32_t nch = got <= 1024 ? 1u : static_cast<uint32_t>((got + 1023) / 1024);
        // the whole file hashed from the pinned buffer, digest written back
        // into it by the kernel: no copy commands (<= 112 KiB: one workgroup;
        // above: 64 KiB groups on as many workgroups, k_small_split)
        uint8_t* hout = hb + cap + 64;
        uint64_t* hoff = reinterpret_cast<uint64_t*>(hb + cap + 128);  // {0}, then the length
        hoff[0] = 0;
        hoff[1] = static_cast<uint64_t>(got);
        const uint32_t* hlen = reinterpret_cast<const uint32_t*>(hoff + 1);
        hipError_t e;
        if (static_cast<uint64_t>(got) <= kHostStageMax)
          e = small_host_launch(hb, hoff, hlen, 1, static_cast<uint32_t>(got), 8, hout, s, c->kt());
        else
          e = small_split_launch(hb, hoff, hlen, 1, SMALL_MAX_BYTES, nch, 8, hout, nullptr,
                                 small_scratch(c, s), s, c->kt());
        if (e != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
          rc = -EIO;
        else
          memcpy(out.data(), hout, 32);
        break;
      }
      if (got != -EFBIG) {
        rc = static_cast<int>(got);
        break;
      }
      if (lseek(fd, 0, SEEK_SET) < 0) {  // grew past 1 MiB since fstat: stream it
        rc = -errno;
        break;
      }
    }
    if ((rc = pipe_slot(c, 0, kSliceBytes)) || (rc = pipe_slot(c, 1, kSliceBytes))) break;
    if (fstat(fd, &st) == 0 && st.st_size > 0 &&
        (rc = grow_dev_keep(c, c->io_b, 32 * (static_cast<uint64_t>(st.st_size) / kSliceBytes + 2) + 256, 0)))
      break;
    if ((rc = ensure_dev(c, c->io_a, 2 * kSliceBytes + 4096))) break;
    uint8_t* dslice[2] = {static_cast<uint8_t*>(c->io_a.p),
                          static_cast<uint8_t*>(c->io_a.p) + kSliceBytes};
    uint8_t* droot = static_cast<uint8_t*>(c->io_a.p) + 2 * kSliceBytes;
    // CV list lives in io_b, grown as slices arrive
    bool eof = false;
    while (!eof) {
      const int k = static_cast<int>(nslices & 1);
      if (inflight[k]) {
        if (hipEventSynchronize(ev[k]) != hipSuccess) { rc = -EIO; break; }
        inflight[k] = false;
      }
      // file_checksum reads BLOCK_LEN = 1 MiB at a time until a short read
      // (hash.rs:14-20); a slice is 64 such reads.
      uint8_t* hb = static_cast<uint8_t*>(hp[k].p);
      size_t got = 0;
      while (got < kSliceBytes) {
        const ssize_t r = read(fd, hb + got, kSliceBytes - got);
        if (r < 0) {
          if (errno == EINTR) continue;
          rc = -errno;
          break;
        }
        if (r == 0) {
          eof = true;
          break;
        }
        got += static_cast<size_t>(r);
      }
      if (rc) break;
      if (got == 0 && nslices > 0) break;  // previous slice ended exactly at EOF
      // peek whether more data follows (to know if this slice is the last)
      if (!eof) {
        uint8_t probe;
        ssize_t r;
        do {
          r = pread(fd, &probe, 1, static_cast<off_t>(total + got));
        } while (r < 0 && errno == EINTR);
        if (r < 0) {
          rc = -errno;
          break;
        }
        if (r == 0) eof = true;
      }
      const bool only = eof && nslices == 0;
      root_done = only;
      if ((rc = grow_dev_keep(c, c->io_b, 32 * (nslices + 1) + 256, 32 * nslices))) break;
      uint8_t* cvs = static_cast<uint8_t*>(c->io_b.p);
      if (got && hipMemcpyAsync(dslice[k], hb, got, hipMemcpyHostToDevice, s) != hipSuccess) {
        rc = -EIO;
        break;
      }
      const TreeSeg seg{dslice[k], got, (total / kChunkLen), only ? 1u : 0u, 0};
      if ((rc = tree_launch(c, &seg, 1, false, only ? droot : cvs + 32 * nslices, s))) break;
      if (hipEventRecord(ev[k], s) != hipSuccess) { rc = -EIO; break; }
      inflight[k] = true;
      total += got;
      ++nslices;
    }
    if (rc) break;
    if (nslices > 1) {
      // fold the slice CVs (equal aligned power-of-two subtrees, last partial)
      const TreeSeg seg{static_cast<uint8_t*>(c->io_b.p), nslices, 0, 1, 0};
      if ((rc = tree_launch(c, &seg, 1, true, droot, s))) break;
    } else if (!root_done) {
      // the probe saw more data but the file was truncated before the next
      // read: the only slice (still in dslice[0]) is the whole message
      const TreeSeg seg{dslice[0], total, 0, 1, 0};
      if ((rc = tree_launch(c, &seg, 1, false, droot, s))) break;
    }
    if (hipMemcpyAsync(out.data(), droot, 32, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = -EIO;
  } while (false);
  if (s) (void)hipStreamSynchronize(s);
  close(fd);
  if (rc) return rc;
  memcpy(digest, out.data(), 32);
  return 0;
}

}  // namespace

int sdgpu_file_checksum(sdgpu_ctx* c, const char* path, char out_hex[65]) {
  if (!c || !path || !out_hex) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  uint8_t d[32];
  SD_TRY_RC(file_checksum_locked(c, path, d));
  to_hex(d, 32, out_hex);
  return 0;
}

// Batched object validator (validator_job.rs:126-169 runs file_checksum one
// file per step): files up to kValidateBatchMax are read whole by a thread
// pool into pinned slabs; each slab is hashed by ONE tree launch (a segment
// per file, K2/K3) while the next slab is read.  Larger files -- and files
// that grew past their reserved room -- take the streamed single-file path.
int sdgpu_checksum_files(sdgpu_ctx* c, const char* const* paths, uint32_t n, uint8_t (*out32)[32],
                         int32_t* status) {
  if (!c || (n && (!paths || !out32))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, nullptr);
  std::vector<int64_t> size(n);
  parallel_for(n, [&](uint32_t i) {
    struct stat st;
    if (stat(paths[i], &st) != 0) size[i] = -errno;
    else if (S_ISDIR(st.st_mode)) size[i] = -EISDIR;
    else size[i] = st.st_size;
  });
  std::vector<int32_t> st(n, 0);
  std::vector<uint8_t> deferred(n, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (size[i] < 0) st[i] = static_cast<int32_t>(size[i]);
    else if (static_cast<uint64_t>(size[i]) > kValidateBatchMax) deferred[i] = 1;
  }
  struct VSlab {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    hipEvent_t done = nullptr;
    bool busy = false;
    std::vector<uint32_t> files;
  };
  // [arena | digests], the arena sized for this call's batched files
  uint64_t want = 0;
  for (uint32_t j = 0; j < n && want < kSlabBytes; ++j)
    if (st[j] == 0 && !deferred[j]) want += align_up(static_cast<uint64_t>(size[j]) + 4096, 256);
  const uint64_t arena_cap = std::clamp<uint64_t>(want, 4096, kSlabBytes);
  const size_t out_off = align_up(arena_cap, 256);
  const size_t slab_total = out_off + 32ull * kSlabFiles;
  VSlab slabs[2];
  int rc = 0;
  for (int k = 0; k < 2 && rc == 0; ++k) {
    if ((rc = pipe_slot(c, k, slab_total)) != 0) break;
    slabs[k].h = static_cast<uint8_t*>(c->pipe_h[k].p);
    slabs[k].d = static_cast<uint8_t*>(c->pipe_d[k].p);
    slabs[k].done = c->pipe_evt[k];
  }
  auto drain = [&](VSlab& sl) -> int {
    if (!sl.busy) return 0;
    if (hipEventSynchronize(sl.done) != hipSuccess) return -EIO;
    sl.busy = false;
    const uint8_t* dg = sl.h + out_off;
    for (size_t j = 0; j < sl.files.size(); ++j) memcpy(out32[sl.files[j]], dg + 32 * j, 32);
    return 0;
  };
  uint32_t i = 0, k = 0;
  std::vector<uint64_t> off, cap;
  std::vector<int64_t> got;
  while (rc == 0) {
    while (i < n && (st[i] != 0 || deferred[i])) ++i;
    if (i >= n) break;
    VSlab& sl = slabs[k & 1];
    if ((rc = drain(sl)) != 0) break;
    sl.files.clear();
    off.clear();
    cap.clear();
    uint64_t pos = 0;
    for (; i < n && sl.files.size() < kSlabFiles; ++i) {
      if (st[i] != 0 || deferred[i]) continue;
      const uint64_t room = align_up(static_cast<uint64_t>(size[i]) + 4096, 256);
      if (pos + room > arena_cap) break;
      sl.files.push_back(i);
      off.push_back(pos);
      cap.push_back(room);
      pos += room;
    }
    const uint32_t cnt = static_cast<uint32_t>(sl.files.size());
    got.assign(cnt, 0);
    uint8_t* hb = sl.h;
    parallel_for(cnt, [&](uint32_t j) {
      got[j] = read_whole(paths[sl.files[j]], hb + off[j], static_cast<size_t>(cap[j]));
    });
    uint8_t* db = sl.d;
    std::vector<TreeSeg> segs;
    std::vector<uint32_t> kept;
    segs.reserve(cnt);
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint32_t f = sl.files[j];
      if (got[j] == -EFBIG) {
        deferred[f] = 1;  // grew since stat: stream it
        continue;
      }
      if (got[j] < 0) {
        st[f] = static_cast<int32_t>(got[j]);
        continue;
      }
      segs.push_back(TreeSeg{db + off[j], static_cast<uint64_t>(got[j]), 0, 1, 0});
      kept.push_back(f);
    }
    sl.files = kept;
    if (segs.empty()) continue;
    if (hipMemcpyAsync(db, hb, pos, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = -EIO;
      break;
    }
    if ((rc = tree_launch(c, segs.data(), static_cast<uint32_t>(segs.size()), false, db + out_off,
                          s)) != 0)
      break;
    if (hipMemcpyAsync(hb + out_off, db + out_off, 32 * segs.size(), hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipEventRecord(sl.done, s) != hipSuccess) {
      rc = -EIO;
      break;
    }
    sl.busy = true;
    ++k;
  }
  for (auto& sl : slabs) {
    const int r2 = drain(sl);
    if (rc == 0) rc = r2;
  }
  (void)hipStreamSynchronize(s);
  if (rc) return rc;
  for (uint32_t j = 0; j < n; ++j)
    if (deferred[j] && st[j] == 0) st[j] = file_checksum_locked(c, paths[j], out32[j]);
  for (uint32_t j = 0; j < n; ++j) {
    if (st[j] != 0) memset(out32[j], 0, 32);
    if (status) status[j] = st[j];
  }
  return 0;
}

// ---- K4-K6 ------------------------------------------------------------------

int sdgpu_group_pairs_device(sdgpu_ctx* c, const uint64_t* d_key, const uint32_t* d_rank,
                             uint64_t n, uint32_t chunk_rows, uint32_t skip_bits, uint32_t* d_rep,
                             void* stream) {
  if (!c || chunk_rows == 0 || skip_bits > 32 || (n && (!d_key || !d_rank || !d_rep)))
    return -EINVAL;
  if (n >= (1ull << 32)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  if (n == 0) return 0;
  SD_TRY_RC(ensure_dev(c, c->dedup_ws, dedup_workspace_bytes(n)));
  GroupInput in;
  in.key = d_key;
  in.rank = d_rank;
  in.n = n;
  SD_TRY(dedup_local_launch(in, chunk_rows, d_rep, true, c->dedup_ws.p, s, c->kt()));
  return 0;
}

int sdgpu_group_rows_device(sdgpu_ctx* c, const uint64_t* d_key, const uint8_t* d_has_key,
                            const uint32_t* d_rank, uint64_t n, uint32_t chunk_rows,
                            uint32_t skip_bits, uint32_t* d_rep, void* stream) {
  if (!c || chunk_rows == 0 || skip_bits > 32 || (n && (!d_key || !d_rep))) return -EINVAL;
  if (n >= (1ull << 32)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  if (n == 0) return 0;
  SD_TRY_RC(ensure_dev(c, c->dedup_ws, dedup_workspace_bytes(n)));
  GroupInput in;
  in.key = d_key;
  in.valid = d_has_key;
  in.rank = d_rank;
  in.n = n;
  SD_TRY(dedup_local_launch(in, chunk_rows, d_rep, true, c->dedup_ws.p, s, c->kt()));
  return 0;
}

int sdgpu_shard_count_device(sdgpu_ctx* c, const uint64_t* d_key, const uint8_t* d_has_key,
                             uint64_t n, uint32_t shard_bits, uint64_t* h_counts, void* stream) {
  if (!c || !h_counts || shard_bits > 8 || (n && !d_key) || n >= (1ull << 32)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  const size_t ws = shard_workspace_bytes(shard_bits);
  SD_TRY_RC(ensure_dev(c, c->shard_ws, ws));
  uint8_t* w = static_cast<uint8_t*>(c->shard_ws.p);
  uint64_t* dcounts = reinterpret_cast<uint64_t*>(w + ws - align_up(8ull << shard_bits, 256));
  SD_TRY(shard_count_launch(d_key, d_has_key, n, shard_bits, dcounts, w, s));
  SD_TRY(hipMemcpyAsync(h_counts, dcounts, 8ull << shard_bits, hipMemcpyDeviceToHost, s));
  SD_TRY(hipStreamSynchronize(s));
  return 0;
}

int sdgpu_shard_partition_device(sdgpu_ctx* c, const uint64_t* d_key, const uint8_t* d_has_key,
                                 const uint32_t* d_rank, uint64_t n, uint32_t shard_bits,
                                 uint64_t* d_out_key, uint32_t* d_out_rank, uint32_t* d_out_pos,
                                 void* stream) {
  if (!c || shard_bits > 8 || (n && (!d_key || !d_out_key || !d_out_rank || !d_out_pos)) ||
      n >= (1ull << 32))
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY_RC(ensure_dev(c, c->shard_ws, shard_workspace_bytes(shard_bits)));
  SD_TRY(shard_partition_launch(d_key, d_has_key, d_rank, n, shard_bits, d_out_key, d_out_rank,
                                d_out_pos, c->shard_ws.p, s, c->kt()));
  return 0;
}

int sdgpu_shard_exchange_device(sdgpu_ctx* c, const uint64_t* d_key, const uint8_t* d_has_key,
                                const uint32_t* d_rank, uint64_t n, uint32_t shard_bits,
                                uint32_t world, uint64_t* d_out_key, uint32_t* d_out_rank,
                                uint32_t* d_out_pos, int64_t* d_dest_counts, void* stream) {
  if (!c || shard_bits == 0 || shard_bits > 8 || world == 0 || world > 64 ||
      world > (1u << shard_bits) || !d_dest_counts || n >= (1ull << 32) ||
      (n && (!d_key || !d_out_key || !d_out_rank || !d_out_pos)))
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY_RC(ensure_dev(c, c->shard_ws, shard_workspace_bytes(shard_bits)));
  SD_TRY(shard_exchange_launch(d_key, d_has_key, d_rank, n, shard_bits, world, d_out_key,
                               d_out_rank, nullptr, d_out_pos, d_dest_counts, c->shard_ws.p, s,
                               c->kt()));
  return 0;
}

int sdgpu_scatter_rep_device(sdgpu_ctx* c, const uint32_t* d_src, const uint32_t* d_pos,
                             uint64_t n, uint32_t* d_dst, uint64_t n_dst, const uint32_t* d_init,
                             int init, void* stream) {
  if (!c || (n && (!d_src || !d_pos)) || ((n || init) && !d_dst)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(scatter_rep_launch(d_src, d_pos, n, d_dst, n_dst, d_init, init != 0, pick(c, stream)));
  return 0;
}

int sdgpu_dedup(sdgpu_ctx* c, const uint64_t* key, const uint8_t* has_key, uint32_t n,
                uint32_t chunk_rows, uint32_t* rep) {
  if (!c || chunk_rows == 0 || (n && (!key || !has_key || !rep))) return -EINVAL;
  if (n == 0) return 0;
  uint8_t* d = nullptr;
  int rc = 0;
  {
    std::lock_guard<std::mutex> g(c->mu);
    SD_TRY(hipSetDevice(c->device));
  }
  // [key n*8 | has n | rep n*4]
  const size_t o_key = 0, o_has = align_up(8ull * n, 256), o_rep = align_up(o_has + n, 256);
  const size_t total = align_up(o_rep + 4ull * n, 256);
  if (hipMalloc(&d, total) != hipSuccess) return -ENOMEM;
  hipStream_t s = c->stream;
  do {
    if (hipMemcpyAsync(d + o_key, key, 8ull * n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d + o_has, has_key, n, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = -EIO;
      break;
    }
    const uint64_t* dk = reinterpret_cast<const uint64_t*>(d + o_key);
    uint32_t* drep = reinterpret_cast<uint32_t*>(d + o_rep);
    if ((rc = sdgpu_group_rows_device(c, dk, d + o_has, nullptr, n, chunk_rows, 0, drep, s)))
      break;
    if (hipMemcpyAsync(rep, drep, 4ull * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = -EIO;
  } while (false);
  (void)hipStreamSynchronize(s);
  (void)hipFree(d);
  return rc;
}

// ---- synthetic corpora -------------------------------------------------------

int sdgpu_synth_cas_arena_device(sdgpu_ctx* c, const uint64_t* d_sizes, const uint64_t* d_seeds,
                                 const uint64_t* d_off, uint32_t n, uint8_t* d_arena, void* stream) {
  if (!c || (n && (!d_sizes || !d_seeds || !d_off || !d_arena))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(synth_cas_arena_launch(d_sizes, d_seeds, d_off, n, d_arena, pick(c, stream)));
  return 0;
}

int sdgpu_synth_file_device(sdgpu_ctx* c, uint64_t seed, uint64_t offset, uint64_t len,
                            uint8_t* d_out, void* stream) {
  if (!c || (len && !d_out) || offset % 8 || reinterpret_cast<uintptr_t>(d_out) % 16)
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(synth_file_launch(seed, offset, len, d_out, pick(c, stream)));
  return 0;
}

// ---- downstream consumers --------------------------------------------------------

int sdgpu_orphan_objects_device(sdgpu_ctx* c, const int32_t* d_object_ids, uint64_t n_objects,
                                const int32_t* d_fp_object_ids, uint64_t n_file_paths,
                                uint32_t max_object_id, int32_t* d_orphans, uint32_t* d_count,
                                void* stream) {
  if (!c || !d_count || (n_objects && (!d_object_ids || !d_orphans)) ||
      (n_file_paths && !d_fp_object_ids) || max_object_id > 0x7FFFFFFFu)
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY_RC(ensure_dev(c, c->link_ws, orphan_workspace_bytes(n_objects, max_object_id)));
  SD_TRY(orphan_objects_launch(d_object_ids, n_objects, d_fp_object_ids, n_file_paths,
                               max_object_id, d_orphans, d_count, c->link_ws.p, s));
  return 0;
}

int sdgpu_thumbnail_shards_device(sdgpu_ctx* c, const uint8_t* d_cas8, const uint8_t* d_valid,
                                  uint64_t n, uint32_t* d_order, uint32_t* d_counts,
                                  void* stream) {
  if (!c || !d_counts || (n && (!d_cas8 || !d_order)) || n >= (1ull << 32)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY_RC(ensure_dev(c, c->link_ws, thumb_workspace_bytes()));
  SD_TRY(thumbnail_shards_launch(d_cas8, d_valid, n, d_order, d_counts, c->link_ws.p, s));
  return 0;
}

int sdgpu_synth_vary_keys_device(sdgpu_ctx* c, uint64_t* d_key, const uint8_t* d_vary,
                                 uint64_t n, uint64_t step, void* stream) {
  if (!c || (n && (!d_key || !d_vary))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(vary_keys_launch(d_key, d_vary, n, step, pick(c, stream)));
  return 0;
}

// ---- instrumentation -----------------------------------------------------------

int sdgpu_set_timing(sdgpu_ctx* c, int enable) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->timing = enable != 0;
  return 0;
}

int sdgpu_timing_reset(sdgpu_ctx* c) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->timer.resolve();
  c->timer.acc.clear();
  return 0;
}

int sdgpu_timing_read(sdgpu_ctx* c, uint32_t idx, char name[32], double* total_ms,
                      uint64_t* launches) {
  if (!c || !name || !total_ms || !launches) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  c->timer.resolve();
  if (idx >= c->timer.acc.size()) return -ENOENT;
  const auto& a = c->timer.acc[idx];
  snprintf(name, 32, "%s", a.name.c_str());
  *total_ms = a.ms;
  *launches = a.n;
  return 0;
}

int sdgpu_valu_probe(sdgpu_ctx* c, double* lane_ops_per_s) {
  return sdgpu_valu_probe_kind(c, 0, lane_ops_per_s);
}

int sdgpu_valu_probe_kind(sdgpu_ctx* c, int kind, double* lane_ops_per_s) {
  if (!c || !lane_ops_per_s || kind < 0 || kind > 5) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY_RC(ensure_dev(c, c->io_b, 1 << 20));
  hipEvent_t a, b;
  SD_TRY(hipEventCreate(&a));
  SD_TRY(hipEventCreate(&b));
  // kind 5 (register-only compressions): 16 waves per CU, 2000 compressions each
  const uint32_t iters = kind == 5 ? 2000 : 4096, blocks = kind == 5 ? 256 * 16 : 256 * 8 * 4;
  uint32_t* sink = static_cast<uint32_t*>(c->io_b.p);
  SD_TRY(valu_probe_launch(kind, sink, 64, blocks, c->stream));  // warm
  SD_TRY(hipEventRecord(a, c->stream));
  SD_TRY(valu_probe_launch(kind, sink, iters, blocks, c->stream));
  SD_TRY(hipEventRecord(b, c->stream));
  SD_TRY(hipEventSynchronize(b));
  float ms = 0;
  SD_TRY(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  // kind 5: 680 VALU per compression; others: per iteration per chain add3,
  // xor, alignbit, add3, xor, alignbit = 6 VALU (kinds 1-4: 6 of one class)
  const double ops = kind == 5 ? double(iters) * 680 * blocks * 256
                               : double(iters) * 8 * 6 * blocks * 256;
  *lane_ops_per_s = ops / (ms * 1e-3);
  return 0;
}

int sdgpu_synth_dedup_rows_device(sdgpu_ctx* c, uint64_t seed, uint64_t total_rows,
                                  uint64_t distinct, uint64_t first_rank, uint64_t n,
                                  uint64_t* d_key, uint8_t* d_has_key, uint32_t* d_rank,
                                  void* stream) {
  if (!c || distinct == 0 || distinct > total_rows || first_rank + n > total_rows ||
      total_rows >= (1ull << 32) || (n && (!d_key || !d_has_key || !d_rank)))
    return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  SD_TRY(synth_dedup_rows_launch(seed, total_rows, distinct, first_rank, n, d_key, d_has_key,
                                 d_rank, pick(c, stream)));
  return 0;
}

}  // extern "C"
