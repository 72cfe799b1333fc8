// Internal (C++) state of a libsdgpu context, shared by the C-ABI translation
// units (sdgpu.cpp: K1-K7 entry points; shard.cpp: Object index and the
// multi-GPU grouping).  Nothing here crosses the public boundary.
#pragma once

#include <errno.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/sdgpu.h"
#include "internal.hpp"

namespace sdgpu {

inline int map_err(hipError_t e) {
  switch (e) {
    case hipSuccess: return 0;
    case hipErrorOutOfMemory: return -ENOMEM;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice: return -ENODEV;
    case hipErrorInvalidValue: return -EINVAL;
    default: return -EIO;
  }
}

#define SD_TRY(expr)                       \
  do {                                     \
    const hipError_t e_ = (expr);          \
    if (e_ != hipSuccess) return map_err(e_); \
  } while (0)

#define SD_TRY_RC(expr)          \
  do {                           \
    const int rc_ = (expr);      \
    if (rc_ != 0) return rc_;    \
  } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
};

constexpr uint64_t kChunkLen = 1024;  // BLAKE3 chunk
constexpr size_t kSlabBytes = size_t(256) << 20;   // pinned staging per slab (max)
constexpr uint64_t kSlabMinBytes = uint64_t(16) << 20;  // smallest slab of a large call
constexpr uint32_t kSlabFiles = 1u << 16;          // files per slab
constexpr size_t kSliceBytes = size_t(64) << 20;   // file_checksum slice = 2^16 chunks
constexpr uint32_t kStageMaxMsg = 8u + (64u << 20);  // largest staged cas message
constexpr size_t kStageSlabBytes = size_t(256) << 20;  // sdgpu_cas_stage_pinned device slab
constexpr uint64_t kValidateBatchMax = uint64_t(16) << 20;  // larger files are streamed
constexpr uint32_t kSmallBatch = 64;  // up to this many messages take the latency kernel

// Brackets kernels with HIP events on their own stream; elapsed times are
// resolved (one sync per event pair) only when read.
struct EventTimer final : KTimer {
  struct Pending {
    std::string name;
    hipEvent_t a, b;
  };
  struct Acc {
    std::string name;
    double ms = 0;
    uint64_t n = 0;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  std::vector<Acc> acc;
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  std::vector<size_t> open;  // pending entries whose scope has not ended (scopes nest)
  void begin(const char* name, hipStream_t s) override {
    Pending p{name, get(), get()};
    (void)hipEventRecord(p.a, s);
    open.push_back(pending.size());
    pending.push_back(p);
  }
  void end(hipStream_t s) override {
    if (open.empty()) return;
    (void)hipEventRecord(pending[open.back()].b, s);
    open.pop_back();
  }
  void resolve() {
    for (auto& p : pending) {
      float ms = 0;
      (void)hipEventSynchronize(p.b);
      (void)hipEventElapsedTime(&ms, p.a, p.b);
      Acc* a = nullptr;
      for (auto& x : acc)
        if (x.name == p.name) a = &x;
      if (!a) {
        acc.push_back(Acc{p.name, 0, 0});
        a = &acc.back();
      }
      a->ms += ms;
      a->n += 1;
      pool.push_back(p.a);
      pool.push_back(p.b);
    }
    pending.clear();
    open.clear();
  }
  // a host-side phase (ms of wall time), reported beside the kernels
  void host(const char* name, double ms) {
    for (auto& x : acc)
      if (x.name == name) {
        x.ms += ms;
        x.n += 1;
        return;
      }
    acc.push_back(Acc{name, ms, 1});
  }
  ~EventTimer() override {
    resolve();
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace sdgpu

struct sdgpu_ctx {
  using DevBuf = sdgpu::DevBuf;
  using PinBuf = sdgpu::PinBuf;
  using EventTimer = sdgpu::EventTimer;
  using KTimer = sdgpu::KTimer;

  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t last = nullptr;
  std::mutex mu;
  DevBuf batch_ws, tree_ws, dedup_ws, shard_ws, io_a, io_b, link_ws, stage_meta;
  DevBuf small_ws;  // k_small_split's group CVs and per-message counters (zeroed once)
  DevBuf stage_slab[3];
  // host staging of the path / host-buffer entry points (identify_files,
  // cas_batch, generate_cas_id, checksum_files, file_checksum): pinned and
  // device slabs kept for the context's lifetime, grown on demand, so a call
  // pays no pinned allocation (a 256 MiB hipHostMalloc costs ~10^5 us)
  static constexpr int kPipeSlabs = 3;
  PinBuf pipe_h[kPipeSlabs];
  DevBuf pipe_d[kPipeSlabs];
  hipEvent_t pipe_evt[kPipeSlabs] = {};
  hipStream_t copy_stream = nullptr;  // H2D of staged slabs (SDMA), created on first use
  hipEvent_t stage_copied[3] = {}, stage_freed[3] = {};
  PinBuf plan_pin;
  hipEvent_t plan_evt = nullptr;
  bool plan_pending = false;
  // stream hand-over (pick): work issued on a new stream waits for the last one
  hipEvent_t handover = nullptr;
  // sharded grouping (shard.cpp): send records / positions / counts, received
  // records, their reps, the returned reps; host copies of the counts
  DevBuf xs_send, xs_recv, xs_back, xs_ret, xs_rback;
  PinBuf xs_counts;
  // padded exchange: two sets of 64 reservation cursors used alternately
  // (each call's k_pad_fill zeroes the other set for the next call), and the
  // keyless-row segments of the write set's partition
  DevBuf xs_cursor, xs_sink;
  // layout agreement messages (shard.cpp agree_layout): [2][W][3] int64
  DevBuf xs_agree;
  uint32_t xs_parity = 0;
  bool xs_cursor_clean = false;
  bool timing = false;
  bool io_uring = false;  // sdgpu_identify_files reads through io_uring (uring.hpp)
  bool io_bounce = true;   // ... or through a per-thread buffer, streamed into the slab
  EventTimer timer;
  KTimer* kt() { return timing ? &timer : nullptr; }
  // resident latency service (f3, sdgpu_latency_service): mailbox + message
  // area in coherent pinned memory, the kernel's own stream
  sdgpu::SvcMailbox* svc_mb = nullptr;
  uint8_t* svc_msg = nullptr;
  hipStream_t svc_stream = nullptr;
  bool svc_enabled = false, svc_launched = false;
  uint32_t svc_seq = 0;
  uint64_t svc_idle_ticks = 0, svc_life_ticks = 0;
  double svc_host_read_us = 0, svc_host_post_us = 0;  // last generate_cas_id (diag)
};

namespace sdgpu {

// The stream a call runs on (NULL = the context's own).  The context's device
// workspaces are shared by every call, so when a call moves to a different
// stream than the previous one it first waits (on the device) for the work
// already queued on that previous stream.
// Ends the resident latency kernel (if any) and waits for it: a bulk call
// gets every CU (K1's persistent grid is sized to the resident capacity).
inline void service_stop(sdgpu_ctx* c) {
  if (!c->svc_launched) return;
  __atomic_store_n(&c->svc_mb->op, kSvcStop, __ATOMIC_RELAXED);
  __atomic_store_n(&c->svc_mb->seq, ++c->svc_seq, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(c->svc_stream);
  c->svc_launched = false;
}

inline hipStream_t pick(sdgpu_ctx* c, void* stream) {
  service_stop(c);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  if (c->last && s != c->last) {
    if (!c->handover) (void)hipEventCreateWithFlags(&c->handover, hipEventDisableTiming);
    if (c->handover && hipEventRecord(c->handover, c->last) == hipSuccess)
      (void)hipStreamWaitEvent(s, c->handover, 0);
  }
  c->last = s;
  return s;
}

// Grow-only device buffer; frees the old one only after the context's work
// has drained (a kernel may still read it).
inline int ensure_dev(sdgpu_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return 0;
  if (b.p) {
    (void)hipStreamSynchronize(c->stream);
    if (c->last && c->last != c->stream) (void)hipStreamSynchronize(c->last);
    (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
  }
  const size_t want = align_up(std::max<size_t>(bytes, 1), size_t(1) << 20);
  SD_TRY(hipMalloc(&b.p, want));
  b.cap = want;
  // SDGPU_POISON_WS=1 (tests only): a new workspace is filled with 0xA5
  // bytes, so a kernel that reads a word no earlier kernel of the call wrote
  // sees garbage rather than a fresh allocation's zeros or the previous
  // call's values (round 6: the class of the SDGPU_SEG_GROUPS fault)
  static const bool poison = std::getenv("SDGPU_POISON_WS") && std::getenv("SDGPU_POISON_WS")[0] == '1';
  if (poison) SD_TRY(hipMemset(b.p, 0xA5, want));
  return 0;
}

// k_small_split's scratch: allocated and zeroed once per context (the kernel
// leaves its counters zero), nullptr on failure.
inline uint32_t* small_scratch(sdgpu_ctx* c, hipStream_t s) {
  if (!c->small_ws.p) {
    const size_t bytes = small_split_scratch_bytes();
    if (ensure_dev(c, c->small_ws, bytes) != 0) return nullptr;
    if (hipMemsetAsync(c->small_ws.p, 0, bytes, s) != hipSuccess) return nullptr;
  }
  return static_cast<uint32_t*>(c->small_ws.p);
}

// Grow-only device buffer that keeps its first `keep` bytes.
inline int grow_dev_keep(sdgpu_ctx* c, DevBuf& b, size_t bytes, size_t keep) {
  if (bytes <= b.cap) return 0;
  void* np = nullptr;
  const size_t want = align_up(std::max<size_t>(bytes, 2 * b.cap), size_t(1) << 20);
  SD_TRY(hipMalloc(&np, want));
  if (b.p) {
    SD_TRY(hipStreamSynchronize(c->stream));
    if (keep) SD_TRY(hipMemcpy(np, b.p, std::min(keep, b.cap), hipMemcpyDeviceToDevice));
    (void)hipFree(b.p);
  }
  b.p = np;
  b.cap = want;
  return 0;
}

inline int ensure_pin(PinBuf& b, size_t bytes) {
  if (bytes <= b.cap) return 0;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const size_t want = align_up(std::max<size_t>(bytes, 1), size_t(1) << 16);
  SD_TRY(hipHostMalloc(&b.p, want, hipHostMallocDefault));
  b.cap = want;
  return 0;
}

}  // namespace sdgpu
