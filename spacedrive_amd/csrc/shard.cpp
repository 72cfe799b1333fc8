// Multi-GPU cas_id -> Object grouping behind the C ABI, and the Object index.
//
// Reference: identifier_job_step's grouping (core/src/object/file_identifier/
// mod.rs:136-333) -- here one library-wide grouping of all rows, hash-sharded
// over the GPUs of a node: every key has exactly one owner
// GPU, so the per-owner grouping is complete and independent; the chunk rule
// needs only the global rank, which travels with the key.
//
// One exchange step per call, on each GPU:
//   1. partition of the GPU's rows by owner GPU (a W-way scatter) into packed
//      12-byte send records {key lo, key hi, rank}, each row's send position
//      (coalesced) and the per-owner counts (device);
//   2. the records to their owners: by default (PADDED, ABI 5) in fixed-
//      capacity messages whose real counts travel in a header slot and are
//      read on the device -- no host synchronisation, the call's outcome
//      (an overflow re-run, -ENOSPC) resolved at the next call; else
//      (COUNTED) an all-to-all of the counts (24 B per pair), one host
//      synchronisation that sizes the payload, then messages of exact size;
//   3. local grouping of the received rows (Object-index probe first when an
//      index is given, creators inserted after), or the write set of the
//      owned rows (the write-set form: no return leg);
//   4. rep form: all-to-all of the reps back to the sources (4 B per row),
//      gathered to row order (keyless rows keep their own rank).
// Transports: RCCL (ncclSend / ncclRecv in one group, over xGMI; one process
// per GPU via sdgpu_comm_init_rank, or one process driving all GPUs via
// sdgpu_comm_init_all); for contexts that share a device (RCCL refuses two
// ranks on one GPU: the one-GPU test box) device-to-device peer copies
// ordered by events (one process) or, one process per rank, a shared host
// mapping (HOST, ABI 6).  All move the same buffers in the same pattern.
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <memory>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "ctx.hpp"

using namespace sdgpu;

namespace {

// One rank's side of one exchange call (all the call's arguments, so a padded
// call can be re-run through the counted exchange when it is resolved).
struct RankJob {
  sdgpu_ctx* c = nullptr;
  sdgpu_comm* comm = nullptr;
  sdgpu_index* idx = nullptr;
  hipStream_t s = nullptr;
  const uint64_t* key = nullptr;
  const uint8_t* has = nullptr;
  const uint32_t* rank = nullptr;
  uint64_t n = 0;
  uint32_t* rep = nullptr;
  // write-set form (sdgpu_group_link_sharded_device): lists of the owned rows
  const uint8_t* valid = nullptr;
  uint32_t* who = nullptr;
  uint32_t* obj = nullptr;
  uint32_t* counts = nullptr;
  uint64_t cap = 0;
  // device workspace
  uint32_t* srec = nullptr;   // [n][3], or padded [W][C1][3]
  uint32_t* spos = nullptr;   // [n] send position of row i (~0: keyless / not sent)
  int64_t* dcnt = nullptr;    // [W] rows to each owner
  int64_t* xmsg = nullptr;    // [W][3] count messages: {rows to the owner, this rank's n, code}
  int64_t* rcnt_d = nullptr;  // [W][3] from each source
  uint32_t* summ = nullptr;   // [8] padded call summary (pad_fill_launch / recv_summary_launch)
  uint32_t* rrec = nullptr;   // [m][3]
  uint32_t* rrep = nullptr;   // [m]
  uint8_t* rvalid = nullptr;  // [m]
  uint32_t* back = nullptr;   // [total] reps of the sent rows, in send order
  int64_t* h = nullptr;       // pinned [6W]: send counts, receive messages; pairs out, pairs in
  std::vector<uint64_t> scnt, rcnt, soff, roff;
  uint64_t total = 0, m = 0;
  uint64_t c1 = 0;            // slots per padded message (header included); 0: counted
  KeylessSink sink;           // padded write set: this rank's valid keyless rows
  // compact return leg
  uint2* ret = nullptr;       // [m] pairs this owner returns, grouped by source
  uint2* rback = nullptr;     // pairs returned to this source
  int64_t* retcnt = nullptr;  // [W] pairs to each source (device)
  int64_t* rretcnt = nullptr; // [W] pairs from each owner (device)
  std::vector<uint64_t> pcnt, pin, poff, pioff;
};

// HOST transport (ABI 6): one rank per process on one host, messages staged
// through a MAP_SHARED file.  Control page: one HostSlot per rank (its
// progress words and this round's message table); then one outbox of `obox`
// bytes per rank.  Round k of a rank: post its messages (posted = k), copy
// every peer's message to it once they are posted, then consumed = k; its
// outbox is rewritten only after every peer consumed round k.  The words are
// lock-free std::atomic in the shared mapping (address-free).
constexpr int kHostMaxRanks = 64;
struct HostSlot {
  std::atomic<uint64_t> joined;    // 1 once the rank has mapped the file
  std::atomic<uint64_t> posted;    // last round whose outbox is written
  std::atomic<uint64_t> consumed;  // last round whose inbound messages are copied
  std::atomic<uint64_t> aborted;   // the rank failed: its peers stop waiting
  uint64_t nranks, obox;           // what the rank joined with (agreement)
  uint64_t pad[2];
  uint64_t off[kHostMaxRanks];     // this round's message to rank p: outbox offset
  uint64_t bytes[kHostMaxRanks];   //   and size
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory progress words");
constexpr size_t kHostCtrlBytes = (sizeof(HostSlot) * kHostMaxRanks + 4095) / 4096 * 4096;

struct HostLink {
  int fd = -1;
  uint8_t* base = nullptr;
  size_t size = 0;
  uint64_t obox = 0;
  uint64_t round = 0;
  std::string path;
  HostSlot* slot(int r) const { return reinterpret_cast<HostSlot*>(base) + r; }
  uint8_t* outbox(int r) const { return base + kHostCtrlBytes + obox * static_cast<uint64_t>(r); }
  ~HostLink() {
    if (base) (void)munmap(base, size);
    if (fd >= 0) (void)close(fd);
  }
};

}  // namespace

struct sdgpu_comm {
  int nranks = 1;
  int rank = 0;
  int transport = SDGPU_TRANSPORT_RCCL;
  int device = 0;
  ncclComm_t nccl = nullptr;
  // RCCL communicators are non-blocking (config.blocking = 0): every wait on
  // a peer is polled against this deadline and the communicator is aborted
  // when it passes, so a rank that never arrives costs -ETIMEDOUT, not a hang
  int timeout_ms = 0;
  bool aborted = false;
  hipStream_t last_stream = nullptr;  // stream of the last exchange (sdgpu_comm_wait)
  // return leg: SDGPU_RETURN_COMPACT (only the linked rows' reps travel back,
  // after a second count exchange), SDGPU_RETURN_FULL (4 B per row, no
  // second synchronisation) or SDGPU_RETURN_AUTO (per call, see
  // compact_pays).  Every rank of a communicator must agree.
  int return_mode = SDGPU_RETURN_AUTO;
  // -ENOSPC of a padded write set resolved at the next call (not that call's
  // result): returned by the next sdgpu_comm_wait
  int deferred_rc = 0;
  // exchange: SDGPU_EXCHANGE_COUNTED / PADDED / AUTO (sdgpu.h).  agreed_n =
  // B, the largest n of the ranks' last call (every rank learns the same
  // value: from the count messages, or from the padded messages' headers
  // when the call is resolved); 0 = unknown (the next call is counted)
  int exchange = SDGPU_EXCHANGE_AUTO;
  uint64_t agreed_n = 0;
  // the padded call not yet resolved: its arguments, and its summary (copied
  // to pinned memory at the end of the call, summ_evt recorded after it)
  bool pending = false;
  bool pending_list = false;
  uint32_t pending_chunk_rows = 0;
  uint64_t pending_call = 0;  // its number in stats.calls
  RankJob pend;
  sdgpu::PinBuf summ;
  hipEvent_t summ_evt = nullptr;
  sdgpu_comm_stats_t stats{};
  // the layout settings changed since the ranks last agreed on them (every
  // communicator starts so): the next one-rank-per-process call checks them
  // with its peers first (agree_layout / the counted call's code)
  bool layout_dirty = true;
  std::unique_ptr<HostLink> host;  // SDGPU_TRANSPORT_HOST
};

struct sdgpu_index {
  sdgpu_ctx* ctx = nullptr;
  DevBuf buf;       // [slots cap*16 | count 8 | special 8]
  IndexRef ref;
  uint64_t ub = 0;  // host upper bound of the stored key count
};

namespace {

constexpr uint32_t kXShardBits = 8;  // 256 shards; rank d owns shards s with s*W>>8 == d

// SDGPU_RETURN_AUTO: the compact return leg saves 2.4 B per returned row on
// every link (8-B pairs for the ~20 % linked rows instead of 4 B for all) but
// costs a second count exchange + host synchronisation and three kernels:
// 0.064 ms in the one-rank rehearsal at 12.5 M rows (r4e
// predicted_scaling).  At ~100 GB/s per xGMI link that pays once a link
// carries more than ~2.7 M rows; with margin for the collective's latency
// at 8 ranks, compact iff the largest rank's rows / W >= 4 M.  The decision
// uses every rank's n, carried in the count messages, so all ranks agree.
constexpr uint64_t kCompactRowsPerPeer = 4ull << 20;
bool compact_pays(uint64_t n_max, int W) {
  return n_max / static_cast<uint64_t>(W) >= kCompactRowsPerPeer;
}

int nccl_err(ncclResult_t r) { return r == ncclSuccess ? 0 : -EIO; }

#define SD_NCCL(expr)                          \
  do {                                         \
    const int rc_ = nccl_err(expr);            \
    if (rc_ != 0) return rc_;                  \
  } while (0)

constexpr int kDefaultCommTimeoutMs = 300000;

// SDGPU_COMM_TIMEOUT_MS, read once per communicator (init), else 300 s.
int default_timeout_ms() {
  const char* e = getenv("SDGPU_COMM_TIMEOUT_MS");
  if (e && *e) {
    const long v = strtol(e, nullptr, 10);
    if (v > 0 && v < (1l << 30)) return static_cast<int>(v);
  }
  return kDefaultCommTimeoutMs;
}

using Clock = std::chrono::steady_clock;

Clock::time_point deadline_of(int timeout_ms) {
  return Clock::now() + std::chrono::milliseconds(timeout_ms);
}

// Spin briefly (the count exchange is on the step's critical path), then back off.
void backoff(int& spins) {
  if (++spins < 2000) {
    std::this_thread::yield();
  } else {
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Abort an RCCL communicator after a local failure or an expired deadline:
// its kernels still queued on the device exit, its peers see their own
// deadline pass (a local error becomes a bounded job-wide failure, never a
// hang).  The communicator is unusable afterwards (-ECONNABORTED).
// (HOST: the rank's aborted word is raised instead, which its peers poll.)
int comm_fail(sdgpu_comm* m, int rc) {
  if (m && m->nccl && !m->aborted) {
    (void)hipSetDevice(m->device);
    (void)ncclCommAbort(m->nccl);
    m->nccl = nullptr;
    m->aborted = true;
  } else if (m && m->host && !m->aborted) {
    m->host->slot(m->rank)->aborted.store(1, std::memory_order_release);
    m->aborted = true;
  }
  return rc;
}

// One rank per process (RCCL, HOST): a call sees only its own rank, its
// padded outcome is resolved at the next call, a failure aborts the
// communicator.
bool per_process(const sdgpu_comm* m) {
  return m->transport == SDGPU_TRANSPORT_RCCL || m->transport == SDGPU_TRANSPORT_HOST;
}

// Waits until the communicator's non-blocking operation settles.
int nccl_settle(sdgpu_comm* m, Clock::time_point deadline) {
  int spins = 0;
  for (;;) {
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(m->nccl, &a) != ncclSuccess) return comm_fail(m, -EIO);
    if (a == ncclSuccess) return 0;
    if (a != ncclInProgress) return comm_fail(m, -EIO);
    if (Clock::now() > deadline) return comm_fail(m, -ETIMEDOUT);
    backoff(spins);
  }
}

// Waits for stream s to drain while the communicator's peers may still be
// missing: polled, with the communicator's asynchronous error checked, up to
// the deadline.
int stream_wait(sdgpu_comm* m, hipStream_t s, Clock::time_point deadline) {
  if (!m->nccl) return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
  int spins = 0;
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return comm_fail(m, map_err(q));
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(m->nccl, &a) != ncclSuccess ||
        (a != ncclSuccess && a != ncclInProgress))
      return comm_fail(m, -EIO);
    if (Clock::now() > deadline) return comm_fail(m, -ETIMEDOUT);
    backoff(spins);
  }
}

// ---- Object index ------------------------------------------------------------

int index_alloc(sdgpu_ctx* c, DevBuf& b, uint64_t cap, IndexRef& r) {
  const size_t bytes = 16 * cap + 16;
  void* p = nullptr;
  SD_TRY(hipMalloc(&p, bytes));
  b.p = p;
  b.cap = bytes;
  r.slots = static_cast<uint4*>(p);
  r.cap = cap;
  r.count = reinterpret_cast<unsigned long long*>(static_cast<uint8_t*>(p) + 16 * cap);
  r.special = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(p) + 16 * cap + 8);
  (void)c;
  return 0;
}

uint64_t pow2_at_least(uint64_t x) {
  uint64_t p = 1024;
  while (p < x) p <<= 1;
  return p;
}

// Make room for `add` more keys at load <= 1/2.  The exact count is read (one
// synchronisation of s) only when the host-side upper bound says it may not fit.
int index_reserve(sdgpu_index* x, uint64_t add, hipStream_t s) {
  if (x->ub + add <= x->ref.cap / 2) {
    x->ub += add;
    return 0;
  }
  unsigned long long cnt = 0;
  SD_TRY(hipMemcpyAsync(&cnt, x->ref.count, 8, hipMemcpyDeviceToHost, s));
  SD_TRY(hipStreamSynchronize(s));
  if (cnt + add > x->ref.cap / 2) {
    DevBuf nb;
    IndexRef nr;
    SD_TRY_RC(index_alloc(x->ctx, nb, pow2_at_least(4 * (cnt + add)), nr));
    SD_TRY(index_rehash_launch(x->ref, nr, s));
    SD_TRY(hipStreamSynchronize(s));
    (void)hipFree(x->buf.p);
    x->buf = nb;
    x->ref = nr;
  }
  x->ub = cnt + add;
  return 0;
}

// Grouping of one GPU's rows (`in`) with optional Object index: probe, group
// the rest, insert the creators.  rep[i] for every row.
// overflow (device, may be null): a padded exchange's "some message
// overflowed" -- the creators are then not inserted (the call is re-run).
int group_with_index(sdgpu_ctx* c, sdgpu_index* idx, GroupInput in, uint32_t chunk_rows,
                     uint32_t* rep, uint8_t* valid_scratch, hipStream_t s,
                     const uint32_t* overflow = nullptr) {
  if (in.n == 0) return 0;
  SD_TRY_RC(ensure_dev(c, c->dedup_ws, dedup_workspace_bytes(in.n)));
  if (!idx) {
    SD_TRY(dedup_local_launch(in, chunk_rows, rep, true, c->dedup_ws.p, s, c->kt()));
    return 0;
  }
  SD_TRY_RC(index_reserve(idx, in.n, s));
  SD_TRY(index_probe_launch(idx->ref, in, chunk_rows, rep, valid_scratch, s, c->kt()));
  GroupInput g = in;
  g.valid = valid_scratch;
  SD_TRY(dedup_local_launch(g, chunk_rows, rep, false, c->dedup_ws.p, s, c->kt()));
  SD_TRY(index_creators_launch(idx->ref, in, rep, valid_scratch, s, c->kt(), overflow));
  return 0;
}

// ---- the sharded grouping engine ------------------------------------------------

// Count-message code: the call's form and return setting, which every rank
// must share (a rank posting the rep return while another does not would
// leave the collectives unmatched until the deadline): checked by every
// receiver of the counts, -EPROTO on a mismatch.
// Since round 6 the exchange mode is part of it, so ranks that would pick
// different layouts (counted vs padded) meet a mismatch, not a hang.
int64_t call_code(const sdgpu_comm* m, bool list) {
  return (list ? 32 : 16) + m->return_mode + 64 * m->exchange;
}

// Agreement message of a padded call {slots per message, B, code | tag}
// (ABI 6; sdgpu.h "Agreement"): 24 B per peer like a count message, and the
// tag keeps the two from matching, so a rank posting counts where its peer
// posts an agreement fails with -EPROTO on both sides.
constexpr int64_t kAgreeTag = int64_t(1) << 40;

// Slots per (source, owner) message of a padded exchange, header included;
// 0 = counted.  C records = a little over the expected share of the largest
// rank's rows, B / W (binomial spread ~sqrt(B / W), a few thousand rows at
// config 4), never more than B (a source cannot send more); C + 1 rounded
// up to 64 slots.  Depends only on what every rank shares (B, W and the
// modes every rank must set alike), so every rank picks the same layout.
uint64_t padded_slots(const sdgpu_comm* m, int W, bool rep_form) {
  if (m->exchange == SDGPU_EXCHANGE_COUNTED) return 0;
  if (rep_form && m->return_mode == SDGPU_RETURN_COMPACT) return 0;
  const uint64_t B = m->agreed_n, w = static_cast<uint64_t>(W);
  if (B == 0 || B >= (1ull << 31)) return 0;
  const uint64_t C = w == 1 ? B : std::min<uint64_t>(B, B / w + B / (128 * w) + 4096);
  const uint64_t c1 = align_up(C + 1, 64);
  if (w * c1 >= (1ull << 32)) return 0;  // slot indices are 32-bit
  return c1;
}

// HOST transport: waits until every rank's progress word `which` reaches k
// (bounded; a peer that raised its aborted word fails the wait at once).
int host_wait_all(sdgpu_comm* m, std::atomic<uint64_t> HostSlot::*which, uint64_t k,
                  Clock::time_point deadline) {
  HostLink& L = *m->host;
  int spins = 0;
  for (int p = 0; p < m->nranks; ++p) {
    HostSlot* sp = L.slot(p);
    while ((sp->*which).load(std::memory_order_acquire) < k) {
      if (sp->aborted.load(std::memory_order_acquire)) return comm_fail(m, -EIO);
      if (Clock::now() > deadline) return comm_fail(m, -ETIMEDOUT);
      backoff(spins);
    }
  }
  return 0;
}

// One all-to-all round over the HOST transport (this process holds one rank,
// J[0]): the messages leave through the rank's outbox once its stream has
// produced them, the inbound ones are copied from the peers' outboxes, the
// self message device to device.  A size that differs from what the peer
// posted is -EPROTO (the RCCL transport would hang on it until the deadline).
template <typename SP, typename RP, typename SB, typename RB>
int host_alltoallv(RankJob& j, int W, Clock::time_point deadline, SP sendp, RP recvp, SB sbytes,
                   RB rbytes) {
  sdgpu_comm* m = j.comm;
  HostLink& L = *m->host;
  const int me = m->rank;
  if (W != m->nranks) return -EINVAL;
  const uint64_t k = ++L.round;
  SD_TRY(hipSetDevice(j.c->device));
  if (hipStreamSynchronize(j.s) != hipSuccess) return comm_fail(m, -EIO);
  HostSlot* mine = L.slot(me);
  uint64_t off = 0;
  for (int p = 0; p < W; ++p) {
    const uint64_t b = p == me ? 0 : sbytes(j, p);
    if (off + b > L.obox) return comm_fail(m, -EMSGSIZE);
    if (b && hipMemcpy(L.outbox(me) + off, sendp(j, p), b, hipMemcpyDeviceToHost) != hipSuccess)
      return comm_fail(m, -EIO);
    mine->off[p] = off;
    mine->bytes[p] = b;
    off = align_up(off + b, 256);
  }
  mine->posted.store(k, std::memory_order_release);
  SD_TRY_RC(host_wait_all(m, &HostSlot::posted, k, deadline));
  for (int p = 0; p < W; ++p) {
    const uint64_t rb = rbytes(j, p);
    if (p == me) {
      if (sbytes(j, p) != rb) return comm_fail(m, -EPROTO);
      if (rb && hipMemcpyAsync(recvp(j, p), sendp(j, p), rb, hipMemcpyDeviceToDevice, j.s) !=
                    hipSuccess)
        return comm_fail(m, -EIO);
      continue;
    }
    const HostSlot* ps = L.slot(p);
    if (ps->bytes[me] != rb) return comm_fail(m, -EPROTO);
    if (rb && hipMemcpyAsync(recvp(j, p), L.outbox(p) + ps->off[me], rb, hipMemcpyHostToDevice,
                             j.s) != hipSuccess)
      return comm_fail(m, -EIO);
  }
  if (hipStreamSynchronize(j.s) != hipSuccess) return comm_fail(m, -EIO);
  mine->consumed.store(k, std::memory_order_release);
  return host_wait_all(m, &HostSlot::consumed, k, deadline);
}

// One all-to-all round: rank j sends bytes(j, p) from sendp(j, p) to every p
// and receives rbytes(j, p) into recvp(j, p) from every p.
template <typename SP, typename RP, typename SB, typename RB>
int alltoallv(std::vector<RankJob>& J, int W, Clock::time_point deadline, SP sendp, RP recvp,
              SB sbytes, RB rbytes) {
  const int transport = J[0].comm->transport;
  if (transport == SDGPU_TRANSPORT_HOST) {
    if (J.size() != 1) return -EINVAL;
    return host_alltoallv(J[0], W, deadline, sendp, recvp, sbytes, rbytes);
  }
  if (transport == SDGPU_TRANSPORT_RCCL) {
    // non-blocking communicators: calls inside the group may report
    // ncclInProgress; ncclGroupEnd's completion is polled per communicator
    auto ok = [](ncclResult_t r) { return r == ncclSuccess || r == ncclInProgress; };
    if (!ok(ncclGroupStart())) return comm_fail(J[0].comm, -EIO);
    bool fail = false;
    for (auto& j : J) {
      for (int p = 0; p < W && !fail; ++p) {
        // a padded exchange's message to this rank itself is already in place
        if (p == j.comm->rank && sbytes(j, p) == 0 && rbytes(j, p) == 0) continue;
        fail |= !ok(ncclSend(sendp(j, p), sbytes(j, p), ncclUint8, p, j.comm->nccl, j.s));
        fail |= !ok(ncclRecv(recvp(j, p), rbytes(j, p), ncclUint8, p, j.comm->nccl, j.s));
      }
    }
    const ncclResult_t e = ncclGroupEnd();
    if (fail || !ok(e)) {
      for (auto& j : J) comm_fail(j.comm, -EIO);
      return -EIO;
    }
    for (auto& j : J) SD_TRY_RC(nccl_settle(j.comm, deadline));
    return 0;
  }
  // peer copies: all ranks live in this process (J holds every rank, J[r] is rank r).
  // An event belongs to the device current at its creation and may only be
  // recorded on a stream of that device (waits may cross devices), so rank r's
  // events are created -- and recorded -- with rank r's device current.
  if (static_cast<int>(J.size()) != W) return -EINVAL;
  std::vector<hipEvent_t> ready(W, nullptr), done(W, nullptr);
  int rc = 0;
  for (int r = 0; r < W && rc == 0; ++r) {
    if (hipSetDevice(J[r].c->device) != hipSuccess ||
        hipEventCreateWithFlags(&ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&done[r], hipEventDisableTiming) != hipSuccess)
      rc = -EIO;
  }
  for (int r = 0; r < W && rc == 0; ++r)
    if (hipSetDevice(J[r].c->device) != hipSuccess || hipEventRecord(ready[r], J[r].s) != hipSuccess)
      rc = -EIO;
  for (int d = 0; d < W && rc == 0; ++d) {  // receiver d pulls from every source
    RankJob& jd = J[d];
    if (hipSetDevice(jd.c->device) != hipSuccess) rc = -EIO;
    for (int src = 0; src < W && rc == 0; ++src) {
      const size_t b = rbytes(jd, src);
      if (b != sbytes(J[src], d)) {
        rc = -EPROTO;
        break;
      }
      if (hipStreamWaitEvent(jd.s, ready[src], 0) != hipSuccess) rc = -EIO;
      if (rc == 0 && b &&
          hipMemcpyPeerAsync(recvp(jd, src), jd.c->device, sendp(J[src], d), J[src].c->device, b,
                             jd.s) != hipSuccess)
        rc = -EIO;
    }
    if (rc == 0 && hipEventRecord(done[d], jd.s) != hipSuccess) rc = -EIO;
  }
  // a source may reuse its send buffer only after every receiver copied it
  for (int src = 0; src < W && rc == 0; ++src) {
    if (hipSetDevice(J[src].c->device) != hipSuccess) rc = -EIO;
    for (int d = 0; d < W && rc == 0; ++d)
      if (hipStreamWaitEvent(J[src].s, done[d], 0) != hipSuccess) rc = -EIO;
  }
  for (int r = 0; r < W; ++r) {
    (void)hipSetDevice(J[r].c->device);
    if (ready[r]) (void)hipEventDestroy(ready[r]);
    if (done[r]) (void)hipEventDestroy(done[r]);
  }
  return rc;
}

// Steps 1-3 of an exchange, shared by the rep and the write-set forms: every
// rank's keyed rows partitioned by owner, then either
//   counted (c1 == 0): the count messages (with every rank's n -> n_max, the
//     same on all ranks, and the call code), the host synchronisation, the
//     records to their owners in messages of their exact size; or
//   padded (c1 > 0): the records at fixed slots of c1-slot messages, their
//     headers and padding written on the device, all messages of one size,
//     the owners' summary of what arrived (rows, overflow, n_max) left on
//     the device -- no host synchronisation.
// count_ms: host time until the counts were known (0 when padded).
int exchange_forward(std::vector<RankJob>& J, int W, Clock::time_point t_start,
                     Clock::time_point deadline, int64_t code, uint64_t c1, bool list,
                     uint64_t& n_max, double& count_ms) {
  auto recv_bufs = [&](RankJob& j) -> int {
    const size_t o_rep = align_up(12 * j.m, 256);
    const size_t o_val = align_up(o_rep + 4 * j.m, 256);
    SD_TRY_RC(ensure_dev(j.c, j.c->xs_recv, o_val + j.m + 256));
    SD_TRY_RC(ensure_dev(j.c, j.c->xs_back, 4 * j.total + 256));
    uint8_t* r = static_cast<uint8_t*>(j.c->xs_recv.p);
    j.rrec = reinterpret_cast<uint32_t*>(r);
    j.rrep = reinterpret_cast<uint32_t*>(r + o_rep);
    j.rvalid = r + o_val;
    j.back = static_cast<uint32_t*>(j.c->xs_back.p);
    return 0;
  };
  // 1. send side: the keyed rows by owner, on each GPU
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    const uint64_t n = j.n;
    j.c1 = c1;
    const uint64_t srecs = c1 ? static_cast<uint64_t>(W) * c1 : n;
    const size_t o_pos = align_up(12 * srecs, 256);
    const size_t o_dcnt = align_up(o_pos + 4 * n, 256);
    const size_t o_xmsg = align_up(o_dcnt + 8ull * W, 256);
    const size_t o_rcnt = align_up(o_xmsg + 24ull * W, 256);
    const size_t o_pcnt = align_up(o_rcnt + 24ull * W, 256);
    const size_t o_rpcnt = align_up(o_pcnt + 8ull * W, 256);
    const size_t o_summ = align_up(o_rpcnt + 8ull * W, 256);
    SD_TRY_RC(ensure_dev(j.c, j.c->xs_send, o_summ + 32));
    SD_TRY_RC(ensure_dev(j.c, j.c->shard_ws, shard_workspace_bytes(kXShardBits)));
    SD_TRY_RC(ensure_pin(j.c->xs_counts, 64ull * W));
    uint8_t* b = static_cast<uint8_t*>(j.c->xs_send.p);
    j.srec = reinterpret_cast<uint32_t*>(b);
    j.spos = reinterpret_cast<uint32_t*>(b + o_pos);
    j.dcnt = reinterpret_cast<int64_t*>(b + o_dcnt);
    j.xmsg = reinterpret_cast<int64_t*>(b + o_xmsg);
    j.rcnt_d = reinterpret_cast<int64_t*>(b + o_rcnt);
    j.retcnt = reinterpret_cast<int64_t*>(b + o_pcnt);
    j.rretcnt = reinterpret_cast<int64_t*>(b + o_rpcnt);
    j.summ = reinterpret_cast<uint32_t*>(b + o_summ);
    j.h = static_cast<int64_t*>(j.c->xs_counts.p);
    if (c1) {
      // fixed slots: the receive buffer is sized now, and the message to
      // this rank itself is written straight into it (no self copy)
      j.total = j.m = static_cast<uint64_t>(W) * c1;
      SD_TRY_RC(recv_bufs(j));
      const uint32_t me = static_cast<uint32_t>(j.comm->rank), cap = static_cast<uint32_t>(c1 - 1);
      // reservation cursors: two sets used alternately, each call's pad
      // fill zeroing the next call's (no memset launch per call)
      sdgpu_ctx* c = j.c;
      SD_TRY_RC(ensure_dev(c, c->xs_cursor, 2 * 64 * sizeof(uint32_t)));
      if (!c->xs_cursor_clean) {
        SD_TRY(hipMemsetAsync(c->xs_cursor.p, 0, 2 * 64 * sizeof(uint32_t), j.s));
        c->xs_cursor_clean = true;
      }
      uint32_t* cur = static_cast<uint32_t*>(c->xs_cursor.p) + 64 * c->xs_parity;
      uint32_t* next = static_cast<uint32_t*>(c->xs_cursor.p) + 64 * (c->xs_parity ^ 1u);
      j.sink = KeylessSink{};
      if (list) {  // the valid keyless rows, collected by the partition
        const uint32_t segs = keyless_sink_segments(), scap = keyless_sink_cap(n);
        const size_t o_cnt = align_up(4ull * segs * scap, 256);
        SD_TRY_RC(ensure_dev(c, c->xs_sink, o_cnt + 4ull * segs));
        j.sink.valid = j.valid;
        j.sink.st = static_cast<uint32_t*>(c->xs_sink.p);
        j.sink.cnt = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(c->xs_sink.p) + o_cnt);
        j.sink.cap = scap;
      }
      c->xs_cursor_clean = false;  // until the pad fill below is queued
      SD_TRY(padded_partition_launch(j.key, j.has, j.rank, n, static_cast<uint32_t>(W), me, cap,
                                     j.srec, j.rrec, list ? nullptr : j.spos, cur,
                                     list ? &j.sink : nullptr, j.s, j.c->kt()));
      SD_TRY(pad_fill_launch(cur, static_cast<uint32_t>(W), me, cap, n, j.srec, j.rrec, j.summ,
                             list ? j.counts : nullptr, next, j.s));
      c->xs_cursor_clean = true;
      c->xs_parity ^= 1u;
    } else {
      SD_TRY(shard_exchange_launch(j.key, j.has, j.rank, n, kXShardBits, W, nullptr, nullptr,
                                   j.srec, list ? nullptr : j.spos, j.dcnt, j.c->shard_ws.p, j.s,
                                   j.c->kt(), j.xmsg, code));
    }
  }
  if (c1) {
    n_max = 0;  // known on the device only (resolution)
    count_ms = 0;
    for (auto& j : J) {
      const int me = j.comm->rank;
      j.scnt.assign(W, c1);
      j.rcnt.assign(W, c1);
      j.scnt[me] = j.rcnt[me] = 0;  // already in place
      j.soff.assign(W + 1, 0);
      j.roff.assign(W + 1, 0);
      for (int p = 0; p < W; ++p) {
        j.soff[p + 1] = j.soff[p] + c1;
        j.roff[p + 1] = j.roff[p] + c1;
      }
    }
  } else {
    // 2. count messages all-to-all ({rows for the peer, my n, code}), then the
    // host synchronisation
    SD_TRY_RC(alltoallv(
        J, W, deadline, [](RankJob& j, int p) -> void* { return j.xmsg + 3 * p; },
        [](RankJob& j, int p) -> void* { return j.rcnt_d + 3 * p; },
        [](RankJob&, int) -> size_t { return 24; }, [](RankJob&, int) -> size_t { return 24; }));
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      SD_TRY(hipMemcpyAsync(j.h, j.dcnt, 8ull * W, hipMemcpyDeviceToHost, j.s));
      SD_TRY(hipMemcpyAsync(j.h + W, j.rcnt_d, 24ull * W, hipMemcpyDeviceToHost, j.s));
    }
    n_max = 0;  // every rank's n arrived with the counts: the same on all ranks
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      if (j.comm->transport == SDGPU_TRANSPORT_RCCL) {
        SD_TRY_RC(stream_wait(j.comm, j.s, deadline));
      } else {
        SD_TRY(hipStreamSynchronize(j.s));
      }
      j.scnt.assign(W, 0);
      j.rcnt.assign(W, 0);
      j.soff.assign(W + 1, 0);
      j.roff.assign(W + 1, 0);
      for (int p = 0; p < W; ++p) {
        const int64_t* msg = j.h + W + 3 * p;
        const int64_t rc = msg[0], np = msg[1];
        if (j.h[p] < 0 || rc < 0 || np < 0) return -EPROTO;
        if (msg[2] != code) return -EPROTO;  // ranks disagree on the form / return leg
        n_max = std::max(n_max, static_cast<uint64_t>(np));
        j.scnt[p] = static_cast<uint64_t>(j.h[p]);
        j.rcnt[p] = static_cast<uint64_t>(rc);
        j.soff[p + 1] = j.soff[p] + j.scnt[p];
        j.roff[p + 1] = j.roff[p] + j.rcnt[p];
      }
      j.total = j.soff[W];
      j.m = j.roff[W];
      if (j.total > j.n || j.m >= (1ull << 32)) return -EPROTO;
      SD_TRY_RC(recv_bufs(j));
    }
    count_ms = std::chrono::duration<double, std::milli>(Clock::now() - t_start).count();
    for (auto& j : J) j.comm->agreed_n = n_max;
  }
  // 3. the rows, one message per (source, owner) pair
  SD_TRY_RC(alltoallv(
      J, W, deadline, [](RankJob& j, int p) -> void* { return j.srec + 3 * j.soff[p]; },
      [](RankJob& j, int p) -> void* { return j.rrec + 3 * j.roff[p]; },
      [](RankJob& j, int p) -> size_t { return 12 * j.scnt[p]; },
      [](RankJob& j, int p) -> size_t { return 12 * j.rcnt[p]; }));
  if (c1 && W > 1)  // (one rank: the pad fill wrote the summary)
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      SD_TRY(recv_summary_launch(j.rrec, static_cast<uint32_t>(W), static_cast<uint32_t>(c1 - 1),
                                 j.summ, j.s));
    }
  return 0;
}

// The received rows of a padded exchange, for the grouping: every slot of
// the W messages (the grouping drops headers and padding), buckets sized for
// the rows the ranks hold (B).
GroupInput received_rows(const RankJob& j) {
  GroupInput in;
  in.rec12 = j.rrec;
  in.n = j.m;
  if (j.c1) in.bits_rows = std::max<uint64_t>(j.comm->agreed_n, 1);
  return in;
}

// Padded call: its summary to pinned memory behind everything it enqueued,
// and the call pending until resolved (single rank per process), or the
// payload counted into the stats now (the caller resolves at once).
int padded_epilogue(std::vector<RankJob>& J, int W, bool rep_form) {
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    sdgpu_comm* m = j.comm;
    SD_TRY_RC(ensure_pin(m->summ, 64));
    if (!m->summ_evt) SD_TRY(hipEventCreateWithFlags(&m->summ_evt, hipEventDisableTiming));
    SD_TRY(hipMemcpyAsync(m->summ.p, j.summ, 32, hipMemcpyDeviceToHost, j.s));
    SD_TRY(hipEventRecord(m->summ_evt, j.s));
    const uint64_t slots = static_cast<uint64_t>(W) * j.c1, mine = j.c1;
    const uint64_t ret = rep_form ? 4 : 0;
    sdgpu_comm_stats_t& st = m->stats;
    st.padded_calls += 1;
    st.bytes_sent += 12 * slots + ret * slots;
    st.bytes_received += 12 * slots + ret * slots;
    st.bytes_remote += 2 * (12 + ret) * (slots - mine);
    if (rep_form) st.rows_returned += 0;  // counted at resolution (rows received)
  }
  return 0;
}

int run_sharded_impl(std::vector<RankJob>& J, int W, uint32_t chunk_rows, uint64_t c1) {
  const auto t_start = Clock::now();
  for (auto& j : J) j.comm->stats.calls += 1;  // attempted calls (nospc_call numbers them)
  const Clock::time_point deadline = deadline_of(J[0].comm->timeout_ms);
  uint64_t n_max = 0;
  double count_ms = 0;
  SD_TRY_RC(exchange_forward(J, W, t_start, deadline, call_code(J[0].comm, false), c1, false,
                             n_max, count_ms));
  // 4. local grouping of the received rows (every key's rows are all here)
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    SD_TRY_RC(group_with_index(j.c, j.idx, received_rows(j), chunk_rows, j.rrep, j.rvalid, j.s,
                               c1 ? j.summ : nullptr));
  }
  // 5. reps back to their sources, gathered to row order (a padded call
  // returns in full: its messages are fixed-size, the compact leg's are not)
  const int mode = J[0].comm->return_mode;
  const bool compact = !c1 && (mode == SDGPU_RETURN_COMPACT ||
                               (mode == SDGPU_RETURN_AUTO && compact_pays(n_max, W)));
  if (!compact) {
    SD_TRY_RC(alltoallv(
        J, W, deadline, [](RankJob& j, int p) -> void* { return j.rrep + j.roff[p]; },
        [](RankJob& j, int p) -> void* { return j.back + j.soff[p]; },
        [](RankJob& j, int p) -> size_t { return 4 * j.rcnt[p]; },
        [](RankJob& j, int p) -> size_t { return 4 * j.scnt[p]; }));
  } else {
    // only the rows whose rep is not their own rank go back, as {index in
    // the source's message, rep}: the owners compact them per source, the
    // pair counts cross (the step's second host synchronisation), the pairs
    // follow, and each source spreads them over its send-order array
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      RetTiles st{};
      st.world = static_cast<uint32_t>(W);
      for (int p = 0; p < W; ++p) {
        st.roff[p] = static_cast<uint32_t>(j.roff[p]);
        st.tstart[p + 1] = st.tstart[p] +
                           static_cast<uint32_t>((j.rcnt[p] + kRetTileRows - 1) / kRetTileRows);
      }
      st.roff[W] = static_cast<uint32_t>(j.roff[W]);
      const size_t o_ws = align_up(8 * j.m + 8, 256);
      SD_TRY_RC(ensure_dev(j.c, j.c->xs_ret, o_ws + ret_workspace_bytes(ret_tiles(st))));
      j.ret = static_cast<uint2*>(j.c->xs_ret.p);
      SD_TRY(ret_compact_launch(st, j.rrec, j.rrep, j.ret,
                                j.retcnt, static_cast<uint8_t*>(j.c->xs_ret.p) + o_ws, j.s,
                                j.c->kt()));
    }
    SD_TRY_RC(alltoallv(
        J, W, deadline, [](RankJob& j, int p) -> void* { return j.retcnt + p; },
        [](RankJob& j, int p) -> void* { return j.rretcnt + p; },
        [](RankJob&, int) -> size_t { return 8; }, [](RankJob&, int) -> size_t { return 8; }));
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      SD_TRY(hipMemcpyAsync(j.h + 4 * W, j.retcnt, 8ull * W, hipMemcpyDeviceToHost, j.s));
      SD_TRY(hipMemcpyAsync(j.h + 5 * W, j.rretcnt, 8ull * W, hipMemcpyDeviceToHost, j.s));
    }
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      if (j.comm->transport == SDGPU_TRANSPORT_RCCL) {
        SD_TRY_RC(stream_wait(j.comm, j.s, deadline));
      } else {
        SD_TRY(hipStreamSynchronize(j.s));
      }
      j.pcnt.assign(W, 0);
      j.pin.assign(W, 0);
      j.poff.assign(W + 1, 0);
      j.pioff.assign(W + 1, 0);
      for (int p = 0; p < W; ++p) {
        const int64_t a = j.h[4 * W + p], b = j.h[5 * W + p];
        if (a < 0 || b < 0 || static_cast<uint64_t>(a) > j.rcnt[p] ||
            static_cast<uint64_t>(b) > j.scnt[p])
          return -EPROTO;
        j.pcnt[p] = static_cast<uint64_t>(a);
        j.pin[p] = static_cast<uint64_t>(b);
        j.poff[p + 1] = j.poff[p] + j.pcnt[p];
        j.pioff[p + 1] = j.pioff[p] + j.pin[p];
      }
      SD_TRY_RC(ensure_dev(j.c, j.c->xs_rback, 8 * j.pioff[W] + 256));
      j.rback = static_cast<uint2*>(j.c->xs_rback.p);
    }
    SD_TRY_RC(alltoallv(
        J, W, deadline, [](RankJob& j, int p) -> void* { return j.ret + j.poff[p]; },
        [](RankJob& j, int p) -> void* { return j.rback + j.pioff[p]; },
        [](RankJob& j, int p) -> size_t { return 8 * j.pcnt[p]; },
        [](RankJob& j, int p) -> size_t { return 8 * j.pin[p]; }));
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      RetApply ap{};
      ap.world = static_cast<uint32_t>(W);
      for (int p = 0; p <= W; ++p) {
        ap.poff[p] = j.pioff[p];
        ap.soff[p] = static_cast<uint32_t>(j.soff[p]);
      }
      SD_TRY(ret_apply_launch(ap, j.rback, j.back, j.total, j.srec, j.s));
    }
  }
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    const uint64_t me = static_cast<uint64_t>(j.comm->rank);
    SD_TRY(gather_rep_launch(j.back, j.spos, j.rank, j.n, j.rep, j.s, c1 ? j.rrep : nullptr,
                             me * c1, (me + 1) * c1));
  }
  if (c1) SD_TRY_RC(padded_epilogue(J, W, true));
  const double call_ms =
      std::chrono::duration<double, std::milli>(Clock::now() - t_start).count();
  for (auto& j : J) {
    sdgpu_comm_stats_t& st = j.comm->stats;
    st.host_ms += call_ms;
    j.comm->last_stream = j.s;
    if (c1) continue;  // the rows are counted when the call is resolved
    // payload of this rank: the 12-B records it sent, the reps it returned
    // as an owner (4 B per received row, or 8-B pairs for the linked ones),
    // and the same for what it received
    const int me = j.comm->rank;
    const uint64_t self_rows = j.scnt[me];
    st.rows_sent += j.total;
    st.rows_received += j.m;
    if (compact) {
      const uint64_t out_p = j.poff[W], in_p = j.pioff[W];
      st.rows_returned += out_p;
      st.bytes_sent += 12 * j.total + 8 * out_p;
      st.bytes_received += 12 * j.m + 8 * in_p;
      st.bytes_remote += 12 * (j.total - self_rows) + 8 * (out_p - j.pcnt[me]) +
                         12 * (j.m - j.rcnt[me]) + 8 * (in_p - j.pin[me]);
    } else {
      st.rows_returned += j.m;
      st.bytes_sent += 12 * j.total + 4 * j.m;
      st.bytes_received += 12 * j.m + 4 * j.total;
      st.bytes_remote += 12 * (j.total - self_rows) + 4 * (j.m - j.rcnt[me]) +
                         12 * (j.m - j.rcnt[me]) + 4 * (j.total - self_rows);
    }
    st.count_wait_ms += count_ms;
  }
  return 0;
}

// The write-set form: after the forward exchange each owner groups the rows
// it received and writes their Object write set itself (the list-writing
// group kernel of sdgpu_group_link_device, ranks from the records), then
// appends its OWN valid keyless rows.  No return leg, no gather: the union of
// the ranks' lists is the write set of all rows (a set, mod.rs:189-333).
int run_lists_impl(std::vector<RankJob>& J, int W, uint32_t chunk_rows, uint64_t c1) {
  const auto t_start = Clock::now();
  for (auto& j : J) j.comm->stats.calls += 1;  // attempted calls (nospc_call numbers them)
  const Clock::time_point deadline = deadline_of(J[0].comm->timeout_ms);
  uint64_t n_max = 0;
  double count_ms = 0;
  SD_TRY_RC(exchange_forward(J, W, t_start, deadline, call_code(J[0].comm, true), c1, true,
                             n_max, count_ms));
  // no collective follows: a rank whose lists do not fit fails alone.
  // Counted: every rank's capacity (owned keyed rows + own keyless rows,
  // i.e. the rows it did not send) is checked before any list kernel runs,
  // with every rank's counts zeroed first.  Padded: the owned
  // rows are known on the device only; the list kernels write nothing past
  // cap and flag it (summary[4]), the call returns -ENOSPC when resolved.
  bool nospc = false;
  for (auto& j : J) {  // (padded: k_pad_fill zeroed the counts)
    SD_TRY(hipSetDevice(j.c->device));
    if (c1) continue;
    SD_TRY(hipMemsetAsync(j.counts, 0, 3 * sizeof(uint32_t), j.s));
    if (j.m + (j.n - j.total) > j.cap) nospc = true;
  }
  if (nospc) {
    for (auto& j : J)
      if (j.m + (j.n - j.total) > j.cap) j.comm->stats.nospc_call = j.comm->stats.calls;
    return -ENOSPC;
  }
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    SD_TRY_RC(ensure_dev(j.c, j.c->dedup_ws, dedup_workspace_bytes(std::max<uint64_t>(j.m, 1))));
    SD_TRY_RC(ensure_dev(j.c, j.c->link_ws, extra_workspace_bytes(j.n)));
    const GroupInput in = received_rows(j);  // {key, global rank}: 12-B bucket records
    const uint32_t cap32 = static_cast<uint32_t>(std::min<uint64_t>(j.cap, 0xFFFFFFFFull));
    uint32_t* flag = c1 ? j.summ + 4 : nullptr;
    // padded: the own valid keyless rows were collected by the partition and
    // the list's finish moves them; counted: the extra-entry pass lists them
    SD_TRY(dedup_list_launch(in, chunk_rows, j.who, j.obj, j.counts, j.c->dedup_ws.p, j.s,
                             j.c->kt(), false, nullptr, cap32, flag, c1 ? &j.sink : nullptr));
    if (!c1)
      SD_TRY(extra_list_launch(j.has, j.valid, nullptr, nullptr, j.rank, 0, j.n, j.who, j.obj,
                               j.counts, j.c->link_ws.p, j.s, j.c->kt()));
  }
  if (c1) SD_TRY_RC(padded_epilogue(J, W, false));
  const double call_ms =
      std::chrono::duration<double, std::milli>(Clock::now() - t_start).count();
  for (auto& j : J) {
    sdgpu_comm_stats_t& st = j.comm->stats;
    st.host_ms += call_ms;
    j.comm->last_stream = j.s;
    if (c1) continue;
    const int me = j.comm->rank;
    st.rows_sent += j.total;
    st.rows_received += j.m;
    st.bytes_sent += 12 * j.total;
    st.bytes_received += 12 * j.m;
    st.bytes_remote += 12 * (j.total - j.scnt[me]) + 12 * (j.m - j.rcnt[me]);
    st.count_wait_ms += count_ms;
  }
  return 0;
}

// The first padded call of a communicator, and its first after a setting
// changed, checks that every rank chose the same layout before any record
// moves (one process per rank: J = this rank).  One 24-B message per peer,
// one host synchronisation; -EPROTO (communicator aborted) on a mismatch.
int agree_layout(std::vector<RankJob>& J, int W, uint64_t c1, int64_t code) {
  RankJob& j = J[0];
  sdgpu_comm* m = j.comm;
  const Clock::time_point deadline = deadline_of(m->timeout_ms);
  SD_TRY(hipSetDevice(j.c->device));
  SD_TRY_RC(ensure_dev(j.c, j.c->xs_agree, 48ull * W));
  SD_TRY_RC(ensure_pin(j.c->xs_counts, 64ull * W));
  int64_t* h = static_cast<int64_t*>(j.c->xs_counts.p);
  int64_t* d = static_cast<int64_t*>(j.c->xs_agree.p);
  const int64_t mine[3] = {static_cast<int64_t>(c1), static_cast<int64_t>(m->agreed_n),
                           code | kAgreeTag};
  for (int p = 0; p < W; ++p)
    for (int q = 0; q < 3; ++q) h[3 * p + q] = mine[q];
  SD_TRY(hipMemcpyAsync(d, h, 24ull * W, hipMemcpyHostToDevice, j.s));
  SD_TRY_RC(alltoallv(
      J, W, deadline, [d](RankJob&, int p) -> void* { return d + 3 * p; },
      [d, W](RankJob&, int p) -> void* { return d + 3 * W + 3 * p; },
      [](RankJob&, int) -> size_t { return 24; }, [](RankJob&, int) -> size_t { return 24; }));
  SD_TRY(hipMemcpyAsync(h + 3 * W, d + 3 * W, 24ull * W, hipMemcpyDeviceToHost, j.s));
  if (m->transport == SDGPU_TRANSPORT_RCCL) {
    SD_TRY_RC(stream_wait(m, j.s, deadline));
  } else {
    SD_TRY(hipStreamSynchronize(j.s));
  }
  for (int p = 0; p < W; ++p)
    for (int q = 0; q < 3; ++q)
      if (h[3 * W + 3 * p + q] != mine[q]) return comm_fail(m, -EPROTO);
  m->layout_dirty = false;
  m->stats.agreements += 1;
  return 0;
}

// Waits (bounded, the communicator's errors polled) for event ev.
int event_wait(sdgpu_comm* m, hipEvent_t ev, Clock::time_point deadline) {
  if (!m->nccl) return hipEventSynchronize(ev) == hipSuccess ? 0 : -EIO;
  int spins = 0;
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return comm_fail(m, map_err(q));
    ncclResult_t a = ncclSuccess;
    if (ncclCommGetAsyncError(m->nccl, &a) != ncclSuccess ||
        (a != ncclSuccess && a != ncclInProgress))
      return comm_fail(m, -EIO);
    if (Clock::now() > deadline) return comm_fail(m, -ETIMEDOUT);
    backoff(spins);
  }
}

// What a finished padded call left in m->summ: the rows it moved are
// counted, B is updated (every rank read the same headers).  Returns
// 1 when some message overflowed (re-run counted), -ENOSPC when this rank's
// lists did not fit (stats.nospc_call = call_no, the call's number), else 0.
int padded_outcome(sdgpu_comm* m, bool list, uint64_t call_no) {
  const uint32_t* sm = static_cast<const uint32_t*>(m->summ.p);
  m->agreed_n = sm[1];
  sdgpu_comm_stats_t& st = m->stats;
  st.rows_sent += sm[3];
  st.rows_received += sm[2];
  if (!list) st.rows_returned += sm[2];
  if (sm[0]) return 1;
  if (!(list && sm[4])) return 0;
  st.nospc_call = call_no;
  return -ENOSPC;
}

int run_counted(std::vector<RankJob>& J, int W, uint32_t chunk_rows, bool list) {
  return list ? run_lists_impl(J, W, chunk_rows, 0) : run_sharded_impl(J, W, chunk_rows, 0);
}

// Resolves the communicator's pending padded call (single rank per process;
// the caller holds the call's context lock): waits for its summary, and
// re-runs it through the counted exchange if some message overflowed --
// every rank reads the same overflow bit and does the same.  Returns the
// call's result.
int resolve_pending(sdgpu_comm* m) {
  if (!m->pending) return 0;
  m->pending = false;
  if (m->aborted) return -ECONNABORTED;
  const auto t0 = Clock::now();
  SD_TRY(hipSetDevice(m->device));
  SD_TRY_RC(event_wait(m, m->summ_evt, deadline_of(m->timeout_ms)));
  m->stats.resolve_wait_ms += std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
  const int o = padded_outcome(m, m->pending_list, m->pending_call);
  if (o <= 0) return o;
  m->stats.overflow_reruns += 1;
  std::vector<RankJob> J(1, m->pend);
  // after whatever the context ran since; the caller's next work is ordered
  // after this stream in turn (run_call picks its own stream again)
  J[0].s = pick(J[0].c, J[0].s);
  const int rc = run_counted(J, m->nranks, m->pending_chunk_rows, m->pending_list);
  if (rc != 0 && rc != -ENOSPC && per_process(m)) comm_fail(m, rc);
  return rc;
}

// One exchange call over J (every rank of the call: one for a process per
// GPU, all for the _all entry points).  Any failure on an RCCL rank aborts
// its communicator (bounded failure for the peers) and is
// returned; -ENOSPC of the write set comes after the last collective and
// leaves the peers fine.  J[k].s: the stream the entry point was given (the
// context's default when NULL); picked here, after the pending call.
// all_form: an _all entry point, which resolves its padded call before it
// returns -- also when it holds a single per-process communicator (one
// context: a one-rank RCCL communicator), whose call would otherwise be
// left pending like a per-process entry point's.
int run_call(std::vector<RankJob>& J, int W, uint32_t chunk_rows, bool list, bool all_form) {
  for (auto& j : J)
    if (j.comm->aborted || (j.comm->transport == SDGPU_TRANSPORT_RCCL && !j.comm->nccl))
      return -ECONNABORTED;
  const bool single = J.size() == 1 && W > 0 && per_process(J[0].comm);
  if (single) {
    // the previous call of this communicator first (its overflow re-run, if
    // any, keeps the collectives in the same order on every rank).  Its
    // -ENOSPC waits for sdgpu_comm_wait (the earliest unreported one stays).
    sdgpu_comm* m = J[0].comm;
    const int prc = resolve_pending(m);
    if (prc == -ENOSPC && !m->deferred_rc) m->deferred_rc = prc;
    if (prc != 0 && prc != -ENOSPC) return prc;
    if (m->aborted) return -ECONNABORTED;
  }
  // This call's stream, picked only now: a re-run above went on the pending
  // call's stream, which the context's hand-over orders this one after (the
  // re-run and this call share the exchange buffers and the communicator;
  // ADVICE r5 high).
  for (auto& j : J) {
    SD_TRY(hipSetDevice(j.c->device));
    j.s = pick(j.c, j.s);
  }
  uint64_t c1 = padded_slots(J[0].comm, W, !list);
  for (auto& j : J)  // the _all forms: every rank's settings must agree
    if (padded_slots(j.comm, W, !list) != c1 || j.comm->exchange != J[0].comm->exchange ||
        j.comm->return_mode != J[0].comm->return_mode)
      return -EINVAL;
  if (single && c1 && J[0].comm->layout_dirty)
    SD_TRY_RC(agree_layout(J, W, c1, call_code(J[0].comm, list)));
  int rc = list ? run_lists_impl(J, W, chunk_rows, c1) : run_sharded_impl(J, W, chunk_rows, c1);
  if (rc == 0 && !c1) J[0].comm->layout_dirty = false;  // the count messages agreed
  if (rc == 0 && c1) {
    if (single && !all_form) {
      sdgpu_comm* m = J[0].comm;
      m->pending = true;
      m->pending_list = list;
      m->pending_chunk_rows = chunk_rows;
      m->pending_call = m->stats.calls;
      m->pend = J[0];
      return 0;
    }
    // all ranks in this process: resolve now (wait, and re-run counted on
    // an overflow, which every rank's summary shows alike)
    bool over = false;
    int local = 0;
    for (auto& j : J) {
      SD_TRY(hipSetDevice(j.c->device));
      rc = event_wait(j.comm, j.comm->summ_evt, deadline_of(j.comm->timeout_ms));
      if (rc) break;
      const int o = padded_outcome(j.comm, list, j.comm->stats.calls);
      if (o > 0) over = true;
      if (o < 0) local = o;
    }
    if (rc == 0 && over) {
      for (auto& j : J) j.comm->stats.overflow_reruns += 1;
      rc = run_counted(J, W, chunk_rows, list);
    } else if (rc == 0) {
      rc = local;
    }
  }
  if (rc != 0 && rc != -ENOSPC)
    for (auto& j : J)
      if (per_process(j.comm)) comm_fail(j.comm, rc);
  return rc;
}

// The stream an exchange entry point was given (run_call picks it after
// resolving the pending call).
hipStream_t given_stream(sdgpu_ctx* c, void* stream) {
  return stream ? static_cast<hipStream_t>(stream) : c->stream;
}

bool same_devices(sdgpu_ctx* const* ctx, int ngpu) {
  for (int a = 0; a < ngpu; ++a)
    for (int b = a + 1; b < ngpu; ++b)
      if (ctx[a]->device == ctx[b]->device) return true;
  return false;
}

}  // namespace

extern "C" {

// ---- communicators -----------------------------------------------------------------

int sdgpu_comm_unique_id(uint8_t id[SDGPU_COMM_ID_BYTES]) {
  if (!id) return -EINVAL;
  static_assert(sizeof(ncclUniqueId) == SDGPU_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  SD_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return 0;
}

int sdgpu_comm_init_rank_timeout(sdgpu_ctx* c, int nranks, int rank,
                                 const uint8_t id[SDGPU_COMM_ID_BYTES], int timeout_ms,
                                 sdgpu_comm** out) {
  if (!c || !id || !out || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks ||
      timeout_ms <= 0)
    return -EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  sdgpu_comm* m = new (std::nothrow) sdgpu_comm;
  if (!m) return -ENOMEM;
  m->nranks = nranks;
  m->rank = rank;
  m->transport = SDGPU_TRANSPORT_RCCL;
  m->device = c->device;
  m->timeout_ms = timeout_ms;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  // non-blocking init: the bootstrap runs while this thread polls the
  // deadline; a rank that never joins aborts the init (-ETIMEDOUT)
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = ncclCommInitRankConfig(&m->nccl, nranks, u, rank, &cfg);
  int rc = 0;
  if (r != ncclSuccess && r != ncclInProgress) {
    rc = m->nccl ? comm_fail(m, -EIO) : -EIO;
  } else {
    rc = nccl_settle(m, deadline_of(timeout_ms));
  }
  if (rc != 0) {
    delete m;
    return rc;
  }
  *out = m;
  return 0;
}

int sdgpu_comm_init_rank(sdgpu_ctx* c, int nranks, int rank, const uint8_t id[SDGPU_COMM_ID_BYTES],
                         sdgpu_comm** out) {
  return sdgpu_comm_init_rank_timeout(c, nranks, rank, id, default_timeout_ms(), out);
}

int sdgpu_comm_init_host(sdgpu_ctx* c, int nranks, int rank, const char* path,
                         uint64_t msg_bytes, int timeout_ms, sdgpu_comm** out) {
  if (!c || !path || !*path || !out || nranks < 1 || nranks > kHostMaxRanks || rank < 0 ||
      rank >= nranks || msg_bytes == 0 || msg_bytes > (1ull << 40) || timeout_ms <= 0)
    return -EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  std::unique_ptr<HostLink> L(new (std::nothrow) HostLink);
  if (!L) return -ENOMEM;
  L->obox = align_up(msg_bytes, 4096);
  L->size = kHostCtrlBytes + L->obox * static_cast<uint64_t>(nranks);
  L->path = path;
  L->fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0600);
  if (L->fd < 0) return -errno;
  struct stat st;
  if (fstat(L->fd, &st) != 0) return -errno;
  // every rank grows the (fresh, all-zero) file to the same size; a rank
  // that asked for a different msg_bytes is caught by the agreement below
  if (static_cast<uint64_t>(st.st_size) < L->size && ftruncate(L->fd, L->size) != 0) return -errno;
  void* p = mmap(nullptr, L->size, PROT_READ | PROT_WRITE, MAP_SHARED, L->fd, 0);
  if (p == MAP_FAILED) return -errno;
  L->base = static_cast<uint8_t*>(p);
  HostSlot* mine = L->slot(rank);
  if (mine->joined.load(std::memory_order_acquire)) return -EEXIST;  // an earlier communicator's file
  mine->nranks = static_cast<uint64_t>(nranks);
  mine->obox = L->obox;
  mine->joined.store(1, std::memory_order_release);
  const Clock::time_point deadline = deadline_of(timeout_ms);
  int spins = 0;
  for (int q = 0; q < nranks; ++q) {
    HostSlot* sq = L->slot(q);
    while (!sq->joined.load(std::memory_order_acquire)) {
      if (Clock::now() > deadline) return -ETIMEDOUT;
      backoff(spins);
    }
    if (sq->nranks != static_cast<uint64_t>(nranks) || sq->obox != L->obox) return -EPROTO;
  }
  sdgpu_comm* m = new (std::nothrow) sdgpu_comm;
  if (!m) return -ENOMEM;
  m->nranks = nranks;
  m->rank = rank;
  m->transport = SDGPU_TRANSPORT_HOST;
  m->device = c->device;
  m->timeout_ms = timeout_ms;
  m->host = std::move(L);
  *out = m;
  return 0;
}

int sdgpu_comm_set_timeout(sdgpu_comm* m, int timeout_ms) {
  if (!m || timeout_ms <= 0) return -EINVAL;
  m->timeout_ms = timeout_ms;
  return 0;
}

int sdgpu_comm_wait(sdgpu_comm* m, void* stream) {
  if (!m) return -EINVAL;
  int rc = 0;
  if (m->pending) {
    // the padded call's summary, and its counted re-run on an overflow
    sdgpu_ctx* c = m->pend.c;
    std::lock_guard<std::mutex> g(c->mu);
    rc = resolve_pending(m);
  }
  // an earlier call's -ENOSPC found by a later call is reported now, once
  // (ADVICE r5): a hard error of this resolution first, then the deferred
  // -ENOSPC, then this resolution's own
  const int deferred = m->deferred_rc;
  m->deferred_rc = 0;
  if (rc != 0 && rc != -ENOSPC) return rc;
  if (deferred) return deferred;
  if (rc) return rc;
  if (m->aborted) return -ECONNABORTED;
  // the given stream, and the stream of the last exchange when it differs
  // (a re-run goes on the pending call's own stream)
  hipStream_t ss[2] = {stream ? static_cast<hipStream_t>(stream) : m->last_stream, m->last_stream};
  if (ss[1] == ss[0]) ss[1] = nullptr;
  SD_TRY(hipSetDevice(m->device));
  for (hipStream_t s : ss) {
    if (!s) continue;
    if (m->transport != SDGPU_TRANSPORT_RCCL || !m->nccl) {
      if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
    } else {
      SD_TRY_RC(stream_wait(m, s, deadline_of(m->timeout_ms)));
    }
  }
  return 0;
}

int sdgpu_comm_set_exchange(sdgpu_comm* m, int mode, uint64_t rows_hint) {
  if (!m || (mode != SDGPU_EXCHANGE_AUTO && mode != SDGPU_EXCHANGE_COUNTED &&
             mode != SDGPU_EXCHANGE_PADDED))
    return -EINVAL;
  m->exchange = mode;
  if (rows_hint) m->agreed_n = rows_hint;
  m->layout_dirty = true;  // checked with the peers at the next call
  return 0;
}

int sdgpu_comm_set_return(sdgpu_comm* m, int mode) {
  if (!m || (mode != SDGPU_RETURN_FULL && mode != SDGPU_RETURN_COMPACT &&
             mode != SDGPU_RETURN_AUTO))
    return -EINVAL;
  m->return_mode = mode;
  m->layout_dirty = true;
  return 0;
}

int sdgpu_comm_stats(sdgpu_comm* m, sdgpu_comm_stats_t* out) {
  if (!m || !out) return -EINVAL;
  *out = m->stats;
  return 0;
}

int sdgpu_comm_init_all(sdgpu_ctx* const* ctx, int ngpu, int transport, sdgpu_comm** out) {
  if (!ctx || !out || ngpu < 1 || ngpu > 64) return -EINVAL;
  for (int i = 0; i < ngpu; ++i)
    if (!ctx[i]) return -EINVAL;
  const bool dup = same_devices(ctx, ngpu);
  if (transport == SDGPU_TRANSPORT_AUTO)
    transport = dup ? SDGPU_TRANSPORT_PEER : SDGPU_TRANSPORT_RCCL;
  if (transport == SDGPU_TRANSPORT_RCCL && dup) return -EINVAL;  // RCCL: one rank per GPU
  if (transport != SDGPU_TRANSPORT_RCCL && transport != SDGPU_TRANSPORT_PEER) return -EINVAL;
  std::vector<ncclComm_t> nc(ngpu, nullptr);
  if (transport == SDGPU_TRANSPORT_RCCL) {
    std::vector<int> devs(ngpu);
    for (int i = 0; i < ngpu; ++i) devs[i] = ctx[i]->device;
    SD_NCCL(ncclCommInitAll(nc.data(), ngpu, devs.data()));
  } else {
    for (int a = 0; a < ngpu; ++a)  // direct xGMI copies where the devices allow it
      for (int b = 0; b < ngpu; ++b)
        if (ctx[a]->device != ctx[b]->device) {
          (void)hipSetDevice(ctx[a]->device);
          (void)hipDeviceEnablePeerAccess(ctx[b]->device, 0);
          (void)hipGetLastError();
        }
  }
  const int tmo = default_timeout_ms();
  for (int i = 0; i < ngpu; ++i) {
    sdgpu_comm* m = new (std::nothrow) sdgpu_comm;
    if (!m) {
      for (int q = 0; q < i; ++q) {
        delete out[q];
        out[q] = nullptr;
      }
      for (int q = i; q < ngpu; ++q)
        if (nc[q]) (void)ncclCommDestroy(nc[q]);
      return -ENOMEM;
    }
    m->nranks = ngpu;
    m->rank = i;
    m->transport = transport;
    m->device = ctx[i]->device;
    m->nccl = nc[i];
    m->timeout_ms = tmo;
    out[i] = m;
  }
  return 0;
}

int sdgpu_comm_destroy(sdgpu_comm* m) {
  if (!m) return -EINVAL;
  // a pending padded call is dropped (its outputs were never final): its
  // summary copy is waited for, not re-run (the peers are going away too)
  if (m->summ_evt) {
    (void)hipSetDevice(m->device);
    if (m->pending && m->nccl)
      (void)event_wait(m, m->summ_evt, deadline_of(m->timeout_ms > 0 ? m->timeout_ms : 10000));
    else
      (void)hipEventSynchronize(m->summ_evt);
    (void)hipEventDestroy(m->summ_evt);
    m->summ_evt = nullptr;
  }
  m->pending = false;
  if (m->nccl) {
    (void)hipSetDevice(m->device);
    // non-blocking communicator: finalize (may report ncclInProgress while
    // peers flush) is settled against the deadline, then destroyed; a peer
    // that never finishes gets the communicator aborted instead
    const ncclResult_t r = ncclCommFinalize(m->nccl);
    bool settled = r == ncclSuccess;
    if (r == ncclInProgress) settled = nccl_settle(m, deadline_of(m->timeout_ms > 0
                                                                        ? m->timeout_ms
                                                                        : 10000)) == 0;
    if (m->nccl) {  // nccl_settle aborts (and clears) on failure
      if (settled)
        (void)ncclCommDestroy(m->nccl);
      else
        (void)ncclCommAbort(m->nccl);
    }
    m->nccl = nullptr;
  }
  if (m->host && m->rank == 0) (void)unlink(m->host->path.c_str());
  if (m->summ.p) (void)hipHostFree(m->summ.p);
  delete m;
  return 0;
}

int sdgpu_comm_info(sdgpu_comm* m, int* nranks, int* rank, int* transport) {
  if (!m) return -EINVAL;
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  if (transport) *transport = m->transport;
  return 0;
}

// ---- Object index --------------------------------------------------------------------

int sdgpu_index_create(sdgpu_ctx* c, uint64_t capacity_hint, sdgpu_index** out) {
  if (!c || !out) return -EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  sdgpu_index* x = new (std::nothrow) sdgpu_index;
  if (!x) return -ENOMEM;
  x->ctx = c;
  int rc = index_alloc(c, x->buf, pow2_at_least(2 * std::max<uint64_t>(capacity_hint, 1)), x->ref);
  if (rc == 0 && index_clear_launch(x->ref, c->stream) != hipSuccess) rc = -EIO;
  if (rc == 0 && hipStreamSynchronize(c->stream) != hipSuccess) rc = -EIO;
  if (rc) {
    if (x->buf.p) (void)hipFree(x->buf.p);
    delete x;
    return rc;
  }
  *out = x;
  return 0;
}

int sdgpu_index_destroy(sdgpu_index* x) {
  if (!x) return -EINVAL;
  {
    std::lock_guard<std::mutex> g(x->ctx->mu);
    (void)hipSetDevice(x->ctx->device);
    (void)hipStreamSynchronize(x->ctx->stream);
    if (x->ctx->last) (void)hipStreamSynchronize(x->ctx->last);
    if (x->buf.p) (void)hipFree(x->buf.p);
  }
  delete x;
  return 0;
}

int sdgpu_index_clear(sdgpu_index* x, void* stream) {
  if (!x) return -EINVAL;
  std::lock_guard<std::mutex> g(x->ctx->mu);
  SD_TRY(hipSetDevice(x->ctx->device));
  SD_TRY(index_clear_launch(x->ref, pick(x->ctx, stream)));
  x->ub = 0;
  return 0;
}

int sdgpu_index_count(sdgpu_index* x, uint64_t* count) {
  if (!x || !count) return -EINVAL;
  std::lock_guard<std::mutex> g(x->ctx->mu);
  SD_TRY(hipSetDevice(x->ctx->device));
  hipStream_t s = pick(x->ctx, nullptr);
  unsigned long long cnt = 0;
  uint32_t sp[2] = {0, 0};
  SD_TRY(hipMemcpyAsync(&cnt, x->ref.count, 8, hipMemcpyDeviceToHost, s));
  SD_TRY(hipMemcpyAsync(sp, x->ref.special, 8, hipMemcpyDeviceToHost, s));
  SD_TRY(hipStreamSynchronize(s));
  *count = cnt + (sp[0] ? 1 : 0);
  return 0;
}

int sdgpu_index_add_objects_device(sdgpu_index* x, const uint64_t* d_key, const uint32_t* d_handle,
                                   uint64_t n, uint32_t world, uint32_t rank, void* stream) {
  if (!x || (n && (!d_key || !d_handle)) || world == 0 || world > 64 || rank >= world)
    return -EINVAL;
  std::lock_guard<std::mutex> g(x->ctx->mu);
  SD_TRY(hipSetDevice(x->ctx->device));
  hipStream_t s = pick(x->ctx, stream);
  SD_TRY_RC(index_reserve(x, n, s));
  SD_TRY(index_objects_launch(x->ref, d_key, d_handle, n, world, rank, s));
  return 0;
}

int sdgpu_group_rows_indexed_device(sdgpu_ctx* c, sdgpu_index* x, const uint64_t* d_key,
                                    const uint8_t* d_has_key, const uint32_t* d_rank, uint64_t n,
                                    uint32_t chunk_rows, uint32_t* d_rep, void* stream) {
  if (!c || !x || x->ctx->device != c->device || chunk_rows == 0 ||
      (n && (!d_key || !d_rep)))
    return -EINVAL;
  if (n >= (1ull << 32)) return -EINVAL;
  // index values are ranks < 2^31 (the top bit marks existing Objects): with
  // implicit ranks (d_rank NULL, rank = i) that bounds n
  if (!d_rank && n > kRepExisting) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  if (n == 0) return 0;
  SD_TRY_RC(ensure_dev(c, c->xs_recv, n + 256));  // the probe's valid mask
  GroupInput in;
  in.key = d_key;
  in.valid = d_has_key;
  in.rank = d_rank;
  in.n = n;
  return group_with_index(c, x, in, chunk_rows, d_rep, static_cast<uint8_t*>(c->xs_recv.p), s);
}

// Fused grouping + Object write set (ABI 4).  With an index: the probe
// decides the rows whose cas_id already has an Object (reps into a scratch
// array, its mask as the grouping's valid), the group kernel lists the other
// keyed rows, the extra pass lists the probe's rows and the valid keyless
// rows, and every grouped row is offered to the index with its rank -- the
// index keeps the minimum, i.e. the creator (a linked row's rank is never
// below its creator's), so this inserts exactly the creators' values.
int sdgpu_group_link_device(sdgpu_ctx* c, sdgpu_index* x, const uint64_t* d_key,
                            const uint8_t* d_has_key, const uint8_t* d_valid,
                            const uint32_t* d_rank, uint32_t first_rank, uint64_t n,
                            uint32_t chunk_rows, uint32_t* d_who, uint32_t* d_obj,
                            uint32_t* d_counts, void* stream) {
  if (!c || chunk_rows == 0 || !d_counts || (n && (!d_key || !d_who || !d_obj))) return -EINVAL;
  if (x && x->ctx->device != c->device) return -EINVAL;
  // ranks stay below the SDGPU_LINKED / SDGPU_REP_EXISTING bit
  if (n >= (1ull << 31) || (!d_rank && first_rank + n > (1ull << 31))) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  hipStream_t s = pick(c, stream);
  SD_TRY(hipMemsetAsync(d_counts, 0, 3 * sizeof(uint32_t), s));
  if (n == 0) return 0;
  SD_TRY_RC(ensure_dev(c, c->dedup_ws, dedup_workspace_bytes(n, !x && d_has_key)));
  SD_TRY_RC(ensure_dev(c, c->link_ws, extra_workspace_bytes(n)));
  GroupInput in;
  in.key = d_key;
  in.valid = d_has_key;
  in.rank = d_rank;
  in.rank_base = first_rank;
  in.n = n;
  if (!x) {  // the valid keyless rows collected by the partition's first pass
    // (the keyless sink; round 4 measured it against a separate extra-entry
    // pass: 0.242 -> 0.227 ms at 12.5 M rows)
    SD_TRY(dedup_list_launch(in, chunk_rows, d_who, d_obj, d_counts, c->dedup_ws.p, s, c->kt(),
                             true, d_valid));
    return 0;
  }
  // probe scratch: reps [n] + mask [n]
  const size_t o_mask = align_up(4 * n, 256);
  SD_TRY_RC(ensure_dev(c, c->xs_recv, o_mask + n + 256));
  uint32_t* hitrep = static_cast<uint32_t*>(c->xs_recv.p);
  uint8_t* mask = static_cast<uint8_t*>(c->xs_recv.p) + o_mask;
  SD_TRY_RC(index_reserve(x, n, s));
  SD_TRY(index_probe_launch(x->ref, in, chunk_rows, hitrep, mask, s, c->kt()));
  GroupInput gi = in;
  gi.valid = mask;
  SD_TRY(dedup_list_launch(gi, chunk_rows, d_who, d_obj, d_counts, c->dedup_ws.p, s, c->kt()));
  SD_TRY(extra_list_launch(d_has_key, d_valid, mask, hitrep, d_rank, first_rank, n, d_who, d_obj,
                           d_counts, c->link_ws.p, s, c->kt()));
  // hitrep[i] == rank for every grouped row: all of them are offered
  SD_TRY(index_creators_launch(x->ref, in, hitrep, mask, s, c->kt()));
  return 0;
}

int sdgpu_dedup_batch(sdgpu_ctx* c, sdgpu_index* x, const uint64_t* key, const uint8_t* has_key,
                      uint32_t first_rank, uint32_t n, uint32_t chunk_rows, uint32_t* rep) {
  if (!c || chunk_rows == 0 || (n && (!key || !has_key || !rep))) return -EINVAL;
  if (n == 0) return 0;
  if (static_cast<uint64_t>(first_rank) + n > kRepExisting) return -EINVAL;
  {
    std::lock_guard<std::mutex> g(c->mu);
    SD_TRY(hipSetDevice(c->device));
  }
  const size_t o_has = align_up(8ull * n, 256), o_rank = align_up(o_has + n, 256),
               o_rep = align_up(o_rank + 4ull * n, 256), total = align_up(o_rep + 4ull * n, 256);
  uint8_t* d = nullptr;
  if (hipMalloc(&d, total) != hipSuccess) return -ENOMEM;
  std::vector<uint32_t> rank(n);
  for (uint32_t i = 0; i < n; ++i) rank[i] = first_rank + i;
  hipStream_t s = c->stream;
  int rc = 0;
  do {
    if (hipMemcpyAsync(d, key, 8ull * n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d + o_has, has_key, n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d + o_rank, rank.data(), 4ull * n, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = -EIO;
      break;
    }
    const uint64_t* dk = reinterpret_cast<const uint64_t*>(d);
    const uint32_t* dr = reinterpret_cast<const uint32_t*>(d + o_rank);
    uint32_t* drep = reinterpret_cast<uint32_t*>(d + o_rep);
    rc = x ? sdgpu_group_rows_indexed_device(c, x, dk, d + o_has, dr, n, chunk_rows, drep, s)
           : sdgpu_group_rows_device(c, dk, d + o_has, dr, n, chunk_rows, 0, drep, s);
    if (rc) break;
    if (hipMemcpyAsync(rep, drep, 4ull * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = -EIO;
  } while (false);
  (void)hipStreamSynchronize(s);
  (void)hipFree(d);
  return rc;
}

// ---- sharded grouping ----------------------------------------------------------------

int sdgpu_group_sharded_device(sdgpu_ctx* c, sdgpu_comm* comm, sdgpu_index* x,
                               const uint64_t* d_key, const uint8_t* d_has_key,
                               const uint32_t* d_rank, uint64_t n, uint32_t chunk_rows,
                               uint32_t* d_rep, void* stream) {
  if (!c || !comm || chunk_rows == 0 || (n && (!d_key || !d_rank || !d_rep))) return -EINVAL;
  if (comm->device != c->device || (x && x->ctx->device != c->device)) return -EINVAL;
  if (!per_process(comm)) return -EINVAL;  // peer: sdgpu_group_sharded_all_device
  // global ranks are < 2^31 and unique, so n < 2^31 (the padded header's
  // count shares its word with the overflow bit)
  if (n >= (1ull << 31)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  std::vector<RankJob> J(1);
  RankJob& j = J[0];
  j.c = c;
  j.comm = comm;
  j.idx = x;
  j.s = given_stream(c, stream);
  j.key = d_key;
  j.has = d_has_key;
  j.rank = d_rank;
  j.n = n;
  j.rep = d_rep;
  return run_call(J, comm->nranks, chunk_rows, false, false);
}

int sdgpu_group_sharded_all_device(sdgpu_ctx* const* ctx, sdgpu_comm* const* comm,
                                   sdgpu_index* const* idx, int ngpu,
                                   const uint64_t* const* d_key, const uint8_t* const* d_has_key,
                                   const uint32_t* const* d_rank, const uint64_t* n,
                                   uint32_t chunk_rows, uint32_t* const* d_rep,
                                   void* const* streams) {
  if (!ctx || !comm || ngpu < 1 || ngpu > 64 || !d_key || !d_rank || !n || !d_rep ||
      chunk_rows == 0)
    return -EINVAL;
  std::vector<RankJob> J(ngpu);
  for (int r = 0; r < ngpu; ++r) {
    if (!ctx[r] || !comm[r] || comm[r]->nranks != ngpu || comm[r]->rank != r ||
        comm[r]->device != ctx[r]->device || comm[r]->transport != comm[0]->transport)
      return -EINVAL;
    if (n[r] && (!d_key[r] || !d_rank[r] || !d_rep[r])) return -EINVAL;
    if (n[r] >= (1ull << 31)) return -EINVAL;
    if (idx && idx[r] && idx[r]->ctx->device != ctx[r]->device) return -EINVAL;
  }
  // contexts may repeat a device (peer transport on one GPU); lock each once
  std::vector<std::unique_lock<std::mutex>> locks;
  for (int r = 0; r < ngpu; ++r) {
    bool seen = false;
    for (int q = 0; q < r; ++q) seen |= ctx[q] == ctx[r];
    if (!seen) locks.emplace_back(ctx[r]->mu);
  }
  for (int r = 0; r < ngpu; ++r) {
    for (int q = 0; q < r; ++q)
      if (ctx[q] == ctx[r]) return -EINVAL;  // one context per rank: workspaces are per context
    RankJob& j = J[r];
    j.c = ctx[r];
    j.comm = comm[r];
    j.idx = idx ? idx[r] : nullptr;
    SD_TRY(hipSetDevice(ctx[r]->device));
    j.s = given_stream(ctx[r], streams ? streams[r] : nullptr);
    j.key = d_key[r];
    j.has = d_has_key ? d_has_key[r] : nullptr;
    j.rank = d_rank[r];
    j.n = n[r];
    j.rep = d_rep[r];
  }
  return run_call(J, ngpu, chunk_rows, false, true);
}

int sdgpu_group_link_sharded_device(sdgpu_ctx* c, sdgpu_comm* comm, const uint64_t* d_key,
                                    const uint8_t* d_has_key, const uint8_t* d_valid,
                                    const uint32_t* d_rank, uint64_t n, uint32_t chunk_rows,
                                    uint32_t* d_who, uint32_t* d_obj, uint64_t cap,
                                    uint32_t* d_counts, void* stream) {
  if (!c || !comm || chunk_rows == 0 || !d_counts || !d_who || !d_obj ||
      (n && (!d_key || !d_rank)))
    return -EINVAL;
  if (comm->device != c->device) return -EINVAL;
  if (!per_process(comm)) return -EINVAL;  // peer: the _all form
  if (n >= (1ull << 31)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  SD_TRY(hipSetDevice(c->device));
  std::vector<RankJob> J(1);
  RankJob& j = J[0];
  j.c = c;
  j.comm = comm;
  j.s = given_stream(c, stream);
  j.key = d_key;
  j.has = d_has_key;
  j.valid = d_valid;
  j.rank = d_rank;
  j.n = n;
  j.who = d_who;
  j.obj = d_obj;
  j.counts = d_counts;
  j.cap = cap;
  return run_call(J, comm->nranks, chunk_rows, true, false);
}

int sdgpu_group_link_sharded_all_device(sdgpu_ctx* const* ctx, sdgpu_comm* const* comm, int ngpu,
                                        const uint64_t* const* d_key,
                                        const uint8_t* const* d_has_key,
                                        const uint8_t* const* d_valid,
                                        const uint32_t* const* d_rank, const uint64_t* n,
                                        uint32_t chunk_rows, uint32_t* const* d_who,
                                        uint32_t* const* d_obj, const uint64_t* cap,
                                        uint32_t* const* d_counts, void* const* streams) {
  if (!ctx || !comm || ngpu < 1 || ngpu > 64 || !d_key || !d_rank || !n || !d_who || !d_obj ||
      !cap || !d_counts || chunk_rows == 0)
    return -EINVAL;
  for (int r = 0; r < ngpu; ++r) {
    if (!ctx[r] || !comm[r] || comm[r]->nranks != ngpu || comm[r]->rank != r ||
        comm[r]->device != ctx[r]->device || comm[r]->transport != comm[0]->transport)
      return -EINVAL;
    if (!d_who[r] || !d_obj[r] || !d_counts[r] || (n[r] && (!d_key[r] || !d_rank[r])))
      return -EINVAL;
    if (n[r] >= (1ull << 31)) return -EINVAL;
    for (int q = 0; q < r; ++q)
      if (ctx[q] == ctx[r]) return -EINVAL;  // one context per rank
  }
  std::vector<std::unique_lock<std::mutex>> locks;
  for (int r = 0; r < ngpu; ++r) locks.emplace_back(ctx[r]->mu);
  std::vector<RankJob> J(ngpu);
  for (int r = 0; r < ngpu; ++r) {
    RankJob& j = J[r];
    j.c = ctx[r];
    j.comm = comm[r];
    SD_TRY(hipSetDevice(ctx[r]->device));
    j.s = given_stream(ctx[r], streams ? streams[r] : nullptr);
    j.key = d_key[r];
    j.has = d_has_key ? d_has_key[r] : nullptr;
    j.valid = d_valid ? d_valid[r] : nullptr;
    j.rank = d_rank[r];
    j.n = n[r];
    j.who = d_who[r];
    j.obj = d_obj[r];
    j.counts = d_counts[r];
    j.cap = cap[r];
  }
  return run_call(J, ngpu, chunk_rows, true, true);
}

int sdgpu_dedup_sharded(sdgpu_ctx* const* ctx, int ngpu, const uint64_t* key,
                        const uint8_t* has_key, uint32_t n, uint32_t chunk_rows, uint32_t* rep) {
  if (!ctx || ngpu < 1 || ngpu > 64 || chunk_rows == 0 || (n && (!key || !has_key || !rep)))
    return -EINVAL;
  if (n == 0) return 0;
  if (n >= kRepExisting) return -EINVAL;
  std::vector<sdgpu_comm*> comm(ngpu, nullptr);
  SD_TRY_RC(sdgpu_comm_init_all(ctx, ngpu, SDGPU_TRANSPORT_AUTO, comm.data()));
  // rows split in ngpu contiguous ranges; rank = global row index
  std::vector<uint64_t> cnt(ngpu), first(ngpu);
  std::vector<uint8_t*> buf(ngpu, nullptr);
  std::vector<const uint64_t*> dk(ngpu);
  std::vector<const uint8_t*> dh(ngpu);
  std::vector<const uint32_t*> dr(ngpu);
  std::vector<uint32_t*> drep(ngpu);
  int rc = 0;
  for (int r = 0; r < ngpu && rc == 0; ++r) {
    first[r] = static_cast<uint64_t>(n) * r / ngpu;
    cnt[r] = static_cast<uint64_t>(n) * (r + 1) / ngpu - first[r];
    const uint64_t m = std::max<uint64_t>(cnt[r], 1);
    const size_t o_has = align_up(8 * m, 256), o_rank = align_up(o_has + m, 256),
                 o_rep = align_up(o_rank + 4 * m, 256), tot = align_up(o_rep + 4 * m, 256);
    if (hipSetDevice(ctx[r]->device) != hipSuccess || hipMalloc(&buf[r], tot) != hipSuccess) {
      rc = -ENOMEM;
      break;
    }
    std::vector<uint32_t> rk(cnt[r]);
    for (uint64_t i = 0; i < cnt[r]; ++i) rk[i] = static_cast<uint32_t>(first[r] + i);
    dk[r] = reinterpret_cast<const uint64_t*>(buf[r]);
    dh[r] = buf[r] + o_has;
    dr[r] = reinterpret_cast<const uint32_t*>(buf[r] + o_rank);
    drep[r] = reinterpret_cast<uint32_t*>(buf[r] + o_rep);
    if (hipMemcpy(buf[r], key + first[r], 8 * cnt[r], hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(buf[r] + o_has, has_key + first[r], cnt[r], hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(buf[r] + o_rank, rk.data(), 4 * cnt[r], hipMemcpyHostToDevice) != hipSuccess)
      rc = -EIO;
  }
  if (rc == 0)
    rc = sdgpu_group_sharded_all_device(ctx, comm.data(), nullptr, ngpu, dk.data(), dh.data(),
                                        dr.data(), cnt.data(), chunk_rows, drep.data(), nullptr);
  for (int r = 0; r < ngpu; ++r) {
    if (!buf[r]) continue;
    (void)hipSetDevice(ctx[r]->device);
    (void)hipStreamSynchronize(ctx[r]->stream);
    if (rc == 0 && hipMemcpy(rep + first[r], drep[r], 4 * cnt[r], hipMemcpyDeviceToHost) != hipSuccess)
      rc = -EIO;
    (void)hipFree(buf[r]);
  }
  for (auto* m : comm)
    if (m) (void)sdgpu_comm_destroy(m);
  return rc;
}

}  // extern "C"
