// Internal (C++) interfaces between the C-ABI layer (sdgpu.cpp) and the HIP
// kernel translation units.  Nothing here crosses the public boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "tree_plan.hpp"

namespace sdgpu {

// Optional per-kernel timing: the C-ABI layer passes a recorder that brackets
// each main kernel with HIP events on the stream it is launched on.
struct KTimer {
  virtual void begin(const char* name, hipStream_t s) = 0;
  virtual void end(hipStream_t s) = 0;
  virtual ~KTimer() = default;
};
// name null: no scope (a launch sequence timed as a whole elsewhere)
struct KScope {
  KTimer* t;
  hipStream_t s;
  KScope(KTimer* t_, const char* name, hipStream_t s_) : t(name ? t_ : nullptr), s(s_) {
    if (t) t->begin(name, s);
  }
  ~KScope() {
    if (t) t->end(s);
  }
};

// ---- batched short-message BLAKE3 (cas_id, K1) ------------------------------
// Workspace for one batch of n messages and at most max_chunks chunks.
struct BatchWork {
  uint32_t* n_chunks = nullptr;    // [n]     4-chunk units per message
  uint32_t* chunk_base = nullptr;  // [n + 1] exclusive prefix of the units
  uint32_t* block_sums = nullptr;  // [scan tiles of n]
  uint32_t* chunk_msg = nullptr;   // [max_chunks] unit -> message
  uint32_t* cvs = nullptr;         // [max_chunks][8] CV slots
  uint32_t* total = nullptr;       // [1]   == chunk_base[n] (units of the batch)
  uint32_t* order = nullptr;       // [2n]  lane orders: message items, then fold lanes
  uint32_t* hist = nullptr;        // [2 * 128 * 256 + 1] per-block sort histograms
  uint32_t* hist_sums = nullptr;   // [scan tiles of hist]
  uint32_t* grab = nullptr;        // [1] work-queue counter
  uint64_t max_chunks = 0;         // capacity of chunk_msg / cvs (units + n must fit)
};

// Largest message the batched cas kernel accepts: 8 + 100 KiB (cas.rs:15,27-29).
constexpr uint32_t CAS_MAX_MSG_LEN = 8u + 100u * 1024u;

// Hash n messages arena[off[i] .. off[i]+len[i]) (off 16-B aligned) and write
// out_words (2 => cas_id's 8 bytes, 8 => full 32-byte digest) words per message.
// status[i] = 0, -EINVAL for len > max_len / misaligned offset / a message
// ending past arena_bytes, or -ENOBUFS (every message) when the batch's CV
// slots (units + n) exceed w.max_chunks (overlapping messages).
// All pointers are device pointers; fully asynchronous on `s`.
hipError_t batch_hash_launch(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* off,
                             const uint32_t* len, uint32_t n, uint32_t max_len,
                             uint32_t out_words, uint8_t* out, int32_t* status,
                             const BatchWork& w, hipStream_t s, KTimer* timer = nullptr);

// Latency path for a few messages of at most 1 MiB each (SMALL_MAX_BYTES):
// ONE launch.  max_chunks = largest chunk count in the batch.  Same status /
// out semantics as batch_hash_launch.
constexpr uint32_t SMALL_MAX_BYTES = 1024u * 1024u;
// Messages of <= SMALL_MAX_BYTES each (device or pinned host memory, 16-B
// aligned offsets, readable up to the next 16 bytes), each split into 64 KiB groups hashed by one workgroup apiece and folded by
// the message's last group: the latency path for messages above one CU's
// worth of chunks; n <= 64.  scratch: small_split_scratch_bytes() device bytes
// whose counters (the first 64 words) start zeroed (the kernel leaves them so).
size_t small_split_scratch_bytes();
hipError_t small_split_launch(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                              uint32_t n, uint32_t max_len, uint32_t max_chunks,
                              uint32_t out_words, uint8_t* out, int32_t* status, uint32_t* scratch,
                              hipStream_t s, KTimer* timer = nullptr);
// A few messages of at most kHostStageMax bytes read straight from pinned
// host memory (16-B aligned offsets; off / len in pinned memory too), one
// workgroup each, digest words written straight to pinned host memory: the
// single-file and small-batch callers' path without copy commands.
constexpr uint32_t kHostStageMax = 112u * 1024u;
hipError_t small_host_launch(const uint8_t* h_arena, const uint64_t* h_off, const uint32_t* h_len,
                             uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* h_out,
                             hipStream_t s, KTimer* timer = nullptr);

// Resident latency service (the single-file callers, f3): ONE workgroup that
// stays on the device and polls a mailbox in coherent pinned host memory;
// each request's message (<= kHostStageMax bytes, already in the pinned
// message area) is copied into LDS, hashed like k_small_host, and its digest
// words and sequence number written back -- a call costs no launch, no copy
// command and no stream synchronisation.  The kernel returns on a stop
// request, after idle_ticks of wall clock without a request, or after
// life_ticks in total (so it always ends, whatever the host does), setting
// state = kSvcExited first.  Fields sit on separate 64-B lines.
struct alignas(64) SvcMailbox {
  uint32_t seq;        // host: request number, written last (release)
  uint32_t op;         // kSvcHash / kSvcStop
  uint32_t len;        // message bytes at the message area
  uint32_t out_words;  // digest words to return (2: cas_id, 8: checksum)
  uint32_t pad0[12];
  uint32_t done;       // device: the last request number answered (release)
  uint32_t state;      // kSvcRunning (host, before a launch) / kSvcExited (device)
  uint32_t pad1[14];
  uint32_t digest[16];
  // device wall clock (s_memrealtime) of the last request: seen, message in
  // LDS, digest written -- the latency breakdown (sdgpu_latency_service_diag)
  uint64_t t_seen, t_loaded, t_done;
};
constexpr uint32_t kSvcHash = 0, kSvcStop = 1;
constexpr uint32_t kSvcRunning = 1, kSvcExited = 2;
hipError_t service_launch(SvcMailbox* mb, const uint8_t* msg, uint32_t last_seq,
                          uint64_t idle_ticks, uint64_t life_ticks, hipStream_t s);

// ---- tree BLAKE3 of large segments (file_checksum, K2/K3) -------------------
// TreeSeg: tree_plan.hpp
// cv_input: every segment's `data` holds `len` 32-byte chaining values of
// consecutive equal, aligned power-of-two subtrees (the last may be partial);
// they are folded into the digest / CV of their concatenation.
size_t tree_workspace_bytes(const TreeSeg* segs, uint32_t nseg, bool cv_input);
// Bytes of the plan prefix of the workspace (what h_ws must hold).
size_t tree_plan_bytes(uint32_t nseg);
// d_ws: device workspace of tree_workspace_bytes(); h_ws: host scratch of
// tree_plan_bytes() (pinned; must stay untouched until the plan copy on `s`
// has executed).  out: device [nseg][32].
hipError_t tree_hash_launch(const TreeSeg* segs, uint32_t nseg, bool cv_input, uint8_t* out,
                            void* d_ws, void* h_ws, hipStream_t s, KTimer* timer = nullptr);

// ---- synthetic corpora (bench / tests only) -----------------------------------
hipError_t synth_cas_arena_launch(const uint64_t* sizes, const uint64_t* seeds,
                                  const uint64_t* off, uint32_t n, uint8_t* arena, hipStream_t s);
hipError_t synth_file_launch(uint64_t seed, uint64_t offset, uint64_t len, uint8_t* out,
                             hipStream_t s);
// Integer VALU throughput microbenchmark (add3/xor/alignbit mix of BLAKE3's G).
// kind 0: BLAKE3-G mix; 1 v_xor_b32; 2 v_add3_u32; 3 v_alignbit_b32; 4 v_add_u32.
hipError_t valu_probe_launch(int kind, uint32_t* sink, uint32_t iters, uint32_t blocks,
                             hipStream_t s);
hipError_t vary_keys_launch(uint64_t* key, const uint8_t* vary, uint64_t n, uint64_t step,
                            hipStream_t s);
hipError_t synth_dedup_rows_launch(uint64_t seed, uint64_t total_rows, uint64_t distinct,
                                   uint64_t first_rank, uint64_t n, uint64_t* key,
                                   uint8_t* has_key, uint32_t* rank, hipStream_t s);

// ---- dedup (K4-K6) ------------------------------------------------------------
// Rows of one grouping call: either the caller's arrays (key[i], valid[i]
// (null: all keyed), rank[i] (null: rank_base + i)) or packed 12-byte exchange
// records {key lo, key hi, rank} (rec12, all keyed unless valid is given).
struct GroupInput {
  const uint64_t* key = nullptr;
  const uint32_t* rec12 = nullptr;
  const uint8_t* valid = nullptr;
  const uint32_t* rank = nullptr;
  uint32_t rank_base = 0;
  uint64_t n = 0;
  // rows the buckets are sized for (0: n) -- a padded exchange receive's n
  // counts its header and padding slots, which the grouping drops
  uint64_t bits_rows = 0;
};
// with_sink: room for the fused call's keyless sink (sdgpu_group_link_device
// without an index)
size_t dedup_workspace_bytes(uint64_t n, bool with_sink = false);
// rep[i] for row i of `in` (the canonical rule over ranks; rows without a key
// get rep = their rank when init_rep, and are left untouched otherwise).
hipError_t dedup_local_launch(const GroupInput& in, uint32_t chunk_rows, uint32_t* rep,
                              bool init_rep, void* ws, hipStream_t s, KTimer* timer = nullptr);
// The grouping as the Object write set (ListOut in dedup.hip): per bucket, in
// its record range, creators from the front (who = rank) and linked rows from
// the back (who = rank | SDGPU_LINKED, obj = creator rank); no rep array.
// counts[0..2] (zeroed by the caller) += creators, linked; counts[2] = keyed
// entries.  sink_keyless (caller's rows with a has_key array): the first
// partition pass also lists the valid keyless rows (keyless_valid[i] != 0,
// null: all) as creators behind the keyed entries -- what extra_list_launch
// does without an index, with no pass of its own.
// The valid keyless rows of a write set collected by a partition pass into
// per-wave segments (dedup.hip XSink): kPartBlocks x 16 segments of cap rows
// (keyless_sink_cap of the partitioned rows), their counts in cnt.
struct KeylessSink {
  const uint8_t* valid = nullptr;  // null: every keyless row is valid
  uint32_t* st = nullptr;
  uint32_t* cnt = nullptr;
  uint32_t cap = 0;
};
uint32_t keyless_sink_segments();
uint32_t keyless_sink_cap(uint64_t n);
// nospc (non-null): who / obj hold cap entries; a bucket past them writes
// nothing and sets *nospc (the sharded write set's -ENOSPC, decided on the
// device).  moved (may be null): keyless-row segments filled earlier (the
// padded exchange's partition) that the list's finish moves behind the keyed
// entries.
hipError_t dedup_list_launch(const GroupInput& in, uint32_t chunk_rows, uint32_t* who,
                             uint32_t* obj, uint32_t* counts, void* ws, hipStream_t s,
                             KTimer* timer = nullptr, bool sink_keyless = false,
                             const uint8_t* keyless_valid = nullptr, uint32_t cap = 0xFFFFFFFFu,
                             uint32_t* nospc = nullptr, const KeylessSink* moved = nullptr);
// extra_list_launch then appends, in row order, the valid keyless rows and
// (with an index: grouped = the probe's mask, hitrep = its reps) the keyed
// rows the probe decided -- the index path and the owner's keyless rows of
// the sharded write set.
size_t extra_workspace_bytes(uint64_t n);
hipError_t extra_list_launch(const uint8_t* has, const uint8_t* valid, const uint8_t* grouped,
                             const uint32_t* hitrep, const uint32_t* rank, uint32_t first_rank,
                             uint64_t n, uint32_t* who, uint32_t* obj, uint32_t* counts, void* ws,
                             hipStream_t s, KTimer* timer = nullptr, uint32_t cap = 0xFFFFFFFFu,
                             uint32_t* nospc = nullptr);
// Compact return leg of the exchange (dedup.hip): the received rows are cut
// into tiles of 4096 that never straddle a source's segment [roff[p],
// roff[p + 1]); tstart[p] = first tile of segment p, tstart[world] = tiles.
constexpr uint32_t kMaxWorld = 64;
struct RetTiles {
  uint32_t world;
  uint32_t tstart[kMaxWorld + 1];
  uint32_t roff[kMaxWorld + 1];
};
// Source side: pairs from owner d at [poff[d], poff[d + 1]) of the received
// pairs; its rows were sent at [soff[d], ...) of the send order.
struct RetApply {
  uint32_t world;
  uint64_t poff[kMaxWorld + 1];
  uint32_t soff[kMaxWorld + 1];
};
constexpr uint32_t kRetTileRows = 4096;
uint32_t ret_tiles(const RetTiles& st);
size_t ret_workspace_bytes(uint32_t tiles);
// pairs {index in the source's message, rep} of the received rows whose rep
// is not their rank (rrec: 12-B records {key, rank}), grouped by source;
// retcnt[p] (int64, device) = pairs for source p.  No synchronisation.
hipError_t ret_compact_launch(const RetTiles& st, const uint32_t* rrec, const uint32_t* rrep,
                              uint2* ret, int64_t* retcnt, void* ws, hipStream_t s,
                              KTimer* timer = nullptr);
// back[p] = the rank of send record p (srec12, p < n_back: a row no pair
// came back for keeps its own Object), then back[soff[d] + idx] = rep for
// every received pair
hipError_t ret_apply_launch(const RetApply& ap, const uint2* rback, uint32_t* back,
                            uint64_t n_back, const uint32_t* srec12, hipStream_t s);
size_t shard_workspace_bytes(uint32_t shard_bits);
// Shard of a key = top shard_bits bits of mix64(key) (rows_device.hpp row_hash).
hipError_t shard_count_launch(const uint64_t* key, const uint8_t* has_key, uint64_t n,
                              uint32_t shard_bits, uint64_t* d_counts, void* ws, hipStream_t s);
hipError_t shard_partition_launch(const uint64_t* key, const uint8_t* has_key,
                                  const uint32_t* rank, uint64_t n, uint32_t shard_bits,
                                  uint64_t* out_key, uint32_t* out_rank, uint32_t* out_pos,
                                  void* ws, hipStream_t s, KTimer* timer = nullptr);
// partition by destination rank (one hist + scan + scatter; shard s = top 8
// hash bits belongs to rank s * world >> 8) and, on device, the rows per
// destination rank (int64[world]); no host synchronisation.  Output either
// separate key / rank arrays + out_pos[p] = source row of packed row p, or
// packed 12-byte records (out_rec12 non-null) + out_pos[i] = send position of
// source row i (~0 = keyless).
hipError_t shard_exchange_launch(const uint64_t* key, const uint8_t* has_key,
                                 const uint32_t* rank, uint64_t n, uint32_t shard_bits,
                                 uint32_t world, uint64_t* out_key, uint32_t* out_rank,
                                 uint32_t* out_rec12, uint32_t* out_pos, int64_t* d_dest_counts,
                                 void* ws, hipStream_t s, KTimer* timer = nullptr,
                                 int64_t* d_count_msgs = nullptr, int64_t msg_code = 0);
// rep[i] = pos[i] == ~0 ? rank[i] : back[pos[i]] (the exchange's return
// path); positions in [self_lo, self_hi) read self[pos] instead (the padded
// exchange's message to this rank itself: its reps never travel)
hipError_t gather_rep_launch(const uint32_t* back, const uint32_t* pos, const uint32_t* rank,
                             uint64_t n, uint32_t* rep, hipStream_t s, const uint32_t* self = nullptr,
                             uint64_t self_lo = 0, uint64_t self_hi = 0);
// Padded exchange (fixed-capacity messages of cap + 1 12-byte slots per
// destination rank, dedup.hip k_part_padded / k_pad_fill): one pass writes
// the keyed rows into their owners' messages -- the message to rank `me`
// into self_rec12 (the receive buffer), the others into rec12 -- reserving
// slots through cursor[world] (device u32, zero on entry); out_pos (may be
// null): send slot of each row, ~0 for keyless / unsent rows; sink (may be
// null, the write set): the valid keyless rows collected.  Then the headers
// + padding from the cursors; summary (device u32[8]): [3] rows sent, [4] =
// 0 (one rank: [0..2] too, nothing is received); zero3 (may be null) and
// next_cursor[world] (the next call's cursors) zeroed.
hipError_t padded_partition_launch(const uint64_t* key, const uint8_t* has_key,
                                   const uint32_t* rank, uint64_t n, uint32_t world, uint32_t me,
                                   uint32_t cap, uint32_t* out_rec12, uint32_t* self_rec12,
                                   uint32_t* out_pos, uint32_t* cursor, const KeylessSink* sink,
                                   hipStream_t s, KTimer* timer = nullptr);
hipError_t pad_fill_launch(const uint32_t* cursor, uint32_t world, uint32_t me, uint32_t cap,
                           uint64_t n, uint32_t* rec12, uint32_t* self_rec12, uint32_t* summary,
                           uint32_t* zero3, uint32_t* next_cursor, hipStream_t s);
// summary [0] some message overflowed (every rank alike), [1] largest source
// n, [2] rows received, from the received headers.
hipError_t recv_summary_launch(const uint32_t* rrec12, uint32_t world, uint32_t cap,
                               uint32_t* summary, hipStream_t s);
hipError_t scatter_rep_launch(const uint32_t* src, const uint32_t* pos, uint64_t n, uint32_t* dst,
                              uint64_t n_dst, const uint32_t* init, bool do_init, hipStream_t s);

// ---- Object index (index.hip) -----------------------------------------------------
// rep values with this bit name a pre-existing Object handle, not a row rank.
constexpr uint32_t kRepExisting = 0x80000000u;
struct IndexRef {
  uint4* slots = nullptr;              // [cap] {key lo, key hi, value, 0}
  uint64_t cap = 0;                    // power of two
  unsigned long long* count = nullptr; // distinct keys stored (device)
  uint32_t* special = nullptr;         // [2]: key ~0 present, its value
};
hipError_t index_clear_launch(const IndexRef& t, hipStream_t s);
hipError_t index_rehash_launch(const IndexRef& from, const IndexRef& to, hipStream_t s);
hipError_t index_objects_launch(const IndexRef& t, const uint64_t* key, const uint32_t* handle,
                                uint64_t n, uint32_t world, uint32_t rank, hipStream_t s);
// rep[i] / valid_out[i] for every row (see index.hip); valid_out = rows left
// for the batch's own grouping.
hipError_t index_probe_launch(const IndexRef& t, const GroupInput& in, uint32_t chunk_rows,
                              uint32_t* rep, uint8_t* valid_out, hipStream_t s,
                              KTimer* timer = nullptr);
// skip (device, may be null): nothing is inserted when *skip != 0 (a padded
// exchange that overflowed: re-run counted).
hipError_t index_creators_launch(const IndexRef& t, const GroupInput& in, const uint32_t* rep,
                                 const uint8_t* grouped, hipStream_t s, KTimer* timer = nullptr,
                                 const uint32_t* skip = nullptr);

// ---- downstream consumers (consumers.hip) ---------------------------------------
size_t orphan_workspace_bytes(uint64_t n_obj, uint32_t max_id);
hipError_t orphan_objects_launch(const int32_t* obj, uint64_t n_obj, const int32_t* fp_obj,
                                 uint64_t n_fp, uint32_t max_id, int32_t* out, uint32_t* d_count,
                                 void* ws, hipStream_t s);
size_t thumb_workspace_bytes();
hipError_t thumbnail_shards_launch(const uint8_t* cas8, const uint8_t* valid, uint64_t n,
                                   uint32_t* order, uint32_t* counts, void* ws, hipStream_t s);

// ---- Object link batch (K7) ----------------------------------------------------
size_t link_workspace_bytes(uint64_t n);
// rank may be null (rank = first_rank + i), valid may be null (all rows valid).
// d_counts[0] = rows creating an Object, d_counts[1] = rows linking to one.
hipError_t link_batch_launch(const uint32_t* rep, const uint32_t* rank, const uint8_t* valid,
                             uint32_t first_rank, uint64_t n, uint32_t* create, uint32_t* link_row,
                             uint32_t* link_obj, uint32_t* d_counts, void* ws, hipStream_t s,
                             KTimer* timer = nullptr);

}  // namespace sdgpu
