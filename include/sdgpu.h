/*
 * sdgpu.h -- C ABI of libsdgpu.so: MI355X (gfx950) content identification for
 * Spacedrive's sd-core.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json: the
 * sampled-BLAKE3 cas_id, the full-file BLAKE3 integrity checksum and the
 * cas_id -> Object grouping step.  Every entry point below replaces a
 * reference function; the replaced interface is cited (file:line, paths
 * relative to the Spacedrive repository).  INTEGRATION.md shows the Rust FFI
 * binding (`extern "C"` block + wrappers keeping the reference signatures).
 *
 * Conventions
 *  - Plain C types only; no C++ or torch types cross this boundary.
 *  - Return value: 0 on success, a negative errno on failure (-EINVAL bad
 *    argument, -ENOMEM allocation, -ENODEV no usable GPU, -EIO HIP runtime
 *    error, or the -errno of a failed open/read/seek).  Per-item statuses use
 *    the same encoding, so a Rust caller maps them with
 *    io::Error::from_raw_os_error(-status) (FileIOError, core/src/util/error.rs:5-20).
 *  - "_device" entry points take device pointers and a hipStream_t passed as
 *    `void* stream` (NULL = the context's own stream, a blocking stream ordered
 *    with the null stream) and return without
 *    synchronising; all others take host pointers and return when done.
 *  - A context is used by one host thread at a time (the reference runs one
 *    job at a time, core/src/job/manager.rs:32); its device workspace is
 *    shared by all calls made through it.
 *  - Hex formatting stays with the caller: cas_id = lowercase hex of the 8
 *    returned bytes (cas.rs:61 `to_hex()[..16]`), checksum = lowercase hex of
 *    the 32 returned bytes (validation/hash.rs:21-23).  The path-based helpers
 *    additionally return the formatted strings.
 */
#ifndef SDGPU_H
#define SDGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDGPU_ABI_VERSION 6

/* cas.rs:10-15 */
#define SDGPU_CAS_SAMPLE_COUNT 4u
#define SDGPU_CAS_SAMPLE_SIZE 10240u
#define SDGPU_CAS_HEADER_OR_FOOTER_SIZE 8192u
#define SDGPU_CAS_MINIMUM_FILE_SIZE 102400u
/* Largest cas message: u64 size || whole 100 KiB file. */
#define SDGPU_CAS_MAX_MSG_LEN (8u + SDGPU_CAS_MINIMUM_FILE_SIZE)
/* Message of a sampled (> 100 KiB) file: 8 + 8192 + 4 * 10240 + 8192. */
#define SDGPU_CAS_SAMPLED_MSG_LEN 57352u
/* identifier_job_step batch size, file_identifier/mod.rs:36 */
#define SDGPU_IDENTIFIER_CHUNK_SIZE 100u

typedef struct sdgpu_ctx sdgpu_ctx;

int sdgpu_abi_version(void);
const char *sdgpu_strerror(int rc);

/* ---- context / memory ------------------------------------------------------ */
int sdgpu_device_count(int *count);
int sdgpu_open(int device, sdgpu_ctx **out);
/* Frees the context.  Destroy its indexes (sdgpu_index_destroy) and
 * communicators (sdgpu_comm_destroy) first: they point into it. */
int sdgpu_close(sdgpu_ctx *ctx);
/* Waits for all work issued through ctx (its stream and the last stream
 * passed to a _device call). */
int sdgpu_sync(sdgpu_ctx *ctx);
/* The context's hipStream_t. */
void *sdgpu_stream(sdgpu_ctx *ctx);
int sdgpu_alloc_pinned(sdgpu_ctx *ctx, size_t bytes, void **out);
int sdgpu_free_pinned(sdgpu_ctx *ctx, void *p);
int sdgpu_alloc_device(sdgpu_ctx *ctx, size_t bytes, void **out);
int sdgpu_free_device(sdgpu_ctx *ctx, void *p);
/* Asynchronous copy on `stream` (direction inferred by the runtime). */
int sdgpu_memcpy_async(sdgpu_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);

/* ---- K1: sampled cas_id ------------------------------------------------------
 * Replaces the hashing of generate_cas_id (core/src/object/cas.rs:23-62) for a
 * whole batch of files (identifier_job_step, file_identifier/mod.rs:107-134).
 * Message i is msg_arena[msg_off[i] .. msg_off[i] + msg_len[i]) and must be
 * the exact byte sequence the reference feeds its Hasher:
 *   u64 size little-endian || file bytes          (size <= 100 KiB, cas.rs:27-29)
 *   u64 size LE || file[0,8192) || 4 x file[8192 + k*((size-16384)/4), +10240)
 *     || file[len-8192, len)                       (size > 100 KiB, cas.rs:30-58)
 * msg_off[i] % 16 == 0 and msg_len[i] <= SDGPU_CAS_MAX_MSG_LEN, else
 * status[i] = -EINVAL and out8[i] is zeroed.  out8[i] = BLAKE3(M_i)[0..8).
 * status may be NULL. */
int sdgpu_cas_batch(sdgpu_ctx *ctx, const uint8_t *msg_arena, const uint64_t *msg_off,
                    const uint32_t *msg_len, uint32_t n, uint8_t (*out8)[8], int32_t *status);
/* Device-resident variant.  arena_bytes bounds the arena and sizes the K1
 * workspace (arena_bytes / 1024 + n chaining-value slots, enough for disjoint
 * messages inside the arena).  A message ending past arena_bytes gets
 * status -EINVAL.  Messages may overlap (e.g. duplicates sharing one copy) as
 * long as their 4-chunk units plus n fit that bound; otherwise EVERY message
 * gets -ENOBUFS and nothing is hashed (no write past the workspace). */
int sdgpu_cas_batch_device(sdgpu_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes,
                           const uint64_t *d_off, const uint32_t *d_len, uint32_t n,
                           uint8_t *d_out8, int32_t *d_status, void *stream);

/* Pinned-host staged variant (the identifier's "pinned async staging", BASELINE
 * config 5): the messages live in caller-owned PINNED host memory (e.g. where
 * the pread of the cas windows landed, sdgpu_alloc_pinned), in file order
 * (h_off ascending, 16-B aligned).  The library streams the arena through a
 * ring of device slabs -- H2D on its own copy stream overlapped with K1 on
 * `stream` -- and leaves the cas bytes in device memory (d_out8 [n][8],
 * d_status [n] or NULL) for the grouping step.  Asynchronous: h_arena must
 * stay untouched until sdgpu_sync; h_off/h_len are consumed before return. */
int sdgpu_cas_stage_pinned(sdgpu_ctx *ctx, const uint8_t *h_arena, const uint64_t *h_off,
                           const uint32_t *h_len, uint32_t n, uint8_t *d_out8, int32_t *d_status,
                           void *stream);

/* Path-based drop-in for generate_cas_id(path, size) (cas.rs:23): same reads
 * as the reference (open, header, 4 samples by seek, footer from the actual
 * end), hash on the GPU, out_hex = 16 lowercase hex chars + NUL. */
int sdgpu_generate_cas_id(sdgpu_ctx *ctx, const char *path, uint64_t size, char out_hex[17]);

/* Batched file identifier staging (file_identifier/mod.rs:107-134 join_all of
 * FileMetadata::new -> generate_cas_id): reads the cas windows of n files with
 * pread into pinned buffers, pipelines H2D copies with K1 in slabs.  size[i] is
 * the fs::metadata length (mod.rs:65,80-81); size 0 yields status 0 and
 * has_key[i] = 0 (cas_id None, mod.rs:80-88); I/O errors yield status -errno
 * and has_key 0 (row dropped, mod.rs:113,127).  has_key may be NULL.
 * size may be NULL (ABI 6): every path is stat-ed by the read pool first --
 * the reference's fresh fs::metadata(path).len() at identification time, not
 * a size stored with the row; a failed stat is status -errno, a directory
 * -EISDIR (the reference asserts the path is not one, mod.rs:69-72). */
int sdgpu_identify_files(sdgpu_ctx *ctx, const char *const *paths, const uint64_t *size,
                         uint32_t n, uint8_t (*out8)[8], uint8_t *has_key, int32_t *status);

/* ---- K2/K3: full-file checksum -------------------------------------------------
 * Replaces file_checksum (core/src/object/validation/hash.rs:10-24). */
/* BLAKE3 of a host buffer. */
int sdgpu_checksum(sdgpu_ctx *ctx, const void *bytes, uint64_t len, uint8_t out32[32]);
/* BLAKE3 of n device-resident files (pointers 16-B aligned); d_files and lens
 * are HOST arrays of device addresses / byte lengths, d_out32 is device [n][32]. */
int sdgpu_checksum_batch_device(sdgpu_ctx *ctx, const uint8_t *const *d_files,
                                const uint64_t *lens, uint32_t n, uint8_t *d_out32, void *stream);
/* Chaining value of one aligned subtree slice (for streaming hosts): len bytes
 * starting at chunk counter chunk_offset; chunk_offset must be a multiple of
 * the slice's chunk count rounded up to a power of two.  root=1 gives the digest
 * of a whole message (chunk_offset 0). */
int sdgpu_subtree_device(sdgpu_ctx *ctx, const uint8_t *d_bytes, uint64_t len,
                         uint64_t chunk_offset, int root, uint8_t *d_out32, void *stream);
/* Digest of a message from the chaining values of its consecutive aligned
 * subtree slices (sdgpu_subtree_device with root=0): d_cvs is device [n][32]
 * (16-B aligned), n >= 2, every slice of the same power-of-two chunk count
 * except a shorter last one.  One large file split over several GPUs: each
 * GPU computes its slices' CVs, one GPU combines them. */
int sdgpu_combine_subtrees_device(sdgpu_ctx *ctx, const uint8_t *d_cvs, uint64_t n,
                                  uint8_t *d_out32, void *stream);
/* Latency service for the single-file callers (watcher/utils.rs:236,411,467,
 * non_indexed.rs:161): with enable != 0, sdgpu_generate_cas_id and
 * sdgpu_file_checksum hash messages of at most 112 KiB (every cas message;
 * files up to 112 KiB for the checksum) on a workgroup that stays resident
 * on the device and polls a mailbox in pinned memory -- no launch, copy
 * command or stream synchronisation per call.  The workgroup occupies part
 * of one CU until 20 ms after the last such call (then it ends itself; the
 * next call restarts it) and is stopped before any other call of the context
 * launches work.
 * Crossover for the watcher / non-indexed callers (MI355X, measured,
 * profiles/r3/check_r3R_bench.json): the workgroup hashes in quads of lanes
 * (one compression spread over 4 lanes); generate_cas_id through the service
 * 23 / 25 / 28 / 35 us at 4 / 16 / 32 / 64 KiB and 32 us for a sampled file
 * (57 352-B message), against 7.7 / 22 / 40 / 78 / 69 us on one CPU thread
 * of the AVX2 port.  So: hash on the CPU below ~20 KiB of message, on the
 * GPU above (every file > 100 KiB for generate_cas_id; files > 20 KiB for
 * file_checksum, where 1 MiB takes 78 us vs 1.1 ms). */
int sdgpu_latency_service(sdgpu_ctx *ctx, int enable);
/* Path-based drop-in for file_checksum(path): streams the file in 64 MiB
 * power-of-two slices through double-buffered pinned memory; out_hex = 64
 * lowercase hex chars + NUL. */
int sdgpu_file_checksum(sdgpu_ctx *ctx, const char *path, char out_hex[65]);

/* Batched object validator: file_checksum of n files (validator_job.rs:126-169
 * checksums one file per job step).  Files up to 16 MiB are read whole by a
 * thread pool into pinned slabs and each slab is hashed by one tree launch;
 * larger files are streamed like sdgpu_file_checksum.  out32[i] = BLAKE3 of
 * file i (lowercase hex of it = the reference's integrity_checksum);
 * status[i] = 0 or -errno (out32 zeroed), status may be NULL. */
int sdgpu_checksum_files(sdgpu_ctx *ctx, const char *const *paths, uint32_t n,
                         uint8_t (*out32)[32], int32_t *status);

/* ---- K4-K6: cas_id -> Object grouping ------------------------------------------
 * Replaces the Object link/create decisions of identifier_job_step
 * (file_identifier/mod.rs:167-333) over the orphan rows in ascending id order
 * processed in chunks of chunk_rows (=100, mod.rs:36; file_identifier_job.rs:286-309).
 * Rows are identified by their rank r (position in id order, < 2^31).  Output
 * rep[r]: the rank of the row whose Object row r is linked to:
 *   - has_key[r] == 0 (empty file, cas_id None): rep[r] = r;
 *   - r in the chunk holding the lowest-rank row f of its key: rep[r] = r
 *     (a new Object per row, mod.rs:233-297);
 *   - otherwise rep[r] = f (linked to an existing Object, mod.rs:189-225).
 * key = the 8 cas bytes read as a little-endian u64 (equality is all the
 * grouping uses, mod.rs:136-141,196-203).
 * The calls below group the rows they are given.  Objects that exist BEFORE
 * the rows (earlier batches of the run, earlier runs, other locations: the
 * library-wide find_many of mod.rs:168-185) come from an Object index, see
 * sdgpu_index_* and sdgpu_group_rows_indexed_device. */
int sdgpu_dedup(sdgpu_ctx *ctx, const uint64_t *key, const uint8_t *has_key, uint32_t n,
                uint32_t chunk_rows, uint32_t *rep);
/* Device-resident, one GPU: rows given as (key, rank) pairs (rows without a
 * key are simply not passed); writes rep for each pair at the same index.
 * skip_bits: accepted for ABI 1 compatibility and ignored (bucket digits come
 * from a hash of the key since ABI 2, so shards need no skipped bits). */
int sdgpu_group_pairs_device(sdgpu_ctx *ctx, const uint64_t *d_key, const uint32_t *d_rank,
                             uint64_t n, uint32_t chunk_rows, uint32_t skip_bits, uint32_t *d_rep,
                             void *stream);
/* Device-resident, one GPU, whole rows: rep[i] for every row i; rows with
 * d_has_key[i] == 0 get rep[i] = rank[i].  d_has_key NULL = every row keyed;
 * d_rank NULL = rank i (rows already in id order; the partition then moves
 * 12-byte bucket records instead of 16-byte ones, ~10 % faster).  skip_bits
 * ignored. */
int sdgpu_group_rows_device(sdgpu_ctx *ctx, const uint64_t *d_key, const uint8_t *d_has_key,
                            const uint32_t *d_rank, uint64_t n, uint32_t chunk_rows,
                            uint32_t skip_bits, uint32_t *d_rep, void *stream);

/* ---- Object index: Objects that exist before a batch ------------------------
 * Replaces the library-wide lookup of identifier_job_step
 * (file_identifier/mod.rs:168-185: Objects owning a file_path whose cas_id is
 * in the step's set) and the link of matching rows to them (:189-225, :233-241).
 * A device hash table key -> value lives with one context.  Values are either
 * a row rank (the Object created by that row in an earlier batch of the same
 * run) or SDGPU_REP_EXISTING | handle for an Object registered by the caller
 * (handle < 2^31, e.g. the Object's database id).  A key keeps the canonical
 * "first" Object: a registered (pre-existing) Object before any
 * Object created during the run, whatever the order of the calls (find_many,
 * mod.rs:168-185, returns Objects already in the database); the lowest handle
 * among registered ones, the lowest rank among created ones.  Row ranks must
 * be < 2^31 (SDGPU_REP_EXISTING is the top bit).
 * Grouping batches in id order through one index yields exactly the grouping
 * of the whole run (tests/test_gpu_index.py). */
#define SDGPU_REP_EXISTING 0x80000000u
typedef struct sdgpu_index sdgpu_index;
int sdgpu_index_create(sdgpu_ctx *ctx, uint64_t capacity_hint, sdgpu_index **out);
int sdgpu_index_destroy(sdgpu_index *idx);
int sdgpu_index_clear(sdgpu_index *idx, void *stream);
/* Distinct keys stored (synchronises). */
int sdgpu_index_count(sdgpu_index *idx, uint64_t *count);
/* Register pre-existing Objects: d_key[i] -> SDGPU_REP_EXISTING | d_handle[i].
 * Only keys whose shard belongs to `rank` of `world` are kept (world = 1: all),
 * so every GPU of a sharded grouping can be given the same list.  May
 * synchronise `stream` when the table grows. */
int sdgpu_index_add_objects_device(sdgpu_index *idx, const uint64_t *d_key,
                                   const uint32_t *d_handle, uint64_t n, uint32_t world,
                                   uint32_t rank, void *stream);
/* sdgpu_group_rows_device against the index: a keyed row whose key is in the
 * index gets rep = the index value if it is an existing Object, else (a rank
 * f of an earlier batch) rep = r when r and f share a chunk and f otherwise;
 * the other rows are grouped among themselves; afterwards every row that
 * created an Object (rep == rank) is inserted with its rank.  May synchronise
 * `stream` when the table grows. */
int sdgpu_group_rows_indexed_device(sdgpu_ctx *ctx, sdgpu_index *idx, const uint64_t *d_key,
                                    const uint8_t *d_has_key, const uint32_t *d_rank, uint64_t n,
                                    uint32_t chunk_rows, uint32_t *d_rep, void *stream);
/* Host arrays, one batch of n rows with ranks first_rank + i (an identifier
 * job step over a whole batch); idx may be NULL (group the batch alone). */
int sdgpu_dedup_batch(sdgpu_ctx *ctx, sdgpu_index *idx, const uint64_t *key,
                      const uint8_t *has_key, uint32_t first_rank, uint32_t n,
                      uint32_t chunk_rows, uint32_t *rep);

/* ---- multi-GPU grouping: hash-sharded over a node, RCCL all-to-all over xGMI --
 * Every key has one owner GPU (shard = top 8 bits of mix64(key), rank d owns
 * shards s with s * world / 256 == d); each GPU sends its keyed rows to their
 * owners as packed 12-byte {key, rank} records, the owners group their rows
 * (and probe their share of the Object index), and the reps return (4 B per
 * row).  Two exchanges (sdgpu_comm_set_exchange): COUNTED -- a count
 * all-to-all sizes the messages, one host synchronisation per call; PADDED
 * (ABI 5, the default once a communicator has run one call) -- every
 * (source, owner) message has a fixed capacity agreed by all ranks, its
 * real count travels in its first slot and is read on the device, and the
 * call enqueues everything without waiting for the host.
 * Transports: SDGPU_TRANSPORT_RCCL (grouped ncclSend/ncclRecv; one rank per
 * GPU), SDGPU_TRANSPORT_PEER (device-to-device copies between contexts of one
 * process; also contexts sharing a GPU), AUTO = RCCL unless devices repeat,
 * SDGPU_TRANSPORT_HOST (ABI 6, sdgpu_comm_init_host: one process per rank on
 * one host, ranks may share a GPU). */
#define SDGPU_COMM_ID_BYTES 128
#define SDGPU_TRANSPORT_AUTO 0
#define SDGPU_TRANSPORT_RCCL 1
#define SDGPU_TRANSPORT_PEER 2
#define SDGPU_TRANSPORT_HOST 3
typedef struct sdgpu_comm sdgpu_comm;
/* Failure model (ABI 3).  RCCL communicators are created non-blocking; every
 * wait on a peer (joining, the count exchange's one synchronisation,
 * sdgpu_comm_wait) is bounded by the communicator's timeout.  When it passes,
 * or a local step of the exchange fails, the communicator is aborted (its
 * queued kernels exit) and the call returns -ETIMEDOUT (or the local error);
 * the peers then time out too, so a missing or failed rank ends the job with
 * an error on every rank instead of a hang.  An aborted communicator returns
 * -ECONNABORTED from every later exchange; destroy it. */
int sdgpu_comm_unique_id(uint8_t id[SDGPU_COMM_ID_BYTES]);
/* One process per GPU: rank 0 creates the id, every rank receives it out of
 * band and joins; returns when all nranks have joined, or -ETIMEDOUT after
 * timeout_ms (> 0).  The timeout also bounds the communicator's exchanges. */
int sdgpu_comm_init_rank_timeout(sdgpu_ctx *ctx, int nranks, int rank,
                                 const uint8_t id[SDGPU_COMM_ID_BYTES], int timeout_ms,
                                 sdgpu_comm **out);
/* The same with the timeout from env SDGPU_COMM_TIMEOUT_MS (default 300 s). */
int sdgpu_comm_init_rank(sdgpu_ctx *ctx, int nranks, int rank,
                         const uint8_t id[SDGPU_COMM_ID_BYTES], sdgpu_comm **out);
/* One process per rank on one host, through a shared file mapping (ABI 6):
 * the same messages, in the same order, as the RCCL transport, staged
 * through host memory -- each rank's outbox of msg_bytes holds its messages
 * of one all-to-all round; a round waits for the rank's stream, posts the
 * outbox, waits (bounded by timeout_ms) for every peer's, copies its
 * inbound messages and waits until every peer has copied its own.  The
 * exchange calls (sdgpu_group_sharded_device, sdgpu_group_link_sharded_
 * device) run exactly the per-process state machine they run under RCCL
 * (a padded call left pending and resolved at the next call / wait / destroy,
 * the overflow re-run, the deferred -ENOSPC, the bounded failure), so ranks
 * that share a GPU -- which RCCL refuses -- can exercise it.  Host-
 * synchronous: a test and fallback transport, not a fast one.  path names a
 * file every rank opens (created by the first; it must not hold an earlier
 * communicator's state: -EEXIST); rank 0 unlinks it on destroy.  A round
 * whose messages exceed msg_bytes fails with -EMSGSIZE.  -ETIMEDOUT when not
 * every rank joins within timeout_ms (> 0), -EPROTO when the ranks disagree
 * on nranks or msg_bytes. */
int sdgpu_comm_init_host(sdgpu_ctx *ctx, int nranks, int rank, const char *path,
                         uint64_t msg_bytes, int timeout_ms, sdgpu_comm **out);
/* One process driving ngpu contexts: out[r] is rank r's communicator. */
int sdgpu_comm_init_all(sdgpu_ctx *const *ctx, int ngpu, int transport, sdgpu_comm **out);
int sdgpu_comm_destroy(sdgpu_comm *comm);
int sdgpu_comm_info(sdgpu_comm *comm, int *nranks, int *rank, int *transport);
int sdgpu_comm_set_timeout(sdgpu_comm *comm, int timeout_ms);
/* Waits, bounded by the timeout, until `stream` (NULL: the stream of the
 * communicator's last exchange) has drained -- i.e. the reps of the last
 * sdgpu_group_sharded_device are written -- and resolves a padded exchange
 * (below): if any message of it overflowed, the call is re-run through the
 * counted exchange before this returns.  Returns that call's result (e.g.
 * -ENOSPC of a write set that did not fit).  -ETIMEDOUT (communicator
 * aborted) if a peer never completes its side. */
int sdgpu_comm_wait(sdgpu_comm *comm, void *stream);
/* Exchange of the one-process-per-GPU calls (sdgpu_group_sharded_device,
 * sdgpu_group_link_sharded_device; ABI 5):
 *   COUNTED: counts first, then the records; one host synchronisation per
 *     call, the results final when the stream reaches them.
 *   PADDED: no host synchronisation.  The message from each source to each
 *     owner holds C = min(B, B / nranks + B / (128 nranks) + 4096) records
 *     (a little over its expected share; B = the largest n of the ranks'
 *     previous call, which every rank learns from the headers, or rows_hint)
 *     plus a header slot; the owners drop the padding on the device.  A
 *     message that needed more than C records (a cas_id held by many rows,
 *     a rank with more rows than B) sets an overflow bit every rank sees.
 *     The call is RESOLVED at the next exchange call on the communicator,
 *     sdgpu_comm_wait or destroy: overflowed calls are then re-run through
 *     the counted exchange on the same stream, on every rank alike.  Until
 *     it is resolved, the call's inputs must not change and its outputs are
 *     not final (read them after sdgpu_comm_wait).  The rep form with an
 *     explicit SDGPU_RETURN_COMPACT stays counted.
 *   AUTO (default): PADDED once B is known (after the first call), else
 *     COUNTED.
 * Every rank of a communicator must set the same mode (and rows_hint, which
 * sets B when > 0).  The _all entry points (one process, all ranks) resolve
 * a padded call before they return -- also with ngpu = 1, whose communicator
 * is a one-rank per-process one.
 * Agreement (ABI 6): a communicator's first call and its first call after
 * sdgpu_comm_set_exchange / sdgpu_comm_set_return (which every rank must
 * call alike, between the same two exchange calls) check that every rank
 * chose the same layout -- a counted call through the code in its count
 * messages (form, return mode, exchange mode), a padded call through one
 * 24-byte agreement message per peer {slots per message, B, code} of the
 * same shape, before any record moves -- and fail with -EPROTO (communicator
 * aborted) when they differ, instead of posting messages of different sizes.
 * -ENOSPC of a padded write set that is resolved by a later call is returned
 * by the next sdgpu_comm_wait (the earliest unreported one; stats.nospc_call
 * names the call); a hard error found by the same wait takes precedence. */
#define SDGPU_EXCHANGE_AUTO 0
#define SDGPU_EXCHANGE_COUNTED 1
#define SDGPU_EXCHANGE_PADDED 2
int sdgpu_comm_set_exchange(sdgpu_comm *comm, int mode, uint64_t rows_hint);
/* Cumulative exchange volume of this rank (bytes = 12-B records + 4-B reps). */
typedef struct sdgpu_comm_stats_t {
  uint64_t calls;
  uint64_t rows_sent, rows_received;      /* keyed rows to / from every rank incl. self */
  uint64_t bytes_sent, bytes_received;    /* payload incl. the self share: 12-B records,
                                             plus the reps this rank returned as an owner
                                             (sent) / got back as a source (received);
                                             padded calls: the whole fixed-size messages */
  uint64_t bytes_remote;                  /* payload that crossed to / from other ranks */
  double count_wait_ms;                   /* host ms until the counts were known (0 for
                                             padded calls) */
  double host_ms;                         /* host ms inside the exchange calls */
  uint64_t rows_returned;                 /* (ABI 4) received rows whose rep went back */
  uint64_t padded_calls;                  /* (ABI 5) calls through the padded exchange */
  uint64_t overflow_reruns;               /* (ABI 5) padded calls re-run counted */
  double resolve_wait_ms;                 /* (ABI 5) host ms waiting to resolve them */
  uint64_t agreements;                    /* (ABI 6) layout agreement rounds (below) */
  uint64_t nospc_call;                    /* (ABI 6) `calls` number of the last call that
                                             failed with -ENOSPC (0: none) */
} sdgpu_comm_stats_t;
/* Return leg of the exchange (ABI 4).  COMPACT: an owner sends back only the
 * received rows whose rep is not their own rank, as 8-B {index, rep} pairs
 * after a second count exchange (a second host synchronisation); ~1.6 B per
 * row instead of 4 at config 4's 20 % duplicates.  FULL: every received row's
 * 4-B rep, one synchronisation per call.  AUTO (the default): COMPACT when the
 * largest rank's rows / nranks >= 4 Mi (the bytes it saves per link outweigh
 * the second synchronisation), else FULL -- decided per call from every
 * rank's n, which travels with the counts, so all ranks agree.  All ranks of
 * a communicator must set the same mode. */
#define SDGPU_RETURN_FULL 0
#define SDGPU_RETURN_COMPACT 1
#define SDGPU_RETURN_AUTO 2
int sdgpu_comm_set_return(sdgpu_comm *comm, int mode);
int sdgpu_comm_stats(sdgpu_comm *comm, sdgpu_comm_stats_t *out);
/* Collective, one process per GPU (RCCL): every rank calls it with its own
 * rows (global ranks in d_rank, required, each < 2^31); rep for each of its
 * rows.  idx (may be NULL) is this rank's share of the Object index. */
int sdgpu_group_sharded_device(sdgpu_ctx *ctx, sdgpu_comm *comm, sdgpu_index *idx,
                               const uint64_t *d_key, const uint8_t *d_has_key,
                               const uint32_t *d_rank, uint64_t n, uint32_t chunk_rows,
                               uint32_t *d_rep, void *stream);
/* The same from one process for all ngpu ranks at once (arrays indexed by
 * rank; idx, d_has_key and streams may be NULL). */
int sdgpu_group_sharded_all_device(sdgpu_ctx *const *ctx, sdgpu_comm *const *comm,
                                   sdgpu_index *const *idx, int ngpu,
                                   const uint64_t *const *d_key, const uint8_t *const *d_has_key,
                                   const uint32_t *const *d_rank, const uint64_t *n,
                                   uint32_t chunk_rows, uint32_t *const *d_rep,
                                   void *const *streams);
/* Sharded grouping + Object write set, with no return leg: each rank writes
 * the write-set entries (as sdgpu_group_link_device: who = rank, or rank |
 * SDGPU_LINKED with obj = the creator's rank) of the keyed rows it OWNS --
 * their cas_id hashes to its shard, whichever rank identified them -- and of
 * its own valid keyless rows.  The union over the ranks is the write set of
 * all rows (a set, mod.rs:189-333), so only the 12-B records cross xGMI.
 * Global ranks in d_rank (required, < 2^31).  d_who / d_obj hold cap
 * entries: -ENOSPC (the peers are unaffected; the lists are not valid) when
 * this rank's owned keyed rows + own keyless rows exceed cap -- up to
 * nranks x n when every row shares one cas_id.  The counted exchange
 * returns it from the call, before any list is written; the padded one
 * finds it on the device (no entry is written past cap) and returns it when
 * the call is resolved (sdgpu_comm_wait).
 * d_counts (device) = [creators, linked, entries].  No Object index (use
 * sdgpu_group_sharded_device with one). */
int sdgpu_group_link_sharded_device(sdgpu_ctx *ctx, sdgpu_comm *comm, const uint64_t *d_key,
                                    const uint8_t *d_has_key, const uint8_t *d_valid,
                                    const uint32_t *d_rank, uint64_t n, uint32_t chunk_rows,
                                    uint32_t *d_who, uint32_t *d_obj, uint64_t cap,
                                    uint32_t *d_counts, void *stream);
/* The same from one process for all ngpu ranks (arrays indexed by rank;
 * d_has_key, d_valid and streams may be NULL). */
int sdgpu_group_link_sharded_all_device(sdgpu_ctx *const *ctx, sdgpu_comm *const *comm, int ngpu,
                                        const uint64_t *const *d_key,
                                        const uint8_t *const *d_has_key,
                                        const uint8_t *const *d_valid,
                                        const uint32_t *const *d_rank, const uint64_t *n,
                                        uint32_t chunk_rows, uint32_t *const *d_who,
                                        uint32_t *const *d_obj, const uint64_t *cap,
                                        uint32_t *const *d_counts, void *const *streams);
/* SURVEY §8(b)'s sdgpu_dedup(ctx[], ngpu, ...): host arrays in rank order,
 * split into ngpu contiguous ranges, grouped across the ngpu contexts
 * (communicators created and destroyed inside). */
int sdgpu_dedup_sharded(sdgpu_ctx *const *ctx, int ngpu, const uint64_t *key,
                        const uint8_t *has_key, uint32_t n, uint32_t chunk_rows, uint32_t *rep);

/* Sharding helpers (single steps of the exchange, for hosts that bring their
 * own collectives, e.g. torch.distributed): shard of a key = top shard_bits
 * bits of mix64(key).  count: h_counts[s] = rows with has_key destined to
 * shard s (host array of 2^shard_bits; synchronises).  partition: packs those
 * rows by shard into d_out_key/d_out_rank (shard s at exclusive prefix of
 * counts) and records each packed row's source index in d_out_pos. */
int sdgpu_shard_count_device(sdgpu_ctx *ctx, const uint64_t *d_key, const uint8_t *d_has_key,
                             uint64_t n, uint32_t shard_bits, uint64_t *h_counts, void *stream);
int sdgpu_shard_partition_device(sdgpu_ctx *ctx, const uint64_t *d_key, const uint8_t *d_has_key,
                                 const uint32_t *d_rank, uint64_t n, uint32_t shard_bits,
                                 uint64_t *d_out_key, uint32_t *d_out_rank, uint32_t *d_out_pos,
                                 void *stream);
/* The send side of the sharded grouping's exchange in one call, with no host
 * synchronisation: the partition of sdgpu_shard_partition_device (one
 * histogram pass) plus d_dest_counts[d] (int64, device) = packed rows destined
 * to rank d, where shard s belongs to rank (s * world) >> shard_bits.  Ranks'
 * segments are contiguous and in rank order in d_out_*; sized n rows (keyless
 * rows are dropped, so the tail is unused).  world <= 64, world <= 2^shard_bits. */
int sdgpu_shard_exchange_device(sdgpu_ctx *ctx, const uint64_t *d_key, const uint8_t *d_has_key,
                                const uint32_t *d_rank, uint64_t n, uint32_t shard_bits,
                                uint32_t world, uint64_t *d_out_key, uint32_t *d_out_rank,
                                uint32_t *d_out_pos, int64_t *d_dest_counts, void *stream);
/* d_dst[d_pos[i]] = d_src[i] for i < n.  With init != 0 every row of d_dst is
 * first set to d_init[r] (or to r when d_init is NULL), so rows without a key
 * keep their own rank (mod.rs:238-239). */
int sdgpu_scatter_rep_device(sdgpu_ctx *ctx, const uint32_t *d_src, const uint32_t *d_pos,
                             uint64_t n, uint32_t *d_dst, uint64_t n_dst, const uint32_t *d_init,
                             int init, void *stream);

/* ---- K7: Object link batch ------------------------------------------------------
 * The write set of identifier_job_step (file_identifier/mod.rs:189-333) for a
 * whole batch of rows, from the grouping's rep[]: rows with rep == own rank
 * create an Object (object::create_many, mod.rs:243-297), the others connect
 * to the Object of row rep (mod.rs:189-225); rows with d_valid[i] == 0 (I/O
 * error, mod.rs:113,127) are in neither list.  Row i has rank d_rank[i]
 * (d_rank NULL: first_rank + i).  Outputs (device): d_create[0..C) creator
 * ranks, d_link_row/d_link_obj[0..L) (row rank, creator rank), both in row
 * order; d_counts[0] = C, d_counts[1] = L.  Each output holds n entries. */
int sdgpu_link_batch_device(sdgpu_ctx *ctx, const uint32_t *d_rep, const uint32_t *d_rank,
                            const uint8_t *d_valid, uint32_t first_rank, uint64_t n,
                            uint32_t *d_create, uint32_t *d_link_row, uint32_t *d_link_obj,
                            uint32_t *d_counts, void *stream);

/* Fused grouping + Object write set (ABI 4): the grouping of
 * sdgpu_group_rows_device and the lists of sdgpu_link_batch_device in one
 * pass, with no rep array in between (the group kernel writes the lists
 * directly, coalesced; file_identifier/mod.rs:189-333).  Rows: d_key[i],
 * d_has_key[i] (NULL = every row keyed), d_valid[i] (NULL = every row valid;
 * a row with valid == 0 must have has_key == 0 and is in no list: it stays an
 * orphan, mod.rs:113,127), rank d_rank[i] or first_rank + i (d_rank NULL),
 * ranks < 2^31.  Output (device), one entry per keyed row and per valid
 * keyless row, n entries each:
 *   d_who[e] = rank                  the row creates an Object
 *   d_who[e] = rank | SDGPU_LINKED   the row connects to the Object created by
 *                                    the row of rank d_obj[e]
 * Keyed rows come first, grouped by an internal hash bucket (creators before
 * linked rows inside a bucket); the valid keyless rows (own Objects,
 * mod.rs:238-239) follow them.  The ORDER of the entries is not
 * part of the contract (the reference's writes are a set; compare as sets).
 * d_counts[0] = creators, [1] = linked rows, [2] = entries (= [0] + [1]). */
#define SDGPU_LINKED 0x80000000u
/* idx (may be NULL): the Object index, as in sdgpu_group_rows_indexed_device:
 * a row whose cas_id already has an Object (registered, or created by an
 * earlier batch) links to it -- obj = SDGPU_REP_EXISTING | handle, or the
 * creator's rank -- and the creators of this batch are added to the index.
 * May synchronise `stream` when the index grows. */
int sdgpu_group_link_device(sdgpu_ctx *ctx, sdgpu_index *idx, const uint64_t *d_key,
                            const uint8_t *d_has_key, const uint8_t *d_valid,
                            const uint32_t *d_rank, uint32_t first_rank, uint64_t n,
                            uint32_t chunk_rows, uint32_t *d_who, uint32_t *d_obj,
                            uint32_t *d_counts, void *stream);

/* ---- downstream consumers of the grouping ---------------
 * Orphan remover (core/src/object/orphan_remover.rs:57-90: Objects with no
 * file_path, `object::file_paths::none`, deleted 512 at a time): d_orphans
 * receives the ids of d_object_ids that no entry of d_fp_object_ids (a
 * file_path's object_id; negative = NULL) references, in list order;
 * d_count[0] = how many.  Object ids must lie in [0, max_object_id]; the
 * context keeps a workspace of max_object_id + 1 bytes (a mark per id). */
int sdgpu_orphan_objects_device(sdgpu_ctx *ctx, const int32_t *d_object_ids, uint64_t n_objects,
                                const int32_t *d_fp_object_ids, uint64_t n_file_paths,
                                uint32_t max_object_id, int32_t *d_orphans, uint32_t *d_count,
                                void *stream);
/* Thumbnail shards (core/src/object/media/thumbnail/shard.rs:4-8: directory =
 * cas_id[0..2] = the first digest byte): d_order = the rows (d_valid[i] != 0,
 * or all when NULL) ordered by shard directory, stable within a directory;
 * d_counts[256] = rows per directory. */
int sdgpu_thumbnail_shards_device(sdgpu_ctx *ctx, const uint8_t *d_cas8, const uint8_t *d_valid,
                                  uint64_t n, uint32_t *d_order, uint32_t *d_counts, void *stream);

/* ---- synthetic corpora (bench / tests; same content function as oracle/) ---- */
int sdgpu_synth_cas_arena_device(sdgpu_ctx *ctx, const uint64_t *d_sizes, const uint64_t *d_seeds,
                                 const uint64_t *d_off, uint32_t n, uint8_t *d_arena, void *stream);
int sdgpu_synth_file_device(sdgpu_ctx *ctx, uint64_t seed, uint64_t offset, uint64_t len,
                            uint8_t *d_out, void *stream);
/* Dedup corpus (BASELINE config 4 shape): global rows [first_rank, first_rank+n)
 * of a table of total_rows rows whose keys are a random permutation of
 * `distinct` distinct keys plus (total_rows - distinct) duplicates of them;
 * one row in 1000 has no key.  Writes key, has_key and rank (= global row). */
int sdgpu_synth_dedup_rows_device(sdgpu_ctx *ctx, uint64_t seed, uint64_t total_rows,
                                  uint64_t distinct, uint64_t first_rank, uint64_t n,
                                  uint64_t *d_key, uint8_t *d_has_key, uint32_t *d_rank,
                                  void *stream);

/* Config-5 run (bench): step `step` of a run over one pinned pool of files --
 * rows with d_vary[i] != 0 stand for files with new content (key' =
 * mix64(key ^ step * 0x9E3779B97F4A7C15), a bijection); the others are the
 * same files in every step.  step 0 leaves every key unchanged. */
int sdgpu_synth_vary_keys_device(sdgpu_ctx *ctx, uint64_t *d_key, const uint8_t *d_vary,
                                 uint64_t n, uint64_t step, void *stream);

/* ---- instrumentation (bench / profiling) ---------------------------------------
 * With timing enabled every main kernel launched through ctx is bracketed by
 * HIP events on its own stream; sdgpu_timing_read returns, per kernel name
 * (e.g. "cas_chunks", "tree_leaves", "bucket_group"), the accumulated device
 * milliseconds and launch count (-ENOENT past the last entry). */
int sdgpu_set_timing(sdgpu_ctx *ctx, int enable);
int sdgpu_timing_reset(sdgpu_ctx *ctx);
int sdgpu_timing_read(sdgpu_ctx *ctx, uint32_t idx, char name[32], double *total_ms,
                      uint64_t *launches);
/* Measured int32 VALU issue rate (lane-ops/s) of a BLAKE3-G-shaped
 * add3/xor/alignbit stream at full occupancy: the VALU roofline's peak. */
int sdgpu_valu_probe(sdgpu_ctx *ctx, double *lane_ops_per_s);
/* Same for one instruction class: 0 the G mix above, 1 v_xor_b32, 2 v_add3_u32,
 * 3 v_alignbit_b32, 4 v_add_u32; 5 = whole BLAKE3 compressions with everything
 * in registers (680 VALU each): the attainable roof of K1/K2's stream. */
int sdgpu_valu_probe_kind(sdgpu_ctx *ctx, int kind, double *lane_ops_per_s);
/* Latency breakdown of the last service request (sdgpu_latency_service) in
 * microseconds: [0] message copied into LDS, [1] hashed and digest written
 * (device wall clock), [2] host: post -> answer seen, [3] host: the file read
 * (the last two for sdgpu_generate_cas_id). */
int sdgpu_latency_service_diag(sdgpu_ctx *ctx, double out_us[4]);

#ifdef __cplusplus
}
#endif

#endif /* SDGPU_H */
