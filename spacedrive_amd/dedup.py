"""cas_id -> Object grouping (K4-K6), one GPU or sharded over a node.

Replaces the grouping half of identifier_job_step
(/root/reference/core/src/object/file_identifier/mod.rs:136-333) with the
canonical rule of SURVEY.md §8 a6 (see include/sdgpu.h, sdgpu_dedup):
rep[r] = r for rows without a key and for rows in the chunk of their key's
lowest-rank row f; rep[r] = f otherwise.

Multi-GPU: rows are hash-partitioned by the top 8 bits of mix64(key) (256
shards, shard s owned by rank s*W//256), exchanged by all-to-all of (key,
rank), grouped locally (the chunk rule only needs the global rank carried in
the payload) and the representatives return with a second all-to-all.  The
product path runs the whole exchange inside libsdgpu over RCCL
(group_sharded / group_sharded_all / dedup_sharded: sdgpu_group_sharded_*),
callable from the Rust host.  `sharded_group_reps` below is the same
algorithm over a pluggable exchange (torch.distributed, gloo in the CPU tests)
built from libsdgpu's single steps.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._native import check, default_context

CHUNK_SIZE = 100  # file_identifier/mod.rs:36


def group_reps(key, has_key, chunk_rows: int = CHUNK_SIZE, ctx=None) -> np.ndarray:
    """rep (uint32, ranks) for rows in rank order; host arrays, one GPU."""
    ctx = ctx or default_context()
    key = np.ascontiguousarray(key, np.uint64)
    has_key = np.ascontiguousarray(has_key, np.uint8)
    rep = np.zeros(key.size, np.uint32)
    check(ctx.lib.sdgpu_dedup(ctx.h, key.ctypes.data, has_key.ctypes.data, key.size, chunk_rows,
                              rep.ctypes.data), "sdgpu_dedup")
    return rep


class HipOps:
    """Local steps of the sharded dedup on device tensors (libsdgpu kernels)."""

    def __init__(self, ctx=None):
        self.ctx = ctx

    def _c(self, t):
        return self.ctx or default_context(t.device.index)

    @staticmethod
    def _s(t):
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    def shard_counts(self, key, has_key, shard_bits: int) -> np.ndarray:
        import ctypes
        ctx = self._c(key)
        counts = (ctypes.c_uint64 * (1 << shard_bits))()
        check(ctx.lib.sdgpu_shard_count_device(ctx.h, key.data_ptr(), has_key.data_ptr(),
                                               key.numel(), shard_bits, counts, self._s(key)),
              "sdgpu_shard_count_device")
        return np.array(counts[:], dtype=np.int64)

    def partition(self, key, has_key, rank, shard_bits: int, total: int):
        import torch
        ctx = self._c(key)
        okey = torch.empty(total, dtype=torch.int64, device=key.device)
        orank = torch.empty(total, dtype=torch.int32, device=key.device)
        opos = torch.empty(total, dtype=torch.int32, device=key.device)
        check(ctx.lib.sdgpu_shard_partition_device(
            ctx.h, key.data_ptr(), has_key.data_ptr(), rank.data_ptr() if rank is not None else None,
            key.numel(), shard_bits, okey.data_ptr(), orank.data_ptr(), opos.data_ptr(),
            self._s(key)), "sdgpu_shard_partition_device")
        return okey, orank, opos

    def exchange_partition(self, key, has_key, rank, shard_bits: int, world: int):
        """Send side in one pass, no host sync: rows packed by destination rank
        (n-row buffers, keyless rows dropped) + int64 rows per destination on
        the device (sdgpu_shard_exchange_device)."""
        import torch
        ctx = self._c(key)
        n = key.numel()
        okey = torch.empty(max(n, 1), dtype=torch.int64, device=key.device)
        orank = torch.empty(max(n, 1), dtype=torch.int32, device=key.device)
        opos = torch.empty(max(n, 1), dtype=torch.int32, device=key.device)
        dest = torch.empty(world, dtype=torch.int64, device=key.device)
        check(ctx.lib.sdgpu_shard_exchange_device(
            ctx.h, key.data_ptr(), has_key.data_ptr(), rank.data_ptr() if rank is not None else None,
            n, shard_bits, world, okey.data_ptr(), orank.data_ptr(), opos.data_ptr(),
            dest.data_ptr(), self._s(key)), "sdgpu_shard_exchange_device")
        return okey, orank, opos, dest

    def group(self, key, rank, chunk_rows: int, skip_bits: int):
        import torch
        ctx = self._c(key)
        rep = torch.empty(key.numel(), dtype=torch.int32, device=key.device)
        if key.numel():
            check(ctx.lib.sdgpu_group_pairs_device(ctx.h, key.data_ptr(), rank.data_ptr(),
                                                   key.numel(), chunk_rows, skip_bits,
                                                   rep.data_ptr(), self._s(key)),
                  "sdgpu_group_pairs_device")
        return rep

    def group_rows(self, key, has_key, rank, chunk_rows: int, skip_bits: int):
        """rep for every row (rows without a key keep their own rank)."""
        import torch
        ctx = self._c(key)
        rep = torch.empty(key.numel(), dtype=torch.int32, device=key.device)
        if key.numel():
            check(ctx.lib.sdgpu_group_rows_device(
                ctx.h, key.data_ptr(), has_key.data_ptr() if has_key is not None else None,
                rank.data_ptr() if rank is not None else None, key.numel(), chunk_rows,
                skip_bits, rep.data_ptr(), self._s(key)), "sdgpu_group_rows_device")
        return rep

    def scatter(self, src, pos, n: int, init):
        import torch
        ctx = self._c(src)
        out = torch.empty(n, dtype=torch.int32, device=src.device)
        check(ctx.lib.sdgpu_scatter_rep_device(
            ctx.h, src.data_ptr(), pos.data_ptr(), src.numel(), out.data_ptr(), n,
            init.data_ptr() if init is not None else None, 1, self._s(src)),
            "sdgpu_scatter_rep_device")
        return out


def shard_plan(world: int):
    """(shard_bits, owner-of-shard array, skip_bits) for `world` ranks.  Shards
    are the top 8 bits of mix64(key) (shard_of); skip_bits is kept for the ABI
    and unused (bucket digits are hash bits below the shard byte)."""
    if world <= 1:
        return 0, np.zeros(1, np.int64), 0
    bits = 8
    owner = (np.arange(1 << bits, dtype=np.int64) * world) >> bits
    return bits, owner, 0


class TorchDistExchange:
    """The exchange of the sharded grouping over torch.distributed (RCCL on
    ROCm, gloo in the CPU tests)."""

    def __init__(self, group=None):
        self.group = group

    def world_size(self) -> int:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group)
        return 1

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        import torch.distributed as dist
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)


def sharded_group_reps(key, has_key, rank, chunk_rows: int = CHUNK_SIZE, group=None, ops=None,
                       timings: dict | None = None, exchange=None):
    """Grouping of this rank's rows against the rows of every rank in `group`.

    key: int64 tensor (u64 cas keys), has_key: uint8, rank: int32 (global
    ranks, u32).  Returns int32 rep (global ranks) for this rank's rows.
    Collective: every rank of `group` must call it.  `exchange` replaces the
    torch.distributed all-to-alls (default TorchDistExchange(group))."""
    import torch
    ops = ops or HipOps()
    exchange = exchange or TorchDistExchange(group)
    world = exchange.world_size()
    n = key.numel()
    if world == 1:  # no exchange: group the rows in place (no compaction pass)
        return ops.group_rows(key, has_key, rank, chunk_rows, 0)
    bits, owner, skip = shard_plan(world)
    # partition + per-destination counts on the device, counts exchanged
    # device to device: the step's ONE host synchronisation is the read of the
    # send and receive counts that size the payload all-to-alls
    skey, srank, spos, sc = ops.exchange_partition(key, has_key, rank, bits, world)
    dev = key.device
    rc = torch.empty_like(sc)
    exchange.all_to_all(rc, sc)
    both = torch.cat([sc, rc]).cpu().numpy().astype(np.int64)
    s_list, r_list = both[:world].tolist(), both[world:].tolist()
    total, m = int(sum(s_list)), int(sum(r_list))
    if timings is not None:  # exchange volume of this call (payload bytes sent / received)
        timings["sent_rows"] = total
        timings["recv_rows"] = m
    skey, srank, spos = skey[:total], srank[:total], spos[:total]
    rkey = torch.empty(m, dtype=torch.int64, device=dev)
    rrank = torch.empty(m, dtype=torch.int32, device=dev)
    exchange.all_to_all(rkey, skey, r_list, s_list)
    exchange.all_to_all(rrank, srank, r_list, s_list)
    rrep = ops.group(rkey, rrank, chunk_rows, skip)
    rep_sent = torch.empty(total, dtype=torch.int32, device=dev)
    exchange.all_to_all(rep_sent, rrep, s_list, r_list)
    return ops.scatter(rep_sent, spos, n, rank)


# ---- Object index (objects that exist before a batch) -------------------------

REP_EXISTING = 0x80000000  # include/sdgpu.h SDGPU_REP_EXISTING


class ObjectIndex:
    """Device hash table of cas key -> Object (sdgpu_index_*): the library-wide
    lookup of identifier_job_step (file_identifier/mod.rs:168-185).  Values are
    ranks of rows that created an Object in an earlier batch of the run, or
    REP_EXISTING | handle for Objects registered with add_objects."""

    def __init__(self, ctx=None, capacity: int = 1 << 20):
        import ctypes
        self.ctx = ctx or default_context()
        h = ctypes.c_void_p()
        check(self.ctx.lib.sdgpu_index_create(self.ctx.h, capacity, ctypes.byref(h)),
              "sdgpu_index_create")
        self.h = h
        self.ctx.adopt(self)

    def close(self):
        if self.h:
            self.ctx.lib.sdgpu_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def count(self) -> int:
        import ctypes
        c = ctypes.c_uint64()
        check(self.ctx.lib.sdgpu_index_count(self.h, ctypes.byref(c)), "sdgpu_index_count")
        return c.value

    def clear(self, stream=None):
        check(self.ctx.lib.sdgpu_index_clear(self.h, stream), "sdgpu_index_clear")

    def add_objects(self, key, handle, world: int = 1, rank: int = 0):
        """Pre-existing Objects (device tensors: int64 keys, int32 handles <
        2^31); with world > 1 only this rank's shards are kept."""
        import torch
        s = torch.cuda.current_stream(key.device).cuda_stream
        check(self.ctx.lib.sdgpu_index_add_objects_device(
            self.h, key.data_ptr(), handle.data_ptr(), key.numel(), world, rank, s),
            "sdgpu_index_add_objects_device")


def group_rows_indexed(key, has_key, rank, index: ObjectIndex, chunk_rows: int = CHUNK_SIZE):
    """rep (int32, device) of one batch of rows against `index`, which then
    also holds the batch's new Objects (sdgpu_group_rows_indexed_device)."""
    import torch
    ctx = index.ctx
    rep = torch.empty(key.numel(), dtype=torch.int32, device=key.device)
    s = torch.cuda.current_stream(key.device).cuda_stream
    check(ctx.lib.sdgpu_group_rows_indexed_device(
        ctx.h, index.h, key.data_ptr(), has_key.data_ptr() if has_key is not None else None,
        rank.data_ptr() if rank is not None else None, key.numel(), chunk_rows, rep.data_ptr(), s),
        "sdgpu_group_rows_indexed_device")
    return rep


def dedup_batch(key, has_key, first_rank: int, index: ObjectIndex | None = None,
                chunk_rows: int = CHUNK_SIZE, ctx=None) -> np.ndarray:
    """Host arrays: rep of one batch (ranks first_rank + i) via sdgpu_dedup_batch."""
    ctx = ctx or (index.ctx if index is not None else default_context())
    key = np.ascontiguousarray(key, np.uint64)
    has_key = np.ascontiguousarray(has_key, np.uint8)
    rep = np.zeros(key.size, np.uint32)
    check(ctx.lib.sdgpu_dedup_batch(ctx.h, index.h if index is not None else None,
                                    key.ctypes.data, has_key.ctypes.data, first_rank, key.size,
                                    chunk_rows, rep.ctypes.data), "sdgpu_dedup_batch")
    return rep


# ---- multi-GPU grouping inside libsdgpu (RCCL / peer transport) -----------------

TRANSPORT_AUTO, TRANSPORT_RCCL, TRANSPORT_PEER, TRANSPORT_HOST = 0, 1, 2, 3


RETURN_FULL, RETURN_COMPACT, RETURN_AUTO = 0, 1, 2  # SDGPU_RETURN_*
EXCHANGE_AUTO, EXCHANGE_COUNTED, EXCHANGE_PADDED = 0, 1, 2  # SDGPU_EXCHANGE_*


class CommStats(ctypes.Structure):
    """sdgpu_comm_stats_t (include/sdgpu.h)."""
    _fields_ = [("calls", ctypes.c_uint64), ("rows_sent", ctypes.c_uint64),
                ("rows_received", ctypes.c_uint64), ("bytes_sent", ctypes.c_uint64),
                ("bytes_received", ctypes.c_uint64), ("bytes_remote", ctypes.c_uint64),
                ("count_wait_ms", ctypes.c_double), ("host_ms", ctypes.c_double),
                ("rows_returned", ctypes.c_uint64), ("padded_calls", ctypes.c_uint64),
                ("overflow_reruns", ctypes.c_uint64), ("resolve_wait_ms", ctypes.c_double),
                ("agreements", ctypes.c_uint64), ("nospc_call", ctypes.c_uint64)]


class Comm:
    """A libsdgpu communicator (sdgpu_comm_*)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle
        self._hold = None  # an unresolved padded call's tensors (_held)
        ctx.adopt(self)

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        buf = (ctypes.c_uint8 * 128)()
        check(default_context().lib.sdgpu_comm_unique_id(buf), "sdgpu_comm_unique_id")
        return bytes(buf)

    @classmethod
    def init_rank(cls, ctx, nranks: int, rank: int, uid: bytes,
                  timeout_ms: int | None = None) -> "Comm":
        """One process per GPU (RCCL): every rank joins with rank 0's id.
        Raises SdgpuError(-ETIMEDOUT) when not every rank joins within
        timeout_ms (None: SDGPU_COMM_TIMEOUT_MS or 300 s), which also bounds
        every later exchange of the communicator."""
        import ctypes
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        if timeout_ms is None:
            check(ctx.lib.sdgpu_comm_init_rank(ctx.h, nranks, rank, buf, ctypes.byref(h)),
                  "sdgpu_comm_init_rank")
        else:
            check(ctx.lib.sdgpu_comm_init_rank_timeout(ctx.h, nranks, rank, buf, int(timeout_ms),
                                                       ctypes.byref(h)),
                  "sdgpu_comm_init_rank_timeout")
        return cls(ctx, h)

    @classmethod
    def init_host(cls, ctx, nranks: int, rank: int, path: str, msg_bytes: int = 64 << 20,
                  timeout_ms: int = 60000) -> "Comm":
        """One process per rank on one host, through a shared file mapping
        (sdgpu_comm_init_host, ABI 6): the per-process exchange of the RCCL
        transport, host-staged, for ranks that share a GPU.  path: a fresh
        file name every rank passes; msg_bytes: one rank's messages of one
        all-to-all round."""
        h = ctypes.c_void_p()
        check(ctx.lib.sdgpu_comm_init_host(ctx.h, nranks, rank, os.fsencode(path), int(msg_bytes),
                                           int(timeout_ms), ctypes.byref(h)),
              "sdgpu_comm_init_host")
        return cls(ctx, h)

    def set_timeout(self, timeout_ms: int):
        check(self.ctx.lib.sdgpu_comm_set_timeout(self.h, int(timeout_ms)),
              "sdgpu_comm_set_timeout")

    def wait(self, stream=None):
        """Bounded wait for the last exchange's stream, resolving a padded
        call (re-run counted on an overflow; its -ENOSPC raised here)
        (sdgpu_comm_wait)."""
        check(self.ctx.lib.sdgpu_comm_wait(self.h, stream), "sdgpu_comm_wait")
        self._hold = None  # the resolved call's tensors (see _held)

    def set_return(self, mode: int):
        """SDGPU_RETURN_COMPACT (only the linked rows' reps travel back, one
        more count exchange), SDGPU_RETURN_FULL (4 B per row) or
        SDGPU_RETURN_AUTO (the default: compact for large calls, sdgpu.h)."""
        check(self.ctx.lib.sdgpu_comm_set_return(self.h, mode), "sdgpu_comm_set_return")

    def set_exchange(self, mode: int, rows_hint: int = 0):
        """SDGPU_EXCHANGE_PADDED (fixed-capacity messages, no host
        synchronisation; an overflowed call is re-run counted when resolved),
        SDGPU_EXCHANGE_COUNTED or SDGPU_EXCHANGE_AUTO (the default: padded
        once the ranks' row count is known).  rows_hint > 0 sets that count
        (every rank alike)."""
        check(self.ctx.lib.sdgpu_comm_set_exchange(self.h, mode, int(rows_hint)),
              "sdgpu_comm_set_exchange")

    def stats(self) -> dict:
        """Cumulative exchange volume / host time of this rank (sdgpu_comm_stats)."""
        st = CommStats()
        check(self.ctx.lib.sdgpu_comm_stats(self.h, ctypes.byref(st)), "sdgpu_comm_stats")
        return {f: getattr(st, f) for f, _ in CommStats._fields_}

    @classmethod
    def init_all(cls, ctxs, transport: int = TRANSPORT_AUTO) -> list:
        import ctypes
        n = len(ctxs)
        arr = (ctypes.c_void_p * n)(*[c.h.value for c in ctxs])
        out = (ctypes.c_void_p * n)()
        check(ctxs[0].lib.sdgpu_comm_init_all(arr, n, transport, out), "sdgpu_comm_init_all")
        return [cls(ctxs[i], ctypes.c_void_p(out[i])) for i in range(n)]

    def info(self):
        import ctypes
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.ctx.lib.sdgpu_comm_info(self.h, ctypes.byref(a), ctypes.byref(b),
                                           ctypes.byref(c)), "sdgpu_comm_info")
        return a.value, b.value, c.value

    def close(self):
        if self.h:
            self.ctx.lib.sdgpu_comm_destroy(self.h)
            self.h = None
        self._hold = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _held(comm: Comm, tensors):
    """Keeps an unresolved padded call's tensors alive until the call is
    resolved (sdgpu.h: until then its inputs must not change, and an overflow
    re-run, enqueued by the next exchange call or Comm.wait(), still reads and
    writes them): held on the communicator until the next call or wait."""
    comm._hold = tensors


def group_sharded(key, has_key, rank, comm: Comm, index: ObjectIndex | None = None,
                  chunk_rows: int = CHUNK_SIZE, out=None, wait: bool = True):
    """This rank's rep (int32, device) of the grouping over all ranks of `comm`
    (collective; sdgpu_group_sharded_device: RCCL all-to-all inside libsdgpu).
    wait=True resolves the call before returning (sdgpu_comm_wait: a padded
    exchange that overflowed is re-run counted); wait=False leaves it to the
    next exchange call or Comm.wait() -- rep is final only then."""
    import torch
    ctx = comm.ctx
    rep = out if out is not None else torch.empty(key.numel(), dtype=torch.int32,
                                                  device=key.device)
    s = torch.cuda.current_stream(key.device).cuda_stream
    check(ctx.lib.sdgpu_group_sharded_device(
        ctx.h, comm.h, index.h if index is not None else None, key.data_ptr(),
        has_key.data_ptr() if has_key is not None else None, rank.data_ptr(), key.numel(),
        chunk_rows, rep.data_ptr(), s), "sdgpu_group_sharded_device")
    _held(comm, (key, has_key, rank, rep, index))
    if wait:
        comm.wait(s)
    return rep


def group_sharded_all(keys, hass, ranks, comms, indexes=None, chunk_rows: int = CHUNK_SIZE):
    """All ranks from one process (sdgpu_group_sharded_all_device): lists of
    device tensors per rank -> list of int32 reps."""
    import ctypes
    import torch
    W = len(keys)
    vp = ctypes.c_void_p
    reps = [torch.empty(k.numel(), dtype=torch.int32, device=k.device) for k in keys]
    arr = lambda xs: (vp * W)(*xs)  # noqa: E731
    ctxs = [c.ctx for c in comms]
    n = (ctypes.c_uint64 * W)(*[k.numel() for k in keys])
    check(ctxs[0].lib.sdgpu_group_sharded_all_device(
        arr([c.h.value for c in ctxs]), arr([c.h.value for c in comms]),
        arr([i.h.value for i in indexes]) if indexes else None, W,
        arr([k.data_ptr() for k in keys]),
        arr([h.data_ptr() if h is not None else None for h in hass]) if hass else None,
        arr([r.data_ptr() for r in ranks]), n, chunk_rows, arr([r.data_ptr() for r in reps]),
        arr([torch.cuda.current_stream(k.device).cuda_stream for k in keys])),
        "sdgpu_group_sharded_all_device")
    return reps


def dedup_sharded(ctxs, key, has_key, chunk_rows: int = CHUNK_SIZE) -> np.ndarray:
    """SURVEY §8(b)'s sdgpu_dedup(ctx[], ngpu, ...) on host arrays."""
    import ctypes
    key = np.ascontiguousarray(key, np.uint64)
    has_key = np.ascontiguousarray(has_key, np.uint8)
    rep = np.zeros(key.size, np.uint32)
    arr = (ctypes.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    check(ctxs[0].lib.sdgpu_dedup_sharded(arr, len(ctxs), key.ctypes.data, has_key.ctypes.data,
                                          key.size, chunk_rows, rep.ctypes.data),
          "sdgpu_dedup_sharded")
    return rep


def shard_of(key: np.ndarray, bits: int = 8) -> np.ndarray:
    """Shard of cas keys: top `bits` bits of mix64(key) (csrc/rows_device.hpp)."""
    z = np.asarray(key, np.uint64).copy()
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(64 - bits)).astype(np.int64)


def link_batch_device(rep, rank=None, valid=None, first_rank: int = 0, ctx=None,
                      trim: bool = True):
    """K7 (sdgpu_link_batch_device): the Object write set of a batch of rows.

    rep int32 (u32 ranks), rank int32 or None (= first_rank + i), valid uint8 or
    None.  Returns device tensors (create, link_row, link_obj) trimmed to their
    counts: creator ranks (object::create_many, file_identifier/mod.rs:243-297)
    and (row, creator) connect pairs (mod.rs:189-225), both in row order.
    trim=False skips the host read of the counts (no synchronisation) and
    returns the full-length lists plus the device counts tensor [C, L]."""
    import torch
    dev = rep.device
    ctx = ctx or default_context(dev.index)
    n = rep.numel()
    create = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    lrow = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    lobj = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    # no fill kernel: the K7 scans write both counts (a null-stream fill here would
    # order the host behind the whole queued step on the context stream)
    counts = torch.empty(2, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_link_batch_device(
        ctx.h, rep.data_ptr(), rank.data_ptr() if rank is not None else None,
        valid.data_ptr() if valid is not None else None, first_rank, n, create.data_ptr(),
        lrow.data_ptr(), lobj.data_ptr(), counts.data_ptr(), s), "sdgpu_link_batch_device")
    if not trim:
        return create, lrow, lobj, counts
    c, l = (int(x) for x in counts.cpu().tolist())
    return create[:c], lrow[:l], lobj[:l]


LINKED = 0x80000000  # SDGPU_LINKED: the entry's row connects to an Object


def group_link_device(key, has_key=None, valid=None, rank=None, first_rank: int = 0,
                      chunk_rows: int = 100, ctx=None, trim: bool = True, index=None):
    """Fused grouping + Object write set (sdgpu_group_link_device, ABI 4):
    what group_rows + link_batch_device compute, without a rep array.

    key int64 (u64 cas keys), has_key / valid uint8 or None, rank int32 or None
    (= first_rank + i).  Returns device tensors (who, obj) trimmed to the
    entry count and the host counts (creators, linked): who[e] = rank (a new
    Object, file_identifier/mod.rs:243-297) or rank | LINKED (connects to the
    Object of creator rank obj[e], mod.rs:189-225); bucket order, not row
    order (a set).  trim=False: full-length tensors + the device counts [3],
    no synchronisation.  index: an ObjectIndex (rows whose cas_id already
    has an Object link to it: obj = REP_EXISTING | handle or the creator's
    rank from an earlier batch; this batch's creators are added)."""
    import torch
    dev = key.device
    ctx = ctx or default_context(dev.index)
    n = key.numel()
    who = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    obj = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(3, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    check(ctx.lib.sdgpu_group_link_device(ctx.h, index.h if index is not None else None,
                                          key.data_ptr(), ptr(has_key), ptr(valid), ptr(rank),
                                          first_rank, n, chunk_rows, who.data_ptr(),
                                          obj.data_ptr(), counts.data_ptr(), s),
          "sdgpu_group_link_device")
    if not trim:
        return who, obj, counts
    c, l, e = (int(x) for x in counts.cpu().tolist())
    return who[:e], obj[:e], (c, l)


def group_link_sharded(key, has_key, valid, rank, comm, chunk_rows: int = 100,
                       cap: int | None = None, trim: bool = True):
    """Sharded grouping + Object write set with no return leg
    (sdgpu_group_link_sharded_device): this rank's lists hold the entries of
    the keyed rows it OWNS (hash shard) and of its own valid keyless rows; the
    union over the ranks is the write set of all rows.  rank: int32 global
    ranks (required).  cap: list capacity (default nranks x n + n: enough
    when every row shares one cas_id and the ranks hold equal shares).
    Returns (who, obj, (c, l)) trimmed after resolving the call (Comm.wait:
    a padded exchange that overflowed is re-run counted, -ENOSPC raised), or
    full-length tensors + device counts with trim=False (final after the
    next exchange call or Comm.wait())."""
    import torch
    dev = key.device
    ctx = comm.ctx
    n = key.numel()
    nranks = comm.info()[0]
    cap = cap if cap is not None else max(1, nranks * n + n)
    who = torch.empty(cap, dtype=torch.int32, device=dev)
    obj = torch.empty(cap, dtype=torch.int32, device=dev)
    counts = torch.empty(3, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    check(ctx.lib.sdgpu_group_link_sharded_device(ctx.h, comm.h, key.data_ptr(), ptr(has_key),
                                                  ptr(valid), rank.data_ptr(), n, chunk_rows,
                                                  who.data_ptr(), obj.data_ptr(), cap,
                                                  counts.data_ptr(), s),
          "sdgpu_group_link_sharded_device")
    _held(comm, (key, has_key, valid, rank, who, obj, counts))
    if not trim:
        return who, obj, counts
    comm.wait(s)
    c, l, e = (int(x) for x in counts.cpu().tolist())
    return who[:e], obj[:e], (c, l)


def group_link_sharded_all(keys, hass, valids, ranks, comms, chunk_rows: int = 100):
    """All ranks from one process (sdgpu_group_link_sharded_all_device): lists
    of device tensors per rank -> [(who, obj, (c, l))] per rank, trimmed."""
    import ctypes
    import torch
    W = len(keys)
    vp = ctypes.c_void_p
    arr = lambda xs: (vp * W)(*xs)  # noqa: E731
    ctxs = [c.ctx for c in comms]
    n = [k.numel() for k in keys]
    caps = [max(1, sum(n) + m) for m in n]  # every keyed row may land on one owner
    whos = [torch.empty(c_, dtype=torch.int32, device=k.device) for c_, k in zip(caps, keys)]
    objs = [torch.empty(c_, dtype=torch.int32, device=k.device) for c_, k in zip(caps, keys)]
    cnts = [torch.empty(3, dtype=torch.int32, device=k.device) for k in keys]
    opt = lambda xs: arr([x.data_ptr() if x is not None else None for x in xs]) if xs else None  # noqa: E731
    check(ctxs[0].lib.sdgpu_group_link_sharded_all_device(
        arr([c.h.value for c in ctxs]), arr([c.h.value for c in comms]), W,
        arr([k.data_ptr() for k in keys]), opt(hass), opt(valids),
        arr([r.data_ptr() for r in ranks]), (ctypes.c_uint64 * W)(*n), chunk_rows,
        arr([w.data_ptr() for w in whos]), arr([o.data_ptr() for o in objs]),
        (ctypes.c_uint64 * W)(*caps), arr([c.data_ptr() for c in cnts]),
        arr([torch.cuda.current_stream(k.device).cuda_stream for k in keys])),
        "sdgpu_group_link_sharded_all_device")
    out = []
    for w, o, c in zip(whos, objs, cnts):
        cc, ll, e = (int(x) for x in c.cpu().tolist())
        out.append((w[:e], o[:e], (cc, ll)))
    return out


def split_link_lists(who: np.ndarray, obj: np.ndarray):
    """(create, link_row, link_obj) of a fused write set, each sorted by row
    rank: the same lists link_batch_device returns (row order), for comparing
    the two as sets."""
    w = np.asarray(who).view(np.uint32)
    o = np.asarray(obj).view(np.uint32)
    lk = (w & np.uint32(LINKED)) != 0
    create = np.sort(w[~lk])
    lr = w[lk] & np.uint32(LINKED - 1)
    order = np.argsort(lr, kind="stable")
    return create, lr[order], o[lk][order]


def object_stats(rep: np.ndarray, has_key: np.ndarray, ok: np.ndarray | None = None):
    """(created, linked) Object counts the reference's job would report
    (identifier_job_step returns (total_created, updated_file_paths.len()),
    mod.rs:335): a row whose rep is itself creates an Object; others link."""
    rep = np.asarray(rep, np.int64)
    r = np.arange(rep.size, dtype=np.int64)
    valid = np.ones(rep.size, bool) if ok is None else np.asarray(ok, bool)
    created = int(np.count_nonzero((rep == r) & valid))
    linked = int(np.count_nonzero((rep != r) & valid))
    return created, linked
