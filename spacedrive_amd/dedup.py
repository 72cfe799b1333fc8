"""cas_id -> Object grouping (K4-K6), one GPU or sharded over a node.

Replaces the grouping half of identifier_job_step
(/root/reference/core/src/object/file_identifier/mod.rs:136-333) with the
canonical rule of SURVEY.md §8 a6 (see include/sdgpu.h, sdgpu_dedup):
rep[r] = r for rows without a key and for rows in the chunk of their key's
lowest-rank row f; rep[r] = f otherwise.

Multi-GPU (one process per GPU, torch.distributed over RCCL/xGMI): rows are
hash-partitioned by the top 8 bits of the cas key (256 shards, shard s owned
by rank s*W//256), exchanged by all-to-all of (key, rank), grouped locally
(the chunk rule only needs the global rank carried in the payload) and the
representatives return with a second all-to-all.  The exchange logic below is
backend-agnostic (`ops`), so it is tested with gloo on CPU; the product ops are
the HIP kernels of libsdgpu.
"""
from __future__ import annotations

import math

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
    """(shard_bits, owner-of-shard array, skip_bits) for `world` ranks."""
    if world <= 1:
        return 0, np.zeros(1, np.int64), 0
    bits = 8
    owner = (np.arange(1 << bits, dtype=np.int64) * world) >> bits
    skip = int(math.floor(math.log2(world)))
    return bits, owner, skip


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
