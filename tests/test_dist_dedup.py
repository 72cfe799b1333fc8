"""CPU, multi-process: the sharded dedup exchange (spacedrive_amd.dedup.
sharded_group_reps) over gloo with world sizes 2 and 3.  The local steps are
numpy stand-ins (the GPU runs libsdgpu's kernels through the same interface);
what is under test is the partition -> all-to-all -> group -> all-to-all back ->
scatter logic, checked against the oracle's whole-table grouping."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class NumpyOps:
    """CPU stand-ins with the HipOps interface (test-only)."""

    @staticmethod
    def _digit(k, bits):
        from spacedrive_amd.dedup import shard_of  # the product's shard function
        return shard_of(k, bits) if bits else np.zeros(k.size, np.int64)

    def shard_counts(self, key, has_key, bits):
        k = key.numpy().view(np.uint64)
        h = has_key.numpy().astype(bool)
        return np.bincount(self._digit(k[h], bits), minlength=1 << bits).astype(np.int64)

    def partition(self, key, has_key, rank, bits, total):
        k = key.numpy().view(np.uint64)
        idx = np.flatnonzero(has_key.numpy())
        order = np.argsort(self._digit(k[idx], bits), kind="stable")
        sel = idx[order]
        assert sel.size == total
        r = rank.numpy() if rank is not None else sel.astype(np.int32)
        return (torch.from_numpy(k[sel].view(np.int64).copy()),
                torch.from_numpy(np.ascontiguousarray(r[sel], np.int32)),
                torch.from_numpy(sel.astype(np.int32)))

    def exchange_partition(self, key, has_key, rank, bits, world):
        counts = self.shard_counts(key, has_key, bits)
        owner = (np.arange(1 << bits, dtype=np.int64) * world) >> bits
        dest = np.bincount(owner, weights=counts, minlength=world).astype(np.int64)
        okey, orank, opos = self.partition(key, has_key, rank, bits, int(dest.sum()))
        pad = key.numel() - okey.numel()  # n-row buffers, as the HIP op returns
        z64, z32 = torch.zeros(pad, dtype=torch.int64), torch.zeros(pad, dtype=torch.int32)
        return (torch.cat([okey, z64]), torch.cat([orank, z32]), torch.cat([opos, z32]),
                torch.from_numpy(dest))

    def group(self, key, rank, chunk_rows, skip):
        k = key.numpy().view(np.uint64)
        r = rank.numpy().view(np.uint32).astype(np.int64)
        rep = r.copy()
        if k.size:
            order = np.lexsort((r, k))
            ks = k[order]
            head = np.ones(ks.size, bool)
            head[1:] = ks[1:] != ks[:-1]
            seg = np.cumsum(head) - 1
            first = r[order][head][seg]
            rr = r[order]
            rep[order] = np.where(rr // chunk_rows == first // chunk_rows, rr, first)
        return torch.from_numpy(rep.astype(np.uint32).view(np.int32))

    def group_rows(self, key, has_key, rank, chunk_rows, skip):
        h = has_key.numpy().astype(bool)
        r = rank.numpy() if rank is not None else np.arange(key.numel(), dtype=np.int32)
        out = torch.from_numpy(np.ascontiguousarray(r, np.int32).copy())
        idx = np.flatnonzero(h)
        g = self.group(torch.from_numpy(key.numpy()[idx].copy()),
                       torch.from_numpy(np.ascontiguousarray(r[idx], np.int32)), chunk_rows, skip)
        out[torch.from_numpy(idx)] = g
        return out

    def scatter(self, src, pos, n, init):
        out = init.clone() if init is not None else torch.arange(n, dtype=torch.int32)
        out[pos.long()] = src
        return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, distinct, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from spacedrive_amd import dedup
        per = total // world
        first = rank * per
        n = per if rank < world - 1 else total - first
        k, h, r = O.synth_dedup_rows(11, total, distinct, first, n)
        rep = dedup.sharded_group_reps(torch.from_numpy(k.view(np.int64)),
                                       torch.from_numpy(h), torch.from_numpy(r.view(np.int32)),
                                       100, ops=NumpyOps())
        q.put((rank, rep.numpy().view(np.uint32).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dedup_gloo(world):
    from oracle import oracle as O
    total, distinct = 30_000, 20_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, distinct, q))
             for r in range(world)]
    for p in procs:
        p.start()
    parts = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rep = np.concatenate([parts[r] for r in range(world)])
    k, h, _ = O.synth_dedup_rows(11, total, distinct, 0, total)
    np.testing.assert_array_equal(rep, O.group_reps(k, h, 100))


def test_shard_plan_balanced():
    from spacedrive_amd.dedup import shard_plan
    for w in (2, 3, 4, 6, 8):
        bits, owner, skip = shard_plan(w)
        counts = np.bincount(owner, minlength=w)
        assert counts.min() >= 256 // w and counts.max() <= 256 // w + 1
        assert np.all(np.diff(owner) >= 0)  # contiguous shard ranges per rank
        assert (1 << skip) <= w


def test_single_process_path_matches_oracle():
    from oracle import oracle as O
    from spacedrive_amd import dedup
    k, h, r = O.synth_dedup_rows(5, 20_000, 15_000, 0, 20_000)
    rep = dedup.sharded_group_reps(torch.from_numpy(k.view(np.int64)), torch.from_numpy(h),
                                   torch.from_numpy(r.view(np.int32)), 100, ops=NumpyOps())
    np.testing.assert_array_equal(rep.numpy().view(np.uint32), O.group_reps(k, h, 100))
