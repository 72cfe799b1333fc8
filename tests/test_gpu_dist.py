"""GPU, multi-process: the sharded grouping with libsdgpu's own kernels in every
rank -- the destination partition (k_part_hist / k_part_scatter with the
packed 12-byte send records), the local grouping of the received rows and the
gather of the returned reps (spacedrive_amd.dedup.HipOps) -- exchanged by
torch.distributed all-to-alls over gloo between 2 and 3 processes sharing the
box's one GPU (RCCL refuses two ranks on one device; the RCCL transport is
covered by test_gpu_sharded.py).  tests/test_dist_dedup.py runs the same
exchange logic with numpy stand-ins on the CPU; here the steps are the
product's.  Checked against the oracle's whole-table grouping
(file_identifier/mod.rs:136-241, canonical rule)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


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
        from spacedrive_amd._native import default_context
        torch.cuda.set_device(0)
        ctx = default_context(0)
        per = total // world
        first = rank * per
        n = per if rank < world - 1 else total - first
        k, h, r = O.synth_dedup_rows(23, total, distinct, first, n)
        timings = {}
        rep = dedup.sharded_group_reps(torch.from_numpy(k.view(np.int64)).cuda(),
                                       torch.from_numpy(h).cuda(),
                                       torch.from_numpy(r.view(np.int32)).cuda(), 100,
                                       ops=dedup.HipOps(ctx), timings=timings)
        torch.cuda.synchronize()
        q.put((rank, rep.cpu().numpy().view(np.uint32).copy(), timings))
    except BaseException as e:  # reported to the parent, which fails the test
        q.put((rank, None, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_grouping_product_kernels_gloo(world):
    from oracle import oracle as O
    total, distinct = 400_000, 300_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, distinct, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    parts = {}
    for rank, rep, info in got:
        assert rep is not None, f"rank {rank}: {info}"
        parts[rank] = rep
        # every rank sent and received rows of the other ranks' shards
        assert info["sent_rows"] > 0 and info["recv_rows"] > 0
    for p in procs:
        assert p.exitcode == 0
    rep = np.concatenate([parts[r] for r in range(world)])
    k, h, _ = O.synth_dedup_rows(23, total, distinct, 0, total)
    np.testing.assert_array_equal(rep, O.group_reps(k, h, 100))
