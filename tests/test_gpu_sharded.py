"""GPU parity: the multi-GPU grouping inside libsdgpu (sdgpu_dedup_sharded,
sdgpu_group_sharded_all_device, sdgpu_group_sharded_device) against the
oracle's whole-table grouping.  On the one-GPU test box every "GPU" is a
separate context on device 0 and the exchange takes the peer transport
(RCCL refuses two ranks on one device); the RCCL transport itself runs here
as a one-rank communicator (grouped self send/recv through the same code) and
on the driver's 8-GPU node through bench.py."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    from spacedrive_amd._native import Context
    cs = [Context(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("ngpu", [1, 2, 3, 8])
def test_dedup_sharded_host_api(ctxs, ngpu):
    """SURVEY §8(b)'s sdgpu_dedup(ctx[], ngpu, ...): bit-exact at 1/2/3/8."""
    from spacedrive_amd import dedup
    k, h, _ = O.synth_dedup_rows(21, 400_000, 280_000, 0, 400_000)
    k[::997] = np.uint64(2**64 - 1)
    for chunk in (100, 1):
        rep = dedup.dedup_sharded(ctxs[:ngpu], k, h, chunk)
        np.testing.assert_array_equal(rep, O.group_reps(k, h, chunk))


def test_dedup_sharded_two_level_per_rank(ctxs):
    """2 ranks x 13.5 M rows: every rank receives ~13.5 M exchanged 12-B
    records, so its local grouping takes the two-level partition with packed
    records as input."""
    from spacedrive_amd import dedup
    n = 27_000_000
    k, h, _ = O.synth_dedup_rows(31, n, int(n * 0.8), 0, n)
    rep = dedup.dedup_sharded(ctxs[:2], k, h, 100)
    np.testing.assert_array_equal(rep, O.group_reps(k, h, 100))


@pytest.mark.parametrize("world,mode", [(2, 1), (3, 1), (8, 1), (3, 0), (3, 2)])
def test_sharded_all_device_with_index_batches(ctxs, world, mode):
    """Device API over `world` ranks, two batches through per-rank Object
    indexes (each rank holds its shards' keys), plus pre-existing Objects
    registered on every rank: equals the oracle over the union."""
    import torch
    from spacedrive_amd import dedup
    total, batch = 300_000, 150_000
    k, h, _ = O.synth_dedup_rows(23, total, 180_000, 0, total)
    rng = np.random.default_rng(world)
    ek = rng.choice(k, 2000)
    eh = np.arange(ek.size, dtype=np.uint32) + 5
    comms = dedup.Comm.init_all(ctxs[:world])
    assert comms[0].info() == (world, 0, dedup.TRANSPORT_PEER)
    for c in comms:
        c.set_return(mode)  # compact (1) / full (0) / auto (2) return leg
    idxs = [dedup.ObjectIndex(c, 1000) for c in ctxs[:world]]
    for r, ix in enumerate(idxs):  # every rank gets the full list, keeps its share
        ix.add_objects(torch.from_numpy(ek.view(np.int64)).cuda(),
                       torch.from_numpy(eh.view(np.int32)).cuda(), world, r)
    torch.cuda.synchronize()
    assert sum(ix.count() for ix in idxs) == np.unique(ek).size
    out = np.zeros(total, np.uint32)
    for b0 in range(0, total, batch):
        keys, hass, ranks, spans = [], [], [], []
        for r in range(world):  # uneven per-rank shares
            a = b0 + batch * r // world
            b = b0 + batch * (r + 1) // world
            spans.append((a, b))
            keys.append(torch.from_numpy(k[a:b].view(np.int64)).cuda())
            hass.append(torch.from_numpy(h[a:b]).cuda())
            ranks.append(torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda())
        reps = dedup.group_sharded_all(keys, hass, ranks, comms, idxs, 100)
        torch.cuda.synchronize()
        for (a, b), rp in zip(spans, reps):
            out[a:b] = rp.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(out, O.group_reps_existing(k, h, 100, ek, eh))
    for c in comms:
        c.close()


def test_auto_return_takes_the_compact_leg_for_large_calls(ctxs):
    """SDGPU_RETURN_AUTO (the default): two ranks of 8.5 M rows each exceed
    4 Mi rows per peer, so every rank takes the compact leg (pairs for the
    linked rows only), decided from the n in the count messages; a second
    call with uneven shares (one rank 1 M rows, the other 8.5 M) takes it too
    -- the larger rank decides for both -- and a small call the full leg."""
    import torch
    from spacedrive_amd import dedup
    per = 8_500_000
    total = 2 * per
    k, h, _ = O.synth_dedup_rows(37, total, int(total * 0.8), 0, total)
    ref = O.group_reps(k, h, 100)
    comms = dedup.Comm.init_all(ctxs[:2])
    for c in comms:  # the counted exchange's return legs (a padded call returns in full)
        c.set_exchange(dedup.EXCHANGE_COUNTED)

    def run(bounds):
        keys, hass, ranks = [], [], []
        for a, b in bounds:
            keys.append(torch.from_numpy(k[a:b].view(np.int64)).cuda())
            hass.append(torch.from_numpy(h[a:b]).cuda())
            ranks.append(torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda())
        before = [c.stats() for c in comms]
        reps = dedup.group_sharded_all(keys, hass, ranks, comms, None, 100)
        torch.cuda.synchronize()
        for (a, b), rp in zip(bounds, reps):
            np.testing.assert_array_equal(rp.cpu().numpy().view(np.uint32), ref[a:b])
        after = [c.stats() for c in comms]
        return [{x: a_[x] - b_[x] for x in ("rows_received", "rows_returned", "bytes_sent")}
                for a_, b_ in zip(after, before)]

    for d in run([(0, per), (per, total)]):              # 8.5 M rows per rank: compact
        assert 0 < d["rows_returned"] < d["rows_received"] // 2
    for d in run([(0, 1_000_000), (1_000_000, total)]):  # the larger rank decides
        assert 0 < d["rows_returned"] < d["rows_received"] // 2
    for d in run([(0, 200_000), (200_000, 400_000)]):    # small: the full leg
        assert d["rows_returned"] == d["rows_received"]
    for c in comms:
        c.close()


def _lists_union(parts):
    from spacedrive_amd import dedup
    w = np.concatenate([p[0].cpu().numpy() for p in parts])
    o = np.concatenate([p[1].cpu().numpy() for p in parts])
    return dedup.split_link_lists(w, o), sum(p[2][0] for p in parts), sum(p[2][1] for p in parts)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_link_sharded_union_is_the_write_set(ctxs, world):
    """sdgpu_group_link_sharded_all_device (peer transport, all ranks in one
    process): each rank lists the rows it owns + its own keyless rows; the
    union over the ranks equals the oracle's link batch over the grouping of
    all rows, as sets -- uneven shares, keyless and invalid rows, a key
    repeated 40 k times (one owner gets all its rows).  Once through the
    counted exchange, once through the padded one (round 5), whose messages
    overflow on the 40 k-row key at 2 / 3 / 8 ranks and are re-run counted."""
    import torch
    from spacedrive_amd import dedup
    total = 400_000
    rng = np.random.default_rng(world + 40)
    pool = rng.integers(0, 2**64 - 1, 250_000, dtype=np.uint64, endpoint=True)
    k = pool[rng.integers(0, pool.size, total)]
    k[rng.choice(total, 40_000, replace=False)] = pool[3]
    valid = (rng.random(total) > 0.02).astype(np.uint8)
    h = ((rng.random(total) > 0.01) & (valid != 0)).astype(np.uint8)
    comms = dedup.Comm.init_all(ctxs[:world])
    keys, hass, vals, ranks = [], [], [], []
    for r in range(world):
        a, b = total * r * r // (world * world), total * (r + 1) * (r + 1) // (world * world)
        keys.append(torch.from_numpy(k[a:b].view(np.int64)).cuda())
        hass.append(torch.from_numpy(h[a:b]).cuda())
        vals.append(torch.from_numpy(valid[a:b]).cuda())
        ranks.append(torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda())
    rc, rlr, rlo = O.link_batch(O.group_reps(k, h, 100), None, valid, 0)
    for mode in (dedup.EXCHANGE_COUNTED, dedup.EXCHANGE_PADDED):
        for cm in comms:
            cm.set_exchange(mode, max(x.numel() for x in keys))
        before = [cm.stats() for cm in comms]
        parts = dedup.group_link_sharded_all(keys, hass, vals, ranks, comms, 100)
        (c, lr, lo), nc, nl = _lists_union(parts)
        assert (nc, nl) == (rc.size, rlr.size)
        np.testing.assert_array_equal(c, rc)
        np.testing.assert_array_equal(lr, rlr)
        np.testing.assert_array_equal(lo, rlo)
        for cm, b in zip(comms, before):
            st = cm.stats()
            d = {x: st[x] - b[x] for x in st}
            assert d["rows_returned"] == 0
            if mode == dedup.EXCHANGE_COUNTED:
                assert d["bytes_sent"] == 12 * d["rows_sent"] and d["padded_calls"] == 0
            else:
                assert d["padded_calls"] == 1
                assert d["overflow_reruns"] == (1 if world > 1 else 0)
    for cm in comms:
        cm.close()


def test_link_sharded_one_rank_rccl(ctx):
    """The write-set form through a one-rank RCCL communicator (the N > 1
    headline step's code path): equal to the oracle, counted (12 B per row on
    the wire) and padded (round 5: no count exchange, no host wait), and
    -ENOSPC for lists that do not fit -- from the call when counted, from
    Comm.wait() when padded (the list kernels write nothing past cap) --
    leaves the communicator usable."""
    import errno
    import torch
    from spacedrive_amd import dedup
    from spacedrive_amd._native import SdgpuError
    comm = dedup.Comm.init_rank(ctx, 1, 0, dedup.Comm.unique_id())
    n = 1_000_000
    k, h, rk = O.synth_dedup_rows(41, n, 800_000, 0, n)
    dk = torch.from_numpy(k.view(np.int64)).cuda()
    dh = torch.from_numpy(h).cuda()
    dr = torch.from_numpy(rk.view(np.int32)).cuda()
    rc, rlr, rlo = O.link_batch(O.group_reps(k, h, 100), None, None, 0)

    def check(who, obj, c, l):
        fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
        assert (c, l) == (rc.size, rlr.size)
        np.testing.assert_array_equal(fc, rc)
        np.testing.assert_array_equal(flr, rlr)
        np.testing.assert_array_equal(flo, rlo)

    for mode in (dedup.EXCHANGE_COUNTED, dedup.EXCHANGE_AUTO):
        comm.set_exchange(mode)
        s0 = comm.stats()
        for _ in range(2):
            who, obj, (c, l) = dedup.group_link_sharded(dk, dh, None, dr, comm, 100)
            check(who, obj, c, l)
        d = {x: comm.stats()[x] - s0[x] for x in s0}
        if mode == dedup.EXCHANGE_COUNTED:
            assert d["rows_returned"] == 0 and d["bytes_sent"] == 12 * d["rows_sent"]
        else:  # one rank: the message holds all n rows, header + 64-slot rounding
            assert d["padded_calls"] == 2 and d["overflow_reruns"] == 0
            assert d["count_wait_ms"] == 0
            assert d["bytes_sent"] == 2 * 12 * ((n + 1 + 63) // 64 * 64)
        with pytest.raises(SdgpuError) as e:
            dedup.group_link_sharded(dk, dh, None, dr, comm, 100, cap=1000)
        assert e.value.rc == -errno.ENOSPC
        who, obj, (c, l) = dedup.group_link_sharded(dk, dh, None, dr, comm, 100)
        check(who, obj, c, l)
    # trim=False calls back to back, resolved by the next call / wait
    comm.set_exchange(dedup.EXCHANGE_AUTO)
    outs = [dedup.group_link_sharded(dk, dh, None, dr, comm, 100, trim=False) for _ in range(3)]
    comm.wait()
    for who, obj, cnt in outs[-1:]:
        c, l, e = (int(x) for x in cnt.cpu().tolist())
        check(who[:e], obj[:e], c, l)
    # a padded message too small (B below this call's rows): overflow, re-run counted
    comm.set_exchange(dedup.EXCHANGE_PADDED, n // 2)
    s0 = comm.stats()
    who, obj, (c, l) = dedup.group_link_sharded(dk, dh, None, dr, comm, 100)
    check(who, obj, c, l)
    d = {x: comm.stats()[x] - s0[x] for x in s0}
    assert d["padded_calls"] == 1 and d["overflow_reruns"] == 1
    comm.close()


def test_rccl_transport_one_rank(ctx):
    """The RCCL code path on hardware: a one-rank communicator from
    sdgpu_comm_unique_id + sdgpu_comm_init_rank, the whole exchange through
    grouped ncclSend/ncclRecv to itself, repeated (workspace reuse) and with an
    Object index."""
    import torch
    from spacedrive_amd import dedup
    uid = dedup.Comm.unique_id()
    comm = dedup.Comm.init_rank(ctx, 1, 0, uid)
    assert comm.info() == (1, 0, dedup.TRANSPORT_RCCL)
    comm.set_exchange(dedup.EXCHANGE_COUNTED)  # the padded exchange: test_gpu_padded.py
    comm.set_return(dedup.RETURN_COMPACT)  # the default (AUTO) picks FULL at this size
    k, h, rk = O.synth_dedup_rows(29, 500_000, 400_000, 0, 500_000)
    dk = torch.from_numpy(k.view(np.int64)).cuda()
    dh = torch.from_numpy(h).cuda()
    dr = torch.from_numpy(rk.view(np.int32)).cuda()
    ref = O.group_reps(k, h, 100)
    for _ in range(3):
        rep = dedup.group_sharded(dk, dh, dr, comm, None, 100)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(rep.cpu().numpy().view(np.uint32), ref)
    idx = dedup.ObjectIndex(ctx)
    out = []
    for a, b in ((0, 200_000), (200_000, 500_000)):
        out.append(dedup.group_sharded(dk[a:b], dh[a:b], dr[a:b], comm, idx, 100).cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(out).view(np.uint32), ref)
    comm.wait()                       # bounded wait for the last exchange's stream
    st = comm.stats()
    keyed = int(h.sum())
    assert st["calls"] == 5
    assert st["rows_sent"] == st["rows_received"] == 4 * keyed   # 3 whole + 2 halves
    # compact return leg: 12-B records out,
    # 8-B {index, rep} pairs back for the linked rows only
    linked = int(np.count_nonzero(ref != np.arange(ref.size)))
    assert st["rows_returned"] == 4 * linked
    assert st["bytes_sent"] == 12 * st["rows_sent"] + 8 * st["rows_returned"]
    assert st["bytes_sent"] / st["rows_sent"] <= 14.0
    assert st["bytes_remote"] == 0    # one rank: every record is a self-send
    # the full return leg (4 B per row, one synchronisation): same reps
    comm.set_return(dedup.RETURN_FULL)
    rep = dedup.group_sharded(dk, dh, dr, comm, None, 100)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rep.cpu().numpy().view(np.uint32), ref)
    st2 = comm.stats()
    assert st2["bytes_sent"] - st["bytes_sent"] == 16 * keyed
    # AUTO (the default): 500 k rows on one rank is below the compact
    # threshold (4 Mi rows per rank), so the full leg runs
    comm.set_return(dedup.RETURN_AUTO)
    rep = dedup.group_sharded(dk, dh, dr, comm, None, 100)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rep.cpu().numpy().view(np.uint32), ref)
    st3 = comm.stats()
    assert st3["bytes_sent"] - st2["bytes_sent"] == 16 * keyed
    assert st3["rows_returned"] - st2["rows_returned"] == keyed
    comm.close()


_MISSING_PEER = r'''
import errno, json, sys, time
sys.path.insert(0, sys.argv[1])
import torch
from spacedrive_amd import dedup
from spacedrive_amd._native import Context, SdgpuError
ctx = Context(0)
uid = dedup.Comm.unique_id()
t0 = time.monotonic()
try:
    dedup.Comm.init_rank(ctx, 2, 0, uid, timeout_ms=int(sys.argv[2]))
    rc = 0
except SdgpuError as e:
    rc = e.rc
print(json.dumps({"rc": rc, "s": time.monotonic() - t0}), flush=True)
'''


def test_rccl_missing_peer_times_out():
    """a 2-rank communicator whose second rank never
    joins returns -ETIMEDOUT within the deadline instead of blocking forever
    (non-blocking ncclCommInitRankConfig polled, ncclCommAbort on expiry).
    Run in a fresh child process so an abort cannot disturb this one."""
    import errno
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _MISSING_PEER, root, "4000"], capture_output=True,
                       text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["rc"] == -errno.ETIMEDOUT, res
    assert 3.5 < res["s"] < 60, res


def test_config4_100m_rows_one_gpu_and_8_ranks(ctx, ctxs):
    """BASELINE config 4 at full size (100 M rows) grouped on ONE GPU (2^15
    buckets, every bucket in LDS) -- the strong-scaling base -- and as 8 ranks
    through sdgpu_group_sharded_all_device; both bit-exact vs the oracle."""
    import torch
    from spacedrive_amd import corpus, dedup
    total = 100_000_000
    key, has, rank = corpus.synth_dedup_rows_device(4, total, int(total * 0.8), 0, total, ctx=ctx)
    ops = dedup.HipOps(ctx)
    rep1 = ops.group_rows(key, has, rank, 100, 0)
    torch.cuda.synchronize()
    hk = key.cpu().numpy().view(np.uint64)
    hh = has.cpu().numpy()
    ref = O.group_reps(hk, hh, 100)
    np.testing.assert_array_equal(rep1.cpu().numpy().view(np.uint32), ref)
    del rep1
    # the variant bench.py times (config4_full_one_gpu): no rank array, so
    # 12-byte records through k_part_private -> k_part2_runs -> k_bucket_group12_pk
    # at 2^15 buckets
    rep0 = ops.group_rows(key, has, None, 100, 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rep0.cpu().numpy().view(np.uint32), ref)
    del rep0
    # the fused write set at full size (sdgpu_group_link_device, no rep array):
    # the oracle's link batch over the same grouping, as sets
    who, obj, (nc, nl) = dedup.group_link_device(key, has, None, None, 0, 100, ctx=ctx)
    fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
    del who, obj
    rc, rlr, rlo = O.link_batch(ref, None, None, 0)
    assert (nc, nl) == (rc.size, rlr.size)
    np.testing.assert_array_equal(fc, rc)  # rc is in row order: already sorted
    np.testing.assert_array_equal(flr, rlr)
    np.testing.assert_array_equal(flo, rlo)
    del fc, flr, flo, rc, rlr, rlo
    comms = dedup.Comm.init_all(ctxs)
    per = total // 8
    reps = dedup.group_sharded_all([key[r * per:(r + 1) * per] for r in range(8)],
                                   [has[r * per:(r + 1) * per] for r in range(8)],
                                   [rank[r * per:(r + 1) * per] for r in range(8)], comms)
    torch.cuda.synchronize()
    got = np.concatenate([x.cpu().numpy().view(np.uint32) for x in reps])
    np.testing.assert_array_equal(got, ref)
    for c in comms:
        c.close()
