"""GPU parity: K4-K6 grouping against the oracle's canonical rule."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_golden_grouping_fixture(ctx):
    from spacedrive_amd import dedup
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "grouping_10k.npz"))
    rep = dedup.group_reps(z["key"], z["has_key"], int(z["chunk_rows"][0]), ctx)
    np.testing.assert_array_equal(rep, z["rep"])


@pytest.mark.parametrize("n,pool", [(0, 1), (1, 1), (2, 1), (1000, 10), (200_000, 150_000),
                                    (1_000_000, 900_000), (300_000, 1), (500_000, 7)])
def test_random_vs_oracle(ctx, n, pool):
    """Includes buckets far beyond the LDS table (one key 300k times: the
    global-table path) and a sentinel-valued key."""
    from spacedrive_amd import dedup
    rng = np.random.default_rng(n + pool)
    keys = rng.integers(0, 2**64 - 1, max(pool, 1), dtype=np.uint64, endpoint=True)
    keys[0] = np.uint64(2**64 - 1)
    key = keys[rng.integers(0, keys.size, n)] if n else np.zeros(0, np.uint64)
    has = (rng.random(n) > 0.01).astype(np.uint8)
    for chunk in (100, 1, 7):
        rep = dedup.group_reps(key, has, chunk, ctx)
        np.testing.assert_array_equal(rep, O.group_reps(key, has, chunk))


def test_skip_bits_shard(ctx):
    """Keys of one shard of an 8-GPU partition (top 3 bits constant)."""
    import torch
    rng = np.random.default_rng(3)
    n = 400_000
    key = rng.integers(0, 2**61, n, dtype=np.uint64) | np.uint64(5 << 61)
    key[rng.integers(0, n, n // 5)] = key[rng.integers(0, n, n // 5)]
    rank = rng.permutation(n).astype(np.uint32)
    from spacedrive_amd import dedup
    ops = dedup.HipOps(ctx)
    dk = torch.from_numpy(key.view(np.int64)).cuda()
    dr = torch.from_numpy(rank.view(np.int32)).cuda()
    rep = ops.group(dk, dr, 100, 3).cpu().numpy().view(np.uint32)
    # oracle: rows in rank order
    order = np.argsort(rank)
    ref_rank_order = O.group_reps(key[order], np.ones(n, np.uint8), 100)
    np.testing.assert_array_equal(rep[order], ref_rank_order)


def test_config4_shape_single_gpu(ctx):
    """12.5 M rows of the config-4 table (one GPU's share at 8 GPUs)."""
    import torch
    from spacedrive_amd import corpus, dedup
    total = 12_500_000
    key, has, rank = corpus.synth_dedup_rows_device(4, total, int(total * 0.8), 0, total, ctx=ctx)
    rep = dedup.sharded_group_reps(key, has, rank, 100, ops=dedup.HipOps(ctx))
    torch.cuda.synchronize()
    hk = key.cpu().numpy().view(np.uint64)
    hh = has.cpu().numpy()
    k2, h2, _ = O.synth_dedup_rows(4, total, int(total * 0.8), 0, 200_000)
    np.testing.assert_array_equal(hk[:200_000], k2)
    np.testing.assert_array_equal(hh[:200_000], h2)
    np.testing.assert_array_equal(rep.cpu().numpy().view(np.uint32), O.group_reps(hk, hh, 100))


class ThreadExchange:
    """W 'ranks' as threads of one process on one GPU: all_to_all moves the
    device tensors between them through shared slots (a test stand-in for
    RCCL that exercises every HipOps step of the N > 1 path on the GPU)."""

    def __init__(self, rank, world, shared):
        self.rank, self.world, self.shared = rank, world, shared

    def world_size(self):
        return self.world

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        import torch
        W = self.world
        ins = in_splits or [inp.numel() // W] * W
        outs = out_splits or [out.numel() // W] * W
        torch.cuda.synchronize()
        self.shared["slots"][self.rank] = list(torch.split(inp, ins))
        self.shared["barrier"].wait()
        parts = [self.shared["slots"][src][self.rank] for src in range(W)]
        assert [p.numel() for p in parts] == outs
        torch.cat(parts, out=out) if out.numel() else None
        torch.cuda.synchronize()
        self.shared["barrier"].wait()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_path_all_hip_ops_on_gpu(ctx, world):
    """The N-GPU grouping (partition -> exchange -> group -> return ->
    scatter) with the HIP kernels, W ranks emulated in one process."""
    import threading
    import torch
    from spacedrive_amd import dedup
    total, distinct = 300_000, 200_000
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world)}
    results, errors = {}, []

    def run(r):
        try:
            per = total // world
            first = r * per
            n = per if r < world - 1 else total - first
            k, h, rk = O.synth_dedup_rows(11, total, distinct, first, n)
            rep = dedup.sharded_group_reps(
                torch.from_numpy(k.view(np.int64)).cuda(), torch.from_numpy(h).cuda(),
                torch.from_numpy(rk.view(np.int32)).cuda(), 100, ops=dedup.HipOps(ctx),
                exchange=ThreadExchange(r, world, shared))
            torch.cuda.synchronize()
            results[r] = rep.cpu().numpy().view(np.uint32)
        except Exception as e:  # surface thread failures
            errors.append(e)
            shared["barrier"].abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    rep = np.concatenate([results[r] for r in range(world)])
    k, h, _ = O.synth_dedup_rows(11, total, distinct, 0, total)
    np.testing.assert_array_equal(rep, O.group_reps(k, h, 100))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_exchange_partition_matches_count_and_partition(ctx, world):
    """sdgpu_shard_exchange_device (one pass, device counts) packs exactly what
    sdgpu_shard_count_device + sdgpu_shard_partition_device do."""
    import torch
    from spacedrive_amd import dedup
    k, h, rk = O.synth_dedup_rows(13, 500_000, 350_000, 0, 500_000)
    key = torch.from_numpy(k.view(np.int64)).cuda()
    has = torch.from_numpy(h).cuda()
    rank = torch.from_numpy(rk.view(np.int32)).cuda()
    ops = dedup.HipOps(ctx)
    bits, owner, _ = dedup.shard_plan(world)
    counts = ops.shard_counts(key, has, bits)
    dest_ref = np.bincount(owner, weights=counts, minlength=world).astype(np.int64)
    total = int(dest_ref.sum())
    rk_, rr_, rp_ = ops.partition(key, has, rank, bits, total)
    ok, orr, op, dest = ops.exchange_partition(key, has, rank, bits, world)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dest.cpu().numpy(), dest_ref)
    assert total == int(h.sum())
    # order inside a (shard, block) bucket is not fixed (LDS cursors): compare
    # each destination's segment as a set of source rows, and every packed
    # row against its source
    ok, orr, op = (t[:total].cpu().numpy() for t in (ok, orr, op))
    ref_pos = rp_.cpu().numpy()
    np.testing.assert_array_equal(ok.view(np.uint64), k[op])
    np.testing.assert_array_equal(orr.view(np.uint32), rk[op])
    bounds = np.concatenate([[0], np.cumsum(dest_ref)])
    for d in range(world):
        seg = slice(bounds[d], bounds[d + 1])
        np.testing.assert_array_equal(np.sort(op[seg]), np.sort(ref_pos[seg]))
        assert np.all(owner[dedup.shard_of(k[op[seg]], bits)] == d)


def _one_bucket_keys(rng, n, count):
    """`count` distinct random keys that all land in bucket 0 of an n-row
    grouping (bucket = the hash bits below the shard byte, csrc/dedup.hip
    bucket_bits_for / digit_of)."""
    from spacedrive_amd.dedup import shard_of
    bits = 1
    while bits < 15 and (n >> bits) > 3072:
        bits += 1
    out = []
    while sum(x.size for x in out) < count:
        k = rng.integers(0, 2**64 - 1, 1 << 20, dtype=np.uint64, endpoint=True)
        digit = shard_of(k, 8 + bits) & ((1 << bits) - 1)
        out.append(k[digit == 0])
    return np.unique(np.concatenate(out))[:count]


@pytest.mark.parametrize("n", [4607, 4608, 4609, 6144, 6145, 9000])
def test_single_bucket_at_lds_capacity(ctx, n):
    """Every key in one bucket: rows just under, at and over the LDS table's
    capacity (4608 rows of 6144 slots) take the LDS path or the global-table
    path, with ~30% duplicates (the all-ones key, the table's empty value, is
    checked by test_random_vs_oracle)."""
    from spacedrive_amd import dedup
    rng = np.random.default_rng(n)
    keys = _one_bucket_keys(rng, n, int(n * 0.7))
    key = keys[rng.integers(0, keys.size, n)]
    has = np.ones(n, np.uint8)  # every row in the bucket
    for chunk in (100, 1):
        rep = dedup.group_reps(key, has, chunk, ctx)
        np.testing.assert_array_equal(rep, O.group_reps(key, has, chunk))


@pytest.mark.timeout(400)
def test_config4_full_100m_rows_eight_ranks(ctx):
    """BASELINE config 4 at its full size: 100 M rows (80 M distinct keys, 20 M
    duplicates, 0.1 % keyless) as 8 ranks of 12.5 M rows, the whole N = 8
    sharded path (partition -> exchange -> group -> return -> scatter) on the
    HIP kernels, against the oracle's grouping of the whole table."""
    import threading
    import torch
    from spacedrive_amd import corpus, dedup
    world, total = 8, 100_000_000
    per = total // world
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world)}
    inputs, results, errors = {}, {}, []
    for r in range(world):
        inputs[r] = corpus.synth_dedup_rows_device(4, total, int(total * 0.8), r * per, per,
                                                   ctx=ctx)
    torch.cuda.synchronize()

    def run(r):
        try:
            k, h, rk = inputs[r]
            rep = dedup.sharded_group_reps(k, h, rk, 100, ops=dedup.HipOps(ctx),
                                           exchange=ThreadExchange(r, world, shared))
            torch.cuda.synchronize()
            results[r] = rep.cpu().numpy().view(np.uint32)
        except Exception as e:  # surface thread failures
            errors.append(e)
            shared["barrier"].abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    rep = np.concatenate([results[r] for r in range(world)])
    key = np.concatenate([inputs[r][0].cpu().numpy().view(np.uint64) for r in range(world)])
    has = np.concatenate([inputs[r][1].cpu().numpy() for r in range(world)])
    rank = np.concatenate([inputs[r][2].cpu().numpy().view(np.uint32) for r in range(world)])
    del inputs
    np.testing.assert_array_equal(rank, np.arange(total, dtype=np.uint32))
    assert abs(int(total - has.sum()) - total // 1000) < total // 5000  # ~0.1 % keyless
    ref = O.group_reps(key, has, 100)
    np.testing.assert_array_equal(rep, ref)
    # the config's shape: 20 % of the keyed rows link to an earlier row's Object
    linked = np.count_nonzero(rep != rank)
    assert 0.15 * total < linked < 0.21 * total


@pytest.mark.parametrize("n,chunk", [(13_000_000, 100), (26_000_000, 7)])
def test_two_level_partition(ctx, n, chunk):
    """Past 2^12 buckets the partition runs in two passes (coarse, then 9-bit
    staged per segment, offsets from the coarse pass's fine counts): 13 M rows
    (16 segments) and 26 M rows (32), with a key repeated 60 k times (a bucket
    past the LDS table) and keyless rows."""
    from spacedrive_amd import dedup
    rng = np.random.default_rng(n)
    pool = rng.integers(0, 2**64 - 1, int(n * 0.7), dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    key[rng.choice(n, 60_000, replace=False)] = pool[5]
    has = (rng.random(n) > 0.002).astype(np.uint8)
    rep = dedup.group_reps(key, has, chunk, ctx)
    np.testing.assert_array_equal(rep, O.group_reps(key, has, chunk))


def test_two_level_fine_count_overflow(ctx):
    """One key on the first 150 k rows of a 20 M-row table: the first coarse
    block's tile (~78 k rows) holds more than 65 535 rows of one final bucket,
    so its 16-bit fine counter overflows and the second pass's offsets are
    recounted from the records (k_fine_recount).  Bit-exact with the oracle,
    and a second call (flag reset) too."""
    from spacedrive_amd import dedup
    n = 20_000_000
    rng = np.random.default_rng(20)
    key = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    key[: n // 4] = key[rng.integers(0, n, n // 4)]  # duplicates elsewhere too
    key[:150_000] = np.uint64(0x5EED)
    has = (rng.random(n) > 0.001).astype(np.uint8)
    ref = O.group_reps(key, has, 100)
    np.testing.assert_array_equal(dedup.group_reps(key, has, 100, ctx), ref)
    np.testing.assert_array_equal(dedup.group_reps(key, has, 100, ctx), ref)
    key2 = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)  # no overflow now
    np.testing.assert_array_equal(dedup.group_reps(key2, has, 100, ctx), O.group_reps(key2, has, 100))


@pytest.mark.parametrize("n,chunk", [(12_500_000, 100), (7_000_000, 7), (13_000_000, 100)])
def test_implicit_rank_12_byte_records(ctx, n, chunk):
    """Rows without a rank array (rank = row): the 12-bit and the two-level
    (13 M rows) paths move 12-byte records {hash, row}.  Same reps as with the explicit rank array (16-byte
    records) and as the oracle; sentinel-valued keys and keyless rows included."""
    import torch
    from spacedrive_amd import dedup
    rng = np.random.default_rng(n)
    pool = rng.integers(0, 2**64 - 1, int(n * 0.8), dtype=np.uint64, endpoint=True)
    pool[0] = np.uint64(2**64 - 1)
    key = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) > 0.001).astype(np.uint8)
    ops = dedup.HipOps(ctx)
    dk = torch.from_numpy(key.view(np.int64)).cuda()
    dh = torch.from_numpy(has).cuda()
    dr = torch.arange(n, dtype=torch.int32, device="cuda")
    implicit = ops.group_rows(dk, dh, None, chunk, 0).cpu().numpy().view(np.uint32)
    explicit = ops.group_rows(dk, dh, dr, chunk, 0).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(implicit, explicit)
    np.testing.assert_array_equal(implicit, O.group_reps(key, has, chunk))


@pytest.mark.parametrize("key_off,has_off", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_histogram_alignment_paths(ctx, key_off, has_off):
    """k_part_hist reads row pairs with 16-B key / 2-B has_key loads when both
    arrays are so aligned, else row by row: 7 M rows (12-bit path, odd tile
    starts) from views that start 1 element in, same reps as the oracle."""
    import torch
    from spacedrive_amd import dedup
    n = 7_000_001
    rng = np.random.default_rng(77 + key_off * 2 + has_off)
    pool = rng.integers(0, 2**64 - 1, n // 2, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) > 0.01).astype(np.uint8)
    kbuf = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    hbuf = torch.zeros(n + 1, dtype=torch.uint8, device="cuda")
    kbuf[key_off:key_off + n] = torch.from_numpy(key.view(np.int64)).cuda()
    hbuf[has_off:has_off + n] = torch.from_numpy(has).cuda()
    dk, dh = kbuf[key_off:key_off + n], hbuf[has_off:has_off + n]
    rep = dedup.HipOps(ctx).group_rows(dk, dh, None, 100, 0).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(rep, O.group_reps(key, has, 100))


@pytest.mark.parametrize("chunk", [100, 3])
def test_two_level_34m_rows_both_record_sizes(ctx, chunk):
    """The two-level grouping at 34 M rows (32 segments, 2^14 buckets): a key
    repeated 60 k times (its bucket takes the global table), keyless rows,
    implicit (12-B records) and explicit (16-B records) ranks; bit-exact with
    the oracle."""
    import torch
    from spacedrive_amd import dedup
    n = 34_000_000
    rng = np.random.default_rng(34 + chunk)
    pool = rng.integers(0, 2**64 - 1, int(n * 0.8), dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    key[rng.choice(n, 60_000, replace=False)] = pool[9]
    has = (rng.random(n) > 0.001).astype(np.uint8)
    ref = O.group_reps(key, has, chunk)
    ops = dedup.HipOps(ctx)
    dk = torch.from_numpy(key.view(np.int64)).cuda()
    dh = torch.from_numpy(has).cuda()
    implicit = ops.group_rows(dk, dh, None, chunk, 0).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(implicit, ref)
    dr = torch.arange(n, dtype=torch.int32, device="cuda")
    explicit = ops.group_rows(dk, dh, dr, chunk, 0).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(explicit, ref)


def test_two_level_8bit_fine_count_overflow_rep_api(ctx):
    """The rep API over 12-byte records (implicit ranks, two-level at 13 M
    rows): 8-bit fine counters of the 8192-row coarse rounds wrap on a key
    repeated 1000 times in the first tile; reps bit-exact with the oracle."""
    from spacedrive_amd import dedup
    n = 13_000_000
    rng = np.random.default_rng(1000)
    key = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    key[:1000] = np.uint64(0xC0FFEE)
    has = (rng.random(n) > 0.001).astype(np.uint8)
    np.testing.assert_array_equal(dedup.group_reps(key, has, 100, ctx), O.group_reps(key, has, 100))
