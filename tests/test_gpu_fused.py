"""GPU parity of the fused grouping + Object write set (sdgpu_group_link_device,
ABI 4): the create / connect lists the reference's identifier step writes
(file_identifier/mod.rs:189-333), produced by the group kernel itself without
a rep array, equal -- as sets -- the oracle's link batch over the oracle's
grouping (O.link_batch(O.group_reps(...))), on every partition path: the
small-table path (< 2^12 buckets), the one-level 12-bit path, the two-level
path, 12- and 16-byte records (implicit / explicit ranks), buckets past the
LDS table (global table), the hash-sentinel key, keyless and invalid rows."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def inv_mix64(h: int) -> int:
    """The key whose mix64 (splitmix64 finalizer, csrc/rows_device.hpp) is h."""
    c1, c2 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
    z = h
    z ^= (z >> 31) ^ (z >> 62)
    z = (z * pow(c2, -1, 1 << 64)) & M64
    z ^= (z >> 27) ^ (z >> 54)
    z = (z * pow(c1, -1, 1 << 64)) & M64
    z ^= (z >> 30) ^ (z >> 60)
    return z


SENTINEL_KEY = np.uint64(inv_mix64(M64))  # its hash is the LDS table's empty value


def _ref_lists(key, has, valid, rank, first_rank, chunk):
    """The oracle's write set in rank space: rows ordered by rank, grouped,
    then link_batch; lists sorted like split_link_lists."""
    n = key.size
    if rank is None and first_rank:
        # the chunk rule runs on GLOBAL ranks (chunk = rank // chunk_rows):
        # the oracle sees first_rank keyless rows in front, then drops them
        pad = np.zeros(first_rank, np.uint64)
        c, lr, lo = _ref_lists(np.concatenate([pad, key]),
                               np.concatenate([np.zeros(first_rank, np.uint8), has]),
                               None if valid is None else
                               np.concatenate([np.zeros(first_rank, np.uint8), valid]),
                               None, 0, chunk)
        return c[c >= first_rank], lr, lo
    r = (np.arange(n, dtype=np.uint64) + first_rank).astype(np.uint32) if rank is None else rank
    order = np.argsort(r, kind="stable")
    rep = O.group_reps(key[order], has[order], chunk)  # ranks relative to the sorted rows
    rs = r[order]
    rep_r = rs[rep]                                   # as ranks
    v = None if valid is None else valid[order]
    c, lr, lo = O.link_batch(rep_r, rs, v, 0)
    o = np.argsort(lr, kind="stable")
    return np.sort(c), lr[o], lo[o]


def _fused(ctx, key, has, valid, rank, first_rank, chunk):
    import torch
    from spacedrive_amd import dedup
    dk = torch.from_numpy(key.view(np.int64)).cuda()
    dh = torch.from_numpy(has).cuda() if has is not None else None
    dv = torch.from_numpy(valid).cuda() if valid is not None else None
    dr = torch.from_numpy(rank.view(np.int32)).cuda() if rank is not None else None
    who, obj, (c, l) = dedup.group_link_device(dk, dh, dv, dr, first_rank, chunk, ctx=ctx)
    w = who.cpu().numpy().view(np.uint32)
    o = obj.cpu().numpy().view(np.uint32)
    assert w.size == c + l
    return dedup.split_link_lists(w, o), (c, l)


def _check(ctx, key, has, valid=None, rank=None, first_rank=0, chunk=100):
    (c, lr, lo), (nc, nl) = _fused(ctx, key, has, valid, rank, first_rank, chunk)
    rc, rlr, rlo = _ref_lists(key, has if has is not None else np.ones(key.size, np.uint8), valid,
                              rank, first_rank, chunk)
    assert (nc, nl) == (rc.size, rlr.size)
    np.testing.assert_array_equal(c, rc)
    np.testing.assert_array_equal(lr, rlr)
    np.testing.assert_array_equal(lo, rlo)


@pytest.mark.parametrize("n,pool", [(0, 1), (1, 1), (2, 1), (1000, 10), (100_000, 70_000),
                                    (300_000, 1), (500_000, 7), (1_000_000, 800_000)])
def test_fused_small_table_path_vs_oracle(ctx, n, pool):
    """< 2^12 buckets (hist + scan + 16-B records, the 6144-slot table), one
    key 300 k times (global table), the hash-sentinel key, keyless rows."""
    rng = np.random.default_rng(n + 3 * pool)
    keys = rng.integers(0, 2**64 - 1, max(pool, 1), dtype=np.uint64, endpoint=True)
    keys[0] = SENTINEL_KEY
    key = keys[rng.integers(0, keys.size, n)] if n else np.zeros(0, np.uint64)
    has = (rng.random(n) > 0.01).astype(np.uint8)
    for chunk in (100, 1, 7):
        _check(ctx, key, has, chunk=chunk)
    _check(ctx, key, has, first_rank=12345)


@pytest.mark.parametrize("n,chunk", [(7_000_001, 100), (12_500_000, 7), (13_000_000, 100)])
def test_fused_packed_paths_vs_oracle(ctx, n, chunk):
    """The one-level 12-bit path (7 M, 12.5 M rows) and the two-level path
    (13 M rows), implicit ranks (12-byte records) and explicit ranks (16-byte
    records), a key repeated 60 k times (a bucket past the LDS table)."""
    rng = np.random.default_rng(n)
    pool = rng.integers(0, 2**64 - 1, int(n * 0.8), dtype=np.uint64, endpoint=True)
    pool[1] = SENTINEL_KEY
    key = pool[rng.integers(0, pool.size, n)]
    key[rng.choice(n, 60_000, replace=False)] = pool[5]
    has = (rng.random(n) > 0.001).astype(np.uint8)
    _check(ctx, key, has, chunk=chunk)
    _check(ctx, key, has, rank=np.arange(n, dtype=np.uint32), chunk=chunk)


def test_fused_permuted_ranks_and_invalid_rows(ctx):
    """Explicit permuted ranks (rows not in id order) and rows whose metadata
    failed (valid == 0, has_key == 0: in neither list, mod.rs:113,127), next to
    valid keyless rows (own Objects, mod.rs:238-239)."""
    n = 400_000
    rng = np.random.default_rng(11)
    pool = rng.integers(0, 2**64 - 1, 250_000, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    valid = (rng.random(n) > 0.02).astype(np.uint8)
    has = ((rng.random(n) > 0.01) & (valid != 0)).astype(np.uint8)
    rank = rng.permutation(n).astype(np.uint32)
    for chunk in (100, 3):
        _check(ctx, key, has, valid=valid, rank=rank, chunk=chunk)
    _check(ctx, key, has, valid=valid, chunk=100)
    _check(ctx, key, None, chunk=100)  # every row keyed: no keyless pass


@pytest.mark.parametrize("n", [4095, 4096, 4607, 4608, 4609, 9000])
def test_fused_one_bucket_at_table_capacity(ctx, n):
    """Every row in ONE bucket: just under, at and over the packed table's
    4095 records and the 6144-slot table's 4608 (LDS vs global-table path)."""
    from tests.test_gpu_dedup import _one_bucket_keys
    rng = np.random.default_rng(n)
    keys = _one_bucket_keys(rng, n, int(n * 0.7))
    key = keys[rng.integers(0, keys.size, n)]
    has = np.ones(n, np.uint8)
    for chunk in (100, 1):
        _check(ctx, key, has, chunk=chunk)


def test_fused_equals_group_then_link_batch(ctx):
    """Same write set as the two-call path it replaces (sdgpu_group_rows_device
    -> sdgpu_link_batch_device) on the config-4 shape, 12.5 M rows."""
    import torch
    from spacedrive_amd import corpus, dedup
    n = 12_500_000
    key, has, rank = corpus.synth_dedup_rows_device(4, n, int(n * 0.8), 0, n, ctx=ctx)
    ops = dedup.HipOps(ctx)
    rep = ops.group_rows(key, has, None, 100, 0)
    c, lr, lo = (x.cpu().numpy().view(np.uint32)
                 for x in dedup.link_batch_device(rep, None, has, 0, ctx=ctx))
    # the two-call path's valid = has: keyless rows are in neither list there
    who, obj, _ = dedup.group_link_device(key, has, has, None, 0, 100, ctx=ctx)
    fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
    np.testing.assert_array_equal(fc, np.sort(c))
    np.testing.assert_array_equal(flr, lr)
    np.testing.assert_array_equal(flo, lo)
    torch.cuda.synchronize()


@pytest.mark.parametrize("chunk,bounds", [(100, [0, 100_000, 200_000]),
                                          (100, [0, 150, 1000, 50_037, 200_000]),
                                          (7, [0, 3, 70_000, 200_000])])
def test_fused_batches_through_the_object_index(ctx, chunk, bounds):
    """Batches in id order through one Object index, with Objects registered
    before the run (existing handles), via the fused call: the union of the
    batches' write sets equals the oracle's link batch over the whole run's
    grouping against those Objects (O.group_reps_existing, mod.rs:168-241)
    -- rows of a later batch link to Objects of an earlier one or to the
    registered ones (obj = REP_EXISTING | handle); batch bounds split chunks."""
    import torch
    from spacedrive_amd import dedup
    total = bounds[-1]
    rng = np.random.default_rng(chunk + len(bounds))
    pool = rng.integers(0, 2**64 - 1, 120_000, dtype=np.uint64, endpoint=True)
    pool[0] = SENTINEL_KEY
    key = pool[rng.integers(0, pool.size, total)]
    has = (rng.random(total) > 0.01).astype(np.uint8)
    ek = rng.choice(pool, 3000)
    eh = (np.arange(ek.size, dtype=np.uint32) * 7 + 11)
    idx = dedup.ObjectIndex(ctx, 1000)  # small: grows and rehashes on the way
    idx.add_objects(torch.from_numpy(ek.view(np.int64)).cuda(),
                    torch.from_numpy(eh.view(np.int32)).cuda())
    torch.cuda.synchronize()
    ws, os_ = [], []
    nc = nl = 0
    for a, b in zip(bounds[:-1], bounds[1:]):
        dk = torch.from_numpy(key[a:b].view(np.int64)).cuda()
        dh = torch.from_numpy(has[a:b]).cuda()
        who, obj, (c, l) = dedup.group_link_device(dk, dh, None, None, a, chunk, ctx=ctx,
                                                   index=idx)
        ws.append(who.cpu().numpy())
        os_.append(obj.cpu().numpy())
        nc, nl = nc + c, nl + l
    fc, flr, flo = dedup.split_link_lists(np.concatenate(ws), np.concatenate(os_))
    ref = O.group_reps_existing(key, has, chunk, ek, eh)
    rc, rlr, rlo = O.link_batch(ref, None, None, 0)
    assert (nc, nl) == (rc.size, rlr.size)
    np.testing.assert_array_equal(fc, rc)
    np.testing.assert_array_equal(flr, rlr)
    np.testing.assert_array_equal(flo, rlo)


@pytest.mark.parametrize("n", [1, 4095, 4097, 65_537, 5_000_003])
def test_fused_extras_only_and_ragged_tiles(ctx, n):
    """The extra-entry pass alone and at tile edges: every row keyless (the
    group kernels see no record, every valid row is its own Object), then a
    ragged row count with 30 % keyless rows and 5 % invalid ones, so the
    one-block scan runs over more tiles than it has threads (5 M rows: 1221
    tiles) and the last tile is partial."""
    rng = np.random.default_rng(n + 77)
    key = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    _check(ctx, key, np.zeros(n, np.uint8))
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    _check(ctx, key, np.zeros(n, np.uint8), valid=valid, first_rank=300)
    pool = key[: max(1, n // 3)]
    key2 = pool[rng.integers(0, pool.size, n)]
    has = ((rng.random(n) > 0.3) & (valid != 0)).astype(np.uint8)
    _check(ctx, key2, has, valid=valid)


def test_fused_every_row_decided_by_the_index(ctx):
    """A batch whose every cas_id already has an Object (registered before
    the run): the probe decides every keyed row, the group kernels get no
    record, and every entry comes from the extra pass (linked to the
    registered Object); keyless rows stay their own Objects."""
    import torch
    from spacedrive_amd import dedup
    n = 300_000
    rng = np.random.default_rng(5)
    pool = rng.integers(0, 2**64 - 1, 50_000, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) > 0.02).astype(np.uint8)
    eh = np.arange(pool.size, dtype=np.uint32) * 3 + 1
    idx = dedup.ObjectIndex(ctx, 1 << 17)
    idx.add_objects(torch.from_numpy(pool.view(np.int64)).cuda(),
                    torch.from_numpy(eh.view(np.int32)).cuda())
    torch.cuda.synchronize()
    dk = torch.from_numpy(key.view(np.int64)).cuda()
    dh = torch.from_numpy(has).cuda()
    who, obj, (c, l) = dedup.group_link_device(dk, dh, None, None, 0, 100, ctx=ctx, index=idx)
    fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
    ref = O.group_reps_existing(key, has, 100, pool, eh)
    rc, rlr, rlo = O.link_batch(ref, None, None, 0)
    assert (c, l) == (rc.size, rlr.size) and l == int(has.sum())
    np.testing.assert_array_equal(fc, rc)
    np.testing.assert_array_equal(flr, rlr)
    np.testing.assert_array_equal(flo, rlo)


@pytest.mark.parametrize("n", [300_001, 7_000_001])
def test_fused_keyless_sink_on_unaligned_rows(ctx, n):
    """The keyless rows are collected by the first partition pass (XSink in
    dedup.hip).  Key / has_key / valid views that start one row into their
    buffers miss the histogram's paired 16-B / 2-B loads, so the per-row
    path collects them (small-table and 12-bit paths); the aligned case runs
    in the other tests."""
    import torch
    from spacedrive_amd import dedup
    rng = np.random.default_rng(n + 5)
    pool = rng.integers(0, 2**64 - 1, n // 2, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    valid = (rng.random(n) > 0.03).astype(np.uint8)
    has = ((rng.random(n) > 0.1) & (valid != 0)).astype(np.uint8)
    pad = lambda a: np.concatenate([a[:1], a])  # noqa: E731
    dk = torch.from_numpy(pad(key).view(np.int64)).cuda()[1:]
    dh = torch.from_numpy(pad(has)).cuda()[1:]
    dv = torch.from_numpy(pad(valid)).cuda()[1:]
    assert dk.data_ptr() % 16 == 8 and dh.data_ptr() % 2 == 1
    who, obj, (c, l) = dedup.group_link_device(dk, dh, dv, None, 40, 100, ctx=ctx)
    fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
    rc, rlr, rlo = _ref_lists(key, has, valid, None, 40, 100)
    assert (c, l) == (rc.size, rlr.size)
    np.testing.assert_array_equal(fc, rc)
    np.testing.assert_array_equal(flr, rlr)
    np.testing.assert_array_equal(flo, rlo)


def test_fused_two_level_path_all_keyless_tiles(ctx):
    """Two-level path (13 M rows): whole first-pass tiles of keyless rows (a
    block's sink filled to its tile size) next to tiles of keyed ones."""
    n = 13_000_000
    rng = np.random.default_rng(13)
    pool = rng.integers(0, 2**64 - 1, n // 2, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, pool.size, n)]
    has = np.ones(n, np.uint8)
    has[: n // 4] = 0             # the first quarter of the tiles: keyless
    has[n // 2: n // 2 + 1000] = 0
    valid = np.ones(n, np.uint8)
    valid[n // 8: n // 8 + 5000] = 0
    _check(ctx, key, has, valid=valid)


@pytest.mark.parametrize("n,bits,t,distinct", [
    (12_500_000, 12, 4093, 4093), (12_500_000, 12, 4093, 1500), (12_500_000, 12, 4094, 4094),
    (12_500_000, 12, 4094, 2000), (12_500_000, 12, 4095, 4095), (13_000_000, 13, 4093, 4093),
    (13_000_000, 13, 4094, 3000), (12_500_000, 12, 3072, 3072), (12_500_000, 12, 3073, 1000),
    (13_000_000, 13, 3073, 3073)])
def test_fused_packed_bucket_at_capacity(ctx, n, bits, t, distinct):
    """One bucket of exactly kPkCap = 4093 records -- the packed table's
    last record index (lmin's last entry, beside special_min and the output
    scratch in the kernel's word area) -- or more (the global table), with
    all-distinct or repeated keys, on the one-level 12-bit path (12.5 M rows)
    and the two-level path (13 M rows: 13 digit bits): keys built from hashes
    whose digit bits (56 - bits .. 55) name the bucket.  3072 / 3073: the
    last bucket grouped with three records per thread, the first with four."""
    D = 1234
    rng = np.random.default_rng(t * 7 + distinct + bits)
    sh8, shd = np.uint64(8), np.uint64(64 - bits)
    key = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    dig = (O.mix64(key) << sh8) >> shd
    bad = np.flatnonzero(dig == D)
    while bad.size:  # every other row outside bucket D
        key[bad] = rng.integers(0, 2**64 - 1, bad.size, dtype=np.uint64, endpoint=True)
        dig[bad] = (O.mix64(key[bad]) << sh8) >> shd
        bad = bad[dig[bad] == D]
    lo = 56 - bits
    mask = np.uint64(((1 << bits) - 1) << lo)
    hs = (rng.integers(0, 2**63, distinct, dtype=np.uint64) & ~mask) | (np.uint64(D) << np.uint64(lo))
    ks = np.array([inv_mix64(int(h)) for h in hs], np.uint64)
    assert np.all(((O.mix64(ks) << sh8) >> shd) == D)
    pick = ks[rng.integers(0, distinct, t)]
    pick[:distinct] = ks
    key[rng.choice(n, t, replace=False)] = pick
    _check(ctx, key, np.ones(n, np.uint8), chunk=100)


@pytest.mark.parametrize("reps,keyless", [(255, False), (256, False), (300, True), (70_000, False)])
def test_fused_two_level_8bit_fine_count_overflow(ctx, reps, keyless):
    """12-byte records (rows in rank order) take 8192-row coarse rounds and
    8-bit fine counters in k_part_private: one key on the first `reps` rows
    puts that many rows of one final bucket in the first coarse tile, so from
    256 on its counter wraps, the flag is set and k_fine_recount_runs
    rebuilds every count from the records.  255 fills the counter exactly.
    13 M rows (two-level), with and without keyless rows beside (the sink)."""
    n = 13_000_000
    rng = np.random.default_rng(reps)
    key = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    key[: n // 8] = key[rng.integers(0, n, n // 8)]  # duplicates elsewhere too
    key[:reps] = np.uint64(0x5EED)
    has = (rng.random(n) > 0.01).astype(np.uint8) if keyless else np.ones(n, np.uint8)
    has[:reps] = 1
    _check(ctx, key, has)
    _check(ctx, key, has)  # the flag was reset
