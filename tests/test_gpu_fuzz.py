"""Seeded randomized GPU parity sweeps (bounded: ~1 min in all): many small
random configurations of each hot-path kernel against the oracle, bit-exact.
Each case prints nothing unless it fails; the seed identifies it."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# SD_SOAK=k: (1 + k) times the seeds of every sweep (a longer bug hunt)
SOAK = 1 + int(os.environ.get("SD_SOAK", "0"))


def _lengths(rng, n):
    """Message lengths mixing tiny, chunk-edge, sampled (57 352) and large."""
    kind = rng.integers(0, 5, n)
    edge = np.array([0, 1, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097, 57352, 102408])
    out = np.where(kind == 0, rng.integers(0, 130, n),
          np.where(kind == 1, rng.choice(edge, n),
          np.where(kind == 2, 57352,
          np.where(kind == 3, rng.integers(0, 8192, n), rng.integers(0, 102409, n)))))
    return out.astype(np.uint32)


@pytest.mark.parametrize("seed", range(40 * SOAK))
def test_fuzz_k1_device_batches(ctx, seed):
    """K1 over random batches (1..6000 messages, random gaps between 16-B
    aligned messages, random content) through the device entry point."""
    import torch
    from spacedrive_amd import cas
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 6000))
    ln = _lengths(rng, n)
    gaps = rng.integers(0, 4, n) * 16
    off = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += (int(ln[i]) + 15) // 16 * 16
    arena = rng.integers(0, 256, max(pos, 16), dtype=np.uint8)
    out, st = cas.cas_batch_device(torch.from_numpy(arena).cuda(),
                                   torch.from_numpy(off.view(np.int64)).cuda(),
                                   torch.from_numpy(ln.view(np.int32)).cuda(), ctx=ctx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), O.cas_batch(arena, off, ln, 4))


@pytest.mark.parametrize("seed", range(48 * SOAK))
def test_fuzz_grouping_device(ctx, seed):
    """Grouping over random shapes: 1..3 M rows, few to all-distinct keys,
    small-integer or all-ones keys, random ranks (a permutation), chunk sizes
    1..1000, keyless density 0..50 %."""
    import torch
    from spacedrive_amd import dedup
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.choice([1, 2, 99, 100, 101, 5000, 300_000, 3_000_000]))
    distinct = max(1, int(n * rng.choice([0.0001, 0.01, 0.5, 0.9, 1.0])))
    mode = seed % 4
    if mode == 0:
        pool = rng.integers(0, 2**64 - 1, distinct, dtype=np.uint64, endpoint=True)
    elif mode == 1:
        pool = np.arange(distinct, dtype=np.uint64)            # small integers
    elif mode == 2:
        pool = (np.arange(distinct, dtype=np.uint64) << np.uint64(48))  # high bits only
    else:
        pool = np.full(distinct, np.uint64(2**64 - 1))         # the table's empty value
    key = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) >= rng.choice([0.0, 0.01, 0.5])).astype(np.uint8)
    chunk = int(rng.choice([1, 7, 100, 1000]))
    rank = rng.permutation(n).astype(np.uint32)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()
    ops = dedup.HipOps(ctx)
    rep = ops.group_rows(t(key, np.int64), t(has, np.uint8), t(rank, np.int32), chunk, 0)
    rep = rep.cpu().numpy().view(np.uint32)
    key_r = np.empty_like(key)
    has_r = np.empty_like(has)
    key_r[rank] = key
    has_r[rank] = has
    ref = O.group_reps(key_r, has_r, chunk).astype(np.uint32)
    np.testing.assert_array_equal(rep, ref[rank])


@pytest.mark.parametrize("seed", range(8 * SOAK))
def test_fuzz_grouping_large(ctx, seed):
    """The 12-bit path (block-major counts, one-launch offsets) and the
    two-level path (fine counts from the coarse pass) over random large shapes:
    6.5-20 M rows, the same key families as above (random, small integers,
    high bits only, the empty value), random rank permutations, keyless rows."""
    import torch
    from spacedrive_amd import dedup
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.choice([6_500_000, 12_500_000, 12_600_000, 13_000_000, 20_000_000]))
    distinct = max(1, int(n * rng.choice([0.001, 0.5, 0.9, 1.0])))
    mode = seed % 4
    if mode == 0:
        pool = rng.integers(0, 2**64 - 1, distinct, dtype=np.uint64, endpoint=True)
    elif mode == 1:
        pool = np.arange(distinct, dtype=np.uint64)
    elif mode == 2:
        pool = (np.arange(distinct, dtype=np.uint64) << np.uint64(40))
    else:
        pool = np.full(min(distinct, 3), np.uint64(2**64 - 1))
    key = pool[rng.integers(0, pool.size, n)]
    has = (rng.random(n) >= rng.choice([0.0, 0.01])).astype(np.uint8)
    chunk = int(rng.choice([7, 100]))
    rank = rng.permutation(n).astype(np.uint32)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()
    ops = dedup.HipOps(ctx)
    rep = ops.group_rows(t(key, np.int64), t(has, np.uint8), t(rank, np.int32), chunk, 0)
    rep = rep.cpu().numpy().view(np.uint32)
    key_r = np.empty_like(key)
    has_r = np.empty_like(has)
    key_r[rank] = key
    has_r[rank] = has
    ref = O.group_reps(key_r, has_r, chunk).astype(np.uint32)
    np.testing.assert_array_equal(rep, ref[rank])


@pytest.mark.parametrize("seed", range(20 * SOAK))
def test_fuzz_checksum_batches(ctx, seed):
    """Tree hashing of random device-resident file batches (1..40 files,
    0..24 MiB each, lengths near chunk / group / power-of-two edges)."""
    import torch
    from spacedrive_amd import validation
    rng = np.random.default_rng(3000 + seed)
    nf = int(rng.integers(1, 40))
    lens = []
    for _ in range(nf):
        k = int(rng.integers(0, 4))
        if k == 0:
            lens.append(int(rng.integers(0, 5000)))
        elif k == 1:
            lens.append(int(1 << int(rng.integers(10, 25))) + int(rng.integers(-1, 2)))
        elif k == 2:
            lens.append(int(rng.integers(1, 24 << 20)))
        else:
            lens.append(16 * 1024 * int(rng.integers(1, 300)))
    lens = [max(0, x) for x in lens]
    data = [rng.integers(0, 256, x, dtype=np.uint8) for x in lens]
    files = [torch.from_numpy(d).cuda() if d.size else torch.empty(16, dtype=torch.uint8).cuda()[:0]
             for d in data]
    out = validation.checksum_batch_device(files, ctx=ctx).cpu().numpy()
    for i, d in enumerate(data):
        assert bytes(out[i]) == O.blake3(d.tobytes(), 8), (seed, i, lens[i])


@pytest.fixture(scope="module")
def ctxs():
    from spacedrive_amd._native import Context
    cs = [Context(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("seed", range(16 * SOAK))
def test_fuzz_sharded_and_indexed(ctxs, seed):
    """The multi-GPU grouping (peer transport between contexts on the one
    GPU) at a random world size, and the same rows grouped in random batches
    through an Object index with some pre-existing Objects."""
    import torch
    from spacedrive_amd import dedup
    rng = np.random.default_rng(4000 + seed)
    n = int(rng.choice([3, 1000, 50_000, 400_000]))
    world = int(rng.integers(1, 9))
    distinct = max(1, int(n * rng.choice([0.05, 0.7])))
    pool = rng.integers(0, 2**64 - 1, distinct, dtype=np.uint64, endpoint=True)
    key = pool[rng.integers(0, distinct, n)]
    has = (rng.random(n) > 0.02).astype(np.uint8)
    chunk = int(rng.choice([1, 100, 333]))
    rep = dedup.dedup_sharded(ctxs[:world], key, has, chunk)
    np.testing.assert_array_equal(rep, O.group_reps(key, has, chunk))
    # batches through one index, with pre-existing Objects
    ek = rng.choice(key, max(1, n // 50))
    eh = rng.permutation(ek.size).astype(np.uint32) + 1
    idx = dedup.ObjectIndex(ctxs[0], 1024)
    idx.add_objects(torch.from_numpy(ek.view(np.int64)).cuda(),
                    torch.from_numpy(eh.view(np.int32)).cuda())
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n + 1, int(rng.integers(0, 6)))]))
    out = [dedup.dedup_batch(key[a:b], has[a:b], int(a), idx, chunk, ctxs[0])
           for a, b in zip(cuts[:-1], cuts[1:])]
    np.testing.assert_array_equal(np.concatenate(out), O.group_reps_existing(key, has, chunk, ek, eh))
