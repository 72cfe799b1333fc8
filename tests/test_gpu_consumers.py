"""GPU parity of the grouping's downstream consumers:
the orphan remover's query and the thumbnail shard grouping, vs the oracle."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_obj,n_fp", [(0, 10), (1, 0), (1000, 800), (4095, 5000), (4096, 100),
                                         (4097, 9000), (300_000, 1_000_000)])
def test_orphan_objects(ctx, n_obj, n_fp):
    import torch
    from spacedrive_amd import consumers
    rng = np.random.default_rng(n_obj + n_fp)
    objs = rng.permutation(max(n_obj * 2, 1))[:n_obj].astype(np.int32) + 1
    fp = rng.choice(objs, n_fp).astype(np.int32) if n_obj else np.zeros(n_fp, np.int32)
    fp[rng.random(n_fp) < 0.1] = -1                   # file_paths with object_id NULL
    maxid = int(objs.max()) if n_obj else 0
    got = consumers.orphan_objects(torch.from_numpy(objs).cuda(), torch.from_numpy(fp).cuda(),
                                   maxid, ctx)
    np.testing.assert_array_equal(got.cpu().numpy(), O.orphan_objects(objs, fp))
    out, cnt = consumers.orphan_objects(torch.from_numpy(objs).cuda(),
                                        torch.from_numpy(fp).cuda(), maxid, ctx, trim=False)
    np.testing.assert_array_equal(out[:int(cnt.item())].cpu().numpy(), O.orphan_objects(objs, fp))


def test_orphans_after_an_identifier_run(ctx):
    """Objects of a grouping: rows re-pointed elsewhere leave their Objects
    orphaned -- exactly those are found."""
    import torch
    from spacedrive_amd import consumers, dedup
    k, h, _ = O.synth_dedup_rows(31, 200_000, 150_000, 0, 200_000)
    rep = dedup.group_reps(k, h, 100, ctx).astype(np.int64)
    creators = np.flatnonzero(rep == np.arange(rep.size)).astype(np.int32)
    fp = rep.astype(np.int32).copy()                  # file_path -> Object (its creator)
    moved = np.random.default_rng(2).choice(rep.size, 20_000, replace=False)
    fp[moved] = -1                                    # those file_paths were deleted
    got = consumers.orphan_objects(torch.from_numpy(creators).cuda(), torch.from_numpy(fp).cuda(),
                                   int(rep.size), ctx).cpu().numpy()
    np.testing.assert_array_equal(got, O.orphan_objects(creators, fp))


@pytest.mark.parametrize("n", [0, 1, 255, 10_000, 1_000_003])
def test_thumbnail_shards(ctx, n):
    import torch
    from spacedrive_amd import consumers
    rng = np.random.default_rng(n)
    cas8 = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    valid = (rng.random(n) > 0.05).astype(np.uint8)
    order, counts = consumers.thumbnail_shards(torch.from_numpy(cas8).cuda(),
                                               torch.from_numpy(valid).cuda(), ctx)
    eo, ec = O.thumbnail_shards(cas8, valid)
    np.testing.assert_array_equal(counts.cpu().numpy(), ec)
    np.testing.assert_array_equal(order.cpu().numpy(), eo)
    o2, c2 = consumers.thumbnail_shards(torch.from_numpy(cas8).cuda(),
                                        torch.from_numpy(valid).cuda(), ctx, trim=False)
    np.testing.assert_array_equal(c2.cpu().numpy(), ec)
    np.testing.assert_array_equal(o2[:int(ec.sum())].cpu().numpy(), eo)
    if n:
        assert consumers.get_shard_hex(bytes(cas8[0]).hex()) == f"{cas8[0, 0]:02x}"


@pytest.mark.parametrize("values", [(0x5A,), (7, 200), (0, 1, 2, 3, 128, 255)])
def test_thumbnail_shards_skewed_bytes(ctx, values):
    """Few distinct first bytes, so every wave holds long runs of equal bytes
    (the same-byte lane masks of k_thumb_scatter), keyless rows between."""
    import torch
    from spacedrive_amd import consumers
    n = 300_007
    rng = np.random.default_rng(len(values))
    cas8 = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    cas8[:, 0] = np.asarray(values, np.uint8)[rng.integers(0, len(values), n)]
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    order, counts = consumers.thumbnail_shards(torch.from_numpy(cas8).cuda(),
                                               torch.from_numpy(valid).cuda(), ctx)
    eo, ec = O.thumbnail_shards(cas8, valid)
    np.testing.assert_array_equal(counts.cpu().numpy(), ec)
    np.testing.assert_array_equal(order.cpu().numpy(), eo)


@pytest.mark.parametrize("seed", range(12))
def test_orphan_objects_random(ctx, seed):
    """Random shapes: Object ids from 0 up (unique, any order), file_paths
    pointing at Objects, at ids no Object has (also past max_id), NULL (-1),
    or all at one Object; sizes across tile edges. Equal to the oracle."""
    import torch
    from spacedrive_amd import consumers
    rng = np.random.default_rng(4000 + seed)
    n_obj = int(rng.choice([1, 2, 4095, 4097, 65_536, 250_001]))
    n_fp = int(rng.choice([0, 1, 100, 5000, 300_000]))
    objs = rng.permutation(int(n_obj * rng.choice([1, 1.5, 4])))[:n_obj].astype(np.int32)
    maxid = int(objs.max())
    kind = seed % 3
    if kind == 0:
        fp = rng.choice(objs, n_fp).astype(np.int32)
    elif kind == 1:
        fp = rng.integers(-1, 2 * maxid + 3, n_fp).astype(np.int32)
    else:
        fp = np.full(n_fp, objs[0], np.int32)
    fp[rng.random(n_fp) < 0.05] = -1
    got = consumers.orphan_objects(torch.from_numpy(objs).cuda(), torch.from_numpy(fp).cuda(),
                                   maxid, ctx)
    np.testing.assert_array_equal(got.cpu().numpy(), O.orphan_objects(objs, fp))
