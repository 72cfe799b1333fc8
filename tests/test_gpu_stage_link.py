"""GPU parity: pinned-host staged K1 (config 5 path) and the K7 Object link
batch, both bit-exact against the oracle."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _pinned_arena(sizes, seeds):
    import torch
    arena, off, ln = O.synth_arena(sizes, seeds)
    h = torch.empty(arena.size, dtype=torch.uint8).pin_memory()
    h.numpy()[:] = arena
    return h, arena, off, ln


def test_stage_pinned_matches_oracle_across_many_slabs(ctx):
    """~40k config-2 files (~1.7 GB of windows): several 256 MiB slabs cycle
    through the 3-slab ring; every cas id vs the oracle."""
    import torch
    from spacedrive_amd import cas, corpus
    sizes, seeds = corpus.config2_files(40_000, seed=31)
    h, arena, off, ln = _pinned_arena(sizes, seeds)
    out, st = cas.cas_stage_pinned(h, off, ln, ctx=ctx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    ref = O.cas_batch(arena, off, ln, threads=16)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    # a second call reuses the slab ring
    out2, _ = cas.cas_stage_pinned(h, off, ln, ctx=ctx)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out2.cpu().numpy(), ref)


def test_stage_pinned_edge_messages(ctx):
    """Invalid lengths / misaligned offsets get -EINVAL; empty and tiny messages."""
    import torch
    from spacedrive_amd import cas
    lens = np.array([0, 1, 1024, 1025, 4096, 4097, 57352, 102408, 102409, 64], np.uint32)
    off = np.zeros(lens.size, np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += (min(int(n), 102408) + 127) // 128 * 128
    off[-1] = off[-2] + 8  # misaligned
    rng = np.random.default_rng(5)
    arena = rng.integers(0, 256, pos + 256, dtype=np.uint8)
    h = torch.empty(arena.size, dtype=torch.uint8).pin_memory()
    h.numpy()[:] = arena
    out, st = cas.cas_stage_pinned(h, off, lens, ctx=ctx)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert st.tolist() == [0] * 8 + [-22, -22]
    ref = O.cas_batch(arena, off[:8], lens[:8], threads=4)
    np.testing.assert_array_equal(out.cpu().numpy()[:8], ref)
    assert not out.cpu().numpy()[8:].any()


def test_stage_pinned_rejects_unordered_arena(ctx):
    import torch
    from spacedrive_amd import cas
    from spacedrive_amd._native import SdgpuError
    h = torch.zeros(4096, dtype=torch.uint8).pin_memory()
    with pytest.raises(SdgpuError):
        cas.cas_stage_pinned(h, np.array([1024, 0], np.uint64), np.array([10, 10], np.uint32),
                             ctx=ctx)


@pytest.mark.parametrize("n,first_rank,with_valid", [(0, 0, False), (1, 0, False),
                                                     (255, 3, True), (4095, 0, True),
                                                     (4096, 0, False), (4097, 11, True),
                                                     (65_537, 0, True),
                                                     (100_000, 0, True), (2_000_000, 7_000, True)])
def test_link_batch_vs_oracle(ctx, n, first_rank, with_valid):
    import torch
    from spacedrive_amd import dedup
    key, has, rank = O.synth_dedup_rows(4, max(n, 1) * 2, max(n, 1), 0, n)
    rep_h = O.group_reps(key, has, 100) + np.uint32(first_rank)
    valid = (np.random.default_rng(n).random(n) > 0.02).astype(np.uint8) if with_valid else None
    d_rep = torch.from_numpy(rep_h.view(np.int32)).cuda()
    d_valid = torch.from_numpy(valid).cuda() if valid is not None else None
    c, lr, lo = dedup.link_batch_device(d_rep, None, d_valid, first_rank, ctx=ctx)
    rc, rlr, rlo = O.link_batch(rep_h, None, valid, first_rank)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), rc)
    np.testing.assert_array_equal(lr.cpu().numpy().view(np.uint32), rlr)
    np.testing.assert_array_equal(lo.cpu().numpy().view(np.uint32), rlo)
    # explicit ranks give the same lists
    if n:
        d_rank = torch.arange(first_rank, first_rank + n, dtype=torch.int64).to(torch.int32).cuda()
        c2, lr2, lo2 = dedup.link_batch_device(d_rep, d_rank, d_valid, 0, ctx=ctx)
        assert torch.equal(c2, c) and torch.equal(lr2, lr) and torch.equal(lo2, lo)


def test_stage_pinned_piece_split_by_file_count(ctx):
    """More than 65 536 tiny messages: the staged path splits pieces by file
    count, not bytes."""
    import torch
    from spacedrive_amd import cas
    n = 140_000
    rng = np.random.default_rng(13)
    lens = rng.integers(0, 300, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum((lens[:-1].astype(np.uint64) + 15) // 16 * 16)
    total = int(off[-1]) + int(lens[-1]) + 16
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    h = torch.empty(total, dtype=torch.uint8).pin_memory()
    h.numpy()[:] = arena
    out, st = cas.cas_stage_pinned(h, off, lens, ctx=ctx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), O.cas_batch(arena, off, lens, threads=16))


def test_identifier_run_chain_vs_oracle(ctx):
    """the config-5 chain as the bench runs it --
    sdgpu_cas_stage_pinned -> sdgpu_synth_vary_keys_device ->
    sdgpu_group_rows_indexed_device (one Object index for the run) ->
    sdgpu_link_batch_device -- over 3 steps of 100 k files, every step against
    the oracle: cas ids (O.cas_batch), reps of the whole run (O.group_reps over
    all steps' rows in id order, file_identifier/mod.rs:168-241) and the
    create / connect lists (O.link_batch, mod.rs:189-333)."""
    import torch
    from spacedrive_amd import cas, corpus, dedup
    n, steps = 100_000, 3
    sizes, seeds = corpus.config2_files(n, seed=41)
    h, arena, off, ln = _pinned_arena(sizes, seeds)
    cas_ref = O.cas_batch(arena, off, ln, threads=16)
    key0 = np.ascontiguousarray(cas_ref).view(np.uint64).ravel()
    has = (sizes != 0).astype(np.uint8)
    vary = corpus.config5_vary_mask(sizes, seeds)
    keys_ref = [O.vary_keys(key0, vary, s) for s in range(steps)]
    whole = O.group_reps(np.concatenate(keys_ref), np.tile(has, steps), 100)
    d_has = torch.from_numpy(has).cuda()
    d_vary = torch.from_numpy(vary).cuda()
    idx = dedup.ObjectIndex(ctx, 1000)        # grows on the way
    linked_earlier = 0
    for s in range(steps):
        out, st = cas.cas_stage_pinned(h, off, ln, ctx=ctx)
        torch.cuda.synchronize()
        assert int(st.abs().sum()) == 0
        np.testing.assert_array_equal(out.cpu().numpy(), cas_ref)
        key = out.view(torch.int64).view(-1)
        corpus.vary_keys_device(key, d_vary, s, ctx=ctx)
        np.testing.assert_array_equal(key.cpu().numpy().view(np.uint64), keys_ref[s])
        rank = torch.arange(s * n, (s + 1) * n, dtype=torch.int64).to(torch.int32).cuda()
        rep = dedup.group_rows_indexed(key, d_has, rank, idx, 100)
        got = rep.cpu().numpy().view(np.uint32)
        ref = whole[s * n:(s + 1) * n]
        np.testing.assert_array_equal(got, ref)
        c, lr, lo = dedup.link_batch_device(rep, rank, None, 0, ctx=ctx)
        rc, rlr, rlo = O.link_batch(ref, np.arange(s * n, (s + 1) * n, dtype=np.uint32), None, 0)
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), rc)
        np.testing.assert_array_equal(lr.cpu().numpy().view(np.uint32), rlr)
        np.testing.assert_array_equal(lo.cpu().numpy().view(np.uint32), rlo)
        linked_earlier += int(np.count_nonzero(ref < s * n))
    assert linked_earlier > 20_000    # later steps link to earlier steps' Objects
