"""GPU parity: K1 (sampled cas_id) against the CPU oracle, bit-exact."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _host_batch(ctx, sizes, seeds):
    from spacedrive_amd import cas
    arena, off, ln = O.synth_arena(np.array(sizes, np.uint64), np.array(seeds, np.uint64))
    out, st = cas.cas_batch(arena, off, ln, ctx)
    return arena, off, ln, out, st


def test_golden_cas_ids_host_api(ctx, golden):
    from spacedrive_amd import cas
    e = golden["cas_synthetic"]
    _, _, _, out, st = _host_batch(ctx, [x["size"] for x in e], [x["seed"] for x in e])
    assert np.all(st == 0)
    assert cas.hex_ids(out) == [x["cas_id"] for x in e]


def test_every_message_length_up_to_3_chunks(ctx):
    """Arbitrary messages of every length 0..3100 (all block/chunk tails)."""
    from spacedrive_amd import cas
    lens = np.arange(0, 3101, dtype=np.uint32)
    off = np.zeros(lens.size, np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += (int(n) + 15) // 16 * 16
    rng = np.random.default_rng(1)
    arena = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    out, st = cas.cas_batch(arena, off, lens, ctx)
    assert np.all(st == 0)
    ref = O.cas_batch(arena, off, lens, threads=8)
    np.testing.assert_array_equal(out, ref)


def test_invalid_messages_rejected(ctx):
    from spacedrive_amd import cas
    arena = np.zeros(300_000, np.uint8)
    off = np.array([0, 0, 16, 32], np.uint64)
    ln = np.array([102408, 102409, 10, 200_000], np.uint32)
    out, st = cas.cas_batch(arena, off, ln, ctx)
    assert st.tolist() == [0, -22, 0, -22]
    assert not out[1].any() and not out[3].any()
    assert bytes(out[0]).hex() == O.cas_id_of_message(bytes(102408))


def test_device_api_misaligned_offset_status(ctx):
    import torch
    from spacedrive_amd import cas
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 8, 1024], dtype=torch.int64, device="cuda")
    ln = torch.tensor([100, 100, 100], dtype=torch.int32, device="cuda")
    out, st = cas.cas_batch_device(arena, off, ln, ctx=ctx)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0, -22, 0]
    assert bytes(out[0].cpu().numpy()).hex() == O.cas_id_of_message(bytes(100))


def test_device_synth_arena_matches_oracle_bytes(ctx):
    import torch
    from spacedrive_amd import corpus
    sizes, seeds = corpus.config2_files(3000, seed=9)
    d_arena, d_off, d_len = corpus.synth_arena_device(sizes, seeds, ctx=ctx)
    torch.cuda.synchronize()
    arena, off, ln = O.synth_arena(sizes, seeds)
    h = d_arena.cpu().numpy()
    for i in range(sizes.size):
        a, b = int(off[i]), int(off[i]) + int(ln[i])
        assert np.array_equal(h[a:b], arena[a:b]), i


def test_random_config2_subset_device_api(ctx):
    import torch
    from spacedrive_amd import cas, corpus
    sizes, seeds = corpus.config2_files(50_000, seed=21)
    d_arena, d_off, d_len = corpus.synth_arena_device(sizes, seeds, ctx=ctx)
    out, st = cas.cas_batch_device(d_arena, d_off, d_len, ctx=ctx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    ref = O.cas_batch(d_arena.cpu().numpy(), d_off.cpu().numpy().view(np.uint64),
                      d_len.cpu().numpy().view(np.uint32), threads=16)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_full_config2_one_million_files_bit_exact(ctx):
    """BASELINE config 2 at full size: 1 M files, every cas_id vs the oracle."""
    import torch
    from spacedrive_amd import cas, corpus
    sizes, seeds = corpus.config2_files(1_000_000, seed=2)
    d_arena, d_off, d_len = corpus.synth_arena_device(sizes, seeds, ctx=ctx)
    out, st = cas.cas_batch_device(d_arena, d_off, d_len, ctx=ctx)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    got = out.cpu().numpy()
    host = d_arena.cpu().numpy()
    del d_arena
    ref = O.cas_batch(host, d_off.cpu().numpy().view(np.uint64),
                      d_len.cpu().numpy().view(np.uint32), threads=16)
    mism = np.flatnonzero(np.any(got != ref, axis=1))
    assert mism.size == 0, f"{mism.size} mismatching cas ids, first rows {mism[:5]}"
    # duplicates (same size+seed) must share a cas id, distinct content must not collide
    # (empty files all hash the 8 zero bytes of their size: one shared id)
    keys = cas.keys_of(got)
    nz = sizes != 0
    pair = sizes * np.uint64(0x9E3779B97F4A7C15) ^ seeds
    assert np.unique(keys[nz]).size == np.unique(pair[nz]).size
    assert np.unique(keys[~nz]).size == 1


def test_zero_files(ctx):
    from spacedrive_amd import cas
    out, st = cas.cas_batch(np.zeros(16, np.uint8), np.zeros(0, np.uint64),
                            np.zeros(0, np.uint32), ctx)
    assert out.shape == (0, 8)


def _tree_edge_lengths():
    """Message lengths at every chunk-count / unit boundary up to 102 408 B:
    n*1024 + {-64, -1, 0, 1, 8, 65} for n = 1..100, plus 57 352 (sampled)."""
    ls = {57352, 102408, 102407}
    for n in range(1, 101):
        for d in (-64, -1, 0, 1, 8, 65):
            v = n * 1024 + d
            if 0 <= v <= 102408:
                ls.add(v)
    return np.array(sorted(ls), np.uint32)


def test_k1_tree_edges_bit_exact(ctx):
    """K1 on every unit/ragged-tail shape: q = 0..25 four-chunk units with 0..4
    trailing chunks, in both orders in one batch."""
    from spacedrive_amd import cas
    lens = _tree_edge_lengths()
    lens = np.concatenate([lens, lens[::-1]])
    off = np.zeros(lens.size, np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += (int(n) + 127) // 128 * 128
    rng = np.random.default_rng(7)
    arena = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    out, st = cas.cas_batch(arena, off, lens, ctx)
    assert np.all(st == 0)
    ref = O.cas_batch(arena, off, lens, threads=8)
    np.testing.assert_array_equal(out, ref)


def test_device_api_workspace_guards(ctx):
    """sdgpu_cas_batch_device sizes its workspace from arena_bytes: a message
    ending past the arena is -EINVAL; overlapping messages whose CV slots fit
    are hashed normally; overlapping messages that would overflow the workspace
    are all -ENOBUFS (nothing written past it)."""
    import torch
    from spacedrive_amd import cas
    rng = np.random.default_rng(3)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    arena = torch.from_numpy(host).cuda()
    off = torch.tensor([0, 0, 4096, (1 << 20) - 64, (1 << 20) - 48], dtype=torch.int64,
                       device="cuda")
    ln = torch.tensor([102408, 102408, 57352, 64, 64], dtype=torch.int32, device="cuda")
    out, st = cas.cas_batch_device(arena, off, ln, ctx=ctx)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0, 0, 0, 0, -22]
    o = off.cpu().numpy().view(np.uint64)[:4]
    l_ = ln.cpu().numpy().view(np.uint32)[:4]
    np.testing.assert_array_equal(out.cpu().numpy()[:4], O.cas_batch(host, o, l_, threads=4))
    assert not out.cpu().numpy()[4].any()
    # 2000 copies of one 100 KiB message in a 128 KiB arena: 25 units each,
    # far beyond arena_bytes / 1024 + n CV slots
    small = arena[: 128 << 10]
    off2 = torch.zeros(2000, dtype=torch.int64, device="cuda")
    ln2 = torch.full((2000,), 102408, dtype=torch.int32, device="cuda")
    out2, st2 = cas.cas_batch_device(small, off2, ln2, ctx=ctx)
    torch.cuda.synchronize()
    assert set(st2.cpu().tolist()) == {-105}  # -ENOBUFS
    assert not out2.cpu().numpy().any()
    # the context still works afterwards
    out3, st3 = cas.cas_batch_device(arena, off[:3], ln[:3], ctx=ctx)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out3.cpu().numpy(), out.cpu().numpy()[:3])


@pytest.mark.parametrize("n", [1, 3, 64])
def test_small_batch_latency_kernel_bit_exact(ctx, n, tmp_path):
    """Batches of <= 64 messages take the one-launch latency kernel (k_small_host):
    every chunk-count shape up to 101 chunks, through sdgpu_cas_batch."""
    from spacedrive_amd import cas
    lens = _tree_edge_lengths()
    rng = np.random.default_rng(n)
    for start in range(0, lens.size, n):
        ln = lens[start:start + n]
        off = np.zeros(ln.size, np.uint64)
        pos = 0
        for i, m in enumerate(ln):
            off[i] = pos
            pos += (int(m) + 127) // 128 * 128
        arena = rng.integers(0, 256, pos + 16, dtype=np.uint8)
        out, st = cas.cas_batch(arena, off, ln, ctx)
        assert np.all(st == 0)
        np.testing.assert_array_equal(out, O.cas_batch(arena, off, ln, threads=4))


def test_host_pipeline_many_slabs_by_file_count(ctx):
    """sdgpu_cas_batch with more messages than one staging slab holds
    (65 536 files per slab): the double-buffered pipeline drains and refills."""
    from spacedrive_amd import cas
    n = 150_000
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 1500, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum((lens[:-1].astype(np.uint64) + 15) // 16 * 16)
    arena = rng.integers(0, 256, int(off[-1]) + int(lens[-1]) + 16, dtype=np.uint8)
    out, st = cas.cas_batch(arena, off, lens, ctx)
    assert np.all(st == 0)
    np.testing.assert_array_equal(out, O.cas_batch(arena, off, lens, threads=16))


def test_host_pipeline_many_slabs_by_bytes(ctx):
    """~700 MB of maximal messages: the 256 MiB slab fills by bytes first."""
    from spacedrive_amd import cas
    n = 7000
    lens = np.full(n, 102408, np.uint32)
    lens[::7] = 57352
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum((lens[:-1].astype(np.uint64) + 127) // 128 * 128)
    arena = np.random.default_rng(12).integers(0, 256, int(off[-1]) + 102408 + 16,
                                                dtype=np.uint8)
    out, st = cas.cas_batch(arena, off, lens, ctx)
    assert np.all(st == 0)
    np.testing.assert_array_equal(out, O.cas_batch(arena, off, lens, threads=16))
