"""GPU parity: K2/K3 (full-file BLAKE3 tree) against the CPU oracle."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_golden_checksums(ctx, golden):
    from spacedrive_amd import validation
    for e in golden["checksum_synthetic"]:
        data = O.synth_file_bytes(e["seed"], 0, e["len"])
        assert validation.checksum_bytes(data, ctx).hex() == e["checksum"], e["len"]


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1024, 1025, 16 * 1024 - 1, 16 * 1024,
                               16 * 1024 + 1, 17 * 1024, 256 * 1024, 256 * 1024 + 1,
                               4 * 1024 * 1024 + 4097, 16 * 1024 * 1024 * 17 + 5])
def test_lengths_vs_oracle(ctx, n):
    from spacedrive_amd import validation
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    assert validation.checksum_bytes(data, ctx) == O.blake3(data, threads=8)


def test_batch_device_mixed_lengths(ctx):
    import torch
    from spacedrive_amd import corpus, validation
    lens = [0, 5, 1024, 70_000, 1 << 20, (1 << 20) + 17, 33 * (1 << 20) + 1]
    files = []
    for i, n in enumerate(lens):
        t = torch.empty(max(n, 16), dtype=torch.uint8, device="cuda")[:n] if n else \
            torch.empty(16, dtype=torch.uint8, device="cuda")[:0]
        if n:
            corpus.synth_file_device(500 + i, n, out=t, ctx=ctx)
        files.append(t)
    out = validation.checksum_batch_device(files, ctx=ctx)
    torch.cuda.synchronize()
    for i, n in enumerate(lens):
        ref = O.blake3(O.synth_file_bytes(500 + i, 0, n), threads=8)
        assert bytes(out[i].cpu().numpy()) == ref, n


def test_subtree_slices_compose(ctx):
    """Aligned power-of-two slices' CVs are the tree's interior nodes: the
    root over 4 slices equals the digest of the whole (checked through
    file_checksum's fold), and a single root slice equals the digest."""
    import torch
    from spacedrive_amd import corpus, validation
    n = 4 * (1 << 16) * 1024 + 12345
    whole = corpus.synth_file_device(77, n, ctx=ctx)
    d = validation.subtree_device(whole, 0, True, ctx=ctx)
    torch.cuda.synchronize()
    assert bytes(d.cpu().numpy()) == O.blake3(whole.cpu().numpy(), threads=16)


@pytest.mark.parametrize("slice_chunks,n_slices,tail", [(1 << 16, 4, 12345), (1 << 10, 7, 0),
                                                       (1 << 12, 2, 1), (16, 3, 1000)])
def test_file_split_over_contexts(ctx, slice_chunks, n_slices, tail):
    """One file checksummed as SURVEY 8(e) splits it over GPUs: aligned
    power-of-two slices hashed to chaining values on different contexts
    (separate workspaces and streams, as separate GPUs would), the CVs gathered
    and combined on one: equal to the whole file's digest and the oracle's."""
    import torch
    from spacedrive_amd import corpus, validation
    from spacedrive_amd._native import Context
    others = [Context(0) for _ in range(3)]
    try:
        n = n_slices * slice_chunks * 1024 + tail
        whole = corpus.synth_file_device(91 + n_slices, n, ctx=ctx)
        step = slice_chunks * 1024
        cvs = torch.empty((n_slices + (1 if tail else 0), 32), dtype=torch.uint8, device="cuda")
        for i in range(cvs.shape[0]):
            c = others[i % len(others)]
            part = whole[i * step:min(n, (i + 1) * step)]
            validation.subtree_device(part, i * slice_chunks, False, out=cvs[i], ctx=c)
        torch.cuda.synchronize()
        d = validation.combine_subtrees_device(cvs, ctx=ctx)
        full = validation.subtree_device(whole, 0, True, ctx=ctx)
        torch.cuda.synchronize()
        assert torch.equal(d, full)
        assert bytes(d.cpu().numpy()) == O.blake3(whole.cpu().numpy(), threads=16)
    finally:
        for c in others:
            c.close()


@pytest.mark.parametrize("n", [0, 1, 1 << 20, 64 << 20, (64 << 20) + 1, (128 << 20),
                               (130 << 20) + 5, 3 * (64 << 20) - 1])
def test_file_checksum_path(ctx, tmp_path, n):
    from spacedrive_amd import validation
    p = tmp_path / "f.bin"
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    data.tofile(p)
    assert validation.file_checksum(p, ctx) == O.blake3(data, threads=8).hex()


def test_file_checksum_missing(ctx, tmp_path):
    from spacedrive_amd import validation
    with pytest.raises(OSError) as ei:
        validation.file_checksum(tmp_path / "nope", ctx)
    assert ei.value.errno == 2


def test_four_gib_file_bit_exact(ctx):
    """One config-3 file (4 GiB) on the device vs the multi-threaded oracle."""
    import torch
    from spacedrive_amd import corpus, validation
    f = corpus.synth_file_device(3, 1 << 32, ctx=ctx)
    out = validation.checksum_batch_device([f], ctx=ctx)
    torch.cuda.synchronize()
    host = f.cpu().numpy()
    del f
    assert bytes(out[0].cpu().numpy()) == O.blake3(host, threads=16)


def test_three_four_gib_files_in_one_plan(ctx):
    """Config 3 as the bench times it -- several ~4 GiB files in ONE
    checksum_batch_device plan, so the tree plan's cross-file group bases and
    chunk counters run past 2^32 bytes (b3_tree.hip find_seg / group_base,
    VERDICT r4 item 4): 4 GiB - 1023 (a partial last chunk), 4 GiB (a perfect
    2^22-chunk tree) and 4 GiB + 1 (a one-byte chunk past it), each against
    the multi-threaded oracle."""
    import torch
    from spacedrive_amd import corpus, validation
    lens = [(1 << 32) - 1023, 1 << 32, (1 << 32) + 1]
    files = [corpus.synth_file_device(300 + i, n, ctx=ctx) for i, n in enumerate(lens)]
    out = validation.checksum_batch_device(files, ctx=ctx)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i in range(len(lens)):
        host = files[i].cpu().numpy()
        files[i] = None
        assert bytes(got[i]) == O.blake3(host, threads=16), lens[i]
        del host


@pytest.mark.parametrize("n", [2, 1023, 1025, 4096, 65537, (1 << 19) + 1, (1 << 20) - 1, 1 << 20,
                               (1 << 20) + 1])
def test_file_checksum_latency_path_boundaries(ctx, tmp_path, n):
    """Files up to 1 MiB take the one-launch latency path (k_small_host up to
    112 KiB, k_small_split above); 1 MiB + 1 streams."""
    from spacedrive_amd import validation
    p = tmp_path / "g.bin"
    data = np.random.default_rng(n + 3).integers(0, 256, n, dtype=np.uint8)
    data.tofile(p)
    assert validation.file_checksum(p, ctx) == O.blake3(data, threads=8).hex()
