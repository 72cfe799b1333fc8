"""GPU parity of the single-file latency kernels (k_small_host / k_service:
one workgroup per message of <= 112 KiB; k_small_split: messages of <= 1 MiB
in 64 KiB groups on as many workgroups; every compression spread over a quad
of lanes, the tree level by level in LDS): batches of <= 64 cas messages
(<= 102 408 B), single files through generate_cas_id and file_checksum up to
1 MiB (1024 chunks, the limit); checked bit-exact against the oracle."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CAS_MAX = 102408  # largest cas message (cas.rs:23-62): sdgpu_cas_batch rejects longer
EDGE = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 4104, 8200, 57352, CAS_MAX - 1, CAS_MAX]
FILE_EDGE = EDGE[1:] + [256 * 1024 - 1, 256 * 1024, 256 * 1024 + 1, 300_000, (1 << 20) - 1,
                        1 << 20]


def _arena(lens, seed):
    rng = np.random.default_rng(seed)
    off = np.zeros(len(lens), np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += (int(n) + 15) // 16 * 16 + 16
    arena = rng.integers(0, 256, max(pos, 16), dtype=np.uint8)
    return arena, off, np.asarray(lens, np.uint32)


def _check(ctx, lens, seed):
    from spacedrive_amd import cas
    arena, off, ln = _arena(lens, seed)
    out, st = cas.cas_batch(arena, off, ln, ctx)
    assert np.all(st == 0)
    for i, n in enumerate(ln.tolist()):
        msg = arena[int(off[i]):int(off[i]) + n].tobytes()
        assert bytes(out[i]).hex() == O.cas_id_of_message(msg), (i, n)


@pytest.mark.parametrize("limit", [4096, 64 * 1024, CAS_MAX])
def test_small_batches_random_lengths(ctx, limit):
    rng = np.random.default_rng(limit)
    for rep in range(3):
        lens = rng.integers(0, limit + 1, 64)
        _check(ctx, lens, 100 * rep + 7)


def test_small_batch_edge_lengths(ctx):
    # every edge alone (one message per launch), then all together
    for n in EDGE:
        _check(ctx, [n], n)
    _check(ctx, EDGE, 3)


def test_file_checksum_small_files(ctx, tmp_path):
    from spacedrive_amd import validation
    rng = np.random.default_rng(5)
    for n in FILE_EDGE:
        p = os.path.join(tmp_path, f"f{n}")
        rng.integers(0, 256, n, dtype=np.uint8).tofile(p)
        assert validation.file_checksum(p, ctx) == O.file_checksum_path(p), n


def test_generate_cas_id_small_files(ctx, tmp_path):
    from spacedrive_amd import cas
    rng = np.random.default_rng(6)
    for n in [1, 100, 1024, 1025, 4096, 65536, 102400, 102401, 500_000]:
        p = os.path.join(tmp_path, f"g{n}")
        rng.integers(0, 256, n, dtype=np.uint8).tofile(p)
        assert cas.generate_cas_id(p, n, ctx) == O.cas_id_path(p, n), n


@pytest.fixture()
def svc_ctx():
    """A separate context with the resident latency service on (f3): the
    single-file drop-ins go through k_service's mailbox."""
    from spacedrive_amd._native import Context
    c = Context(0)
    c.latency_service(True)
    yield c
    c.latency_service(False)
    c.close()


def test_service_generate_cas_id_and_checksum(svc_ctx, tmp_path):
    """Every size class through the resident kernel: empty (size 0 hashes the
    8 zero bytes, non_indexed.rs:161), one chunk, chunk boundaries, the
    100 KiB cas limit, sampled files (57 352-B messages), files up to the
    112 KiB message area and just past it (one-shot fallback)."""
    from spacedrive_amd import cas, validation
    rng = np.random.default_rng(17)
    sizes = [0, 1, 63, 64, 65, 1023, 1024, 1025, 4096, 65536, 102399, 102400, 102401, 114_688 - 1,
             114_688, 114_689, 500_000, 3 << 20]
    for n in sizes:
        p = os.path.join(tmp_path, f"s{n}")
        rng.integers(0, 256, n, dtype=np.uint8).tofile(p)
        assert cas.generate_cas_id(p, n, svc_ctx) == O.cas_id_path(p, n), n
        assert validation.file_checksum(p, svc_ctx) == O.file_checksum_path(p), n


def test_service_survives_idle_exit_and_bulk_calls(svc_ctx, tmp_path):
    """The resident kernel ends itself after 20 ms without a request and is
    stopped by any bulk call; the next single-file call relaunches it.  Both
    orders, repeated, stay bit-exact; a missing file still reports ENOENT."""
    import time
    from spacedrive_amd import cas, validation
    from spacedrive_amd._native import SdgpuError
    rng = np.random.default_rng(18)
    p = os.path.join(tmp_path, "f")
    rng.integers(0, 256, 4096, dtype=np.uint8).tofile(p)
    want_cas, want_ck = O.cas_id_path(p, 4096), O.file_checksum_path(p)
    arena, off, ln = _arena([4096, 57352, 1], 3)
    for it in range(6):
        assert cas.generate_cas_id(p, 4096, svc_ctx) == want_cas
        if it % 2:
            time.sleep(0.05)                                  # idle exit
        else:
            out, st = cas.cas_batch(arena, off, ln, svc_ctx)   # bulk call stops it
            assert np.all(st == 0)
        assert validation.file_checksum(p, svc_ctx) == want_ck
    with pytest.raises(SdgpuError) as ei:
        cas.generate_cas_id(os.path.join(tmp_path, "missing"), 10, svc_ctx)
    assert ei.value.errno == 2
    for _ in range(200):                                      # back-to-back requests
        assert cas.generate_cas_id(p, 4096, svc_ctx) == want_cas


@pytest.mark.parametrize("service", [False, True])
def test_quad_tree_shapes(ctx, svc_ctx, tmp_path, service):
    """The latency kernels hash in quads of lanes and build the tree level by
    level (odd CVs carried): every chunk-count class the carries produce --
    2-9, 15-17, 31-33, 63-65 and 111-112 chunks, ragged and whole last chunks
    -- through file_checksum (the message is the file) on the launch path
    (k_small_host) and through the resident service (k_service)."""
    from spacedrive_amd import validation
    c = svc_ctx if service else ctx
    rng = np.random.default_rng(19)
    chunks = [2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 111, 112]
    for k in chunks:
        for n in {1024 * (k - 1) + 1, 1024 * (k - 1) + 700, 1024 * k}:
            p = os.path.join(tmp_path, f"q{n}")
            rng.integers(0, 256, n, dtype=np.uint8).tofile(p)
            assert validation.file_checksum(p, c) == O.file_checksum_path(p), (k, n)


def test_split_group_shapes(ctx, tmp_path):
    """file_checksum of files in (112 KiB, 1 MiB]: k_small_split hashes every
    64 KiB group on its own workgroup and the message's last group folds the
    group CVs -- 2..16 groups, a last group of 1 chunk (a lone chunk CV, no
    parent), of a ragged chunk, of 63 / 64 chunks; repeated calls (the group
    counters reset themselves)."""
    from spacedrive_amd import validation
    rng = np.random.default_rng(23)
    G = 64 * 1024
    sizes = [112 * 1024 + 1, 2 * G, 2 * G + 1, 2 * G + 1024, 2 * G + 1025, 3 * G - 1024, 3 * G - 1,
             5 * G + 7, 8 * G, 9 * G + 1, 15 * G + 1024, 16 * G - 1, 16 * G]
    for n in sizes:
        p = os.path.join(tmp_path, f"g{n}")
        rng.integers(0, 256, n, dtype=np.uint8).tofile(p)
        want = O.file_checksum_path(p)
        for _ in range(3):
            assert validation.file_checksum(p, ctx) == want, n

