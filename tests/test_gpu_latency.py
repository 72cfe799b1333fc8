"""GPU parity of the single-file latency kernel (k_small: one workgroup per
message, a lane per chunk, the tree level by level in LDS): batches of <= 64
cas messages (<= 102 408 B), single files through generate_cas_id and
file_checksum up to 1 MiB (1024 chunks, the kernel's limit); checked
bit-exact against the oracle."""
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
