"""CPU: the oracle itself -- pinned by the reference KAT, two independent
restatements agreeing, the cas.rs message semantics and the grouping rule."""
import os

import numpy as np
import pytest

from oracle import blake3_py as P
from oracle import oracle as O
from tests.golden.make_golden import KAT_CONTEXT, KAT_EXPECTED, KAT_MATERIAL, pattern


def test_reference_derive_key_kat(golden):
    # /root/reference/crates/crypto/src/keys/hashing.rs:324-327 (derive_b3)
    assert golden["derive_key_kat"]["expected_hex"] == KAT_EXPECTED.hex()
    assert O.derive_key(KAT_CONTEXT, KAT_MATERIAL) == KAT_EXPECTED
    assert P.derive_key(KAT_CONTEXT, KAT_MATERIAL) == KAT_EXPECTED


def _balloon_cases():
    from tests.golden import make_golden as G
    for i, s_cost in enumerate(G.BALLOON_S_COST):
        yield s_cost, b"", G.BALLOON_EXPECTED[i]
        yield s_cost, G.BALLOON_SECRET, G.BALLOON_WITH_SECRET_EXPECTED[i]


def test_reference_balloon_blake3_kats(golden):
    """The six HASH_B3BALLOON_* vectors (/root/reference/crates/crypto/src/keys/
    hashing.rs:180-208, tests :269-321): Balloon (balloon-hash 0.4.0) over BLAKE3
    in hash mode, the mode cas.rs and hash.rs use.  C oracle, six runs in
    parallel (the ctypes call releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    from tests.golden import make_golden as G
    cases = list(_balloon_cases())
    assert [v["expected_hex"] for v in golden["balloon_blake3_kats"]["vectors"]] == \
        [e.hex() for _, _, e in cases]
    with ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda c: O.balloon_blake3(G.BALLOON_PASSWORD, G.BALLOON_SALT, c[1],
                                                      c[0], G.BALLOON_T_COST), cases))
    for (s_cost, secret, exp), g in zip(cases, got):
        assert g == exp, (s_cost, bool(secret))


@pytest.mark.parametrize("with_secret", [False, True])
def test_balloon_kat_messages_through_python_hasher(with_secret):
    """The pure-Python BLAKE3 on the KAT's own messages: every 9973rd message the
    standard-params Balloon run hashes (40/72/24/74-byte shapes, ~280 of them,
    recorded by the C run that reproduces the reference vector) hashes to the
    same digest in blake3_py.  (A full pure-Python Balloon run is ~2.7 M hashes
    at ~0.35 ms each, too slow for the suite; the Python Balloon driver itself is
    checked against the C one at small costs below.)"""
    from tests.golden import make_golden as G
    secret = G.BALLOON_SECRET if with_secret else b""
    exp = (G.BALLOON_WITH_SECRET_EXPECTED if with_secret else G.BALLOON_EXPECTED)[0]
    d, trace = O.balloon_blake3_trace(G.BALLOON_PASSWORD, G.BALLOON_SALT, secret,
                                      G.BALLOON_S_COST[0], G.BALLOON_T_COST, 9973, 400)
    assert d == exp
    assert len(trace) > 250 and {len(m) for m, _ in trace} >= {24, 40, 72}
    for m, dg in trace:
        assert P.blake3(m) == dg


@pytest.mark.parametrize("s_cost,t_cost,secret", [(1, 1, b""), (3, 2, bytes([0x55] * 18)),
                                                  (16, 3, b""), (37, 2, b"ab"),
                                                  (64, 1, bytes([0x55] * 18)), (100, 2, b"")])
def test_balloon_python_restatement_agrees(s_cost, t_cost, secret):
    """Independent pure-Python Balloon + BLAKE3 == the C restatement, including
    s_cost that are not powers of two (the 256-bit `other` reduction)."""
    assert P.balloon(b"password", bytes([0xFF] * 16), secret, s_cost, t_cost) == \
        O.balloon_blake3(b"password", bytes([0xFF] * 16), secret, s_cost, t_cost)


def test_empty_input_spec_value():
    h = "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
    assert O.blake3(b"").hex() == h
    assert P.blake3(b"").hex() == h


def test_golden_pattern_hashes(golden):
    for n, h in golden["blake3_pattern"].items():
        d = pattern(int(n))
        assert O.blake3(d).hex() == h
        if int(n) <= 8192:
            assert P.blake3(d).hex() == h


@pytest.mark.parametrize("n", [0, 1, 64, 1024, 1025, 2048, 3 * 1024 + 1, 17 * 1024, 33 * 1024 + 7,
                               100 * 1024 + 8, 131072, 300_001])
def test_tree_shapes_agree(n):
    """Recursive (C), incremental stack (C, odd update sizes), multi-threaded
    subtree split (C) and incremental (python) must agree."""
    rng = np.random.default_rng(n)
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    ref = O.blake3(d)
    assert O.blake3_incremental(d, 777) == ref
    assert O.blake3_incremental(d, 1 << 20) == ref
    assert O.blake3(d, threads=4) == ref
    if n <= 40_000:
        assert P.blake3(d) == ref


def test_keyed_hash_agrees():
    key = bytes(range(32))
    d = pattern(5000)
    assert O.keyed_hash(key, d) == P.keyed_hash(key, d)


def test_cas_message_layout_small_and_sampled():
    size = 250_000
    fb = O.synth_file_bytes(7, 0, size)
    msg = O.cas_build_message(fb, size)
    assert len(msg) == 57352
    assert msg[:8] == size.to_bytes(8, "little")
    jump = (size - 16384) // 4
    assert msg[8:8 + 8192] == fb[:8192]
    for k in range(4):
        o = 8192 + k * jump
        assert msg[8 + 8192 + k * 10240: 8 + 8192 + (k + 1) * 10240] == fb[o:o + 10240]
    assert msg[-8192:] == fb[-8192:]
    # synthetic message builder == message built from the whole file
    assert O.synth_cas_message(size, 7) == msg
    small = O.synth_file_bytes(9, 0, 5000)
    assert O.cas_build_message(small) == (5000).to_bytes(8, "little") + small


def test_cas_size_argument_semantics():
    """The samples use the passed size (cas.rs:41) but the footer the ACTUAL
    end (SeekFrom::End, cas.rs:54); a file shorter than a sample read fails
    with UnexpectedEof (read_exact)."""
    fb = O.synth_file_bytes(11, 0, 300_000)
    a = O.cas_id_of_file_bytes(fb, 300_000)
    b = O.cas_id_of_file_bytes(fb, 290_000)  # stale stat size: different samples
    assert a != b
    assert P.cas_id_of_file_bytes(fb, 290_000) == b
    with pytest.raises(EOFError):
        O.cas_id_of_file_bytes(fb[:120_000], 400_000)


def test_golden_cas_ids(golden):
    for e in golden["cas_synthetic"]:
        msg = O.synth_cas_message(e["size"], e["seed"])
        assert len(msg) == e["msg_len"]
        assert O.cas_id_of_message(msg) == e["cas_id"]


def test_path_oracle_matches_memory_oracle(tmp_path):
    for i, size in enumerate([0, 1, 1024, 102400, 102401, 250_000, 1_000_003]):
        p = tmp_path / f"f{i}"
        data = O.synth_file_bytes(100 + i, 0, size)
        p.write_bytes(data)
        assert O.cas_id_path(str(p), size) == O.cas_id_of_file_bytes(data, size)
        assert O.file_checksum_path(str(p)) == O.blake3(data).hex()
    with pytest.raises(FileNotFoundError):
        O.cas_id_path(str(tmp_path / "missing"), 10)


def test_golden_checksums(golden):
    for e in golden["checksum_synthetic"]:
        data = O.synth_file_bytes(e["seed"], 0, e["len"])
        assert O.blake3(data).hex() == e["checksum"]


def test_grouping_fixture():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "grouping_10k.npz"))
    rep = O.group_reps(z["key"], z["has_key"], int(z["chunk_rows"][0]))
    np.testing.assert_array_equal(rep, z["rep"])
    # k0 > 1 cases exist: a key first seen several times inside one chunk
    key, has = z["key"], z["has_key"]
    assert np.count_nonzero((z["rep"] == np.arange(key.size)) & (has == 1)) > 1500


def test_grouping_rule_properties():
    rng = np.random.default_rng(5)
    n = 50_000
    key = rng.integers(0, 3000, n).astype(np.uint64)
    has = (rng.random(n) > 0.05).astype(np.uint8)
    rep = O.group_reps(key, has, 100).astype(np.int64)
    r = np.arange(n)
    assert np.all(rep <= r)                      # representative never later
    assert np.all(rep[rep] == rep)               # idempotent
    assert np.all(key[rep] == key)               # same key
    assert np.all(rep[has == 0] == r[has == 0])  # keyless rows are singletons


def test_synth_arena_layout_matches_corpus_layout():
    from spacedrive_amd import corpus
    sizes, seeds = corpus.config2_files(2000, seed=3)
    arena, off, ln = O.synth_arena(sizes, seeds)
    off2, ln2, total = corpus.arena_layout(sizes)
    np.testing.assert_array_equal(off, off2)
    np.testing.assert_array_equal(ln, ln2)
    for i in range(0, 2000, 97):
        m = O.synth_cas_message(int(sizes[i]), int(seeds[i]))
        assert arena[int(off[i]):int(off[i]) + len(m)].tobytes() == m


def test_config2_distribution():
    from spacedrive_amd import corpus
    sizes, seeds = corpus.config2_files(200_000, seed=2)
    small = np.count_nonzero(sizes <= 102400) / sizes.size
    assert 0.55 < small < 0.62                   # ~58.7% <= 100 KiB
    assert np.count_nonzero(sizes == 0) == 200
    pairs = sizes.astype(np.uint64) * np.uint64(1_000_003) ^ seeds
    uniq = np.unique(pairs).size
    assert 0.78 < uniq / sizes.size < 0.82        # ~20% exact duplicates


def test_dedup_corpus_rows():
    key, has, rank = O.synth_dedup_rows(4, 100_000, 80_000, 0, 100_000)
    np.testing.assert_array_equal(rank, np.arange(100_000, dtype=np.uint32))
    assert np.unique(key).size == 80_000
    assert 60 < np.count_nonzero(has == 0) < 150
    k2, h2, r2 = O.synth_dedup_rows(4, 100_000, 80_000, 50_000, 1000)
    np.testing.assert_array_equal(k2, key[50_000:51_000])


def test_link_batch_oracle_matches_object_stats():
    """K7's oracle agrees with the (created, linked) accounting of
    identifier_job_step (file_identifier/mod.rs:335) on a grouped table."""
    from spacedrive_amd.dedup import object_stats
    key, has, _ = O.synth_dedup_rows(4, 20_000, 15_000, 0, 20_000)
    valid = (np.arange(key.size) % 37 != 0).astype(np.uint8)
    # failed rows are grouped without a key (file_identifier.identifier_job)
    rep = O.group_reps(key, has & valid, 100)
    create, lrow, lobj = O.link_batch(rep, None, valid)
    created, linked = object_stats(rep, has, valid.astype(bool))
    assert (create.size, lrow.size) == (created, linked)
    # every link target is a creator, and creators link to themselves
    assert np.isin(lobj, create).all()
    assert np.all(rep[create] == create)
    assert np.all(rep[lrow] == lobj)


def test_simd_cpu_baseline_matches_scalar_oracle():
    """The AVX2 8-way CPU-baseline hashing is bit-exact with the scalar oracle on
    every chunk-count / tail shape and on a config-2 sample."""
    from spacedrive_amd import corpus
    lens = np.array(sorted({n * 1024 + d for n in range(0, 101) for d in (-64, -1, 0, 1, 8, 65)
                            if 0 <= n * 1024 + d <= 102408} | {57352}), np.uint32)
    off = np.zeros(lens.size, np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += (int(n) + 127) // 128 * 128
    arena = np.random.default_rng(3).integers(0, 256, pos + 16, dtype=np.uint8)
    np.testing.assert_array_equal(O.cas_batch_simd(arena, off, lens, 4),
                                  O.cas_batch(arena, off, lens, 4))
    sizes, seeds = corpus.config2_files(3000, seed=8)
    ar, of, ln = O.synth_arena(sizes, seeds)
    np.testing.assert_array_equal(O.cas_batch_simd(ar, of, ln, 4), O.cas_batch(ar, of, ln, 4))


def test_simd_paths_baseline_matches_path_oracle(tmp_path):
    """The config-1 CPU baseline (reference reads per file + AVX2 hashing, C
    threads) is bit-exact with the scalar path-based oracle, errors included."""
    from spacedrive_amd import corpus
    paths, sizes = corpus.write_config1_dir(str(tmp_path / "c1"), 300, seed=4)
    paths = paths + [str(tmp_path / "missing")]
    sizes = np.concatenate([sizes, np.array([10], np.uint64)])
    out, st = O.cas_paths_simd(paths, sizes, 4)
    assert st[-1] == -2 and np.all(st[:-1] == 0)
    for p, s, o in zip(paths[:-1], sizes[:-1].tolist(), out[:-1]):
        assert bytes(o).hex() == O.cas_id_path(p, s)


def test_simd_file_hasher_matches_oracle():
    """The config-3 CPU baseline's AVX2 subtree hasher (1024-chunk subtrees on
    the CV stack, tail through the incremental hasher) is bit-exact with the
    recursive oracle around every subtree boundary it has."""
    S = 1024 * 1024
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 5 * S + 3000, dtype=np.uint8)
    for n in (0, 1, 1024, 1025, S - 1, S, S + 1, 2 * S, 2 * S + 1, 3 * S + 777, 4 * S,
              4 * S + 1024, 5 * S + 3000):
        assert O.blake3_simd(data[:n]) == O.blake3(data[:n].tobytes()), n
    assert O.checksum_simd_mt(data[:3 * S + 5], 3, 2) == O.blake3(data[:3 * S + 5].tobytes())


def test_simd_widths_agree_with_the_scalar_oracle():
    """The CPU baseline's SIMD hashers at both widths (AVX-512 16-way where the
    host has it, AVX2 8-way forced by ORC_SIMD_WIDTH=8, in a subprocess since
    the width is chosen once per process) against the scalar oracle."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
rng = np.random.default_rng(3)
lens = [1025, 8 * 1024, 16 * 1024, 16 * 1024 + 5, 24 * 1024 + 1, 57352, 102408]
buf = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
arena = np.concatenate(buf)
off = np.cumsum([0] + lens[:-1]).astype(np.uint64)
ln = np.array(lens, np.uint32)
assert np.array_equal(O.cas_batch(arena, off, ln), O.cas_batch_simd(arena, off, ln))
d = rng.integers(0, 256, (3 << 20) + 77, dtype=np.uint8)
assert O.blake3(d) == O.blake3_simd(d)
print(O.simd_isa())
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for env in ({}, {"ORC_SIMD_WIDTH": "8"}):
        r = subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True,
                           env={**os.environ, **env}, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        if env:
            assert r.stdout.strip() == "AVX2 8-way"
