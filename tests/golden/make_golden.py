"""Generates the golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

Every value is computed by the C oracle (oracle/sd_oracle.c) AND by the
independent pure-Python restatement (oracle/blake3_py.py); the script refuses
to write a fixture on any disagreement.  Both restatements are pinned by the
reference's own BLAKE3 known-answer tests (derive_b3,
/root/reference/crates/crypto/src/keys/hashing.rs:210-213,324-327, the first
entry of golden.json; and the six hash-mode Balloon-BLAKE3 vectors, :180-208,
269-321, the second).  No reference code is executed or copied: the
reference is Rust and its toolchain / the blake3 crate are absent.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import blake3_py as P  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# derive_b3 KAT (hashing.rs:121 context, :132-141 KEY/SALT, types.rs:164-166 order)
KAT_CONTEXT = "spacedrive 2023-02-09 17:44:14 test key derivation"
KAT_MATERIAL = bytes([0x23] * 32 + [0xFF] * 16)
KAT_EXPECTED = bytes([27, 34, 251, 101, 201, 89, 78, 90, 20, 175, 62, 206, 200, 153, 166, 103,
                      118, 179, 194, 44, 216, 26, 48, 120, 137, 157, 60, 234, 234, 53, 46, 60])

# Balloon-BLAKE3 KATs (hashing.rs:130 password, :138-141 salt, :143-146 secret,
# :58-63 params, expected :180-208; tests :269-321).  [0] standard, [1] hardened,
# [2] paranoid -- BLAKE3 in hash mode, the mode of cas.rs / hash.rs.
BALLOON_PASSWORD = b"password"
BALLOON_SALT = bytes([0xFF] * 16)
BALLOON_SECRET = bytes([0x55] * 18)
BALLOON_S_COST = [131_072, 262_144, 524_288]
BALLOON_T_COST = 2
BALLOON_EXPECTED = [
    bytes([105, 36, 165, 219, 22, 136, 156, 19, 32, 143, 237, 150, 236, 194, 70, 113, 73, 137,
           243, 106, 80, 31, 43, 73, 207, 210, 29, 251, 88, 6, 132, 77]),
    bytes([179, 71, 60, 122, 54, 72, 132, 209, 146, 96, 15, 115, 41, 95, 5, 75, 214, 135, 6, 122,
           82, 42, 158, 9, 117, 19, 19, 40, 48, 233, 207, 237]),
    bytes([233, 60, 62, 184, 29, 152, 111, 46, 239, 126, 98, 90, 211, 255, 151, 0, 10, 189, 61,
           84, 229, 11, 245, 228, 47, 114, 87, 74, 227, 67, 24, 141]),
]
BALLOON_WITH_SECRET_EXPECTED = [
    bytes([188, 0, 43, 39, 137, 199, 91, 142, 97, 31, 98, 6, 130, 75, 251, 71, 150, 109, 29, 62,
           237, 171, 210, 22, 139, 108, 94, 190, 91, 74, 134, 47]),
    bytes([19, 247, 102, 192, 129, 184, 29, 147, 68, 215, 234, 146, 153, 221, 65, 134, 68, 120,
           207, 209, 184, 246, 127, 131, 9, 245, 91, 250, 220, 61, 76, 248]),
    bytes([165, 240, 162, 25, 172, 3, 232, 2, 43, 230, 226, 128, 174, 28, 211, 61, 139, 136, 221,
           197, 16, 83, 221, 18, 212, 190, 138, 79, 239, 148, 89, 215]),
]

HASH_LENGTHS = [0, 1, 2, 63, 64, 65, 127, 128, 129, 1023, 1024, 1025, 2047, 2048, 2049, 3072,
                3073, 4096, 4097, 5120, 5121, 6144, 7168, 8192, 8193, 16384, 31744, 31745, 65536,
                102400, 102408, 102409]
CAS_SIZES = [0, 1, 55, 56, 57, 63, 64, 65, 1015, 1016, 1017, 1023, 1024, 1025, 2040, 2048, 4096,
             8192, 16384, 65536, 102391, 102392, 102399, 102400, 102401, 102402, 118784, 131072,
             1 << 20, (1 << 20) + 3, 10 * (1 << 20) + 7, (1 << 32) + 1]
CHECKSUM_LENGTHS = [0, 1, 1024, 1025, 16384, 16385, (1 << 20) - 1, 1 << 20, (1 << 20) + 1,
                    3 * (1 << 20) + 12345]


def pattern(n: int) -> bytes:
    """BLAKE3 test-vector style input: byte i = i % 251."""
    return bytes(i % 251 for i in range(n))


def main():
    assert O.derive_key(KAT_CONTEXT, KAT_MATERIAL) == KAT_EXPECTED, "C oracle fails the KAT"
    assert P.derive_key(KAT_CONTEXT, KAT_MATERIAL) == KAT_EXPECTED, "py oracle fails the KAT"
    g = {"derive_key_kat": {"context": KAT_CONTEXT, "material_hex": KAT_MATERIAL.hex(),
                            "expected_hex": KAT_EXPECTED.hex(),
                            "source": "crates/crypto/src/keys/hashing.rs:210-213,324-327"}}
    bal = []
    for i, s_cost in enumerate(BALLOON_S_COST):
        for secret, exp in ((b"", BALLOON_EXPECTED[i]), (BALLOON_SECRET, BALLOON_WITH_SECRET_EXPECTED[i])):
            got = O.balloon_blake3(BALLOON_PASSWORD, BALLOON_SALT, secret, s_cost, BALLOON_T_COST)
            assert got == exp, ("C oracle fails a Balloon-BLAKE3 KAT", s_cost, bool(secret))
            bal.append({"s_cost": s_cost, "t_cost": BALLOON_T_COST, "secret_hex": secret.hex(),
                        "expected_hex": exp.hex()})
    g["balloon_blake3_kats"] = {"password_hex": BALLOON_PASSWORD.hex(), "salt_hex": BALLOON_SALT.hex(),
                                "vectors": bal,
                                "source": "crates/crypto/src/keys/hashing.rs:58-63,95-114,180-208,269-321"}
    hashes = {}
    for n in HASH_LENGTHS:
        d = pattern(n)
        a, b = O.blake3(d).hex(), P.blake3(d).hex()
        assert a == b, n
        hashes[str(n)] = a
    g["blake3_pattern"] = hashes
    assert hashes["0"] == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"

    cas = []
    for i, size in enumerate(CAS_SIZES):
        seed = 0x1234_5678_9ABC_0000 + i
        msg = O.synth_cas_message(size, seed)
        cid = O.cas_id_of_message(msg)
        if size <= (1 << 21):  # independent check from whole file bytes (python path)
            fb = O.synth_file_bytes(seed, 0, size)
            assert P.cas_id_of_file_bytes(fb, size) == cid, size
            assert O.cas_id_of_file_bytes(fb, size) == cid, size
        else:
            assert P.blake3(msg).hex()[:16] == cid, size
        cas.append({"size": size, "seed": seed, "msg_len": len(msg), "cas_id": cid})
    g["cas_synthetic"] = cas

    cks = []
    for i, n in enumerate(CHECKSUM_LENGTHS):
        seed = 0xC0FFEE_0000 + i
        data = O.synth_file_bytes(seed, 0, n)
        h = O.blake3(data).hex()
        assert O.blake3_incremental(data, 1 << 20) == bytes.fromhex(h)
        if n <= 64 * 1024:
            assert P.blake3(data).hex() == h, n
        cks.append({"len": n, "seed": seed, "checksum": h})
    g["checksum_synthetic"] = cks

    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)

    # grouping fixture: 10 000 rows, keys drawn from a small pool so most keys
    # repeat, several times inside one 100-row chunk (k0 > 1), 1% empty rows.
    rng = np.random.default_rng(20240601)
    n = 10_000
    pool = rng.integers(0, 2**63, 1500, dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        np.uint64(1)
    key = pool[rng.integers(0, pool.size, n)]
    key[rng.choice(n, 40, replace=False)] = np.uint64(2**64 - 1)  # sentinel-valued key
    has = (rng.random(n) > 0.01).astype(np.uint8)
    rep = O.group_reps(key, has, 100)
    # independent check of the rule in plain numpy/python
    first = {}
    for r in range(n):
        if has[r] and int(key[r]) not in first:
            first[int(key[r])] = r
    for r in range(n):
        if not has[r]:
            assert rep[r] == r
        else:
            f = first[int(key[r])]
            assert rep[r] == (r if r // 100 == f // 100 else f)
    np.savez_compressed(os.path.join(OUT, "grouping_10k.npz"), key=key, has_key=has, rep=rep,
                        chunk_rows=np.array([100]))
    print("wrote golden.json and grouping_10k.npz")


if __name__ == "__main__":
    main()
