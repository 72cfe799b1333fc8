"""The C ABI from a plain C host (tests/c/abi_demo.c, tests/c/ranks_demo.c):
the header compiles as C99 and the programs link against libsdgpu.so on the
CPU; on the GPU box abi_demo runs against the golden vectors and ranks_demo
runs the sharded write set with one process per rank against the oracle."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "spacedrive_amd")


def _build(out, src="abi_demo.c"):
    cmd = ["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c", src), "-L", LIBDIR, "-lsdgpu",
           f"-Wl,-rpath,{LIBDIR}", "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_header_is_c99_and_links(tmp_path):
    _build(tmp_path / "abi_demo")
    assert (tmp_path / "abi_demo").exists()
    _build(tmp_path / "ranks_demo", "ranks_demo.c")
    assert (tmp_path / "ranks_demo").exists()


def _splitmix64(x):
    import numpy as np
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_c_host_one_process_per_rank(tmp_path, world):
    """tests/c/ranks_demo.c: a plain C host forks one process per rank before
    any GPU call; every rank joins the communicator and runs the write-set
    exchange (counted, then two padded calls resolved across the processes)
    through the C ABI alone.  The union of the ranks' lists is the oracle's
    write set of all rows (file_identifier/mod.rs:189-333)."""
    import numpy as np
    from oracle import oracle as O
    from spacedrive_amd import dedup
    exe = tmp_path / "ranks_demo"
    _build(exe, "ranks_demo.c")
    total, distinct = 300_000, 240_000
    r = subprocess.run([str(exe), str(world), str(total), str(distinct), str(tmp_path)],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "c ranks ok" in r.stdout
    g = np.arange(total, dtype=np.uint64)
    key = _splitmix64(np.uint64(0x5D00) + g % np.uint64(distinct))
    has = (g % np.uint64(997) != 0).astype(np.uint8)
    who, obj = [], []
    for rk in range(world):
        raw = np.fromfile(tmp_path / f"rank{rk}.bin", dtype=np.uint32)
        e = int(raw[0])
        who.append(raw[1:1 + e])
        obj.append(raw[1 + e:1 + 2 * e])
    c, lr, lo = dedup.split_link_lists(np.concatenate(who), np.concatenate(obj))
    rc, rlr, rlo = O.link_batch(O.group_reps(key, has, 100), None, None, 0)
    np.testing.assert_array_equal(c, rc)
    np.testing.assert_array_equal(lr, rlr)
    np.testing.assert_array_equal(lo, rlo)
    # every rank: one counted call, then the padded ones
    for line in r.stdout.splitlines():
        if line.startswith("rank "):
            assert "calls 3 padded 2" in line, line


@pytest.mark.gpu
def test_c_host_end_to_end(tmp_path):
    exe = tmp_path / "abi_demo"
    _build(exe)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    vec = tmp_path / "vectors.txt"
    vec.write_text("".join(f"{n} {h}\n" for n, h in g["blake3_pattern"].items()))
    r = subprocess.run([str(exe), str(vec), str(tmp_path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "c abi ok" in r.stdout
