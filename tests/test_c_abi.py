"""The C ABI from a plain C host (tests/c/abi_demo.c): the header compiles as
C99 and the program links against libsdgpu.so on the CPU; on the GPU box it
runs against the golden vectors."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "spacedrive_amd")


def _build(out):
    cmd = ["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c", "abi_demo.c"), "-L", LIBDIR, "-lsdgpu",
           f"-Wl,-rpath,{LIBDIR}", "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_header_is_c99_and_links(tmp_path):
    _build(tmp_path / "abi_demo")
    assert (tmp_path / "abi_demo").exists()


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
