"""CPU: the oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5 'race detection / sanitizers': host code only; GPU ASan is not
available on this pool).  Builds oracle/sd_oracle.c with oracle/sanitize_main.c
into a temporary binary and runs it."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "oracle_san"
    cmd = ["gcc", "-O1", "-g", "-march=x86-64-v3", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-pthread",
           os.path.join(ROOT, "oracle", "sd_oracle.c"),
           os.path.join(ROOT, "oracle", "sanitize_main.c"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    # verify_asan_link_order=0: the environment may preload its own library
    # ahead of the ASan runtime; it is left in place
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ok" in r.stdout


def _build_run_host(tmp_path, flags, env_extra):
    exe = tmp_path / "host_san"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-pthread",
           os.path.join(ROOT, "tests", "c", "host_sanitize.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    data = tmp_path / "files"
    data.mkdir()
    env = dict(os.environ, **env_extra)
    r = subprocess.run([str(exe), str(data)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_io_and_tree_plan_clean_under_asan_ubsan(tmp_path):
    """libsdgpu's host-only C++ (file reads with cas.rs semantics, the thread
    pool, slab layout, the checksum tree plan: csrc/host_io.hpp, tree_plan.hpp)
    under AddressSanitizer + UndefinedBehaviorSanitizer."""
    _build_run_host(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                    {"ASAN_OPTIONS": "detect_leaks=1:verify_asan_link_order=0",
                     "UBSAN_OPTIONS": "print_stacktrace=1"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_thread_pool_clean_under_tsan(tmp_path):
    """The same driver under ThreadSanitizer (parallel_for's work counter and the
    per-index callbacks the staging producers run concurrently)."""
    _build_run_host(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
