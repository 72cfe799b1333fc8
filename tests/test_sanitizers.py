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
