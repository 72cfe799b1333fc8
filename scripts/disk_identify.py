#!/usr/bin/env python3
"""Config 5 ON DISK (VERDICT r2 missing 3): the identifier's
staging from real files at scale.  Writes N sparse files with the config-2
size distribution (only the bytes generate_cas_id reads hold data, cas.rs:
27-58; content = the synthetic-corpus function of (size, seed), so duplicates
are real duplicates), then times sdgpu_identify_files over all of them (pread
or io_uring into pinned slabs -> H2D -> K1) with a warm page cache, checks
every cas id against the oracle's hash of the same messages, and times the
CPU port behind the reference's per-file reads (oracle orc_cas_paths_simd) on
the same files and threads.  Prints one JSON line.

    python scripts/disk_identify.py [--files 200000] [--root DIR] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_files(root, sizes, seeds):
    from oracle import oracle as O
    hf, ss = 8192, 10240
    paths = []
    for i, (sz, sd) in enumerate(zip(sizes.tolist(), seeds.tolist())):
        d = os.path.join(root, f"d{i // 4096:03d}")
        if i % 4096 == 0:
            os.makedirs(d, exist_ok=True)
        p = os.path.join(d, f"f{i:07d}")
        msg = O.synth_cas_message(sz, sd)[8:]
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            if sz <= 100 * 1024:
                os.pwrite(fd, msg, 0)
            else:
                jump = (sz - 2 * hf) // 4
                spans = [(0, hf)] + [(hf + k * jump, ss) for k in range(4)] + [(sz - hf, hf)]
                pos = 0
                for o, ln in spans:
                    os.pwrite(fd, msg[pos:pos + ln], o)
                    pos += ln
                os.ftruncate(fd, sz)
        finally:
            os.close(fd)
        paths.append(p)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=200_000)
    ap.add_argument("--root", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    from oracle import oracle as O
    from spacedrive_amd import corpus
    from spacedrive_amd import file_identifier as fi
    from spacedrive_amd._native import default_context
    root = args.root or tempfile.mkdtemp(prefix="sd_cfg5_disk_")
    free = shutil.disk_usage(root).free
    sizes, seeds = corpus.config2_files(args.files, seed=55)
    t0 = time.perf_counter()
    paths = write_files(root, sizes, seeds)
    t_write = time.perf_counter() - t0
    used = sum(os.stat(p).st_blocks * 512 for p in paths[:: max(1, len(paths) // 2000)]) * \
        max(1, len(paths) // 2000)
    try:
        ctx = default_context(0)
        plist = fi.PathList(paths)
        res = fi.identify(plist, sizes=sizes, ctx=ctx)          # warm the page cache
        ts = []
        for _ in range(args.reps):
            t1 = time.perf_counter()
            res = fi.identify(plist, sizes=sizes, ctx=ctx)
            ts.append(time.perf_counter() - t1)
        ctx.set_timing(True)
        fi.identify(plist, sizes=sizes, ctx=ctx)
        phases = {k: {"ms": v[0], "n": v[1]} for k, v in ctx.kernel_times().items()}
        ctx.set_timing(False)
        # parity: every cas id vs the oracle's hash of the same messages
        arena, off, ln = O.synth_arena(sizes, seeds)
        ref = O.cas_batch(arena, off, ln, threads=args.threads)
        keyed = sizes != 0
        bad = int(np.count_nonzero(np.any(res.cas8[keyed] != ref[keyed], axis=1)))
        bad += int(np.count_nonzero(res.has_key[keyed] != 1)) + int(np.count_nonzero(res.status))
        del arena
        # the CPU port behind the reference's reads, same files and threads
        O.cas_paths_simd(paths[:2000], sizes[:2000], args.threads)
        t2 = time.perf_counter()
        cpu8, cst = O.cas_paths_simd(paths, sizes, args.threads)
        t_cpu = time.perf_counter() - t2
        bad_cpu = int(np.count_nonzero(np.any(cpu8[keyed] != ref[keyed], axis=1)))
        best = min(ts)
        print(json.dumps({
            "workload": f"config 5 on disk: {len(paths)} sparse config-2 files (seed 55), warm "
                        "page cache, sdgpu_identify_files (reads into pinned slabs -> H2D -> K1)",
            "files": len(paths), "gpu_files_per_s": len(paths) / best,
            "gpu_seconds": ts, "phases_one_call": phases,
            "cpu_port_files_per_s": len(paths) / t_cpu, "cpu_threads": args.threads,
            "gpu_vs_cpu": t_cpu / best,
            "cas_id_mismatches_vs_oracle": bad, "cpu_port_mismatches": bad_cpu,
            "write_seconds": t_write, "disk_bytes_est": used, "disk_free_before": free,
            "window_bytes": int(ln.astype(np.int64).sum()),
        }), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
