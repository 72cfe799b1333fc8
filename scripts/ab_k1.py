#!/usr/bin/env python3
"""Interleaved A/B of K1 variants in ONE process (config 2, 1 M files).
Usage: python scripts/ab_k1.py [variants=0,1] [rounds=5] [files=1000000]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from spacedrive_amd import cas, corpus
    from spacedrive_amd._native import default_context
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    ctx = default_context(0)
    sizes, seeds = corpus.config2_files(n, seed=2)
    arena, off, ln = corpus.synth_arena_device(sizes, seeds, ctx=ctx)
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = None
    res = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            os.environ["SDGPU_K1_VARIANT"] = str(v)
            cas.cas_batch_device(arena, off, ln, out, st, ctx=ctx)  # warm
            torch.cuda.synchronize()
            ctx.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(3):
                cas.cas_batch_device(arena, off, ln, out, st, ctx=ctx)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / 3
            kt = ctx.kernel_times()
            ctx.set_timing(False)
            got = out.cpu().numpy()
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), f"variant {v} differs"
            res[v].append((wall * 1e3, {k: t[0] / 3 for k, t in kt.items()}))
    for v in variants:
        walls = np.array([w for w, _ in res[v]])
        names = sorted(res[v][0][1])
        per = {k: np.median([d[k] for _, d in res[v]]) for k in names}
        ks = " | ".join(f"{k} {per[k]:.3f}" for k in names)
        print(f"K1 variant {v}: wall ms median {np.median(walls):.3f} min {walls.min():.3f} | "
              f"{ks} | files/s {n / np.median(walls) * 1e3:.3e}  (bit-identical to variant "
              f"{variants[0]})")


if __name__ == "__main__":
    main()
