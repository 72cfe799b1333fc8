#!/usr/bin/env python3
"""Where does the identifier job step's time beyond K1 go?  Config 2, 1 M
files: K1 alone, K1 + grouping, K1 + grouping + link batch, and the grouping /
link batch alone (device-resident inputs), wall time per step."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from spacedrive_amd import cas, corpus, dedup
    from spacedrive_amd._native import default_context
    ctx = default_context(0)
    n = 1_000_000
    sizes, seeds = corpus.config2_files(n, seed=2)
    arena, off, ln = corpus.synth_arena_device(sizes, seeds, ctx=ctx)
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    has = torch.from_numpy((sizes != 0).astype(np.uint8)).cuda()
    grank = torch.arange(0, n, dtype=torch.int64, device="cuda").to(torch.int32)
    ops = dedup.HipOps(ctx)

    def k1():
        cas.cas_batch_device(arena, off, ln, out, st, ctx=ctx)

    def grp():
        return dedup.sharded_group_reps(out.view(torch.int64).view(-1), has, grank, 100, ops=ops)

    def link(rep):
        dedup.link_batch_device(rep, grank, None, 0, ctx=ctx, trim=False)

    def t(fn, k):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    k1()
    rep = grp()
    for r in range(3):
        a = t(k1, 5)
        b = t(lambda: (k1(), grp()), 5)
        c = t(lambda: link(grp()) if k1() is None else None, 5)
        g = t(grp, 50)
        gl = t(lambda: link(grp()), 50)
        lk = t(lambda: link(rep), 50)
        print(f"round {r}: K1 {a:.3f} ms | K1+group {b:.3f} | K1+group+link {c:.3f} | "
              f"group {g:.3f} | group+link {gl:.3f} | link {lk:.3f}", flush=True)


if __name__ == "__main__":
    main()
