"""Timing of the f4 consumers (thumbnail-shard grouping of 1 M rows, orphan
remover over 10 M Objects / 12.5 M file_paths) for an A/B of libsdgpu builds
(AB_LIB, as scripts/exp/exp_seg_groups.py).  Prints one JSON line.

    AB_LIB=build/ab/libsdgpu_prev.so python scripts/exp/exp_consumers.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    if os.environ.get("AB_LIB"):
        from spacedrive_amd import _native
        _native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from spacedrive_amd import consumers
    from spacedrive_amd._native import default_context
    ctx = default_context(0)
    rng = np.random.default_rng(5)
    cas8 = torch.from_numpy(rng.integers(0, 256, (1_000_000, 8), dtype=np.uint8)).cuda()
    obj = torch.arange(10_000_000, dtype=torch.int32, device="cuda")
    fp = torch.from_numpy(rng.integers(-1, 10_000_000, 12_500_000, dtype=np.int64).astype(np.int32)).cuda()

    def timed(fn, steps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        best = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            best.append(1e3 * (time.perf_counter() - t0) / steps)
        return sorted(best)[1]

    th = timed(lambda: consumers.thumbnail_shards(cas8, ctx=ctx, trim=False))
    orph = timed(lambda: consumers.orphan_objects(obj, fp, 10_000_000, ctx, trim=False))
    o, c = consumers.thumbnail_shards(cas8, ctx=ctx)
    print(json.dumps({"lib": os.environ.get("AB_LIB", "tree"), "thumbnail_ms": th, "orphan_ms": orph,
                      "digest": int(o.to(torch.int64).sum().item()) ^ int(c.sum().item())}))


if __name__ == "__main__":
    main()
