"""The padded exchange's partition (k_part_padded, timer "shard_padded") at
W ranks on one GPU (peer transport, one context per rank): per-rank kernel
time of sdgpu_group_link_sharded_all_device calls over `rows` rows in all,
for an A/B of libsdgpu builds (AB_LIB, as exp_seg_groups.py).

    AB_LIB=build/ab/libsdgpu_prev.so python scripts/exp/exp_padded_world.py [world] [rows]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    if os.environ.get("AB_LIB"):
        from spacedrive_amd import _native
        _native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from spacedrive_amd import corpus, dedup
    from spacedrive_amd._native import Context
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 12_500_000
    ctxs = [Context(0) for _ in range(world)]
    key, has, rank = corpus.synth_dedup_rows_device(4, 100_000_000, 80_000_000, 0, rows, ctx=ctxs[0])
    per = rows // world
    keys = [key[r * per:(r + 1) * per] for r in range(world)]
    hass = [has[r * per:(r + 1) * per] for r in range(world)]
    vals = [torch.ones(per, dtype=torch.uint8, device="cuda") for _ in range(world)]
    ranks = [rank[r * per:(r + 1) * per] for r in range(world)]
    comms = dedup.Comm.init_all(ctxs)
    for c in comms:
        c.set_exchange(dedup.EXCHANGE_PADDED, per)
    for _ in range(3):
        parts = dedup.group_link_sharded_all(keys, hass, vals, ranks, comms, 100)
    torch.cuda.synchronize()
    for c in ctxs:
        c.set_timing(True)
    for _ in range(10):
        parts = dedup.group_link_sharded_all(keys, hass, vals, ranks, comms, 100)
    torch.cuda.synchronize()
    t = [c.kernel_times().get("shard_padded", (0.0, 1)) for c in ctxs]
    digest = sum(int(p[2][0]) * 3 + int(p[2][1]) for p in parts)
    print(json.dumps({"lib": os.environ.get("AB_LIB", "tree"), "world": world, "rows": rows,
                      "shard_padded_ms": float(np.mean([a / max(n, 1) for a, n in t])),
                      "reruns": comms[0].stats()["overflow_reruns"], "digest": digest}))
    for c in comms:
        c.close()


if __name__ == "__main__":
    main()
