"""Per-kernel device times of the one-GPU grouping at several table sizes
(config-4 rows; HIP events on the launch stream).  Usage:
python scripts/exp/exp_dedup_kernels.py 12500000 100000000"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spacedrive_amd import corpus, dedup  # noqa: E402
from spacedrive_amd._native import default_context  # noqa: E402

ctx = default_context(0)
ops = dedup.HipOps(ctx)
for n in [int(x) for x in sys.argv[1:]] or [12_500_000]:
    key, has, rank = corpus.synth_dedup_rows_device(4, n, int(n * 0.8), 0, n, ctx=ctx)
    for _ in range(3):
        ops.group_rows(key, has, None, 100, 0)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        ops.group_rows(key, has, None, 100, 0)
    ev[1].record()
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    ctx.set_timing(False)
    print(json.dumps({"rows": n, "wall_ms_per_call": ev[0].elapsed_time(ev[1]) / 10,
                      "kernels_ms": {k: v[0] / v[1] for k, v in kt.items()}}))
    del key, has, rank
    torch.cuda.empty_cache()
