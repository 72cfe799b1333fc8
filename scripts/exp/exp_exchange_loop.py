"""Exchange-path timing on one GPU (round 5): back-to-back sharded calls of
12.5 M config-4 rows through a ONE-rank RCCL communicator, per exchange mode
(counted / padded) and form (write set / rep), plus the fused one-GPU call
for reference.  Prints one JSON line; run under rocprofv3 --kernel-trace to
see the timeline (scripts/exp/timeline.py).

    python scripts/exp/exp_exchange_loop.py [rows] [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from spacedrive_amd import corpus, dedup
    from spacedrive_amd._native import default_context
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = default_context(0)
    key, has, rank = corpus.synth_dedup_rows_device(4, 100_000_000, 80_000_000, 0, rows, ctx=ctx)
    torch.cuda.synchronize()
    comm = dedup.Comm.init_rank(ctx, 1, 0, dedup.Comm.unique_id(), timeout_ms=60000)
    res = {"rows": rows, "steps": steps}

    def timed(name, fn):
        fn()
        comm.wait()
        torch.cuda.synchronize()
        s0 = comm.stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        comm.wait()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / steps
        s1 = comm.stats()
        res[name] = {"ms": 1e3 * t, "padded": s1["padded_calls"] - s0["padded_calls"],
                     "reruns": s1["overflow_reruns"] - s0["overflow_reruns"],
                     "resolve_wait_ms": (s1["resolve_wait_ms"] - s0["resolve_wait_ms"]) / steps,
                     "count_wait_ms": (s1["count_wait_ms"] - s0["count_wait_ms"]) / steps,
                     "host_ms": (s1["host_ms"] - s0["host_ms"]) / steps}

    modes = os.environ.get("MODES", "fused,write_set_counted,rep_counted,write_set_padded,"
                           "rep_padded").split(",")
    sel = lambda name, fn: timed(name, fn) if name in modes else None  # noqa: E731
    sel("fused", lambda: dedup.group_link_device(key, has, has, rank, 0, 100, ctx=ctx, trim=False))
    ws = lambda: dedup.group_link_sharded(key, has, None, rank, comm, 100, trim=False)  # noqa: E731
    rp = lambda: dedup.group_sharded(key, has, rank, comm, None, 100, wait=False)  # noqa: E731
    comm.set_exchange(dedup.EXCHANGE_COUNTED)
    sel("write_set_counted", ws)
    sel("rep_counted", rp)
    comm.set_exchange(dedup.EXCHANGE_AUTO)
    sel("write_set_padded", ws)
    sel("rep_padded", rp)
    comm.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
