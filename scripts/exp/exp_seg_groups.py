"""A/B of the fused grouping + write set (sdgpu_group_link_device) over
config-4 rows: timed back to back, plus a digest of its write set (sorted
who / obj) so two builds (AB_LIB) or two settings of an env knob can be
compared for equality.  (Written in round 5 for the SDGPU_SEG_GROUPS
interleave, deleted in round 6; the file name stayed for the logs.)

    python scripts/exp/exp_seg_groups.py [rows] [steps]
"""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    if os.environ.get("AB_LIB"):  # A/B against another build of libsdgpu (scripts/gpu_r5_pk.sh)
        from spacedrive_amd import _native
        _native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from spacedrive_amd import corpus, dedup
    from spacedrive_amd._native import default_context
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = default_context(0)
    key, has, _ = corpus.synth_dedup_rows_device(4, rows, int(rows * 0.8), 0, rows, ctx=ctx)
    fn = lambda: dedup.group_link_device(key, has, None, None, 0, 100, ctx=ctx, trim=False)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0) / steps)
    ctx.set_timing(True)
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    ctx.set_timing(False)
    who, obj, cnt = fn()
    c, l, e = (int(x) for x in cnt.cpu().tolist())
    w = who[:e].to(torch.int64) & 0xFFFFFFFF
    o = torch.where(w >= 2**31, obj[:e].to(torch.int64) & 0xFFFFFFFF, torch.zeros_like(w))
    packed = torch.sort((w << 32) | o).values.cpu().numpy()
    print(json.dumps({"lib": os.environ.get("AB_LIB", "tree"), "rows": rows,
                      "ms_per_call": sorted(ts)[1], "rounds_ms": ts, "counts": [c, l, e],
                      "digest": hashlib.sha1(packed.tobytes()).hexdigest(),
                      "kernels": {k: v[0] / max(v[1], 1) for k, v in kt.items()}}))


if __name__ == "__main__":
    main()
