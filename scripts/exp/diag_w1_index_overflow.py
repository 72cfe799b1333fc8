"""Diagnostic (round 6): a padded call that overflows at ONE peer rank with an
Object index.  Runs the failing batch sequence of
test_random_batches_through_sharded_indexes[1] and variants
(counted, two and three ranks), and classifies the mismatching rows against
the oracle.  Found in round 6: at one rank the _all entry point left the
overflowed padded call pending (its reps returned unresolved); fixed in
shard.cpp run_call (all_form), after which every batch equals the oracle
(profiles/r6/r6z5_diag_before_fix.log, r6z6_diag_after_fix.log)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from spacedrive_amd import dedup  # noqa: E402
from spacedrive_amd._native import Context  # noqa: E402

EXIST = np.uint32(0x80000000)


def run(world, use_index, mode_over, cuts, k, h, ek, eh, ref, ctxs, label):
    comms = dedup.Comm.init_all(ctxs[:world])
    idxs = [dedup.ObjectIndex(c, 1000) for c in ctxs[:world]] if use_index else None
    if idxs:
        for r, ix in enumerate(idxs):
            ix.add_objects(torch.from_numpy(ek.view(np.int64)).cuda(),
                           torch.from_numpy(eh.view(np.int32)).cuda(), world, r)
    out = np.zeros(k.size, np.uint32)
    for bi, (b0, b1) in enumerate(zip(cuts[:-1], cuts[1:])):
        m = b1 - b0
        if bi == 1:
            mode, hint = mode_over, max(1, m // (8 * world))
        else:
            mode, hint = dedup.EXCHANGE_COUNTED, m // world + 1
        for c in comms:
            c.set_exchange(mode, hint)
            c.set_return(dedup.RETURN_AUTO)
        spans = [(b0 + m * r // world, b0 + m * (r + 1) // world) for r in range(world)]
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        reps = dedup.group_sharded_all(
            [dev(k[a:b].view(np.int64)) for a, b in spans], [dev(h[a:b]) for a, b in spans],
            [torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda() for a, b in spans],
            comms, idxs, 100)
        for (a, b), rp in zip(spans, reps):
            out[a:b] = rp.cpu().numpy().view(np.uint32)
        r_ = ref[b0:b1]
        bad = np.flatnonzero(out[b0:b1] != r_)
        st = comms[0].stats()
        msg = f"{label} batch {bi} [{b0},{b1}) mode {mode} hint {hint}: {bad.size} bad"
        if bad.size:
            g, w = out[b0:b1][bad], r_[bad]
            rows = bad + b0
            cats = {
                "ref_self": int(np.sum(w == rows)),
                "ref_existing": int(np.sum((w & EXIST) != 0)),
                "ref_earlier_batch": int(np.sum(((w & EXIST) == 0) & (w < b0))),
                "ref_this_batch_other": int(np.sum(((w & EXIST) == 0) & (w >= b0) & (w != rows))),
                "got_self": int(np.sum(g == rows)),
                "got_existing": int(np.sum((g & EXIST) != 0)),
                "got_earlier": int(np.sum(((g & EXIST) == 0) & (g < b0))),
                "got_this_other": int(np.sum(((g & EXIST) == 0) & (g >= b0) & (g != rows))),
            }
            msg += f" {cats} e.g. rows {rows[:4]} got {g[:4]} want {w[:4]}"
        print(msg, "reruns", st["overflow_reruns"], "padded", st["padded_calls"], flush=True)
    for c in comms:
        c.close()
    if idxs:
        for ix in idxs:
            ix.close()


def main():
    world = 1
    rng = np.random.default_rng(1200 + world)
    total = 600_000
    k, h, _ = O.synth_dedup_rows(1300 + world, total, 400_000, 0, total)
    hot = rng.choice(total, 30_000, replace=False)
    k[hot[hot > 100_000]] = k[17]
    ek = rng.choice(k, 2000)
    ek[0] = k[17]
    eh = np.arange(ek.size, dtype=np.uint32) + 5
    eh[0] = 0x7FFFFFFF
    ref = O.group_reps_existing(k, h, 100, ek, eh)
    cuts = np.array([0, 65489, 231439, 400000, 600000])
    ctxs = [Context(0) for _ in range(3)]
    run(1, True, dedup.EXCHANGE_PADDED, cuts, k, h, ek, eh, ref, ctxs, "W1 index padded-overflow")
    run(1, True, dedup.EXCHANGE_COUNTED, cuts, k, h, ek, eh, ref, ctxs, "W1 index counted")
    run(2, True, dedup.EXCHANGE_PADDED, cuts, k, h, ek, eh, ref, ctxs, "W2 index padded-overflow")
    run(3, True, dedup.EXCHANGE_PADDED, cuts, k, h, ek, eh, ref, ctxs, "W3 index padded-overflow")
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
