"""GPU: no kernel reads workspace that no earlier kernel of its call wrote.

Round 6: the SDGPU_SEG_GROUPS fault was a group kernel
reading a bucket end that nothing had written yet -- harmless on a warm
workspace (the previous call's value), fatal on a fresh one.  With
SDGPU_POISON_WS=1 every workspace the library allocates starts as 0xA5
bytes (csrc/ctx.hpp ensure_dev), so such a read yields garbage instead of a
lucky zero or a stale-but-right value.  A fresh child process (the knob is
read once) runs the grouping paths on their FIRST calls -- the one-level
12-bit and the two-level partitions, the fused write set, the rep API, the
Object index, the padded exchange through a one-rank communicator -- and
every result must equal the oracle (file_identifier/mod.rs:136-333).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
from oracle import oracle as O
from spacedrive_amd import dedup
from spacedrive_amd._native import Context

ctx = Context(0)
out = {}


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


for n in (4_000_000, 13_000_000):  # one-level 12-bit, two-level
    k, h, rk = O.synth_dedup_rows(300 + n % 7, n, int(n * 0.8), 0, n)
    ref = O.group_reps(k, h, 100)
    rc, rlr, rlo = O.link_batch(ref, None, None, 0)
    dk, dh = dev(k.view(np.int64)), dev(h)
    # fused grouping + write set (implicit ranks), first call of this size
    who, obj, cnt = dedup.group_link_device(dk, dh, None, None, 0, 100, ctx=ctx, trim=False)
    torch.cuda.synchronize()
    c, l, e = (int(x) for x in cnt.cpu().tolist())
    fc, flr, flo = dedup.split_link_lists(who[:e].cpu().numpy(), obj[:e].cpu().numpy())
    out[f"fused_{n}"] = int(not (np.array_equal(fc, rc) and np.array_equal(flr, rlr)
                                 and np.array_equal(flo, rlo)))
    # the rep API with explicit ranks (16-byte records)
    dr = dev(rk.view(np.int32))
    rep = dedup.HipOps(ctx).group_rows(dk, dh, dr, 100, 0)
    torch.cuda.synchronize()
    out[f"rep_{n}"] = int(np.count_nonzero(rep.cpu().numpy().view(np.uint32) != ref))
# Object index + padded exchange through a one-rank communicator (fresh buffers)
n = 2_000_000
k, h, rk = O.synth_dedup_rows(77, n, 1_600_000, 0, n)
ref = O.group_reps(k, h, 100)
dk, dh, dr = dev(k.view(np.int64)), dev(h), dev(rk.view(np.int32))
comm = dedup.Comm.init_rank(ctx, 1, 0, dedup.Comm.unique_id())
comm.set_exchange(dedup.EXCHANGE_PADDED, n)
idx = dedup.ObjectIndex(ctx)
parts = [dedup.group_sharded(dk[a:b], dh[a:b], dr[a:b], comm, idx, 100).cpu().numpy()
         for a, b in ((0, n // 2), (n // 2, n))]
out["indexed_padded"] = int(np.count_nonzero(np.concatenate(parts).view(np.uint32) != ref))
who, obj, (c, l) = dedup.group_link_sharded(dk, dh, None, dr, comm, 100)
rc, rlr, rlo = O.link_batch(ref, None, None, 0)
fc, flr, flo = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
out["write_set_padded"] = int(not (np.array_equal(fc, rc) and np.array_equal(flr, rlr)
                                   and np.array_equal(flo, rlo)))
comm.close()
print(json.dumps(out), flush=True)
'''


def test_first_calls_on_poisoned_workspace():
    env = dict(os.environ, SDGPU_POISON_WS="1")
    p = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res and all(v == 0 for v in res.values()), res
