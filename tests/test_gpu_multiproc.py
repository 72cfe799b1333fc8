"""GPU: shard.cpp's one-rank-per-process exchange with W > 1 processes
(VERDICT r5 item 2 / missing 1).

Each rank is its own process on the one GPU, joined through
sdgpu_comm_init_host (SDGPU_TRANSPORT_HOST, ABI 6: the same messages in the
same order as the RCCL transport, staged through a shared host mapping,
because RCCL refuses two ranks on one device).  So every call goes through
the path `bench.py --gpus N` takes under RCCL: run_call's single-rank branch,
a padded call left pending and resolved by the next call or Comm.wait()
(resolve_pending), agreed_n learned by each rank on its own, the overflow
re-run issued by every rank in the same collective order, the deferred
-ENOSPC, the layout agreement and the bounded failure when a rank leaves.
Every result is checked against the oracle's grouping of all rows
(file_identifier/mod.rs:136-333; O.group_reps / O.link_batch) by this parent
process; the ranks (tests/_host_rank.py) never import the oracle.
"""
import errno
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from oracle import oracle as O
from spacedrive_amd import dedup

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = ("uniform", "one_key_40k", "all_one_key")
TOTAL = 300_000


def _rows(case, total, seed):
    rng = np.random.default_rng(seed)
    if case == "uniform":
        k, h, _ = O.synth_dedup_rows(seed, total, int(total * 0.8), 0, total)
        return k, h
    pool = rng.integers(0, 2**64 - 1, total, dtype=np.uint64, endpoint=True)
    k = pool[rng.integers(0, pool.size // 2, total)]
    if case == "one_key_40k":
        k[rng.choice(total, 40_000, replace=False)] = pool[7]
    else:
        k[:] = pool[7]
    h = (rng.random(total) > 0.01).astype(np.uint8)
    return k, h


def _spans(total, world):  # uneven shares, contiguous, in rank order
    return np.array([(total * r * (r + 1) // (world * (world + 1)),
                      total * (r + 1) * (r + 2) // (world * (world + 1))) for r in range(world)],
                    np.int64)


def _run_ranks(work, world, scenarios, timeout_ms=60000, proc_timeout=150):
    # PYTHONFAULTHANDLER: a rank that dies on a signal names its Python frame.
    # Each rank writes to files, not pipes: a pipe read only after an earlier
    # rank exits fills up (64 KiB) and blocks the later rank mid-exchange --
    # the ranks then wait on each other until the communicator times out
    env = dict(os.environ, SD_HOST_TIMEOUT_MS=str(timeout_ms), PYTHONFAULTHANDLER="1")
    files = [(open(os.path.join(work, f"rank{r}.out"), "w+"), open(os.path.join(work, f"rank{r}.err"), "w+"))
             for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_host_rank.py"),
                               ROOT, str(world), str(r), work, ",".join(scenarios)],
                              stdout=files[r][0], stderr=files[r][1], text=True, env=env)
             for r in range(world)]
    outs = []
    try:
        errs = []
        for r, p in enumerate(procs):
            p.wait(timeout=proc_timeout)
            fo, fe = files[r]
            fo.seek(0)
            fe.seek(0)
            out, err = fo.read(), fe.read()
            if p.returncode != 0:
                errs.append(f"rank {r} rc {p.returncode}: {err[-2500:]}")
            outs.append([json.loads(x) for x in out.splitlines() if x.startswith("{")])
        assert not errs, "\n".join(errs)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for fo, fe in files:
            fo.close()
            fe.close()
    return outs  # [rank][scenario] -> dict


def _load(work, sc, world):
    return [dict(np.load(os.path.join(work, f"{sc}_{r}.npz"))) for r in range(world)]


def _check_union(parts, ref_link, tag):
    w = np.concatenate([p[f"{tag}_who"] for p in parts])
    o = np.concatenate([p[f"{tag}_obj"] for p in parts])
    c, lr, lo = dedup.split_link_lists(w, o)
    np.testing.assert_array_equal(c, ref_link[0], err_msg=tag)
    np.testing.assert_array_equal(lr, ref_link[1], err_msg=tag)
    np.testing.assert_array_equal(lo, ref_link[2], err_msg=tag)


@pytest.fixture(scope="module", params=[2, 3, 4])
def world_run(request):
    """All scenarios but the rank exit, one process per rank, W = 2, 3 and 4."""
    world = request.param
    work = tempfile.mkdtemp(prefix=f"sd_mp{world}_")
    data, refs = {}, {}
    for i, case in enumerate(CASES):
        k, h = _rows(case, TOTAL, 90 + 7 * world + i)
        sp = _spans(TOTAL, world)
        data[f"k_{case}"], data[f"h_{case}"], data[f"span_{case}"] = k, h, sp
        ref = O.group_reps(k, h, 100)
        refs[case] = (ref, O.link_batch(ref, None, np.ones(TOTAL, np.uint8), 0))
        data[f"B_{case}"] = np.int64((sp[:, 1] - sp[:, 0]).max())
    data["msg_bytes"] = np.int64(16 * world * (TOTAL + 4096))
    np.savez(os.path.join(work, "data.npz"), **data)
    scenarios = [f"mix_{c}" for c in CASES] + ["hint_overflow", "nospc", "agree_hint", "agree_mode"]
    outs = _run_ranks(work, world, scenarios)
    res = {sc: [outs[r][i] for r in range(world)] for i, sc in enumerate(scenarios)}
    return world, work, res, refs, data


@pytest.mark.parametrize("case", CASES)
def test_mixed_forms_pending_across_processes(world_run, case):
    """rep (counted) -> write set (padded, pending) -> rep (padded; resolves
    the write set) -> write set (padded; resolves the rep call) -> wait: every
    result equals the oracle, every rank re-ran the same calls."""
    world, work, res, refs, data = world_run
    ref, ref_link = refs[case]
    assert all(r["wait"] == 0 for r in res[f"mix_{case}"]), res[f"mix_{case}"]
    parts = _load(work, f"mix_{case}", world)
    for tag in ("r1", "r3"):
        np.testing.assert_array_equal(np.concatenate([p[tag] for p in parts]).view(np.uint32),
                                      ref, err_msg=tag)
    _check_union(parts, ref_link, "l2")
    _check_union(parts, ref_link, "l4")
    sts = [r["stats"] for r in res[f"mix_{case}"]]
    assert all(st["padded_calls"] == 3 for st in sts), sts
    reruns = {st["overflow_reruns"] for st in sts}
    assert len(reruns) == 1, sts  # every rank saw the same overflow bits
    if case == "uniform":
        assert reruns == {0}
    else:
        assert reruns.pop() >= 1
    assert sum(st["rows_sent"] for st in sts) == sum(st["rows_received"] for st in sts)


def test_forced_overflow_rerun_in_order(world_run):
    """B set to a quarter of the rows on every rank: the first padded call
    overflows everywhere and is re-run counted when the second call (the
    other form) resolves it; all three results equal the oracle."""
    world, work, res, refs, data = world_run
    ref, ref_link = refs["uniform"]
    parts = _load(work, "hint_overflow", world)
    for tag in ("r1", "r3"):
        np.testing.assert_array_equal(np.concatenate([p[tag] for p in parts]).view(np.uint32),
                                      ref, err_msg=tag)
    _check_union(parts, ref_link, "l2")
    sts = [r["stats"] for r in res["hint_overflow"]]
    assert all(st["overflow_reruns"] == 1 and st["padded_calls"] == 3 for st in sts), sts
    assert all(st["agreements"] == 1 for st in sts), sts  # set_exchange -> one agreement round


def test_deferred_enospc_reported_once(world_run):
    """Rank 0's first write set exceeds its capacity: found when the second
    call resolves the first, reported by the next wait (once, naming call 1);
    the other ranks and the later calls are unaffected."""
    world, work, res, refs, data = world_run
    ref, ref_link = refs["uniform"]
    rs = res["nospc"]
    assert rs[0]["wait1"] == -errno.ENOSPC and rs[0]["wait2"] == 0, rs[0]
    assert rs[0]["stats"]["nospc_call"] == 1
    for r in rs[1:]:
        assert r["wait1"] == 0 and r["wait2"] == 0 and r["stats"]["nospc_call"] == 0, r
    parts = _load(work, "nospc", world)
    _check_union(parts, ref_link, "l2")
    _check_union(parts, ref_link, "l3")


@pytest.mark.parametrize("sc", ["agree_hint", "agree_mode"])
def test_layout_disagreement_is_eproto(world_run, sc):
    """Ranks that set different rows_hint, or counted against padded, fail
    with -EPROTO on every rank before any record moves, and the
    aborted communicator refuses the next call."""
    world, work, res, refs, data = world_run
    for r in res[sc]:
        assert r["rc1"] == -errno.EPROTO and r["rc2"] == -errno.ECONNABORTED, r


@pytest.mark.parametrize("world", [2, 3, 4])
def test_random_call_sequences_across_processes(world):
    """Seeded random sequences of exchange calls, the same on every rank:
    rep and write-set forms, resolved at once or left pending for the next
    call, exchange layouts (padded with a hint of 1/4, 1 or 2 times the rows,
    auto, counted) and return legs changed between calls, over uniform keys,
    one key 40 k times and all one key.  Every call's result equals the
    oracle's grouping of all rows (file_identifier/mod.rs:136-333), and every
    rank re-ran the same overflowed calls."""
    work = tempfile.mkdtemp(prefix=f"sd_mpf{world}_")
    data, refs = {}, {}
    for i, case in enumerate(CASES):
        k, h = _rows(case, TOTAL, 300 + 7 * world + i)
        sp = _spans(TOTAL, world)
        data[f"k_{case}"], data[f"h_{case}"], data[f"span_{case}"] = k, h, sp
        data[f"B_{case}"] = np.int64((sp[:, 1] - sp[:, 0]).max())
        ref = O.group_reps(k, h, 100)
        refs[case] = (ref, O.link_batch(ref, None, np.ones(TOTAL, np.uint8), 0))
    data["cases"] = np.array(CASES)
    data["fuzz_ops"] = np.int64(20)
    data["msg_bytes"] = np.int64(16 * world * (TOTAL + 4096))
    np.savez(os.path.join(work, "data.npz"), **data)
    soak = int(os.environ.get("SD_SOAK", "0"))  # SD_SOAK=k: 5 k more seeds
    seeds = [f"fuzz_{world * 100 + s}" for s in range(5 + 5 * soak)]
    outs = _run_ranks(work, world, seeds, proc_timeout=150 + 30 * soak)
    calls = reruns = padded = 0
    for j, sc in enumerate(seeds):
        rs = [outs[r][j] for r in range(world)]
        assert all(r["wait"] == 0 for r in rs), rs
        assert all(r["ops"] == rs[0]["ops"] for r in rs)
        assert len({r["stats"]["overflow_reruns"] for r in rs}) == 1, [r["stats"] for r in rs]
        parts = _load(work, sc, world)
        for op in rs[0]["ops"]:
            if op[0] not in ("rep", "list"):
                continue
            form, case, _, i = op
            ref, ref_link = refs[case]
            if form == "rep":
                np.testing.assert_array_equal(
                    np.concatenate([p[f"op{i}_rep"] for p in parts]).view(np.uint32), ref,
                    err_msg=f"{sc} op {i} {case}")
            else:
                _check_union(parts, ref_link, f"op{i}")
            calls += 1
        reruns += rs[0]["stats"]["overflow_reruns"]
        padded += rs[0]["stats"]["padded_calls"]
    # the sequences reached the paths they are for
    assert calls >= 40 and padded >= 10 and reruns >= 2, (calls, padded, reruns)


@pytest.mark.parametrize("world", [2, 3])
def test_object_index_batches_with_overflow_across_processes(world):
    """Per-rank shares of the Object index over three batches, pre-existing
    Objects (one with handle 0x7FFFFFFF), the second batch
    overflowing (a key 40 k times) and re-run counted by every process; full
    and compact return legs.  The reps equal the oracle's grouping with the
    library's existing Objects (file_identifier/mod.rs:168-241)."""
    work = tempfile.mkdtemp(prefix="sd_mpi_")
    total, batch = 450_000, 150_000
    k, h, _ = O.synth_dedup_rows(61 + world, total, 280_000, 0, total)
    rng = np.random.default_rng(world)
    k[batch + rng.choice(batch, 40_000, replace=False)] = k[5]
    ek = rng.choice(k, 1500)
    ek[0] = k[5]
    eh = np.arange(ek.size, dtype=np.uint32) + 3
    eh[0] = 0x7FFFFFFF
    ref = O.group_reps_existing(k, h, 100, ek, eh)
    np.savez(os.path.join(work, "data.npz"), k_index=k, h_index=h, ek=ek, eh=eh,
             batch=np.int64(batch), msg_bytes=np.int64(16 * world * (batch + 4096)))
    outs = _run_ranks(work, world, ["index_full", "index_compact"])
    for i, sc in enumerate(("index_full", "index_compact")):
        out = np.zeros(total, np.uint32)
        for p in _load(work, sc, world):
            out[p["pos"]] = p["rep"].view(np.uint32)
        bad = np.flatnonzero(out != ref)
        assert bad.size == 0, (sc, bad.size, bad[:5], out[bad[:5]], ref[bad[:5]])
        sts = [o[i]["stats"] for o in outs]
        assert len({st["overflow_reruns"] for st in sts}) == 1, sts
        if sc == "index_full":
            assert all(st["padded_calls"] == 3 and st["overflow_reruns"] == 1 for st in sts), sts
        else:  # compact return leg: counted exchange only
            assert all(st["padded_calls"] == 0 for st in sts), sts


@pytest.mark.parametrize("shares", [(0, 5, 120_000), (60_000, 0, 0, 1)])
def test_empty_and_tiny_ranks_across_processes(shares):
    """Ragged worlds over the per-process path: a rank with no rows or a
    handful still sends headers and padding and receives its owned rows;
    the mixed counted / padded sequence equals the oracle (as
    test_gpu_padded.py's _all form does in one process)."""
    world, total = len(shares), sum(shares)
    work = tempfile.mkdtemp(prefix="sd_mpr_")
    k, h = _rows("uniform", total, 31 + world)
    b = np.concatenate([[0], np.cumsum(shares)]).astype(np.int64)
    sp = np.stack([b[:-1], b[1:]], axis=1)
    np.savez(os.path.join(work, "data.npz"), k_uniform=k, h_uniform=h, span_uniform=sp,
             B_uniform=np.int64(max(shares)), msg_bytes=np.int64(16 * world * (total + 4096)))
    outs = _run_ranks(work, world, ["mix_uniform"])
    assert all(o[0]["wait"] == 0 for o in outs), [o[0] for o in outs]
    ref = O.group_reps(k, h, 100)
    ref_link = O.link_batch(ref, None, np.ones(total, np.uint8), 0)
    parts = _load(work, "mix_uniform", world)
    for tag in ("r1", "r3"):
        np.testing.assert_array_equal(np.concatenate([p[tag] for p in parts]).view(np.uint32),
                                      ref, err_msg=tag)
    _check_union(parts, ref_link, "l2")
    _check_union(parts, ref_link, "l4")
    sts = [o[0]["stats"] for o in outs]
    assert all(st["padded_calls"] == 3 for st in sts), sts
    assert len({st["overflow_reruns"] for st in sts}) == 1, sts


def test_eight_processes_padded_and_overflow():
    """The N = 8 shape of the driver's scaling run, as 8 processes on the one
    GPU (the box allows 16 GPU processes): a counted call, padded calls of
    both forms left pending and resolved across the processes, then a forced
    overflow re-run in the same order on all 8 ranks -- every result equal
    to the oracle."""
    world = 8
    work = tempfile.mkdtemp(prefix="sd_mp8_")
    total = 240_000
    k, h = _rows("uniform", total, 8)
    sp = _spans(total, world)
    np.savez(os.path.join(work, "data.npz"), k_uniform=k, h_uniform=h, span_uniform=sp,
             B_uniform=np.int64((sp[:, 1] - sp[:, 0]).max()),
             msg_bytes=np.int64(16 * world * (total + 4096)))
    outs = _run_ranks(work, world, ["mix_uniform", "hint_overflow"])
    ref = O.group_reps(k, h, 100)
    ref_link = O.link_batch(ref, None, np.ones(total, np.uint8), 0)
    assert all(o[0]["wait"] == 0 for o in outs), [o[0] for o in outs]
    parts = _load(work, "mix_uniform", world)
    for tag in ("r1", "r3"):
        np.testing.assert_array_equal(np.concatenate([p[tag] for p in parts]).view(np.uint32),
                                      ref, err_msg=tag)
    _check_union(parts, ref_link, "l2")
    _check_union(parts, ref_link, "l4")
    parts = _load(work, "hint_overflow", world)
    for tag in ("r1", "r3"):
        np.testing.assert_array_equal(np.concatenate([p[tag] for p in parts]).view(np.uint32),
                                      ref, err_msg=tag)
    _check_union(parts, ref_link, "l2")
    sts = [o[1]["stats"] for o in outs]
    assert all(st["overflow_reruns"] == 1 and st["padded_calls"] == 3 for st in sts), sts


def test_rank_exit_times_out_the_others():
    """Rank 1 leaves after one call: rank 0's next call fails with
    -ETIMEDOUT within the communicator's 3 s timeout (no hang), the one
    after with -ECONNABORTED; the good call equals the oracle."""
    world = 2
    work = tempfile.mkdtemp(prefix="sd_mpx_")
    k, h = _rows("uniform", 100_000, 5)
    sp = _spans(100_000, world)
    np.savez(os.path.join(work, "data.npz"), k_uniform=k, h_uniform=h, span_uniform=sp,
             B_uniform=np.int64((sp[:, 1] - sp[:, 0]).max()),
             msg_bytes=np.int64(16 * world * 110_000))
    outs = _run_ranks(work, world, ["exit"], timeout_ms=3000)
    r0 = outs[0][0]
    assert r0["rc2"] == -errno.ETIMEDOUT, r0
    assert 2.5 < r0["s2"] < 60, r0
    assert r0["rc3"] == -errno.ECONNABORTED, r0
    parts = _load(work, "exit", world)
    np.testing.assert_array_equal(np.concatenate([p["r1"] for p in parts]).view(np.uint32),
                                  O.group_reps(k, h, 100))
