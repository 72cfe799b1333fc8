"""One rank of a multi-process exchange test (tests/test_gpu_multiproc.py).

Run as `python tests/_host_rank.py <root> <world> <rank> <workdir> <scenario,...>`:
every rank is its own process on the same GPU, joined through
sdgpu_comm_init_host (SDGPU_TRANSPORT_HOST, ABI 6), so each call goes
through shard.cpp's per-process path exactly as under RCCL -- its own
sdgpu_comm, run_call's single-rank branch, a padded call left pending and
resolved by the next call / Comm.wait() (resolve_pending), agreed_n learned
independently, the overflow re-run in the same collective order on every
rank.  Inputs come from <workdir>/data.npz (written by the parent, which
holds the oracle); outputs go to <workdir>/<scenario>_<rank>.npz and one
JSON line per scenario on stdout.  No oracle import here: the parent checks.
"""
import json
import os
import sys

import numpy as np


def main():
    root, world, rank, work = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    scenarios = sys.argv[5].split(",")
    sys.path.insert(0, root)
    import torch
    from spacedrive_amd import dedup
    from spacedrive_amd._native import Context, SdgpuError

    ctx = Context(0)
    data = np.load(os.path.join(work, "data.npz"))
    timeout = int(os.environ.get("SD_HOST_TIMEOUT_MS", "60000"))
    trace = os.environ.get("SD_HOST_TRACE") == "1"  # per-call progress on stderr

    def rows(case):
        k, h = data[f"k_{case}"], data[f"h_{case}"]
        a, b = (int(x) for x in data[f"span_{case}"][rank])
        dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
        return (dev(k[a:b].view(np.int64)), dev(h[a:b]), dev(np.ones(b - a, np.uint8)),
                torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda(), b - a)

    def comm_for(name):
        return dedup.Comm.init_host(ctx, world, rank, os.path.join(work, f"comm_{name}"),
                                    msg_bytes=int(data["msg_bytes"]), timeout_ms=timeout)

    def rc_of(fn):
        try:
            fn()
            return 0
        except SdgpuError as e:
            return e.rc

    def lists(out):
        who, obj, cnt = out
        c, l, e = (int(x) for x in cnt.cpu().tolist())
        return who[:e].cpu().numpy(), obj[:e].cpu().numpy()

    for sc in scenarios:
        res = {"scenario": sc, "rank": rank}
        save = {}
        if sc.startswith("mix_"):
            # rep (counted: B unknown) -> list (padded, pending) -> rep (padded,
            # resolves the list call) -> list (padded, resolves the rep call)
            # -> wait (resolves the last)
            # (list capacity: every row of the batch may be owned here -- one
            # cas_id for all rows -- plus this rank's own keyless rows)
            case = sc[4:]
            key, has, val, rk, n = rows(case)
            cap = int(data[f"k_{case}"].size) + n
            comm = comm_for(sc)
            save["r1"] = dedup.group_sharded(key, has, rk, comm, None, 100).cpu().numpy()
            l2 = dedup.group_link_sharded(key, has, val, rk, comm, 100, cap=cap, trim=False)
            r3 = dedup.group_sharded(key, has, rk, comm, None, 100, wait=False)
            l4 = dedup.group_link_sharded(key, has, val, rk, comm, 100, cap=cap, trim=False)
            res["wait"] = rc_of(comm.wait)
            res["counts"] = [l2[2].cpu().tolist(), l4[2].cpu().tolist()]
            save["r3"] = r3.cpu().numpy()
            save["l2_who"], save["l2_obj"] = lists(l2)
            save["l4_who"], save["l4_obj"] = lists(l4)
            res["stats"] = comm.stats()
            comm.close()
        elif sc.startswith("probe_"):
            # diagnostics: the mix sequence with every call resolved at once
            case = sc[6:]
            key, has, val, rk, n = rows(case)
            comm = comm_for(sc)
            calls = []
            for form in ("rep", "list", "rep", "list"):
                try:
                    if form == "rep":
                        dedup.group_sharded(key, has, rk, comm, None, 100)
                        calls.append({"form": form, "rc": 0})
                    else:
                        w, o, cnt = dedup.group_link_sharded(key, has, val, rk, comm, 100,
                                                             trim=False)
                        rc = 0
                        try:
                            comm.wait()
                        except SdgpuError as e:
                            rc = e.rc
                        calls.append({"form": form, "rc": rc, "counts": cnt.cpu().tolist(),
                                      "cap": int(w.numel())})
                except SdgpuError as e:
                    calls.append({"form": form, "rc": e.rc})
                calls[-1]["stats"] = comm.stats()
            res["calls"] = calls
            comm.close()
        elif sc.startswith("index_"):
            # batches through per-rank shares of the Object index, with
            # pre-existing Objects; the second batch overflows (a key 40 k
            # times): its creators must reach the index only through the
            # counted re-run, which every process issues in the same order
            ret = dedup.RETURN_FULL if sc == "index_full" else dedup.RETURN_COMPACT
            k, h = data["k_index"], data["h_index"]
            batch, total = int(data["batch"]), int(data["k_index"].size)
            comm = comm_for(sc)
            comm.set_return(ret)
            comm.set_exchange(dedup.EXCHANGE_AUTO, batch // world + 1)
            idx = dedup.ObjectIndex(ctx, 1000)
            dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
            idx.add_objects(dev(data["ek"].view(np.int64)), dev(data["eh"].view(np.int32)), world, rank)
            pos, reps = [], []
            for b0 in range(0, total, batch):
                a, b = b0 + batch * rank // world, b0 + batch * (rank + 1) // world
                rep = dedup.group_sharded(dev(k[a:b].view(np.int64)), dev(h[a:b]),
                                          torch.arange(a, b, dtype=torch.int64).to(torch.int32).cuda(),
                                          comm, idx, 100)
                pos.append(np.arange(a, b))
                reps.append(rep.cpu().numpy())
            save["pos"], save["rep"] = np.concatenate(pos), np.concatenate(reps)
            res["stats"] = comm.stats()
            comm.close()
        elif sc.startswith("fuzz_"):
            # a random sequence of exchange calls, the same on every rank (a
            # shared seed): rep / write-set forms, resolved at once or left
            # pending, layouts and return legs changed between calls (padded
            # with a hint of a quarter / one / two times the rows, auto,
            # counted; full / compact / auto return), on the three key cases
            rng = np.random.default_rng(int(sc[5:]))
            cases = [str(c) for c in data["cases"]]
            comm = comm_for(sc)
            held, ops = [], []
            for i in range(int(data["fuzz_ops"])):
                u = rng.random()
                if u < 0.15:
                    mode = int(rng.choice([dedup.EXCHANGE_PADDED, dedup.EXCHANGE_AUTO,
                                           dedup.EXCHANGE_COUNTED]))
                    B = int(data[f"B_{cases[int(rng.integers(len(cases)))]}"])
                    hint = int(rng.choice([max(1, B // 4), B, 2 * B]))
                    comm.set_exchange(mode, hint)
                    ops.append(["exchange", mode, hint])
                    continue
                if u < 0.25:
                    ret = int(rng.choice([dedup.RETURN_FULL, dedup.RETURN_COMPACT, dedup.RETURN_AUTO]))
                    comm.set_return(ret)
                    ops.append(["return", ret])
                    continue
                case = cases[int(rng.integers(len(cases)))]
                form = "rep" if rng.random() < 0.5 else "list"
                wait = bool(rng.random() < 0.4)
                key, has, val, rk, n = rows(case)
                if form == "rep":
                    out = dedup.group_sharded(key, has, rk, comm, None, 100, wait=wait)
                else:
                    cap = int(data[f"k_{case}"].size) + n
                    out = dedup.group_link_sharded(key, has, val, rk, comm, 100, cap=cap, trim=False)
                    if wait:
                        comm.wait()
                held.append((i, form, out))
                ops.append([form, case, int(wait), i])
                if trace:
                    print(json.dumps({"rank": rank, "sc": sc, "op": ops[-1], "stats": comm.stats()}),
                          file=sys.stderr, flush=True)
            res["wait"] = rc_of(comm.wait)
            if trace:
                print(json.dumps({"rank": rank, "sc": sc, "final_wait": res["wait"],
                                  "stats": comm.stats()}), file=sys.stderr, flush=True)
            for i, form, out in held:  # every call is resolved now
                if form == "rep":
                    save[f"op{i}_rep"] = out.cpu().numpy()
                else:
                    save[f"op{i}_who"], save[f"op{i}_obj"] = lists(out)
            res["ops"] = ops
            res["stats"] = comm.stats()
            comm.close()
        elif sc == "hint_overflow":
            # B set below the rows: the first padded call overflows on every
            # rank and is re-run counted when the next call resolves it
            key, has, val, rk, n = rows("uniform")
            comm = comm_for(sc)
            comm.set_exchange(dedup.EXCHANGE_PADDED, int(data["B_uniform"]) // 4)
            r1 = dedup.group_sharded(key, has, rk, comm, None, 100, wait=False)
            l2 = dedup.group_link_sharded(key, has, val, rk, comm, 100, trim=False)
            r3 = dedup.group_sharded(key, has, rk, comm, None, 100, wait=False)
            comm.wait()
            save["r1"], save["r3"] = r1.cpu().numpy(), r3.cpu().numpy()
            save["l2_who"], save["l2_obj"] = lists(l2)
            res["stats"] = comm.stats()
            comm.close()
        elif sc == "nospc":
            # rank 0's first write set does not fit; it is found when the
            # second call resolves the first and reported by the next wait,
            # once; the other ranks are unaffected
            key, has, val, rk, n = rows("uniform")
            comm = comm_for(sc)
            comm.set_exchange(dedup.EXCHANGE_PADDED, int(data["B_uniform"]))
            cap = 10 if rank == 0 else None
            dedup.group_link_sharded(key, has, val, rk, comm, 100, cap=cap, trim=False)
            l2 = dedup.group_link_sharded(key, has, val, rk, comm, 100, trim=False)
            res["wait1"] = rc_of(comm.wait)
            res["wait2"] = rc_of(comm.wait)
            save["l2_who"], save["l2_obj"] = lists(l2)
            w3, o3, _ = dedup.group_link_sharded(key, has, val, rk, comm, 100)
            save["l3_who"], save["l3_obj"] = w3.cpu().numpy(), o3.cpu().numpy()
            res["stats"] = comm.stats()
            comm.close()
        elif sc in ("agree_hint", "agree_mode"):
            # ranks that set different layouts fail with -EPROTO before any
            # record moves, then -ECONNABORTED
            key, has, val, rk, n = rows("uniform")
            comm = comm_for(sc)
            B = int(data["B_uniform"])
            if sc == "agree_hint":
                comm.set_exchange(dedup.EXCHANGE_PADDED, B + rank)
            else:
                comm.set_exchange(dedup.EXCHANGE_COUNTED if rank == 0 else dedup.EXCHANGE_PADDED, B)
            res["rc1"] = rc_of(lambda: dedup.group_sharded(key, has, rk, comm, None, 100))
            res["rc2"] = rc_of(lambda: dedup.group_sharded(key, has, rk, comm, None, 100))
            comm.close()
        elif sc == "exit":
            # one good call, then rank 1 leaves: the others' next call fails
            # within the communicator's timeout, later calls are refused
            key, has, val, rk, n = rows("uniform")
            comm = comm_for(sc)
            save["r1"] = dedup.group_sharded(key, has, rk, comm, None, 100).cpu().numpy()
            if rank == 1:
                np.savez(os.path.join(work, f"{sc}_{rank}.npz"), **save)
                print(json.dumps(res), flush=True)
                os._exit(0)
            import time
            t0 = time.monotonic()

            def second():
                dedup.group_sharded(key, has, rk, comm, None, 100, wait=False)
                comm.wait()
            res["rc2"] = rc_of(second)
            res["s2"] = time.monotonic() - t0
            res["rc3"] = rc_of(lambda: dedup.group_sharded(key, has, rk, comm, None, 100))
            comm.close()
        else:
            raise SystemExit(f"unknown scenario {sc}")
        torch.cuda.synchronize()
        np.savez(os.path.join(work, f"{sc}_{rank}.npz"), **save)
        print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
