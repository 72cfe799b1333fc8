#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    (N > 1: launched by torch.distributed.run, one process per GPU, RCCL)

Headline `value` (files/s, whole job): one STEP = one identifier pass over a
batch resident in HBM -- BASELINE config 2 per GPU (1 M synthetic files,
log-normal sizes, 20 % duplicates, 0.1 % empty; only the cas windows exist) --
consisting of K1 (sampled cas_id of every file), the cas_id -> Object
grouping of all files of all GPUs (hash-sharded, RCCL all-to-all at N > 1) and
the Object link batch (K7: create / connect lists).  Weak scaling: every GPU brings its own 1 M files.

Components reported on the same line (each timed the same way, K steps after W
warm-up, barrier + synchronize on both sides, max over ranks):
  cas      K1 alone over config 2                              files/s
  dedup    config 4: 12.5 M rows per GPU (100 M at 8 GPUs)     rows/s
           (+ at N = 1 the whole 100 M-row table on one GPU)
  checksum config 3: 64 x 4 GiB files per GPU, device-resident GB/s
  staged   config 5: a 50 M-file identifier run, steps of 250 k config-2
           files per GPU whose windows sit in pinned host memory, streamed
           H2D + K1 + grouping against the run's Object index + link batch files/s
  dir      config 1: a real 10 k-file directory (sparse files, warm cache)
           through sdgpu_identify_files (pread -> pinned -> K1)         files/s
`roofline` is for the dominant kernel (K1 "cas_leaves"), timed live with HIP
events on its launch stream; `cpu_baseline` times a SIMD C port of
generate_cas_id's hashing (the crate's multi-chunk SIMD idea: AVX-512 16-way
where the host has it, as the crate's hash_many does, else AVX2 8-way) on this host's
cores over a bounded sample, with the scalar oracle and 1-thread figures beside.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# int32 VALU peak: 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz.  BLAKE3's mix of
# 32-bit ops (v_add3_u32, v_alignbit_b32, v_xor_b32, v_add_u32) issues at that
# rate: a register-only compression loop measures ~38.7 T lane-ops/s whatever
# the VOP2/VOP3 split (profiles/r2/exp_g_mix_r2f.log); the
# 157 TFLOP/s FP32 figure counts packed-FMA lanes instead.
VALU_PEAK_SPEC = 256 * 4 * 16 * 2.4e9
HBM_PEAK = 8.0e12                       # B/s (MI355X spec)
ISA_PER_COMPRESSION = 680               # fused VALU instructions per BLAKE3 compression
METRIC = "cas_id files/sec + full-file BLAKE3 GB/s + dedup rows/sec at 1/2/4/8 MI355X"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cgroup_cpu_quota():
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max),
    or None when unlimited / unknown."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(period)
    except (OSError, ValueError):
        return None


def host_cores():
    """(threads, note): every core this process may run on (its CPU affinity),
    capped by its cgroup CPU quota and by OMP_NUM_THREADS when the host sets
    it (the GPU box: 16, the CPU share of one GPU; nproc and os.cpu_count show
    the whole machine there)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = cgroup_cpu_quota()
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = aff
    if quota:
        n = min(n, max(1, int(quota)))
    if cap > 0:
        n = min(n, cap)
    return n, (f"{n} threads: sched_getaffinity {aff}, os.cpu_count {total}, cgroup cpu.max "
               f"{'unlimited' if quota is None else f'{quota:g} CPUs'}, "
               f"OMP_NUM_THREADS {cap or 'unset'}")


def compressions(lens: np.ndarray):
    """(chunk-block compressions, parent compressions) of messages of these lengths."""
    L = lens.astype(np.int64)
    full = L // 1024
    rem = L % 1024
    blocks = full * 16 + (rem + 63) // 64
    blocks = np.where(L == 0, 1, blocks)
    chunks = np.maximum(1, (L + 1023) // 1024)
    return int(blocks.sum()), int((chunks - 1).sum())


def k1_split(lens: np.ndarray):
    """Compressions done by K1 v3's two kernels (b3_batch.hip k_leaves3 / k_fold3):
    leaves = every chunk block + the parents inside 4-chunk units (3 each) and
    inside the 1..4-chunk ragged tail of a message (rem - 1); fold = the
    (q + [rem > 0] - 1) parents above the level-2 nodes of a message."""
    L = lens.astype(np.int64)
    blk, par = compressions(L)
    nch = np.maximum(1, (L + 1023) // 1024)
    q = np.where(nch > 4, (L // 1024) // 4, 0)
    rem = nch - 4 * q
    leaves = blk + int(3 * q.sum()) + int(np.maximum(rem - 1, 0).sum())
    return leaves, blk + par - leaves


# single-file latency sizes (the GPU / CPU crossover for the watcher callers,
# include/sdgpu.h): one chunk chain, 16 / 32 / 64 KiB messages, a sampled file
BURST_FILES = 64
BURST_SIZES = (("4KiB", 4096), ("64KiB", 65536), ("1MiB", 1 << 20))
SINGLE_SIZES = (("4KiB", 4096), ("16KiB", 16384), ("32KiB", 32768), ("64KiB", 65536),
                ("1MiB", 1 << 20))


def pmc_traffic(kernel: str, section: str = "kernels"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/<round>/pmc_traffic.json, written by scripts/pmc_summary.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench's workload; section
    "kernels" = the K1 pass over config 2, "dedup" = the 12.5 M-row grouping,
    "dedup_full" = the 100 M-row two-level grouping)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    for f in reversed(files):  # newest round first (profiles/r1, r2, ...)
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in d.get(section, {}):
            k = d[section][kernel]
            return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


class Runner:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        # one process per GPU; LOCAL_RANK wraps only in the 1-GPU rehearsal
        # (SD_BENCH_BACKEND=gloo: N ranks sharing one card, exchange via host)
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        # nccl = RCCL over xGMI; host = the one-GPU rehearsal of libsdgpu's
        # per-process exchange (SDGPU_TRANSPORT_HOST, ranks sharing the card,
        # torch.distributed over gloo); gloo = the Python exchange (rehearsal)
        backend = os.environ.get("SD_BENCH_BACKEND", "nccl")
        if self.world > 1:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group("gloo" if backend == "host" else backend)
        from spacedrive_amd import dedup
        from spacedrive_amd._native import default_context
        self.ctx = default_context(self.local)
        self.args = args
        self.backend = backend if self.world > 1 else None
        self.ops = dedup.HipOps(self.ctx)
        self.comm = None
        # every wait on an RCCL peer inside libsdgpu is bounded by this (a
        # rank that never joins or dies mid-exchange: -ETIMEDOUT, not a hang)
        self.comm_timeout_ms = int(os.environ.get("SDGPU_COMM_TIMEOUT_MS", "120000"))
        # SD_BENCH_FORCE_COMM=1: also at N = 1 through a one-rank RCCL
        # communicator (rehearses the N > 1 code path on a one-GPU box)
        force = os.environ.get("SD_BENCH_FORCE_COMM") == "1" and self.world == 1
        if force:
            self.backend = "nccl (one-rank rehearsal)"
            self.comm = dedup.Comm.init_rank(self.ctx, 1, 0, dedup.Comm.unique_id(),
                                             timeout_ms=self.comm_timeout_ms)
        if self.world > 1 and backend == "host":
            # the same libsdgpu calls as under RCCL (sdgpu_group_link_sharded_
            # device ...), their messages staged through a shared file: the
            # N > 1 path of this bench rehearsed on a one-GPU box
            import tempfile
            # a fresh private directory (not mktemp's race-prone name); the
            # file inside is created by the first rank to join
            obj = [os.path.join(tempfile.mkdtemp(prefix="sd_bench_comm_"), "comm")
                   if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            rows = max(args.files, args.dedup_rows, args.staged_files)
            self.comm = dedup.Comm.init_host(self.ctx, self.world, self.rank, obj[0],
                                             msg_bytes=16 * rows + (1 << 20),
                                             timeout_ms=self.comm_timeout_ms)
        if self.world > 1 and backend == "nccl":
            # the grouping's exchange runs INSIDE libsdgpu over RCCL (what the
            # Rust host calls): rank 0's communicator id travels over the
            # torch.distributed group, every rank joins
            obj = [dedup.Comm.unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            err = None
            try:
                self.comm = dedup.Comm.init_rank(self.ctx, self.world, self.rank, obj[0],
                                                 timeout_ms=self.comm_timeout_ms)
            except Exception as e:  # reported, and every rank takes the same path
                err = e
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=self.dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                log(f"bench: libsdgpu RCCL communicator unavailable on some rank ({err!r}); "
                    "the exchange runs over torch.distributed instead")
                if self.comm is not None:
                    self.comm.close()
                    self.comm = None

    def world_info(self) -> dict:
        """Launched world and, with a libsdgpu communicator, its RCCL world
        size and this rank's exchange volume / host time so far."""
        w = {"dist_world_size": self.dist.get_world_size() if self.world > 1 else 1,
             "devices_visible": self.torch.cuda.device_count(),
             "backend": self.backend, "exchange": self.exchange_name()}
        if self.comm is not None:
            try:
                nr, rk, tr = self.comm.info()
                w["rccl"] = {"nranks": nr, "rank": rk, "transport": tr,
                             "stats_rank": self.comm.stats()}
            except Exception as e:  # noqa: BLE001 -- e.g. an aborted communicator
                w["rccl"] = {"error": repr(e)[:200]}
        return w

    def free(self):
        self.torch.cuda.empty_cache()

    def drop_samples(self):
        """Releases the CPU leg's samples and the temporary files of the
        latency / config-1 legs."""
        import shutil
        self._cpu_sample = None
        if getattr(self, "_single_root", None):
            shutil.rmtree(self._single_root, ignore_errors=True)
            self._single_root = self._single_sample = None
        if getattr(self, "_dir_sample", None):  # ranks > 0, or --no-cpu
            shutil.rmtree(self._dir_sample[2], ignore_errors=True)
            self._dir_sample = None
        self.free()

    def shutdown(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None
        if self.world > 1:
            self.dist.destroy_process_group()

    def exchange_name(self) -> str:
        if self.comm is not None and self.backend == "host":
            return "libsdgpu host-staged all-to-all (SDGPU_TRANSPORT_HOST rehearsal, one GPU)"
        if self.comm is not None:
            return "libsdgpu RCCL all-to-all (sdgpu_group_sharded_device)"
        if self.world == 1:
            return "none (one GPU: local grouping)"
        return f"torch.distributed {self.backend} all-to-all over libsdgpu steps (rehearsal)"

    def group(self, key, has, rank, timings=None, wait=True):
        """The cas_id -> Object grouping of this rank's rows against all ranks.
        wait=False (timed loops): a padded exchange call is resolved by the
        next call or the barrier's Comm.wait(), not here."""
        from spacedrive_amd import dedup
        if self.comm is not None:
            return dedup.group_sharded(key, has, rank, self.comm, None, 100, wait=wait)
        if self.world == 1:
            return self.ops.group_rows(key, has, rank, 100, 0)
        return dedup.sharded_group_reps(key, has, rank, 100, ops=self.ops, timings=timings)

    def barrier(self):
        if self.comm is not None:
            # the last exchange's reps, waited for against the communicator's
            # deadline (a dead peer raises -ETIMEDOUT here instead of hanging
            # the torch synchronisation below)
            self.comm.wait()
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def timed_kernels(self, fn, steps, warmup):
        """(seconds for `steps` steps, per-kernel event times): the steps are
        timed un-instrumented, then run once more with libsdgpu's per-kernel
        HIP events (on each kernel's launch stream) for the breakdown -- the
        events' own gaps stay out of the reported rate."""
        t = self.timed(fn, steps, warmup)
        self.ctx.set_timing(True)
        for _ in range(steps):
            fn()
        self.torch.cuda.synchronize()
        kt = self.ctx.kernel_times()
        self.ctx.set_timing(False)
        return t, kt

    def timed(self, fn, steps, warmup) -> float:
        torch = self.torch
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        self.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        self.barrier()
        torch.cuda.synchronize()
        return self.max_over_ranks(time.perf_counter() - t0)

    # ---------------------------------------------------------------- config 2
    def run_cas(self, steps, warmup):
        torch = self.torch
        from spacedrive_amd import cas, corpus, dedup
        n = self.args.files
        sizes, seeds = corpus.config2_files(n, seed=2 + 1000 * self.rank)
        arena, off, ln = corpus.synth_arena_device(sizes, seeds, device=self.local, ctx=self.ctx)
        out = torch.empty((n, 8), dtype=torch.uint8, device=self.dev)
        st = torch.empty(n, dtype=torch.int32, device=self.dev)
        has = torch.from_numpy((sizes != 0).astype(np.uint8)).to(self.dev)
        grank = torch.arange(self.rank * n, (self.rank + 1) * n, dtype=torch.int64,
                             device=self.dev).to(torch.int32)
        torch.cuda.synchronize()
        lens = ln.cpu().numpy().view(np.uint32)
        blk, par = compressions(lens)
        res = {}

        def k1():
            cas.cas_batch_device(arena, off, ln, out, st, ctx=self.ctx)

        fused = self.world == 1 and self.comm is None

        def job():
            k1()
            key = out.view(torch.int64).view(-1)
            if fused:
                # one GPU: the grouping and the Object write set in one pass
                # (sdgpu_group_link_device; rows in id order, rank = row)
                dedup.group_link_device(key, has, None, None, 0, 100, ctx=self.ctx, trim=False)
                return
            if self.comm is not None:
                # N GPUs over libsdgpu's RCCL communicator: the records go to
                # their owners and each owner writes the write set of the rows
                # it owns (sdgpu_group_link_sharded_device): no return leg
                dedup.group_link_sharded(key, has, None, grank, self.comm, 100, trim=False)
                return
            rep = self.group(key, has, grank)
            dedup.link_batch_device(rep, grank, None, 0, ctx=self.ctx, trim=False)

        # K1 alone, with live per-kernel event timing on its launch stream
        t_cas, kt = self.timed_kernels(k1, steps, warmup)
        assert int(st.abs().sum()) == 0
        res["cas"] = {"value": self.world * n * steps / t_cas, "unit": "files/s",
                      "ms_per_step": 1e3 * t_cas / steps,
                      "config": {"workload": f"config2: {n} log-normal files/GPU, 20% dup, 0.1% empty",
                                 "files_per_gpu": n, "window_bytes_per_gpu": int(lens.sum())}}
        res["_leaves"] = kt.get("cas_leaves", (0.0, 1))
        res["kernels"] = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]} for k, v in kt.items()}
        # the CPU leg's sample: this step's K1 cas ids of the first files
        self._cpu_sample = (arena, off, ln, min(n, self.args.cpu_files),
                            out[:min(n, self.args.cpu_files)].cpu().numpy())
        # identifier job step: K1 + sharded grouping (RCCL all-to-all at N > 1).
        # A failing exchange (e.g. a peer that never answers: -ETIMEDOUT after
        # the communicator's deadline) is reported; K1's rate stays measured.
        try:
            t_job = self.timed(job, steps, warmup)
            res["job"] = {"value": self.world * n * steps / t_job,
                          "ms_per_step": 1e3 * t_job / steps,
                          "grouping": ("fused group + write set (sdgpu_group_link_device)"
                                       if fused else
                                       "sharded write set, no return leg "
                                       "(sdgpu_group_link_sharded_device)"
                                       if self.comm is not None else
                                       "sharded grouping + link batch (torch.distributed)")}
        except Exception as e:  # noqa: BLE001 -- reported in the line
            log(f"bench: identifier job step failed: {e!r}")
            res["job"] = {"error": repr(e)[:400]}
            return self._finish_cas(res, lens, blk, par)
        if self.world == 1 and self.comm is not None:
            # one-rank rehearsal (SD_BENCH_FORCE_COMM=1): the step through the
            # communicator against the fused one-GPU step in the SAME process,
            # interleaved A B A B ... so K1's clock (which ramps after every
            # idle gap by more than the exchange costs) cancels out
            def job_fused():
                k1()
                dedup.group_link_device(out.view(torch.int64).view(-1), has, None, None, 0, 100,
                                        ctx=self.ctx, trim=False)
            ab = {"comm": [], "fused": []}
            for _ in range(3):
                ab["comm"].append(1e3 * self.timed(job, steps, warmup) / steps)
                ab["fused"].append(1e3 * self.timed(job_fused, steps, warmup) / steps)
            med = {k: sorted(v)[len(v) // 2] for k, v in ab.items()}
            res["job"]["vs_fused_same_process"] = {
                "comm_ms_per_step": med["comm"], "fused_ms_per_step": med["fused"],
                "delta_ms": med["comm"] - med["fused"], "rounds": ab,
                "note": "medians of 3 interleaved rounds of `steps` steps each"}
        if self.world == 1 and self.comm is None:
            # the same step captured once into a HIP graph and replayed (fixed
            # buffers and shapes: what a host re-running same-size device
            # batches can do); every replay recomputes everything
            try:
                s = torch.cuda.Stream(device=self.dev)
                s.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(s):
                    job()
                    job()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    job()
                t_g = self.timed(g.replay, steps, warmup)
                res["job"]["graph_replay"] = {"value": n * steps / t_g,
                                              "ms_per_step": 1e3 * t_g / steps}
                del g
            except Exception as e:  # reported, the eager figure stands
                log(f"bench: graph capture of the job step failed: {e!r}")
                res["job"]["graph_replay"] = {"error": repr(e)[:200]}
        return self._finish_cas(res, lens, blk, par)

    def _finish_cas(self, res, lens, blk, par):
        leaves, fold = k1_split(lens)
        ms_leaves, nl = res.pop("_leaves", (0.0, 1))
        res["roofline_inputs"] = {"chunk_blocks": blk, "parents": par, "leaf_compressions": leaves,
                                  "fold_compressions": fold,
                                  "avg_leaves_s": ms_leaves / max(nl, 1) * 1e-3,
                                  "bytes": int(lens.sum())}
        return res

    # ---------------------------------------------------------------- config 5
    def h2d_peak(self, nbytes=1 << 30, reps=5):
        """Measured pinned host -> device copy rate (B/s) on this GPU's link."""
        torch = self.torch
        h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        d = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        del h, d
        return nbytes * reps / dt

    def run_staged(self):
        """BASELINE config 5: an identifier RUN over `staged_total_files` files
        (all GPUs together), in steps of `staged_files` per GPU.  The cas
        windows sit in PINNED host memory (where the preads land): staged H2D
        through the slab ring overlapped with K1, then the grouping of the step
        against the run's Object index (sharded with the rows over the GPUs at
        N > 1) and the Object link batch.  One pinned pool of config-2 files per
        GPU serves every step; ~81 % of its files stand for new content in each
        step (their keys remapped by a bijection after K1, sdgpu_synth_vary_keys
        _device), the rest are the same files every step -- so later steps link
        to earlier steps' Objects through the index, and the whole run is ONE
        grouping (test_gpu_index.py checks that batching is exact)."""
        torch = self.torch
        from spacedrive_amd import cas, corpus, dedup
        n = self.args.staged_files
        W = self.world
        nsteps = max(1, -(-self.args.staged_total_files // (W * n)))
        sizes, seeds = corpus.config2_files(n, seed=5 + 1000 * self.rank)
        d_arena, d_off, d_len = corpus.synth_arena_device(sizes, seeds, device=self.local,
                                                          ctx=self.ctx)
        torch.cuda.synchronize()
        h_arena = torch.empty(d_arena.numel(), dtype=torch.uint8).pin_memory()
        h_arena.copy_(d_arena)
        off = d_off.cpu().numpy().view(np.uint64).copy()
        ln = d_len.cpu().numpy().view(np.uint32).copy()
        del d_arena, d_off, d_len
        torch.cuda.empty_cache()
        window_bytes = int(ln.astype(np.int64).sum())
        out = torch.empty((n, 8), dtype=torch.uint8, device=self.dev)
        st = torch.empty(n, dtype=torch.int32, device=self.dev)
        has = torch.from_numpy((sizes != 0).astype(np.uint8)).to(self.dev)
        vary = torch.from_numpy(corpus.config5_vary_mask(sizes, seeds)).to(self.dev)
        # global ranks of every step (id order: step, then GPU, then row)
        base = torch.arange(n, dtype=torch.int64, device=self.dev) + self.rank * n
        ranks = [(base + s * W * n).to(torch.int32) for s in range(nsteps + 1)]
        use_index = W == 1 or self.comm is not None
        index = dedup.ObjectIndex(self.ctx, 2 * nsteps * n // W + (1 << 20)) if use_index else None
        peak = self.h2d_peak()

        def step(s):
            cas.cas_stage_pinned(h_arena, off, ln, out, st, ctx=self.ctx)
            key = out.view(torch.int64).view(-1)
            corpus.vary_keys_device(key, vary, s, ctx=self.ctx)
            if self.comm is None and W == 1:
                # one GPU: grouping against the index + the write set in one
                # pass (sdgpu_group_link_device); every row is an entry
                who, obj, cnt = dedup.group_link_device(key, has, None, None, s * n, 100,
                                                        ctx=self.ctx, trim=False, index=index)
                return ("lists", who, obj, cnt)
            if self.comm is not None:
                # resolved before the link batch reads rep (a padded call that
                # overflowed is re-run counted first)
                rep = dedup.group_sharded(key, has, ranks[s], self.comm, index, 100)
            else:  # gloo rehearsal: the exchange has no index
                rep = self.group(key, has, ranks[s])
            dedup.link_batch_device(rep, ranks[s], None, 0, ctx=self.ctx, trim=False)
            return ("rep", rep)

        step(nsteps)  # warm-up on a step outside the run's key space
        torch.cuda.synchronize()
        if index is not None:
            index.clear()

        # N = 1: every step's keys and reps are kept (a device copy of 12 B per
        # row, next to the step's ~42 KB of windows per file) so
        # the run can be checked after timing against ONE grouping of all its
        # rows: batching through the Object index must equal the whole-run rule
        verify = W == 1 and index is not None and not self.args.no_cpu
        if verify:
            keys_all = torch.empty(nsteps * n, dtype=torch.int64, device=self.dev)
            reps_all = torch.empty(nsteps * n, dtype=torch.int32, device=self.dev)
            obj_all = torch.empty(nsteps * n, dtype=torch.int32, device=self.dev)

        def run():
            for s in range(nsteps):
                res = step(s)
                if verify:  # device copies only; decoded after the timing
                    keys_all[s * n:(s + 1) * n].copy_(out.view(torch.int64).view(-1))
                    reps_all[s * n:(s + 1) * n].copy_(res[1][:n])
                    if res[0] == "lists":
                        obj_all[s * n:(s + 1) * n].copy_(res[2][:n])
            self._staged_last = res

        t = self.timed(run, 1, 0)
        whole = None
        last = self._staged_last
        if last[0] == "lists":
            linked_last = int(last[3].cpu()[1])
        else:
            linked_last = int((last[1] != ranks[nsteps - 1]).sum())
        if verify:
            # checked after the timing against the ORACLE's grouping of all the
            # run's rows (staged_oracle leg, rank 0 at N = 1): batching through
            # the Object index must equal the whole-run rule.  The fused steps'
            # write sets (every row one entry) are turned back into reps here.
            reps = reps_all.cpu().numpy().view(np.uint32)
            if last[0] == "lists":
                who = reps
                obj = obj_all.cpu().numpy().view(np.uint32)
                r = who & np.uint32(0x7FFFFFFF)
                reps = np.empty(nsteps * n, np.uint32)
                reps[r] = np.where((who & np.uint32(0x80000000)) != 0, obj, r)
            self._staged_verify = (keys_all.cpu().numpy().view(np.uint64),
                                   np.tile(has.cpu().numpy(), nsteps), reps)
            whole = {"rows": nsteps * n, "checked_by": "staged_oracle leg (O.group_reps)"}
            del keys_all, reps_all, obj_all
        assert int(st.abs().sum()) == 0
        distinct = index.count() if index is not None else None
        files = W * n * nsteps
        per_gpu_Bps = window_bytes * nsteps / t
        del h_arena, ranks
        self._staged_last = None
        if index is not None:
            index.close()
        return {"value": files / t, "unit": "files/s", "ms_per_step": 1e3 * t / nsteps,
                "files_total": files, "steps": nsteps, "seconds": t,
                "window_GBps_per_gpu": per_gpu_Bps / 1e9,
                "h2d_peak_GBps": peak / 1e9, "h2d_frac": per_gpu_Bps / peak,
                "index_keys_rank0": distinct, "linked_rows_last_step_rank0": linked_last,
                "verify_whole_run": whole,
                "config": {"workload": f"config5: identifier run over {files} files "
                                       f"({nsteps} steps x {n} files/GPU x {W} GPU), windows in "
                                       "pinned host memory, staged H2D (3-slab ring) + K1 + "
                                       "grouping against the run's Object index "
                                       + (("(sharded, host-transport rehearsal) + Object link batch"
                                           if self.backend == "host" else
                                           "(sharded, RCCL) + Object link batch")
                                          if self.comm is not None else
                                          "+ Object write set in one pass (one GPU)" if W == 1
                                          else "(no index: rehearsal) + Object link batch"),
                           "files_per_gpu_per_step": n, "window_bytes_per_gpu_per_step": window_bytes}}

    # ---------------------------------------------------------------- config 1
    def run_dir(self, steps):
        """Config 1: the reference's CPU-runnable case -- identify a synthetic
        10 k-file directory (mixed 1 KiB-10 MiB, sparse) from real files:
        stat sizes given, pread of the cas windows into pinned slabs by a thread
        pool, H2D + K1 (sdgpu_identify_files).  Warm page cache (one untimed pass)."""
        import shutil
        import tempfile
        from spacedrive_amd import corpus, file_identifier as fi
        root = tempfile.mkdtemp(prefix=f"sd_cfg1_r{self.rank}_")
        try:
            paths, sizes = corpus.write_config1_dir(root, self.args.dir_files, seed=1)
            # the listing encoded once for the C ABI (as a host holds its
            # CStrings); the CPU port below gets the same pre-encoded array
            paths = fi.PathList(paths)
            # the files were just written: flush them first, so the kernel's
            # writeback of their dirty pages does not run under the timed reads
            # (the first timed call stays ~35 % slower either way, r5s / r5x
            # step_ms: hence the median)
            os.sync()
            fi.identify(paths, sizes=sizes, ctx=self.ctx)  # warm page cache
            self.barrier()
            # each call timed on its own: one call is ~15 ms of host reads,
            # so single outliers (page-cache or scheduler hiccups on the box)
            # swing a mean of a few calls by +-25 %; `value` is the median
            # call, `mean_value` the plain mean (the CPU port is timed alike)
            step_s = []
            t0 = time.perf_counter()
            for _ in range(steps):
                t1 = time.perf_counter()
                res = fi.identify(paths, sizes=sizes, ctx=self.ctx)
                step_s.append(time.perf_counter() - t1)
            dt = self.max_over_ranks(time.perf_counter() - t0)
            med = self.max_over_ranks(float(np.median(step_s)))
            assert np.all(res.status == 0) and np.all(res.has_key == 1)
            # one more call with the library's phase timers on: file reads into
            # the pinned slabs (pool threads), waits for the device, K1 kernels
            self.ctx.set_timing(True)
            t1 = time.perf_counter()
            fi.identify(paths, sizes=sizes, ctx=self.ctx)
            one = 1e3 * (time.perf_counter() - t1)
            phases = {k: {"ms": v[0], "n": v[1]} for k, v in self.ctx.kernel_times().items()}
            self.ctx.set_timing(False)
            phases["call_ms"] = one
            # the GPU's cas ids are compared with the CPU baseline's (same files,
            # the reference's reads) in the cpu_baseline leg
            self._dir_sample = (paths, sizes, root, res.cas8.copy())
            return {"value": self.world * len(paths) / med, "unit": "files/s",
                    "ms_per_step": 1e3 * med, "mean_value": self.world * len(paths) * steps / dt,
                    "step_ms": [round(1e3 * x, 3) for x in step_s], "phases_one_call": phases,
                    "config": {"workload": "config1: 10k-file directory, log-uniform 1 KiB-10 MiB, "
                                           "sparse files, warm page cache, real pread I/O",
                               "files_per_gpu": len(paths)}}
        except BaseException:
            shutil.rmtree(root, ignore_errors=True)
            raise

    # ------------------------------------------------ single-file latency
    def run_single(self, calls=200):
        """Latency of the single-file drop-ins the watcher / non-indexed
        callers use (watcher/utils.rs:236,411,467; non_indexed.rs:161):
        generate_cas_id(path, size) and file_checksum(path), one call at a time,
        warm page cache.  Median microseconds per call."""
        import tempfile
        from spacedrive_amd import cas, validation
        root = tempfile.mkdtemp(prefix=f"sd_single_r{self.rank}_")
        rng = np.random.default_rng(7)
        res = {}
        try:
            # one-shot kernels, then the resident latency service (sdgpu_latency_service)
            for svc in (False, True):
                self.ctx.latency_service(svc)
                tag = "_service" if svc else ""
                for name, size in SINGLE_SIZES:
                    p = os.path.join(root, name)
                    if not os.path.exists(p):
                        rng.integers(0, 256, size, dtype=np.uint8).tofile(p)
                    for fn_name, fn in (("generate_cas_id",
                                         lambda: cas.generate_cas_id(p, size, self.ctx)),
                                        ("file_checksum",
                                         lambda: validation.file_checksum(p, self.ctx))):
                        for _ in range(10):
                            fn()
                        ts = []
                        for _ in range(calls):
                            t0 = time.perf_counter()
                            fn()
                            ts.append(time.perf_counter() - t0)
                        res[f"{fn_name}_{name}{tag}_us"] = float(np.median(ts) * 1e6)
            # where one resident-service call's time goes (device wall clock
            # for the copy and the hash; host clock for the read and the wait)
            p4 = os.path.join(root, "4KiB")
            cas.generate_cas_id(p4, 4096, self.ctx)
            res["service_breakdown_4KiB_cas"] = self.ctx.latency_service_diag()
            self.ctx.latency_service(False)
            self._single_sample = [(os.path.join(root, n), s) for n, s in SINGLE_SIZES]
            res["burst"] = self.run_burst(root, rng)
        finally:
            self._single_root = root
        return res

    def run_burst(self, root, rng, reps=40):
        """Bursts of single-file calls: BURST_FILES files
        that arrive together -- a folder copied into a watched location
        (watcher/utils.rs:236,411,467) or a non-indexed listing
        (non_indexed.rs:161) -- as ONE sdgpu_identify_files batch (what a
        coalescing host does, crates/sd-core-gpu/src/burst.rs) against the
        resident service one call at a time.  Median wall microseconds per
        burst; the CPU port's figures for the same files are in
        cpu_baseline.single_file_burst (merged here after that leg)."""
        from spacedrive_amd import cas
        from spacedrive_amd import file_identifier as FI
        out, self._burst_sample = {}, []
        for name, size in BURST_SIZES:
            paths = []
            for i in range(BURST_FILES):
                p = os.path.join(root, f"burst_{name}_{i}")
                rng.integers(0, 256, size, dtype=np.uint8).tofile(p)
                paths.append(p)
            pl = FI.PathList(paths)
            sizes = np.full(BURST_FILES, size, np.uint64)
            for _ in range(5):
                r = FI.identify(pl, sizes, ctx=self.ctx)
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                r = FI.identify(pl, sizes, ctx=self.ctx)
                ts.append(time.perf_counter() - t0)
            assert int(np.count_nonzero(r.status)) == 0
            batch = float(np.median(ts) * 1e6)
            self.ctx.latency_service(True)
            for p in paths[:8]:
                cas.generate_cas_id(p, size, self.ctx)
            ts = []
            for _ in range(max(3, reps // 4)):
                t0 = time.perf_counter()
                for p in paths:
                    cas.generate_cas_id(p, size, self.ctx)
                ts.append(time.perf_counter() - t0)
            self.ctx.latency_service(False)
            seq = float(np.median(ts) * 1e6)
            out[name] = {"files": BURST_FILES, "file_bytes": size,
                         "gpu_batch_burst_us": batch, "gpu_batch_per_file_us": batch / BURST_FILES,
                         "gpu_service_sequential_burst_us": seq}
            self._burst_sample.append((name, pl, sizes, r.cas8.copy()))
        return out

    # ---------------------------------------------------------------- config 4
    def run_dedup(self, steps, warmup):
        torch = self.torch
        from spacedrive_amd import corpus, dedup
        per = self.args.dedup_rows
        total = per * self.world
        key, has, rank = corpus.synth_dedup_rows_device(4, total, int(total * 0.8),
                                                        self.rank * per, per,
                                                        device=self.local, ctx=self.ctx)
        if self.args.verify:
            self.verify_sharded(key, has, rank)
        # one GPU: the rows are in rank order (synth rank[i] = i), as the job's
        # rows arrive in ascending id order, so the grouping gets no rank array
        # (12-byte bucket records); the explicit-rank call is timed beside it
        implicit = self.world == 1
        assert not implicit or bool((rank == torch.arange(per, dtype=rank.dtype,
                                                          device=rank.device)).all())
        grank = None if implicit else rank
        self.group(key, has, grank)  # first launches (lazy code-object loads) untimed
        t, kt = self.timed_kernels(lambda: self.group(key, has, grank, wait=False), steps, warmup)
        explicit_ms = None
        if implicit and not self.args.no_explicit_rank:
            self.group(key, has, rank)
            explicit_ms = 1e3 * self.timed(lambda: self.group(key, has, rank, wait=False), steps,
                                           warmup) / steps
        xchg = None
        if self.world > 1:
            # payload of one step on this rank: (key, rank) 12-B records out to
            # their owners, 4-B reps back; a 1/W share stays on this GPU
            keyed = int(has.sum())
            xinfo = {}
            if self.comm is None:
                self.group(key, has, rank, timings=xinfo)
            sent = xinfo.get("sent_rows", keyed)
            recv = xinfo.get("recv_rows", keyed)
            fwd, back = 12 * (sent + recv), 4 * (sent + recv)
            remote = (self.world - 1) / self.world
            xchg = {"payload_bytes_per_gpu": fwd + back,
                    "remote_bytes_per_gpu_est": int((fwd + back) * remote),
                    "remote_GBps_per_gpu_over_step": (fwd + back) * remote / (t / steps) / 1e9,
                    "transport": self.exchange_name(),
                    "note": "bytes sent + received per GPU per step over xGMI; rate is over the "
                            "whole step, a lower bound on the link rate"}
        kernels = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]} for k, v in kt.items()}
        roof = None
        if self.world == 1:
            # algorithmic HBM bytes per launch of the one-GPU grouping:
            # hist reads key + has_key; the scatter reads key, rank, has_key and writes one
            # 16-B record per keyed row plus every row's initial rep; the group-by reads
            # the records and writes rep for the rows that link to an earlier chunk
            rep = self.group(key, has, grank)
            nk = int(has.sum())
            linked = int((rep != rank).sum())
            # implicit rank: no rank array read, 12-byte records
            rb, recb = (0, 12) if implicit else (4, 16)
            alg = {"bucket_hist": 9 * per, "bucket_scatter": (13 + rb) * per + recb * nk,
                   "bucket_group": recb * nk + 4 * linked}
            roof = {"bound": "hbm", "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                    "linked_rows": linked,
                    "kernels": {k: {"algorithmic_bytes": b,
                                    "achieved": b / (kernels[k]["avg_ms"] * 1e-3) / 1e9,
                                    "frac": b / (kernels[k]["avg_ms"] * 1e-3) / HBM_PEAK}
                                for k, b in alg.items() if kernels.get(k, {}).get("avg_ms")},
                    "note": "algorithmic bytes of this partition + group-by design "
                            "(DESIGN.md section 4); PMC traffic in profiles/"}
            # PMC HBM bytes per launch (committed FETCH_SIZE / WRITE_SIZE passes of
            # this 12.5 M-row grouping) beside the algorithmic bytes, and the whole
            # step against SURVEY 8(d)'s 16 B per row
            pmc_names = {"bucket_hist": "k_part_hist",
                         "bucket_scatter": ("k_part_scatter_ws" if implicit
                                            else "k_part_scatter_rec_staged"),
                         "bucket_group": "k_bucket_group12_pk" if implicit else "k_bucket_group_pk"}
            src = None
            for k, kn in pmc_names.items():
                b_, src_ = pmc_traffic(kn, "dedup")
                if k in roof["kernels"]:
                    roof["kernels"][k]["pmc_traffic"] = b_
                src = src or src_
            step_s = t / steps
            pmc_sum = [roof["kernels"].get(k, {}).get("pmc_traffic") for k in pmc_names]
            roof["step"] = {"survey_8d_bytes": 16 * per,
                            "achieved": 16 * per / step_s / 1e9,
                            "frac": 16 * per / step_s / HBM_PEAK,
                            "design_bytes": sum(alg.values()),
                            "pmc_traffic": (sum(pmc_sum) if all(x is not None for x in pmc_sum)
                                            else None),
                            "pmc_source": src}
        if self.world == 1 and not self.args.no_cpu:
            self._cpu_dedup = self.cpu_grouping(key, has, rank, grank)
        # K7 Object link batch over the same 12.5 M rows: the
        # create list and the (row, creator) connect pairs as dense arrays
        repv = self.group(key, has, grank)
        link_t, link_kt = self.timed_kernels(
            lambda: dedup.link_batch_device(repv, rank, has, 0, ctx=self.ctx, trim=False),
            steps, warmup)
        c_, l_ = (int(x) for x in dedup.link_batch_device(repv, rank, has, 0, ctx=self.ctx,
                                                          trim=False)[3].cpu().tolist())
        link_bytes = 9 * per + 4 * c_ + 8 * l_
        link = {"value": self.world * per * steps / link_t, "unit": "rows/s",
                "ms_per_step": 1e3 * link_t / steps, "created": c_, "linked": l_,
                "roofline": {"bound": "hbm", "algorithmic_bytes": link_bytes,
                             "achieved": link_bytes / (link_t / steps) / 1e9,
                             "frac": link_bytes / (link_t / steps) / HBM_PEAK, "unit": "GB/s",
                             "note": "reads rep + rank + has_key, writes the create list and "
                                     "the connect pairs; the flag scans' own traffic on top"},
                "kernels": {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]}
                            for k, v in link_kt.items()}}
        del repv
        # the fused step (sdgpu_group_link_device): the same grouping and write
        # set without a rep array -- the group kernel emits the lists itself
        # (valid = has_key, as in the two-call leg above, for the same write set)
        fused = None
        if self.world == 1:
            fz_t, fz_kt = self.timed_kernels(
                lambda: dedup.group_link_device(key, has, has, grank, 0, 100, ctx=self.ctx,
                                                trim=False), steps, warmup)
            fused = {"ms_per_step": 1e3 * fz_t / steps, "value": per * steps / fz_t,
                     "unit": "rows/s",
                     "two_call_ms_per_step": 1e3 * t / steps + link["ms_per_step"],
                     "note": "grouping + Object write set in one pass (no rep array); "
                             "two_call = group_rows + link_batch_device above",
                     "kernels": {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]}
                                 for k, v in fz_kt.items()}}
        xmodel = None
        if self.world == 1 and self.comm is None and not self.args.no_exchange_model:
            try:
                xmodel = self.exchange_model(key, has, rank, steps, warmup, 1e3 * t / steps)
            except Exception as e:  # noqa: BLE001 -- reported, the leg goes on
                log(f"bench: exchange model failed: {e!r}")
                xmodel = {"error": repr(e)[:300]}
        full = None
        if self.world == 1 and self.args.dedup_full_rows:
            full = self.run_dedup_full(steps, warmup)
        return {"value": total * steps / t, "unit": "rows/s", "ms_per_step": 1e3 * t / steps,
                "rank": "implicit (row order, 12-byte records)" if implicit else "explicit array",
                "explicit_rank_ms_per_step": explicit_ms, "exchange": xchg, "roofline": roof, "config4_full_one_gpu": full,
                "link_batch": link, "fused_job": fused, "predicted_scaling": xmodel,
                "config": {"workload": "config4: 80% distinct u64 keys + 20% dups, 0.1% keyless",
                           "rows_per_gpu": per, "rows_total": total},
                "kernels": kernels}

    # per-direction rate of one xGMI link under RCCL's all-to-all: 153 GB/s per
    # link (SURVEY §2.3 / BASELINE.md) at ~65 % protocol efficiency -- an
    # ASSUMPTION of the model below, not a measurement (no 8-GPU node here)
    XGMI_LINK_GBPS = 100.0

    @staticmethod
    def padded_slots(rows: int, n_ranks: int) -> int:
        """Slots (header included) of one padded exchange message at n_ranks
        ranks of `rows` rows each (csrc/shard.cpp padded_slots)."""
        c = rows if n_ranks == 1 else min(rows, rows // n_ranks + rows // (128 * n_ranks) + 4096)
        return -(-(c + 1) // 64) * 64

    def exchange_model(self, key, has, rank, steps, warmup, local_ms):
        """Predicted per-GPU config-4 step at N = 2 / 4 / 8 (DESIGN.md §6;
        VERDICT r3 item 4, r4 item 1).  The whole exchange path runs on this
        GPU through a ONE-rank RCCL communicator -- partition by owner, the
        records' all-to-all (a self send), the local grouping of as many
        received rows as one GPU gets at any N (weak scaling: every GPU sends
        its rows and receives ~as many), the return leg and the gather --
        timed with its kernels; only the xGMI time of the remote share is
        modelled: every GPU sends one message per peer over that peer's own
        link (fully connected node).  Since round 5 the default exchange is
        PADDED (fixed-capacity messages, no host synchronisation; sdgpu.h):
        its messages carry the padded slot count, 12 B each (+ 4 B back for
        the rep form).  The counted forms (count exchange + host sync; the
        compact return) are rehearsed beside it for the A/B."""
        from spacedrive_amd import dedup
        per = int(key.numel())
        comm = dedup.Comm.init_rank(self.ctx, 1, 0, dedup.Comm.unique_id(),
                                    timeout_ms=self.comm_timeout_ms)
        stats = {}

        def rehearse(name, fn, kernels=False):
            fn()
            comm.wait()
            s0 = comm.stats()
            if kernels:
                t_, kt_ = self.timed_kernels(fn, steps, warmup)
            else:
                t_, kt_ = self.timed(fn, steps, warmup), None
            comm.wait()
            s1 = comm.stats()
            calls = max(1, s1["calls"] - s0["calls"])
            stats[name] = {
                "ms_per_step": 1e3 * t_ / steps,
                "count_wait_ms_per_call": (s1["count_wait_ms"] - s0["count_wait_ms"]) / calls,
                "host_ms_per_call": (s1["host_ms"] - s0["host_ms"]) / calls,
                "padded_calls": s1["padded_calls"] - s0["padded_calls"],
                "overflow_reruns": s1["overflow_reruns"] - s0["overflow_reruns"],
                "resolve_wait_ms_per_call": (s1["resolve_wait_ms"] - s0["resolve_wait_ms"]) / calls,
                "bytes_sent_per_row": (s1["bytes_sent"] - s0["bytes_sent"]) / max(
                    1, s1["rows_sent"] - s0["rows_sent"]),
                "rows_returned": s1["rows_returned"] - s0["rows_returned"],
                "rows_received": s1["rows_received"] - s0["rows_received"]}
            if kt_ is not None:
                stats[name]["kernels"] = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]}
                                          for k, v in kt_.items()}
            return 1e3 * t_ / steps

        try:
            # the rep form, counted with the compact return (explicit setting)
            comm.set_return(dedup.RETURN_COMPACT)
            rep_compact = rehearse("rep_counted_compact", lambda: dedup.group_sharded(
                key, has, rank, comm, None, 100, wait=False))
            st = stats["rep_counted_compact"]
            linked_frac = st["rows_returned"] / max(1, st["rows_received"])
            # the rep form, full return: padded (the default) and counted
            comm.set_return(dedup.RETURN_AUTO)
            rep_padded = rehearse("rep_padded", lambda: dedup.group_sharded(
                key, has, rank, comm, None, 100, wait=False), kernels=True)
            comm.set_exchange(dedup.EXCHANGE_COUNTED)
            comm.set_return(dedup.RETURN_FULL)
            rep_counted = rehearse("rep_counted_full", lambda: dedup.group_sharded(
                key, has, rank, comm, None, 100, wait=False))
            comm.set_return(dedup.RETURN_AUTO)
            # the write-set form (sdgpu_group_link_sharded_device): counted, then
            # padded (the N > 1 identifier step's path)
            fl = lambda: dedup.group_link_sharded(key, has, None, rank, comm, 100,  # noqa: E731
                                                  trim=False)
            ws_counted = rehearse("write_set_counted", fl)
            comm.set_exchange(dedup.EXCHANGE_AUTO)
            ws_padded = rehearse("write_set_padded", fl, kernels=True)
        finally:
            comm.close()
        pred, pred_lists = {}, {}
        for n_ in (2, 4, 8):
            c1 = self.padded_slots(per, n_)
            link_b = c1 * 16  # 12-B records out, 4-B reps back, per link direction
            x_ms = link_b / (self.XGMI_LINK_GBPS * 1e9) * 1e3
            step = rep_padded + x_ms
            pred[str(n_)] = {"exchange": "padded, full return", "slots_per_message": c1,
                             "step_ms": step, "xgmi_ms": x_ms, "bytes_per_link": int(link_b),
                             "rows_per_s_total": n_ * per / (step * 1e-3),
                             "weak_scaling_efficiency": local_ms / step}
            link_b = c1 * 12
            x_ms = link_b / (self.XGMI_LINK_GBPS * 1e9) * 1e3
            step = ws_padded + x_ms
            pred_lists[str(n_)] = {"slots_per_message": c1, "step_ms": step, "xgmi_ms": x_ms,
                                   "bytes_per_link": int(link_b),
                                   "rows_per_s_total": n_ * per / (step * 1e-3)}
        return {"rehearsal_ms_per_step": rep_padded,
                "rehearsal_full_return_counted_ms_per_step": rep_counted,
                "rehearsal_compact_counted_ms_per_step": rep_compact,
                "rehearsal_write_set_ms_per_step": ws_padded,
                "rehearsal_write_set_counted_ms_per_step": ws_counted,
                "per_n_write_set": pred_lists,
                "write_set_note": "grouping + Object write set with no return leg "
                                  "(sdgpu_group_link_sharded_device, the N > 1 identifier "
                                  "step's path), padded exchange: 12 B per slot on the wire; "
                                  "against fused_job.ms_per_step at N = 1",
                "count_wait_ms_per_call": stats["write_set_padded"]["count_wait_ms_per_call"],
                "host_ms_per_call": stats["write_set_padded"]["host_ms_per_call"],
                "linked_fraction": linked_frac, "local_only_ms_per_step": local_ms,
                "xgmi_link_GBps_assumed": self.XGMI_LINK_GBPS, "per_n": pred,
                "legs": stats,
                "note": "PREDICTION (unmeasured on hardware at N > 1): the exchange path "
                        "rehearsed on one GPU (one-rank RCCL: partition, padded records (no "
                        "host synchronisation), local grouping of the received rows, full "
                        "return, gather) + the modelled xGMI time of one padded message per "
                        "link; at one rank a message has no slack slots, at N ranks "
                        "slots_per_message ~1.6 % over rows/N (the model's bytes)"}

    def staged_oracle(self):
        """Config 5's parity at full size: the reps of the batched 50 M-file run
        (grouped step by step through the Object index on the GPU) against the
        oracle's grouping of ALL its rows at once (orc_group_reps, C, one
        thread; the canonical rule over global ranks, file_identifier/mod.rs:
        168-241)."""
        from oracle import oracle as O
        keys, has, reps = self._staged_verify
        self._staged_verify = None
        t0 = time.perf_counter()
        ref = O.group_reps(keys, has, 100)
        dt = time.perf_counter() - t0
        bad = int(np.count_nonzero(ref != reps))
        return {"rows": int(keys.size), "mismatches": bad, "oracle_rows_per_s": keys.size / dt,
                "oracle_seconds": dt,
                "note": "reps of the batched run (Object index, step by step) vs the oracle's "
                        "one grouping of all its rows (oracle orc_group_reps, one thread)"}

    def cpu_grouping(self, key, has, rank, grank):
        """CPU leg of config 4: the oracle's C grouping (orc_group_reps, one
        thread: a restatement of the chunk rule over rows in rank order) on the
        same 12.5 M rows, timed; its reps must equal the GPU's (a parity check
        at full size)."""
        from oracle import oracle as O
        order = np.argsort(rank.cpu().numpy().view(np.uint32), kind="stable")
        k = key.cpu().numpy().view(np.uint64)[order]
        h = has.cpu().numpy()[order]
        gpu = self.group(key, has, grank).cpu().numpy().view(np.uint32)[order]
        t0 = time.perf_counter()
        ref = O.group_reps(k, h, 100)
        dt = time.perf_counter() - t0
        return {"value": k.size / dt, "unit": "rows/s", "threads": 1, "kind": "port",
                "gpu_rep_mismatches": int(np.count_nonzero(ref != gpu)),
                "sample": f"config 4: the same {k.size} rows (rank order), oracle orc_group_reps "
                          f"(C, one thread; the reference groups with SQLite queries per "
                          f"100-row chunk), {dt:.1f} s"}

    def run_dedup_full(self, steps, warmup):
        """BASELINE config 4 at its full size on ONE GPU (the strong-scaling
        base of the 1 -> 8 GPU curve): 100 M rows, 2^15 buckets, every bucket
        grouped in LDS."""
        torch = self.torch
        from spacedrive_amd import corpus
        total = self.args.dedup_full_rows
        key, has, rank = corpus.synth_dedup_rows_device(4, total, int(total * 0.8), 0, total,
                                                        device=self.local, ctx=self.ctx)
        # rows in rank order (synth rank[i] = i): no rank array, 12-byte records;
        # the explicit-rank call timed beside it
        assert bool((rank == torch.arange(total, dtype=rank.dtype, device=rank.device)).all())
        self.ops.group_rows(key, has, None, 100, 0)  # two-level kernels' first launches
        torch.cuda.synchronize()
        t, kt = self.timed_kernels(lambda: self.ops.group_rows(key, has, None, 100, 0), steps,
                                   warmup)
        explicit_ms = None
        if not self.args.no_explicit_rank:
            self.ops.group_rows(key, has, rank, 100, 0)
            explicit_ms = 1e3 * self.timed(lambda: self.ops.group_rows(key, has, rank, 100, 0),
                                           steps, warmup) / steps
        from spacedrive_amd import dedup
        fz_t, fz_kt = self.timed_kernels(
            lambda: dedup.group_link_device(key, has, None, None, 0, 100, ctx=self.ctx,
                                            trim=False), steps, warmup)
        fz_lists = None
        if not self.args.no_cpu:
            who, obj, _ = dedup.group_link_device(key, has, None, None, 0, 100, ctx=self.ctx)
            fz_lists = dedup.split_link_lists(who.cpu().numpy(), obj.cpu().numpy())
            del who, obj
        rep = self.ops.group_rows(key, has, None, 100, 0)
        nk = int(has.sum())
        linked = int((rep != rank).sum())
        # parity of the timed variant at full size: the
        # oracle's C grouping of the same 100 M rows (rank order), outside
        # every timed region
        parity = None
        if not self.args.no_cpu:
            from oracle import oracle as O
            hk = key.cpu().numpy().view(np.uint64)
            hh = has.cpu().numpy()
            gpu = rep.cpu().numpy().view(np.uint32)
            t0 = time.perf_counter()
            ref = O.group_reps(hk, hh, 100)
            dt = time.perf_counter() - t0
            parity = int(np.count_nonzero(ref != gpu))
            rc, rlr, rlo = O.link_batch(ref, None, None, 0)
            fc, flr, flo = fz_lists
            fz_bad = (int(abs(fc.size - rc.size) + abs(flr.size - rlr.size)) or
                      int(np.count_nonzero(fc != rc) + np.count_nonzero(flr != rlr) +
                          np.count_nonzero(flo != rlo)))
            del hk, hh, gpu, ref, rc, rlr, rlo, fc, flr, flo, fz_lists
        del key, has, rank, rep
        torch.cuda.empty_cache()
        kernels = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]} for k, v in kt.items()}
        # algorithmic HBM bytes per launch of the two-level path without a
        # histogram pass: the coarse pass (k_part_private)
        # reads key + has_key, writes rep, one record per keyed row into its own
        # tile range, the run table (start + length per block x 4096-row round x
        # coarse digit) and the fine counts (2^15 buckets x 256 blocks x 4 B); the
        # fine scan reads those and writes the 128 block starts per bucket; the
        # second pass (k_part2_runs) moves every record once more; the group-by as
        # in the one-level path (implicit rank: no rank array read, 12-byte records)
        nfine = 1 << 15
        tile = -(-total // 256)  # rows per coarse block (ceil)
        rounds = -(-tile // 4096)
        alg = {"bucket_scatter1": 13 * total + 12 * nk + 8 * 256 * rounds * 64 + 4 * nfine * 256,
               "bucket_fine_scan": 4 * nfine * 256 + 4 * nfine * 128 + 4 * nfine,
               "bucket_scatter": 24 * nk,
               "bucket_group": 12 * nk + 4 * linked}
        pmc_names = {"bucket_scatter1": "k_part_private", "bucket_scatter": "k_part2_runs",
                     "bucket_group": "k_bucket_group12_pk"}
        step_s = t / steps
        roof = {"bound": "hbm", "peak": HBM_PEAK / 1e9, "unit": "GB/s", "linked_rows": linked,
                "kernels": {}, "note": "algorithmic bytes of the two-level partition + group-by "
                                       "(DESIGN.md section 4); PMC traffic in profiles/"}
        src = None
        for k, b in alg.items():
            ms = kernels.get(k, {}).get("avg_ms")
            if not ms:
                continue
            e = {"algorithmic_bytes": b, "achieved": b / (ms * 1e-3) / 1e9,
                 "frac": b / (ms * 1e-3) / HBM_PEAK}
            if k in pmc_names:
                e["pmc_traffic"], src_ = pmc_traffic(pmc_names[k], "dedup_full")
                src = src or src_
            roof["kernels"][k] = e
        roof["step"] = {"survey_8d_bytes": 16 * total, "achieved": 16 * total / step_s / 1e9,
                        "frac": 16 * total / step_s / HBM_PEAK, "design_bytes": sum(alg.values()),
                        "pmc_source": src}
        fused = {"ms_per_step": 1e3 * fz_t / steps, "value": total * steps / fz_t,
                 "unit": "rows/s",
                 "note": "grouping + Object write set (creators / connect pairs) in one pass, "
                         "no rep array (sdgpu_group_link_device, valid = all rows)",
                 "kernels": {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]}
                             for k, v in fz_kt.items()}}
        # the list-writing group kernel: reads every keyed record, writes the
        # write set itself (who for every keyed row, obj for the linked ones)
        # -- no scattered rep stores
        gms = fused["kernels"].get("bucket_group", {}).get("avg_ms")
        if gms:
            gb = 12 * nk + 4 * nk + 4 * linked
            pt, _ = pmc_traffic("k_bucket_group12_pk:ListOut", "dedup_full")
            fused["roofline"] = {"bucket_group": {
                "algorithmic_bytes": gb, "achieved": gb / (gms * 1e-3) / 1e9,
                "frac": gb / (gms * 1e-3) / HBM_PEAK, "pmc_traffic": pt,
                "note": "reads 12 B per keyed record; writes who (4 B per keyed row) and obj "
                        "(4 B per linked row)"}}
        if parity is not None:
            fused["list_mismatches_vs_oracle"] = fz_bad
        out = {"value": total * steps / t, "unit": "rows/s", "ms_per_step": 1e3 * step_s,
               "rows": total, "rank": "implicit (row order, 12-byte records)",
               "explicit_rank_ms_per_step": explicit_ms, "roofline": roof, "kernels": kernels,
               "gpu_rep_mismatches": parity, "fused_job": fused}
        if parity is not None:
            out["oracle_seconds"] = round(dt, 2)
            out["parity_note"] = ("reps of the timed implicit-rank call vs oracle orc_group_reps "
                                  "over all rows (C, one thread)")
        return out

    def verify_sharded(self, key, has, rank):
        """--verify: the sharded grouping over all ranks (the exchange path the
        timed steps use) equals the one-GPU grouping of the gathered table."""
        torch, dist = self.torch, self.dist
        from spacedrive_amd import dedup
        rep = self.group(key, has, rank)
        if self.world > 1:
            parts = [[torch.empty_like(t) for _ in range(self.world)] for t in (key, has, rank, rep)]
            for p, t in zip(parts, (key, has, rank, rep)):
                dist.all_gather(p, t)
            key, has, rank, rep = (torch.cat(p) for p in parts)
        if self.rank == 0:
            ref = self.ops.group_rows(key, has, rank, 100, 0)
            bad = int((ref != rep).sum())
            log(f"verify: sharded grouping of {key.numel()} rows over {self.world} ranks: "
                f"{bad} mismatches vs the one-GPU grouping")
            assert bad == 0, "sharded grouping differs from the one-GPU grouping"
        self.barrier()

    # ------------------------------------------- downstream consumers (§8 f4)
    def run_consumers(self, steps, warmup):
        """The orphan remover's query over 10 M Objects / 12.5 M file_paths
        (orphan_remover.rs:57-90) and the thumbnail-shard grouping of 1 M cas
        ids (media/thumbnail/shard.rs:4-8) on this GPU's own synthetic tables:
        calls back to back with the counts left on the device (trim=False, as
        the other legs), and each call with its count read-back (one host
        synchronisation per call)."""
        torch = self.torch
        from spacedrive_amd import consumers
        n_obj, n_fp, n_th = 10_000_000, 12_500_000, 1_000_000
        g = torch.Generator(device=self.dev)
        g.manual_seed(5 + self.rank)
        obj = torch.arange(n_obj, dtype=torch.int32, device=self.dev)
        fp = torch.randint(0, n_obj, (n_fp,), dtype=torch.int32, device=self.dev, generator=g)
        fp[::1000] = -1                       # file_paths with object_id NULL
        cas8 = torch.randint(0, 256, (n_th, 8), dtype=torch.uint8, device=self.dev, generator=g)
        orphans = int(consumers.orphan_objects(obj, fp, n_obj - 1, ctx=self.ctx).numel())
        t_o = self.timed(lambda: consumers.orphan_objects(obj, fp, n_obj - 1, ctx=self.ctx,
                                                          trim=False), steps, warmup)
        t_os = self.timed(lambda: consumers.orphan_objects(obj, fp, n_obj - 1, ctx=self.ctx),
                          steps, warmup)
        t_t = self.timed(lambda: consumers.thumbnail_shards(cas8, ctx=self.ctx, trim=False),
                         steps, warmup)
        t_ts = self.timed(lambda: consumers.thumbnail_shards(cas8, ctx=self.ctx), steps, warmup)
        del obj, fp, cas8
        # algorithmic bytes: object_id of every file_path (4 B) + a mark byte per
        # Object id, the Object ids (4 B) and the orphan list written (4 B each)
        ob = 4 * n_fp + n_obj + 4 * n_obj + 4 * orphans
        return {"orphan_remover": {"value": self.world * (n_obj + n_fp) * steps / t_o,
                                   "unit": "rows/s", "ms_per_step": 1e3 * t_o / steps,
                                   "objects_per_gpu": n_obj, "file_paths_per_gpu": n_fp,
                                   "orphans_rank0": orphans,
                                   "ms_per_call_with_readback": 1e3 * t_os / steps,
                                   "roofline": {"bound": "hbm", "algorithmic_bytes": ob,
                                                "achieved": ob / (t_o / steps) / 1e9,
                                                "frac": ob / (t_o / steps) / HBM_PEAK,
                                                "unit": "GB/s",
                                                "note": "calls back to back, count on the "
                                                        "device (no per-call synchronisation)"}},
                "thumbnail_shards": {"value": self.world * n_th * steps / t_t, "unit": "rows/s",
                                     "ms_per_step": 1e3 * t_t / steps, "rows_per_gpu": n_th,
                                     "ms_per_call_with_readback": 1e3 * t_ts / steps}}

    # ---------------------------------------------------------------- config 3
    def run_checksum(self, steps, warmup):
        torch = self.torch
        from spacedrive_amd import corpus, validation
        nf, flen = self.args.checksum_files, self.args.checksum_bytes
        files = []
        try:
            for i in range(nf):
                files.append(corpus.synth_file_device(3 + 7919 * i + 104729 * self.rank, flen,
                                                      device=self.local, ctx=self.ctx))
        except (RuntimeError, MemoryError) as e:  # torch OOM
            log(f"checksum: only {len(files)} of {nf} files fit: {e}")
        torch.cuda.synchronize()
        out = torch.empty((len(files), 32), dtype=torch.uint8, device=self.dev)
        t, kt = self.timed_kernels(
            lambda: validation.checksum_batch_device(files, out=out, ctx=self.ctx), steps, warmup)
        nbytes = len(files) * flen
        res = {"value": self.world * nbytes * steps / t / 1e9, "unit": "GB/s",
               "ms_per_step": 1e3 * t / steps,
               "config": {"workload": "config3: 4 GiB files, device-resident",
                          "files_per_gpu": len(files), "file_bytes": flen},
               "kernels": {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]}
                           for k, v in kt.items()}}
        # VALU roofline of the leaf kernel: 16 compressions per chunk + parents
        chunks = nbytes // 1024
        comp = chunks * 16 + (chunks - len(files))
        lv = kt.get("tree_leaves", (0.0, 1))
        if lv[0] > 0:
            res["leaf_valu_frac_spec"] = comp * ISA_PER_COMPRESSION / (lv[0] / lv[1] * 1e-3) \
                / VALU_PEAK_SPEC
        if self.world == 1 and not self.args.no_cpu and files:
            # parity of the timed batch (after the timing; VERDICT r4 item 4;
            # at N = 1 only, like every oracle check of the bench):
            # the first, the last and two middle digests of the ONE plan the
            # bench times (cross-file offsets past 2^32 bytes) against the
            # oracle's multi-threaded AVX-512 hasher over the same bytes
            from oracle import oracle as O
            threads, _ = host_cores()
            picks = sorted({0, len(files) // 3, 2 * len(files) // 3, len(files) - 1})
            got = out.cpu().numpy()
            bad, t0 = 0, time.perf_counter()
            for i in picks:
                host = files[i].cpu().numpy()
                bad += int(bytes(got[i]) != O.blake3(host, threads=threads))
                del host
            res["gpu_digest_mismatches"] = bad
            res["digests_checked"] = {"files": picks, "threads": threads,
                                      "seconds": time.perf_counter() - t0,
                                      "checker": "oracle blake3 (AVX-512 16-way, multi-threaded)"}
        del files
        return res

    def cpu_baseline(self):
        from oracle import oracle as O
        arena, off, ln, m, gpu_cas8 = self._cpu_sample
        h_off = off[:m].cpu().numpy().view(np.uint64)
        h_len = ln[:m].cpu().numpy().view(np.uint32)
        end = int(h_off[-1] + h_len[-1])
        host = arena[:end].cpu().numpy()
        threads, cores_note = host_cores()
        # the reference crate hashes a message's chunks 8/16 at a time with
        # SIMD: time the AVX2 8-way restatement (oracle/sd_oracle.c
        # orc_cas_batch_simd); the scalar oracle is reported beside it
        O.cas_batch_simd(host, h_off[:100], h_len[:100], threads)  # warm
        # repeat the sample until about 10 s of CPU work has been timed
        t0 = time.perf_counter()
        cpu_cas8 = O.cas_batch_simd(host, h_off, h_len, threads)
        t1 = time.perf_counter() - t0
        # the headline step's GPU cas ids of the same files (parity in the bench)
        sample_mism = int(np.count_nonzero(np.any(cpu_cas8 != gpu_cas8, axis=1)))
        assert sample_mism == 0, f"config 2: {sample_mism} GPU cas ids differ from the CPU port"
        reps = int(min(60, max(1, np.ceil(self.args.cpu_seconds / max(t1, 1e-3)))))
        t0 = time.perf_counter()
        for _ in range(reps):
            O.cas_batch_simd(host, h_off, h_len, threads)
        dt = time.perf_counter() - t0
        # one thread (the reference hashes a 100-file chunk on ONE runtime
        # thread, file_identifier/mod.rs:107-134): a 1/16 slice of the sample
        m1 = max(1, m // 16)
        t0 = time.perf_counter()
        O.cas_batch_simd(host, h_off[:m1], h_len[:m1], 1)
        one = m1 / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        O.cas_batch(host, h_off[:m1], h_len[:m1], threads)
        scalar = m1 / (time.perf_counter() - t0)
        dir_res = None
        if getattr(self, "_dir_sample", None):
            import shutil
            from concurrent.futures import ThreadPoolExecutor
            paths, sizes, root, gpu_cas8 = self._dir_sample
            O.cas_paths_simd(paths[:200], sizes[:200], threads)  # warm
            cpu_s = []  # timed like the GPU leg: each pass on its own, the median
            for _ in range(5):
                t0 = time.perf_counter()
                cpu_cas8, dst = O.cas_paths_simd(paths, sizes, threads)
                cpu_s.append(time.perf_counter() - t0)
            ddt = float(np.median(cpu_s))
            assert np.all(dst == 0)
            mism = int(np.count_nonzero(np.any(cpu_cas8 != gpu_cas8, axis=1)))
            assert mism == 0, f"config-1 directory: {mism} GPU cas ids differ from the CPU port"
            with ThreadPoolExecutor(threads) as ex:  # the C oracle releases the GIL
                t0 = time.perf_counter()
                list(ex.map(O.cas_id_path, paths, sizes.tolist()))
                sdt = time.perf_counter() - t0
            dir_res = {"value": len(paths) / ddt, "unit": "files/s", "threads": threads,
                       "mean_value": len(paths) * len(cpu_s) / sum(cpu_s),
                       "pass_ms": [round(1e3 * x, 3) for x in cpu_s],
                       "scalar_value": len(paths) / sdt, "gpu_cas_ids_checked": len(paths),
                       "gpu_cas_id_mismatches": mism,
                       "sample": f"config 1: {len(paths)} real files, warm cache, median of 5 passes, the "
                                 f"reference's reads per file (open, header / 4 samples / "
                                 f"footer, cas.rs:23-62) + {O.simd_isa()} BLAKE3 "
                                 f"(oracle orc_cas_paths_simd), {threads} threads; "
                                 f"scalar_value = scalar oracle cas_id_path, same threads"}
            shutil.rmtree(root, ignore_errors=True)
            self._dir_sample = None
        # config 3's hashing (file_checksum, hash.rs:10-24): the AVX2 subtree
        # hasher, one 256 MiB buffer per thread (one file per thread, as that
        # many validator jobs would run), and on one thread (the reference
        # hashes a file on one blocking-pool thread)
        buf = np.random.default_rng(3).integers(0, 256, 256 << 20, dtype=np.uint8)
        t0 = time.perf_counter()
        O.blake3_simd(buf)
        ck1 = buf.size / (time.perf_counter() - t0)
        ck_reps = int(max(1, min(20, np.ceil(3.0 * ck1 / buf.size))))
        t0 = time.perf_counter()
        O.checksum_simd_mt(buf, threads, ck_reps)
        ckt = time.perf_counter() - t0
        ck = {"value": threads * ck_reps * buf.size / ckt / 1e9, "unit": "GB/s",
              "threads": threads, "value_1thread": ck1 / 1e9,
              "sample": f"{threads} threads x {ck_reps} x 256 MiB in host RAM, {O.simd_isa()} "
                        f"BLAKE3 over 1024-chunk subtrees (oracle orc_checksum_simd_mt)"}
        del buf
        single = None
        if getattr(self, "_single_sample", None):
            single = {}
            for p, size in self._single_sample:
                name = os.path.basename(p)
                for fn_name, fn in (("generate_cas_id", lambda: O.cas_id_path(p, size)),
                                    ("file_checksum", lambda: O.file_checksum_path(p))):
                    for _ in range(10):
                        fn()
                    ts = []
                    for _ in range(200):
                        t0 = time.perf_counter()
                        fn()
                        ts.append(time.perf_counter() - t0)
                    single[f"{fn_name}_{name}_us"] = float(np.median(ts) * 1e6)
        burst = None
        if getattr(self, "_burst_sample", None):
            # the same bursts through the CPU port behind the reference's reads:
            # one thread (a runtime thread taking the calls one by one) and all
            # threads (the blocking pool taking them concurrently)
            burst = {}
            for name, pl, sizes, gpu8 in self._burst_sample:
                cpu8, bst = O.cas_paths_simd(pl, sizes, 1)
                assert np.all(bst == 0)
                mism = int(np.count_nonzero(np.any(cpu8 != gpu8, axis=1)))
                assert mism == 0, f"burst {name}: {mism} GPU cas ids differ from the CPU port"
                row = {"gpu_cas_id_mismatches": mism, "threads": threads}
                for key_, th in (("cpu_1thread_burst_us", 1), ("cpu_threads_burst_us", threads)):
                    ts = []
                    for _ in range(30):
                        t0 = time.perf_counter()
                        O.cas_paths_simd(pl, sizes, th)
                        ts.append(time.perf_counter() - t0)
                    row[key_] = float(np.median(ts) * 1e6)
                burst[name] = row
            self._burst_sample = None
        return {"value": reps * m / dt, "unit": "files/s", "cores": threads, "kind": "port",
                "cores_note": cores_note, "gpu_cas_id_mismatches": sample_mism,
                "value_1thread": one, "scalar_value": scalar,
                "config1_dir": dir_res, "config3_checksum": ck,
                "single_file_1thread": single, "single_file_burst": burst,
                "sample": f"first {m} files of config 2 (their {int(h_len.sum())} window bytes "
                          f"in host RAM) hashed {reps}x, {O.simd_isa()} BLAKE3 port "
                          f"(oracle/sd_oracle.c orc_cas_batch_simd), {threads} threads, "
                          f"{dt:.1f} s wall; scalar_value = scalar oracle, same threads; "
                          f"value_1thread = one thread (the reference hashes a 100-file "
                          f"step on one runtime thread, file_identifier/mod.rs:107-134)"}


def self_launch(n: int) -> int:
    """`bench.py --gpus N` without torch.distributed's environment: start the N
    ranks ourselves (one process per GPU, 127.0.0.1 rendezvous) as a CHILD
    process -- before this process touches the GPU -- and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


class LineWriter:
    """The bench's one JSON line, guarded so it is printed exactly once: at the
    end of a normal run, or by the watchdog when the deadline passes first
    (an auxiliary leg that fails or hangs must not take the
    headline, roofline and cpu_baseline with it)."""

    def __init__(self, out, rank: int):
        import threading
        self.out, self.rank = out, rank
        self.lock = threading.Lock()
        self.done = False
        self.line = {"metric": METRIC, "value": None, "components": {}}

    def emit(self, **extra) -> None:
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank == 0:
                line = dict(self.line)
                line.update(extra)
                print(json.dumps(line, default=str), file=self.out, flush=True)


def start_watchdog(writer: LineWriter, seconds: float, state: dict):
    """Prints the line with what was measured so far and ends the process if
    the run is still going after `seconds` (a hung leg, e.g. a collective whose
    peer died).  Daemon timer thread: ctypes / HIP waits release the GIL."""
    import threading

    def fire():
        leg = state.get("leg")
        log(f"bench: deadline of {seconds:.0f} s passed inside leg {leg!r}; "
            "printing what was measured and exiting")
        comp = writer.line.setdefault("components", {})
        if leg:
            comp.setdefault(leg, {})["error"] = f"deadline: still running after {seconds:.0f} s"
        writer.line["incomplete"] = {"leg": leg, "deadline_s": seconds}
        writer.emit()
        sys.stdout.flush()
        sys.stderr.flush()
        # non-zero either way (a hung leg must not look
        # green): 4 = the headline was measured and is in the line, 3 = not
        os._exit(4 if writer.line.get("value") is not None else 3)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def build_roofline(c, compress_peak, valu_peak, classes):
    """The dominant kernel's roofline (K1 k_leaves3): algorithmic int32 ops per
    launch / its event-timed average duration, against the spec VALU peak."""
    ri = c["roofline_inputs"]
    ops = ri["leaf_compressions"] * ISA_PER_COMPRESSION
    t_leaf = ri["avg_leaves_s"]
    achieved = ops / t_leaf if t_leaf > 0 else 0.0
    traffic, traffic_src = pmc_traffic("k_leaves3")
    return {"bound": "valu", "kernel": "cas_leaves (K1 k_leaves3)",
            "achieved": achieved / 1e12, "peak": VALU_PEAK_SPEC / 1e12, "unit": "Tops/s",
            "frac": achieved / VALU_PEAK_SPEC, "traffic": traffic,
            "traffic_source": traffic_src,
            "peak_measured": compress_peak / 1e12 if compress_peak else None,
            "peak_measured_note": "register-only BLAKE3 compressions (same 680-VALU stream, no "
                                  "memory traffic): the attainable issue roof of this mix",
            "peak_g_mix_probe": valu_peak / 1e12 if valu_peak else None,
            "peak_by_class_measured": classes,
            "frac_of_measured": achieved / compress_peak if compress_peak else None,
            # the guide's SIMD-32 full-rate issue (MI355X_MICROARCH.md: 32
            # lanes per cycle), which only the VOP2 classes above approach;
            # `peak` is the rate of the VOP3 classes the compression needs
            "peak_guide_full_rate": 2 * VALU_PEAK_SPEC / 1e12,
            "frac_of_guide_full_rate": achieved / (2 * VALU_PEAK_SPEC),
            "algorithmic_per_launch": {"compressions": ri["leaf_compressions"],
                                       "int32_ops": ops, "window_bytes": ri["bytes"]},
            "compressions_per_s": ri["leaf_compressions"] / t_leaf if t_leaf else None,
            "hbm_GBps": ri["bytes"] / t_leaf / 1e9 if t_leaf else None,
            "hbm_frac": ri["bytes"] / t_leaf / HBM_PEAK if t_leaf else None}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--files", type=int, default=1_000_000)
    ap.add_argument("--dedup-rows", type=int, default=12_500_000)
    ap.add_argument("--dedup-full-rows", type=int, default=100_000_000,
                    help="config 4 at full size on one GPU (N = 1 only; 0 = skip)")
    ap.add_argument("--checksum-files", type=int, default=64)
    ap.add_argument("--checksum-bytes", type=int, default=1 << 32)
    ap.add_argument("--cpu-files", type=int, default=100_000)
    ap.add_argument("--staged-files", type=int, default=250_000)
    ap.add_argument("--staged-total-files", type=int, default=50_000_000)
    ap.add_argument("--dir-files", type=int, default=10_000)
    ap.add_argument("--components", default="cas,dedup,consumers,checksum,staged,dir,single")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--deadline", type=float,
                    default=float(os.environ.get("SD_BENCH_DEADLINE_S", "480")),
                    help="seconds after which the line is printed with what was measured "
                         "and the process ends (the driver's limit is 600 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-exchange-model", action="store_true",
                    help="skip the one-rank RCCL rehearsal behind the N = 2/4/8 prediction")
    ap.add_argument("--no-explicit-rank", action="store_true",
                    help="skip the explicit-rank grouping timed beside the implicit one "
                         "(PMC passes: one variant per kernel name)")
    ap.add_argument("--verify", action="store_true",
                    help="check the sharded grouping against the one-GPU grouping first")
    return ap.parse_args(argv)


def main(argv=None, runner_cls=None, out=None):
    """Runs the legs; every leg but the headline is guarded (a failure becomes
    components.<leg>.error), and the line is printed once -- at the end, or by
    the watchdog at --deadline."""
    import traceback
    args = parse_args(argv)
    comps = set(args.components.split(","))
    if runner_cls is None:
        if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
            sys.exit(self_launch(args.gpus))
        runner_cls = Runner
    if out is None:
        # stdout carries exactly one JSON line: everything else the process (or
        # a library it loads -- RCCL prints a version banner on communicator
        # init) writes to fd 1 goes to stderr
        sys.stdout.flush()
        out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
    if args.gpus != int(os.environ.get("WORLD_SIZE", "1")):
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}: "
            "reporting the launched world size")
    t_begin = time.perf_counter()
    state = {"leg": "init"}
    writer = LineWriter(out, int(os.environ.get("RANK", "0")))
    start_watchdog(writer, args.deadline, state)
    line = writer.line
    comp = line["components"]
    walls = {}
    line["leg_wall_s"] = walls

    def leg(name, fn, guarded=True):
        state["leg"] = name
        t0 = time.perf_counter()
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line, the run goes on
            if not guarded:
                raise
            log(f"bench: leg {name} failed: {e!r}\n{traceback.format_exc()}")
            comp.setdefault(name, {})["error"] = repr(e)[:400]
            return None
        finally:
            walls[name] = round(time.perf_counter() - t0, 2)
            state["leg"] = None

    R = leg("init", lambda: runner_cls(args), guarded=False)
    writer.rank = R.rank
    line.update({"unit": "files/s", "n_gpus": R.world, "steps": args.steps,
                 "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
                 "vs_baseline": None, "dtype": "u32",
                 "data": "synthetic (BASELINE configs 2/3/4 shapes, generated in HBM)",
                 "config": {"workload": "identifier job step: config2 (1M files/GPU) cas_id + "
                                        "cas_id->Object grouping + Object write set (one fused "
                                        "pass on one GPU; at N > 1 hash-sharded over RCCL, each "
                                        "owner writing its share of the write set, padded "
                                        "exchange)",
                            "files_per_gpu": args.files, "global_files": args.files * R.world,
                            "parallelism": f"dp{R.world} (files) + hash-sharded dedup, "
                                           "RCCL all-to-all"},
                 "world": R.world_info()})

    def peaks():
        v = R.ctx.valu_peak()
        cp = R.ctx.valu_peak(5)  # register-only compressions, 680 VALU each
        cl = {name: R.ctx.valu_peak(k) / 1e12 for k, name in
              [(1, "v_xor_b32"), (2, "v_add3_u32"), (3, "v_alignbit_b32"), (4, "v_add_u32")]}
        log(f"measured int32 VALU peak: {v / 1e12:.1f} T lane-ops/s "
            f"(spec {VALU_PEAK_SPEC / 1e12:.1f}); per class {json.dumps(cl)}")
        return v, cp, cl
    pk = leg("valu_probe", peaks) or (None, None, None)

    c = None
    if "cas" in comps:  # the headline step; only profiling passes leave it out
        c = leg("cas", lambda: R.run_cas(args.steps, args.warmup))
        if c:
            log("cas:", json.dumps(c["cas"]), json.dumps(c["kernels"]))
            comp["cas"] = c["cas"]
            comp["identifier_job"] = c["job"]
            if "error" in c["job"]:
                # no grouping result: no headline (K1 alone is a strict subset of the
                # step and would read faster); K1's rate stays under components.cas
                # and the process exits non-zero after printing the line
                line["value"] = None
                line["ms_per_step"] = None
                line["headline_note"] = ("identifier job step failed (components."
                                         "identifier_job.error); no headline value. "
                                         "K1's cas_id rate alone: components.cas")
            else:
                line["value"] = c["job"]["value"]
                line["ms_per_step"] = c["job"]["ms_per_step"]
            line["kernels"] = c["kernels"]
            line["roofline"] = leg("roofline", lambda: build_roofline(c, pk[1], pk[0], pk[2]))
    if "single" in comps:
        single = leg("single_file_latency", R.run_single)
        if single:
            log("single:", json.dumps(single))
            comp["single_file_latency"] = single
    if "dir" in comps:
        d = leg("dir", lambda: R.run_dir(max(3, min(args.steps, 9))))
        if d:
            log("dir:", json.dumps(d))
            comp["dir"] = d
    cpu = None
    if R.rank == 0 and R.world == 1 and not args.no_cpu and c:  # rank 0 at N = 1 only
        cpu = leg("cpu_baseline", R.cpu_baseline)
        if cpu:
            log("cpu:", json.dumps(cpu))
            # bursts: the CPU port's times beside the GPU's, per burst size
            gb = (comp.get("single_file_latency") or {}).get("burst") or {}
            for name, row in (cpu.get("single_file_burst") or {}).items():
                if name in gb:
                    gb[name].update(row)
                    gb[name]["gpu_batch_vs_cpu_1thread"] = (row["cpu_1thread_burst_us"] /
                                                            gb[name]["gpu_batch_burst_us"])
                    gb[name]["gpu_batch_vs_cpu_threads"] = (row["cpu_threads_burst_us"] /
                                                            gb[name]["gpu_batch_burst_us"])
    line["cpu_baseline"] = cpu
    leg("cleanup", R.drop_samples)
    if "dedup" in comps:
        d = leg("dedup", lambda: R.run_dedup(args.steps, args.warmup))
        if d:
            log("dedup:", json.dumps(d))
            comp["dedup"] = d
            if cpu is not None and getattr(R, "_cpu_dedup", None):
                cpu["config4_grouping"] = R._cpu_dedup
        R._cpu_dedup = None
        R.free()
    if "consumers" in comps:
        k = leg("consumers", lambda: R.run_consumers(args.steps, args.warmup))
        if k:
            log("consumers:", json.dumps(k))
            comp["consumers"] = k
        R.free()
    if "staged" in comps:
        g = leg("staged", R.run_staged)
        if g:
            log("staged:", json.dumps(g))
            comp["staged"] = g
        R.free()
        if g and getattr(R, "_staged_verify", None) is not None:
            v = leg("staged_oracle", R.staged_oracle)
            if v:
                log("staged_oracle:", json.dumps(v))
                g["verify_whole_run"] = v
        R._staged_verify = None
    if "checksum" in comps:
        k = leg("checksum", lambda: R.run_checksum(args.steps, args.warmup))
        if k:
            log("checksum:", json.dumps(k))
            comp["checksum"] = k
        R.free()
    line["world"] = R.world_info()  # after the legs: exchange volume of the run
    if c is None and "cas" not in comps:
        line["note"] = "--components without cas: profiling pass, no headline"
    walls["total"] = round(time.perf_counter() - t_begin, 2)
    writer.emit()
    leg("shutdown", R.shutdown)
    if "cas" in comps and line.get("value") is None:
        sys.exit(3)  # the headline step failed: the line says why


if __name__ == "__main__":
    main()
