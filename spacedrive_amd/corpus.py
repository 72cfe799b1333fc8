"""Synthetic corpora of the BASELINE.json shapes (bench / tests).

File contents are a pure function of (content seed, byte offset) -- see
DESIGN.md "Synthetic corpora" -- so the GPU generator (csrc/synth.hip) and the
CPU oracle produce identical bytes without materialising whole files: only the
cas windows of each file are ever built.
"""
from __future__ import annotations

import numpy as np

from .cas import MINIMUM_FILE_SIZE, SAMPLED_MSG_LEN

GiB = 1 << 30


def config2_files(n: int = 1_000_000, seed: int = 2, dup_frac: float = 0.20,
                  empty_frac: float = 0.001):
    """Config 2: sizes ~ round(exp(N(ln 65536, 2.0))) clipped to [1 B, 1 GiB],
    `empty_frac` forced to 0 bytes, `dup_frac` exact duplicates (the (size,
    content seed) of a uniformly chosen unique file).  Returns (sizes, seeds)
    as uint64 arrays in file_path id order."""
    rng = np.random.default_rng(seed)
    sizes = np.rint(np.exp(rng.normal(np.log(65536.0), 2.0, n))).astype(np.float64)
    sizes = np.clip(sizes, 1, GiB).astype(np.uint64)
    seeds = (rng.integers(0, 2**63 - 1, n, dtype=np.int64).astype(np.uint64)
             | np.uint64(1))
    n_dup = int(round(dup_frac * n))
    dup_rows = rng.choice(n, n_dup, replace=False)
    is_dup = np.zeros(n, bool)
    is_dup[dup_rows] = True
    uniq = np.flatnonzero(~is_dup)
    src = uniq[rng.integers(0, uniq.size, n_dup)]
    sizes[dup_rows] = sizes[src]
    seeds[dup_rows] = seeds[src]
    n_empty = int(round(empty_frac * n))
    if n_empty:
        sizes[rng.choice(n, n_empty, replace=False)] = 0
    return sizes, seeds


def boundary_sizes() -> list[int]:
    """File sizes around every boundary of generate_cas_id and BLAKE3."""
    return [0, 1, 55, 56, 57, 63, 64, 65, 1015, 1016, 1017, 1023, 1024, 1025, 2040, 2048,
            4096, 8192, 16384, 65536, 102391, 102392, 102399, 102400, 102401, 102402, 118784,
            131072, 1 << 20, (1 << 20) + 3, 10 * (1 << 20) + 7, (1 << 32) + 1]


def msg_lengths(sizes: np.ndarray) -> np.ndarray:
    sizes = np.asarray(sizes, np.uint64)
    return np.where(sizes <= MINIMUM_FILE_SIZE, sizes + 8, SAMPLED_MSG_LEN).astype(np.uint32)


def arena_layout(sizes: np.ndarray, align: int = 128):
    """(offsets uint64, lengths uint32, total bytes) of the packed cas arena
    (the same packing as oracle.synth_arena)."""
    ln = msg_lengths(sizes)
    padded = (ln.astype(np.uint64) + np.uint64(align - 1)) & ~np.uint64(align - 1)
    off = np.zeros(ln.size, np.uint64)
    if ln.size:
        np.cumsum(padded[:-1], out=off[1:])
    total = int(off[-1] + padded[-1]) if ln.size else 0
    return off, ln, total


def synth_arena_device(sizes: np.ndarray, seeds: np.ndarray, device=None, ctx=None):
    """Builds the cas-message arena of a synthetic corpus directly in HBM.
    Returns (arena, off, len) torch tensors on `device`."""
    import torch

    from ._native import check, default_context
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    ctx = ctx or default_context(dev.index)
    off, ln, total = arena_layout(sizes)
    arena = torch.empty(total + 128, dtype=torch.uint8, device=dev)
    d_sizes = torch.from_numpy(np.ascontiguousarray(sizes, np.uint64).view(np.int64)).to(dev)
    d_seeds = torch.from_numpy(np.ascontiguousarray(seeds, np.uint64).view(np.int64)).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_synth_cas_arena_device(ctx.h, d_sizes.data_ptr(), d_seeds.data_ptr(),
                                               d_off.data_ptr(), sizes.size, arena.data_ptr(), s),
          "sdgpu_synth_cas_arena_device")
    return arena, d_off, d_len


def synth_file_device(seed: int, length: int, device=None, out=None, ctx=None):
    """Whole synthetic file (content seed `seed`) of `length` bytes in HBM."""
    import torch

    from ._native import check, default_context
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    ctx = ctx or default_context(dev.index)
    if out is None:
        out = torch.empty(length, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_synth_file_device(ctx.h, seed, 0, length, out.data_ptr(), s),
          "sdgpu_synth_file_device")
    return out


def synth_dedup_rows_device(seed: int, total_rows: int, distinct: int, first: int, n: int,
                            device=None, ctx=None):
    """Rows [first, first+n) of the config-4 dedup table: (key int64 [u64 bits],
    has_key uint8, rank int32 [u32 bits]) on `device`."""
    import torch

    from ._native import check, default_context
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    ctx = ctx or default_context(dev.index)
    key = torch.empty(n, dtype=torch.int64, device=dev)
    has = torch.empty(n, dtype=torch.uint8, device=dev)
    rank = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_synth_dedup_rows_device(ctx.h, seed, total_rows, distinct, first, n,
                                                key.data_ptr(), has.data_ptr(), rank.data_ptr(),
                                                s), "sdgpu_synth_dedup_rows_device")
    return key, has, rank


def config1_sizes(n: int = 10_000, seed: int = 1) -> np.ndarray:
    """Config 1: sizes log-uniform in [1 KiB, 10 MiB] (seed 1)."""
    rng = np.random.default_rng(seed)
    return np.rint(np.exp(rng.uniform(np.log(1024.0), np.log(10.0 * (1 << 20)), n))).astype(
        np.uint64)


def write_config1_dir(root: str, n: int = 10_000, seed: int = 1) -> tuple[list[str], np.ndarray]:
    """Writes BASELINE config 1 (a synthetic n-file directory, mixed 1 KiB-10 MiB)
    under `root`.  Files are SPARSE: only the bytes generate_cas_id reads
    (cas.rs:27-58: the whole file up to 100 KiB, else header, the 4 samples and
    the footer) hold random data; the rest is a hole (ftruncate), so 10 k files
    cost ~0.4 GB of disk.  Returns (paths, sizes)."""
    import os
    sizes = config1_sizes(n, seed)
    rng = np.random.default_rng(seed + 1)
    os.makedirs(root, exist_ok=True)
    paths = []
    hf, ss = 8192, 10240
    for i, sz in enumerate(sizes.tolist()):
        p = os.path.join(root, f"f{i:05d}.bin")
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            if sz <= 100 * 1024:
                os.pwrite(fd, rng.integers(0, 256, sz, dtype=np.uint8).tobytes(), 0)
            else:
                jump = (sz - 2 * hf) // 4
                spans = [(0, hf)] + [(hf + k * jump, ss) for k in range(4)] + [(sz - hf, hf)]
                for o, ln in spans:
                    os.pwrite(fd, rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), o)
                os.ftruncate(fd, sz)
        finally:
            os.close(fd)
        paths.append(p)
    return paths, sizes


def config5_vary_mask(sizes: np.ndarray, seeds: np.ndarray, frac16: int = 13) -> np.ndarray:
    """Rows of the config-5 pool that stand for NEW files in every step of a
    run (frac16/16 of the content seeds, ~81 %; duplicates share a seed, so they
    stay duplicates); the rest are the same files in every step.  Empty files
    have no key."""
    sel = ((np.asarray(seeds, np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(60)) < frac16
    return (sel & (np.asarray(sizes) != 0)).astype(np.uint8)


def vary_keys_device(key, vary, step: int, ctx=None):
    """In place: the cas keys of step `step` of a config-5 run
    (sdgpu_synth_vary_keys_device)."""
    import torch
    from ._native import check, default_context
    ctx = ctx or default_context(key.device.index)
    s = torch.cuda.current_stream(key.device).cuda_stream
    check(ctx.lib.sdgpu_synth_vary_keys_device(ctx.h, key.data_ptr(), vary.data_ptr(),
                                               key.numel(), step, s),
          "sdgpu_synth_vary_keys_device")
