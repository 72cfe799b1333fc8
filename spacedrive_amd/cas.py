"""cas_id generation -- host mirror of core/src/object/cas.rs over libsdgpu.

Same names, argument meaning and error behaviour as the reference:

* ``generate_cas_id(path, size) -> str``      (cas.rs:23-62): 16 lowercase hex
  chars; raises OSError (io::Error) on open/read/seek failures, e.g. ENODATA for
  read_exact's UnexpectedEof on a file shorter than its samples.
* constants SAMPLE_COUNT / SAMPLE_SIZE / HEADER_OR_FOOTER_SIZE /
  MINIMUM_FILE_SIZE (cas.rs:10-15).

Batched entry points (what file_identifier uses): ``cas_batch`` over a host
arena of cas messages and ``cas_batch_device`` over device tensors.  All
hashing happens in the K1 HIP kernel (spacedrive_amd/csrc/b3_batch.hip).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._native import SdgpuError, check, default_context, load

SAMPLE_COUNT = 4                  # cas.rs:10
SAMPLE_SIZE = 1024 * 10           # cas.rs:11
HEADER_OR_FOOTER_SIZE = 1024 * 8  # cas.rs:12
MINIMUM_FILE_SIZE = 1024 * 100    # cas.rs:15
MAX_MSG_LEN = 8 + MINIMUM_FILE_SIZE
SAMPLED_MSG_LEN = 8 + 2 * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE  # 57352


def cas_message_len(size: int) -> int:
    """Length of the bytes generate_cas_id feeds BLAKE3 for a consistent file."""
    return 8 + size if size <= MINIMUM_FILE_SIZE else SAMPLED_MSG_LEN


def sample_offsets(size: int) -> list[int]:
    """File offsets of the 4 samples (cas.rs:41-51)."""
    jump = (size - HEADER_OR_FOOTER_SIZE * 2) // SAMPLE_COUNT
    return [HEADER_OR_FOOTER_SIZE + k * jump for k in range(SAMPLE_COUNT)]


def generate_cas_id(path, size: int, ctx=None) -> str:
    """Drop-in for `generate_cas_id(path, size)` (cas.rs:23)."""
    ctx = ctx or default_context()
    out = ctypes.create_string_buffer(17)
    p = os.fsencode(os.fspath(path))
    rc = ctx.lib.sdgpu_generate_cas_id(ctx.h, p, int(size), out)
    if rc:
        raise SdgpuError(rc, os.fspath(path))
    return out.value.decode()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def cas_batch(arena: np.ndarray, off: np.ndarray, length: np.ndarray, ctx=None):
    """cas ids (n x 8 bytes) + per-message status for a HOST arena of messages."""
    ctx = ctx or default_context()
    arena = np.ascontiguousarray(arena, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    n = off.size
    out = np.zeros((n, 8), np.uint8)
    status = np.zeros(n, np.int32)
    check(ctx.lib.sdgpu_cas_batch(ctx.h, _ptr(arena), _ptr(off), _ptr(length), n, _ptr(out),
                                  _ptr(status)), "sdgpu_cas_batch")
    return out, status


def cas_batch_device(arena, off, length, out=None, status=None, ctx=None, stream=None):
    """K1 over device tensors (torch): arena uint8, off int64, length int32.

    Returns (out[n,8] uint8, status[n] int32) on the same device; asynchronous
    on `stream` (default: torch's current stream)."""
    import torch
    ctx = ctx or default_context(arena.device.index)
    n = off.numel()
    if out is None:
        out = torch.empty((n, 8), dtype=torch.uint8, device=arena.device)
    if status is None:
        status = torch.empty(n, dtype=torch.int32, device=arena.device)
    s = stream if stream is not None else torch.cuda.current_stream(arena.device).cuda_stream
    check(ctx.lib.sdgpu_cas_batch_device(ctx.h, arena.data_ptr(), arena.numel(), off.data_ptr(),
                                         length.data_ptr(), n, out.data_ptr(), status.data_ptr(),
                                         s), "sdgpu_cas_batch_device")
    return out, status


def cas_stage_pinned(h_arena, off, length, out=None, status=None, ctx=None, device=None,
                     stream=None):
    """K1 over messages in PINNED host memory (torch pinned uint8 tensor), in
    file order, streamed H2D through device slabs overlapped with hashing
    (sdgpu_cas_stage_pinned).  Returns device (out[n,8] uint8, status[n] int32);
    asynchronous on `stream` -- keep h_arena alive until it has completed."""
    import torch
    if not h_arena.is_pinned():
        raise ValueError("h_arena must be pinned host memory (pin_memory=True)")
    dev = torch.device("cuda", device if device is not None else torch.cuda.current_device())
    ctx = ctx or default_context(dev.index)
    off = np.ascontiguousarray(off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    n = off.size
    if out is None:
        out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    if status is None:
        status = torch.empty(n, dtype=torch.int32, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_cas_stage_pinned(ctx.h, h_arena.data_ptr(), _ptr(off), _ptr(length), n,
                                         out.data_ptr(), status.data_ptr(), s),
          "sdgpu_cas_stage_pinned")
    return out, status


def hex_ids(out8: np.ndarray) -> list[str]:
    """`to_hex()[..16]` of each 8-byte cas digest prefix (cas.rs:61)."""
    return [bytes(r).hex() for r in np.asarray(out8, np.uint8).reshape(-1, 8)]


def keys_of(out8) -> np.ndarray:
    """8 digest bytes as little-endian u64 grouping keys."""
    return np.ascontiguousarray(out8, np.uint8).reshape(-1, 8).view("<u8").reshape(-1)


class Coalescer:
    """Concurrent single-file ``generate_cas_id`` calls coalesced into batches
    (host mirror of crates/sd-core-gpu/src/burst.rs).

    The watcher (location/manager/watcher/utils.rs:236,411,467) and the
    non-indexed listing (location/non_indexed.rs:161) call generate_cas_id
    once per file; when many arrive together (a folder copied into a watched
    location) the calls queued while the worker is busy leave as ONE
    ``sdgpu_identify_files`` batch (the library's read pool + one K1 launch).
    A lone call goes through the resident latency service (the Rust host
    hashes a lone small file on the CPU with the reference's own blake3 crate
    instead; there is no CPU hasher in this package).  No timer: the worker
    drains what is queued when it looks, so a lone call never waits."""

    def __init__(self, ctx=None, batch_from: int = 4, batch_max: int = 1024):
        import queue
        import threading
        self.ctx = ctx or default_context()
        self.batch_from, self.batch_max = batch_from, batch_max
        self.q = queue.Queue()
        self.stats = {"calls": 0, "batches": 0, "batched_calls": 0, "single": 0}
        self._t = threading.Thread(target=self._worker, name="sd-gpu-cas", daemon=True)
        self._t.start()

    def cas_id(self, path, size: int) -> str:
        """generate_cas_id(path, size) (cas.rs:23) through the worker; blocks."""
        import concurrent.futures as cf
        fut = cf.Future()
        self.q.put((os.fspath(path), int(size), fut))
        return fut.result()

    def close(self):
        self.q.put(None)
        self._t.join(timeout=10)

    def _worker(self):
        import queue
        from .file_identifier import identify
        while True:
            first = self.q.get()
            if first is None:
                return
            group = [first]
            while len(group) < self.batch_max:
                try:
                    r = self.q.get_nowait()
                except queue.Empty:
                    break
                if r is None:
                    self.q.put(None)
                    break
                group.append(r)
            self.stats["calls"] += len(group)
            if len(group) >= self.batch_from:
                self.stats["batches"] += 1
                self.stats["batched_calls"] += len(group)
                try:
                    res = identify([p for p, _, _ in group],
                                   np.array([s for _, s, _ in group], np.uint64), ctx=self.ctx)
                except Exception as e:  # noqa: BLE001 -- every caller sees it
                    for _, _, fut in group:
                        fut.set_exception(e)
                    continue
                for i, (p, s, fut) in enumerate(group):
                    if res.status[i] != 0:
                        fut.set_exception(SdgpuError(int(res.status[i]), p))
                    elif s == 0:  # identify treats size 0 as "no cas_id"; the drop-in hashes 8 zeros
                        self._single(p, s, fut)
                    else:
                        fut.set_result(bytes(res.cas8[i]).hex())
                continue
            for p, s, fut in group:
                self.stats["single"] += 1
                self._single(p, s, fut)

    def _single(self, p, s, fut):
        try:
            self.ctx.latency_service(True)
            fut.set_result(generate_cas_id(p, s, self.ctx))
        except Exception as e:  # noqa: BLE001
            fut.set_exception(e)
