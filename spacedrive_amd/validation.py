"""Object validator checksum -- host mirror of core/src/object/validation/hash.rs.

* ``file_checksum(path) -> str`` (hash.rs:10-24): 64 lowercase hex chars of the
  full-file BLAKE3; raises OSError like the reference's io::Error.
  The file is streamed in 64 MiB power-of-two slices (64 of the reference's
  1 MiB BLOCK_LEN reads) through double-buffered pinned memory; every slice is
  hashed by the tree kernels K2/K3 (csrc/b3_tree.hip) and the slice chaining
  values are folded on the GPU.
* ``checksum_bytes(buf)``, ``checksum_batch_device(tensors)`` for in-memory and
  device-resident data (the object-validator bench, BASELINE config 3).
* ``checksum_files(paths)`` / ``validator_job(paths)``: the object validator
  job (core/src/object/validation/validator_job.rs:35-171) over many rows at
  once -- small files are read whole into pinned slabs and hashed one tree
  launch per slab (sdgpu_checksum_files) instead of one file per job step.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._native import SdgpuError, check, default_context

BLOCK_LEN = 1048576  # hash.rs:8


def file_checksum(path, ctx=None) -> str:
    """Drop-in for `file_checksum(path)` (hash.rs:10)."""
    ctx = ctx or default_context()
    out = ctypes.create_string_buffer(65)
    rc = ctx.lib.sdgpu_file_checksum(ctx.h, os.fsencode(os.fspath(path)), out)
    if rc:
        raise SdgpuError(rc, os.fspath(path))
    return out.value.decode()


def checksum_files(paths, ctx=None):
    """(digests [n, 32] uint8, status [n] int32) of many files in one call."""
    ctx = ctx or default_context()
    n = len(paths)
    enc = [os.fsencode(os.fspath(p)) for p in paths]
    arr = (ctypes.c_char_p * max(n, 1))(*enc)
    out = np.zeros((n, 32), np.uint8)
    status = np.zeros(n, np.int32)
    check(ctx.lib.sdgpu_checksum_files(ctx.h, arr, n, out.ctypes.data, status.ctypes.data),
          "sdgpu_checksum_files")
    return out, status


def validator_job(paths, ctx=None):
    """ObjectValidatorJob (validator_job.rs:126-169) over the rows whose
    integrity_checksum is NULL: {path: checksum hex} for the rows written;
    like the reference, the first I/O error fails the job (FileIOError)."""
    out, status = checksum_files(paths, ctx)
    for i, p in enumerate(paths):
        if status[i]:
            raise SdgpuError(int(status[i]), os.fspath(p))
    return {os.fspath(p): bytes(out[i]).hex() for i, p in enumerate(paths)}


def checksum_bytes(data, ctx=None) -> bytes:
    """BLAKE3 digest (32 bytes) of a host buffer, computed on the GPU."""
    ctx = ctx or default_context()
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
        np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    out = np.zeros(32, np.uint8)
    check(ctx.lib.sdgpu_checksum(ctx.h, a.ctypes.data if a.size else None, a.size, out.ctypes.data),
          "sdgpu_checksum")
    return out.tobytes()


def checksum_batch_device(files, out=None, ctx=None, stream=None):
    """Digests of device-resident files (list of 1-D uint8 torch tensors,
    16-byte aligned) -> uint8 tensor [n, 32]; asynchronous on `stream`."""
    import torch
    n = len(files)
    dev = files[0].device
    ctx = ctx or default_context(dev.index)
    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    ptrs = (ctypes.c_uint64 * n)(*[f.data_ptr() for f in files])
    lens = (ctypes.c_uint64 * n)(*[f.numel() for f in files])
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_checksum_batch_device(ctx.h, ptrs, lens, n, out.data_ptr(), s),
          "sdgpu_checksum_batch_device")
    return out


def subtree_device(data, chunk_offset: int, root: bool, out=None, ctx=None, stream=None):
    """Chaining value (root=False) or digest (root=True) of an aligned slice."""
    import torch
    ctx = ctx or default_context(data.device.index)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=data.device)
    s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
    check(ctx.lib.sdgpu_subtree_device(ctx.h, data.data_ptr(), data.numel(), int(chunk_offset),
                                       1 if root else 0, out.data_ptr(), s),
          "sdgpu_subtree_device")
    return out


def combine_subtrees_device(cvs, out=None, ctx=None, stream=None):
    """Digest of a message from the [n, 32] chaining values of its consecutive
    aligned subtree slices (sdgpu_combine_subtrees_device): the last step of a
    file checksummed slice by slice on several GPUs."""
    import torch
    ctx = ctx or default_context(cvs.device.index)
    cvs = cvs.contiguous()
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=cvs.device)
    s = stream if stream is not None else torch.cuda.current_stream(cvs.device).cuda_stream
    check(ctx.lib.sdgpu_combine_subtrees_device(ctx.h, cvs.data_ptr(), cvs.shape[0],
                                                out.data_ptr(), s),
          "sdgpu_combine_subtrees_device")
    return out
