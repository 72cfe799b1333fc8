"""File identifier -- host mirror of core/src/object/file_identifier/mod.rs.

* ``FileMetadata`` / ``file_metadata(location_path, iso_path)``  (mod.rs:50-97):
  stat, refuse directories, cas_id None for empty files, else generate_cas_id.
  (`kind` -- sd-file-ext magic-byte sniffing, mod.rs:75-78 -- is outside the
  hot path and stays ObjectKind::Unknown = 0 here.)
* ``identify(paths)``: the batched form of identifier_job_step's metadata
  phase (mod.rs:107-134) -- every file's cas windows are pread into pinned
  slabs and hashed by K1 while the next slab is read (sdgpu_identify_files).
* ``identifier_job(paths)``: the whole job over orphan rows in id order --
  cas ids, then the Object grouping of every row (dedup.group_reps), with the
  reference's per-step (created, linked) accounting.
"""
from __future__ import annotations

import ctypes
import os
import stat as _stat
from dataclasses import dataclass

import numpy as np

from . import cas as _cas
from . import dedup as _dedup
from ._native import SdgpuError, check, default_context

CHUNK_SIZE = 100  # mod.rs:36


@dataclass
class FileMetadata:
    cas_id: str | None
    kind: int
    size: int


def file_metadata(location_path, iso_file_path, ctx=None) -> FileMetadata:
    """FileMetadata::new (mod.rs:59-97)."""
    path = os.path.join(os.fspath(location_path), os.fspath(iso_file_path))
    st = os.stat(path)
    assert not _stat.S_ISDIR(st.st_mode), "We can't generate cas_id for directories"
    cas_id = _cas.generate_cas_id(path, st.st_size, ctx) if st.st_size != 0 else None
    return FileMetadata(cas_id=cas_id, kind=0, size=st.st_size)


@dataclass
class IdentifyResult:
    cas8: np.ndarray      # [n, 8] uint8 (zeros where has_key == 0)
    has_key: np.ndarray   # [n] uint8: 1 = cas_id present
    status: np.ndarray    # [n] int32: 0 or -errno (row dropped, mod.rs:113,127)
    sizes: np.ndarray     # [n] uint64 (fs::metadata len, mod.rs:65)

    def cas_ids(self) -> list[str | None]:
        return [bytes(self.cas8[i]).hex() if self.has_key[i] else None
                for i in range(self.has_key.size)]


def identify(paths, sizes=None, ctx=None) -> IdentifyResult:
    """cas ids of many files in one pipelined call."""
    ctx = ctx or default_context()
    n = len(paths)
    st = np.zeros(n, np.int32)
    if sizes is None:
        sizes = np.zeros(n, np.uint64)
        for i, p in enumerate(paths):
            try:
                sizes[i] = os.stat(p).st_size
            except OSError as e:
                st[i] = -e.errno
    sizes = np.ascontiguousarray(sizes, np.uint64)
    enc = [os.fsencode(os.fspath(p)) for p in paths]
    arr = (ctypes.c_char_p * n)(*enc)
    out = np.zeros((n, 8), np.uint8)
    has = np.zeros(n, np.uint8)
    status = np.zeros(n, np.int32)
    check(ctx.lib.sdgpu_identify_files(ctx.h, arr, sizes.ctypes.data, n, out.ctypes.data,
                                       has.ctypes.data, status.ctypes.data),
          "sdgpu_identify_files")
    failed_stat = st != 0
    status[failed_stat] = st[failed_stat]
    has[failed_stat] = 0
    return IdentifyResult(out, has, status, sizes)


@dataclass
class JobResult:
    identify: IdentifyResult
    rep: np.ndarray       # [n] uint32: rank of the row whose Object each row joins
    created: int
    linked: int


def identifier_job(paths, chunk_size: int = CHUNK_SIZE, ctx=None) -> JobResult:
    """FileIdentifierJob over orphan rows given in ascending file_path.id order."""
    ident = identify(paths, ctx=ctx)
    ok = ident.status == 0
    key = _cas.keys_of(ident.cas8)
    # rows whose metadata failed are not grouped (they stay orphans)
    rep = _dedup.group_reps(key, ident.has_key & ok.astype(np.uint8), chunk_size, ctx)
    created, linked = _dedup.object_stats(rep, ident.has_key, ok)
    return JobResult(ident, rep, created, linked)


__all__ = ["FileMetadata", "file_metadata", "identify", "identifier_job", "IdentifyResult",
           "JobResult", "SdgpuError"]
