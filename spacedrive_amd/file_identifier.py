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
* ``FileIdentifierJob`` / ``shallow``: the resumable job
  (file_identifier_job.rs:32-309) and the light-scan variant (shallow.rs:26-119)
  over a ``FilePaths`` table: orphan rows fetched in ascending id with the
  reference's cursor (``id >= cursor``, cursor = last fetched id), grouped
  against a device Object index so that steps of many chunks give the same
  Objects as the reference's 100-row steps; pause/resume through a JSON state.
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
    sizes: np.ndarray | None  # [n] uint64 as passed; None: stat-ed by the library

    def cas_ids(self) -> list[str | None]:
        return [bytes(self.cas8[i]).hex() if self.has_key[i] else None
                for i in range(self.has_key.size)]


class PathList:
    """A list of paths encoded once as the C ABI's `const char *const *` (a
    host that identifies the same listing repeatedly -- the bench, a rescan --
    pays the encoding once; a Rust host passes its CString pointers directly)."""

    def __init__(self, paths):
        self.paths = list(paths)
        self._enc = [os.fsencode(os.fspath(p)) for p in self.paths]
        self.c_paths = (ctypes.c_char_p * len(self._enc))(*self._enc)

    def __len__(self):
        return len(self.paths)

    def __iter__(self):
        return iter(self.paths)

    def __getitem__(self, i):
        return self.paths[i]


def identify(paths, sizes=None, ctx=None) -> IdentifyResult:
    """cas ids of many files in one pipelined call (paths: a sequence of
    paths, or a PathList)."""
    ctx = ctx or default_context()
    n = len(paths)
    # sizes None: the library stats every path in its read pool (the
    # reference's fresh fs::metadata(path).len(), mod.rs:65,80-81; a failed
    # stat is status -errno, the row dropped)
    if sizes is not None:
        sizes = np.ascontiguousarray(sizes, np.uint64)
    arr = paths.c_paths if isinstance(paths, PathList) else PathList(paths).c_paths
    out = np.zeros((n, 8), np.uint8)
    has = np.zeros(n, np.uint8)
    status = np.zeros(n, np.int32)
    check(ctx.lib.sdgpu_identify_files(ctx.h, arr, sizes.ctypes.data if sizes is not None else None,
                                       n, out.ctypes.data, has.ctypes.data, status.ctypes.data),
          "sdgpu_identify_files")
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


# ---------------------------------------------------------------------------
# The resumable identifier job and the shallow (light-scan) identifier
# ---------------------------------------------------------------------------

class FilePaths:
    """The file_path rows the identifier reads and writes: the columns of
    file_path_for_file_identifier (core/src/location/file_path_helper/mod.rs:32-40)
    plus cas_id and object_id (core/prisma/schema.prisma:154-201).  An in-memory
    stand-in for the library's table -- the prisma/SQLite store is out of scope
    (SURVEY §2); the job only needs these queries and writes."""

    def __init__(self):
        self.location_id: list[int] = []
        self.materialized_path: list[str] = []   # "/a/b/" for a child of /a/b
        self.name: list[str] = []
        self.is_dir: list[bool] = []
        self.cas_id: list[str | None] = []
        self.object_id: list[int | None] = []
        self.next_object_id = 1
        # per location, the ids of its non-directory rows (ascending: ids are
        # appended in order) -- the index the orphan query walks from the cursor
        self._file_rows: dict[int, list[int]] = {}

    def add(self, location_id: int, materialized_path: str, name: str,
            is_dir: bool = False) -> int:
        """Appends a row; its file_path.id is its index + 1 (ascending ids)."""
        self.location_id.append(location_id)
        self.materialized_path.append(materialized_path)
        self.name.append(name)
        self.is_dir.append(is_dir)
        self.cas_id.append(None)
        self.object_id.append(None)
        fid = len(self.name)
        if not is_dir:
            self._file_rows.setdefault(location_id, []).append(fid)
        return fid

    def __len__(self):
        return len(self.name)

    def rel_path(self, fid: int) -> str:
        i = fid - 1
        return self.materialized_path[i].lstrip("/") + self.name[i]

    def orphans(self, location_id: int, cursor: int | None = None,
                children_of: str | None = None, under: str | None = None,
                limit: int | None = None) -> list[int]:
        """ids of orphan rows in ascending id (orphan_path_filters,
        file_identifier_job.rs:245-268 / shallow.rs:121-139): object_id NULL,
        !is_dir, the location, id >= cursor, and either a subtree
        (materialized_path starts with `under`) or one directory's children;
        at most `limit` of them (the query's LIMIT, :286-309).  Walks the
        location's file rows from the cursor (bisect), so a job step costs
        about its own rows, not a scan of the table."""
        import bisect
        rows = self._file_rows.get(location_id, [])
        out = []
        for j in range(bisect.bisect_left(rows, max(1, cursor or 1)), len(rows)):
            fid = rows[j]
            i = fid - 1
            if self.object_id[i] is not None:
                continue
            mp = self.materialized_path[i]
            if children_of is not None and mp != children_of:
                continue
            if under is not None and not mp.startswith(under):
                continue
            out.append(fid)
            if limit is not None and len(out) >= limit:
                break
        return out

    def count_orphans(self, location_id: int, children_of: str | None = None,
                      under: str | None = None) -> int:
        """count_orphan_file_paths (file_identifier_job.rs:270-284): a count,
        no rows returned."""
        rows = self._file_rows.get(location_id, [])
        n = 0
        for fid in rows:
            i = fid - 1
            if self.object_id[i] is not None:
                continue
            mp = self.materialized_path[i]
            if (children_of is not None and mp != children_of) or \
                    (under is not None and not mp.startswith(under)):
                continue
            n += 1
        return n

    def first_orphan(self, location_id: int, children_of: str | None = None,
                     under: str | None = None) -> int | None:
        """find_first(orphan_path_filters(.., None, ..)) selecting the id
        (file_identifier_job.rs:140-151)."""
        first = self.orphans(location_id, None, children_of, under, limit=1)
        return first[0] if first else None

    def existing_objects_page(self, after: int | None = None, limit: int = 1 << 20):
        """(ids, keys, object ids) of the rows linked to an Object and carrying
        a cas_id, library-wide (what mod.rs:168-175's find_many can return),
        id > after in ascending id, at most `limit`: the Object index is
        filled page by page, never from one materialised table."""
        from .cas import keys_of
        ids, keys, objs = [], [], []
        for i in range(after or 0, len(self.name)):
            c, o = self.cas_id[i], self.object_id[i]
            if c is not None and o is not None:
                ids.append(i + 1)
                keys.append(bytes.fromhex(c))
                objs.append(o)
                if len(ids) >= limit:
                    break
        if not keys:
            return np.zeros(0, np.int64), np.zeros(0, np.uint64), np.zeros(0, np.uint32)
        k = keys_of(np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 8))
        return np.asarray(ids, np.int64), k, np.asarray(objs, np.uint32)

    def existing_objects(self):
        """(key, object id) of every row linked to an Object (all pages)."""
        ks, os_ = [], []
        after = None
        while True:
            ids, k, o = self.existing_objects_page(after)
            if not ids.size:
                break
            ks.append(k)
            os_.append(o)
            after = int(ids[-1])
        if not ks:
            return np.zeros(0, np.uint64), np.zeros(0, np.uint32)
        return np.concatenate(ks), np.concatenate(os_)


@dataclass
class IdentifierRunMetadata:
    """FileIdentifierJobRunMetadata (file_identifier_job.rs:53-68)."""
    cursor: int = 0
    total_orphan_paths: int = 0
    total_objects_created: int = 0
    total_objects_linked: int = 0
    total_objects_ignored: int = 0


class FileIdentifierJob:
    """FileIdentifierJobInit (file_identifier_job.rs:72-243) over a FilePaths
    table, run on the GPU.

    init: counts the orphans (early finish if none, :130-136), task_count =
    ceil(n / 100) steps of CHUNK_SIZE rows, cursor = first orphan id (:140-170).
    A reference step fetches the next 100 orphans with id >= cursor in id order
    (:286-309), identifies and groups them (mod.rs:100-336) and sets the cursor
    to the last fetched id (mod.rs:384-392).  Here one execute_step runs
    `chunks_per_step` such steps as ONE GPU batch: the chunk boundaries are
    replayed exactly (a failed last row is fetched again by the next chunk, as
    the `id >= cursor` query does), every fetched row gets rank = step * 100 +
    position, and the grouping runs against a device Object index holding the
    library's existing Objects and this run's creators -- so the Objects are
    the reference's whatever the step size.  state() / resume() persist the
    cursor and counters (the JobState of job/mod.rs:701-720); a resumed job
    re-registers the Objects already in the table."""

    def __init__(self, table: FilePaths, location_id: int, location_path: str,
                 sub_path: str | None = None, chunks_per_step: int = 64, ctx=None,
                 _shallow_dir: str | None = None):
        self.table = table
        self.location_id = location_id
        self.location_path = location_path
        self.sub_path = sub_path
        self.chunks_per_step = max(1, int(chunks_per_step))
        self.ctx = ctx or default_context()
        self._children_of = _shallow_dir
        self._under = None
        if sub_path:
            sp = "/" + sub_path.strip("/") + "/"
            self._under = sp
        self.meta = IdentifierRunMetadata()
        self.step_number = 0      # reference steps (chunks of 100) done
        self.task_count = 0
        self._creator_object: dict[int, int] = {}  # rank -> Object id (this run)
        self.index = None

    # ---- reference: init (file_identifier_job.rs:80-172) -------------------------
    def init(self) -> "FileIdentifierJob":
        # a count and a find_first (file_identifier_job.rs:120-156), not the rows
        count = self.table.count_orphans(self.location_id, self._children_of, self._under)
        if count == 0:
            raise EarlyFinish("Found no orphan file paths to process")
        first = self.table.first_orphan(self.location_id, self._children_of, self._under)
        self.meta = IdentifierRunMetadata(cursor=first, total_orphan_paths=count)
        self.task_count = -(-count // CHUNK_SIZE)
        self._open_index()
        return self

    def _orphans(self, cursor, limit=None):
        return self.table.orphans(self.location_id, cursor, self._children_of, self._under, limit)

    def _open_index(self, page: int = 1 << 20):
        """The library's existing Objects into the device index, page by page
        (the index grows as it fills)."""
        import torch
        self.index = _dedup.ObjectIndex(self.ctx, max(1024, 2 * self.meta.total_orphan_paths))
        dev = torch.device("cuda", self.ctx.device)
        after = None
        while True:
            ids, ek, eh = self.table.existing_objects_page(after, page)
            if not ids.size:
                break
            # copies: the views may be read-only (torch.from_numpy warns on them)
            self.index.add_objects(torch.from_numpy(ek.view(np.int64).copy()).to(dev),
                                   torch.from_numpy(eh.view(np.int32).copy()).to(dev))
            if ids.size < page:
                break
            after = int(ids[-1])

    def done(self) -> bool:
        return self.step_number >= self.task_count

    # ---- reference: execute_step, chunks_per_step of them at once -----------------
    def execute_step(self) -> IdentifierRunMetadata:
        if self.done():
            return self.meta
        nchunks = min(self.chunks_per_step, self.task_count - self.step_number)
        cand = self._orphans(self.meta.cursor, nchunks * CHUNK_SIZE + nchunks)
        if not cand:
            raise EarlyFinish("Expected orphan Paths not returned from database query for this chunk")
        paths = [os.path.join(self.location_path, self.table.rel_path(f)) for f in cand]
        ident = identify(paths, ctx=self.ctx)
        ok = {f: ident.status[i] == 0 for i, f in enumerate(cand)}
        pos = {f: i for i, f in enumerate(cand)}
        # replay the reference's fetches: chunk c = the next 100 orphans with
        # id >= cursor (a failed last row stays orphan and is fetched again)
        fetched, cursor = [], self.meta.cursor
        for _ in range(nchunks):
            chunk = []
            for f in cand:
                if f < cursor or (fetched and f == cursor and ok[f]):
                    continue  # below the cursor, or identified by the previous chunk
                chunk.append(f)
                if len(chunk) == CHUNK_SIZE:
                    break
            if not chunk:
                break
            fetched.append(chunk)
            cursor = chunk[-1]
        rows = [f for ch in fetched for f in ch]
        first_rank = self.step_number * CHUNK_SIZE
        key = np.zeros(len(rows), np.uint64)
        has = np.zeros(len(rows), np.uint8)
        valid = np.zeros(len(rows), bool)
        keys8 = _cas.keys_of(ident.cas8)
        for j, f in enumerate(rows):
            i = pos[f]
            valid[j] = ok[f]
            has[j] = ident.has_key[i] if ok[f] else 0
            key[j] = keys8[i]
        rep = _dedup.dedup_batch(key, has, first_rank, self.index, CHUNK_SIZE, self.ctx)
        created = linked = 0
        t = self.table
        for j, f in enumerate(rows):  # the write set, in rank order (mod.rs:144-333)
            if not valid[j]:
                continue
            i = f - 1
            t.cas_id[i] = bytes(ident.cas8[pos[f]]).hex() if has[j] else None
            r = first_rank + j
            if rep[j] == r:
                obj = t.next_object_id
                t.next_object_id += 1
                self._creator_object[r] = obj
                created += 1
            elif rep[j] & _dedup.REP_EXISTING:
                obj = int(rep[j] & 0x7FFFFFFF)
                linked += 1
            else:
                obj = self._creator_object[int(rep[j])]
                linked += 1
            t.object_id[i] = obj
        self.step_number += len(fetched)
        self.meta.cursor = cursor
        self.meta.total_objects_created += created
        self.meta.total_objects_linked += linked
        self.meta.total_objects_ignored += int((~valid).sum())
        return self.meta

    def run(self, max_steps: int | None = None) -> IdentifierRunMetadata:
        k = 0
        while not self.done() and (max_steps is None or k < max_steps):
            self.execute_step()
            k += 1
        return self.meta

    # ---- pause / resume (job/mod.rs:701-720, cold_resume job/manager.rs:269-320) ---
    def state(self) -> dict:
        from dataclasses import asdict
        return {"location_id": self.location_id, "location_path": self.location_path,
                "sub_path": self.sub_path, "shallow_dir": self._children_of,
                "chunks_per_step": self.chunks_per_step, "step_number": self.step_number,
                "task_count": self.task_count, "run_metadata": asdict(self.meta)}

    @classmethod
    def resume(cls, table: FilePaths, state: dict, ctx=None) -> "FileIdentifierJob":
        job = cls(table, state["location_id"], state["location_path"], state["sub_path"],
                  state["chunks_per_step"], ctx, state.get("shallow_dir"))
        job.meta = IdentifierRunMetadata(**state["run_metadata"])
        job.step_number = state["step_number"]
        job.task_count = state["task_count"]
        job._open_index()  # this run's earlier Objects are existing Objects now
        return job

    def close(self):
        if self.index is not None:
            self.index.close()
            self.index = None


class EarlyFinish(Exception):
    """JobError::EarlyFinish (file_identifier_job.rs:131-136, 197-203)."""


def shallow(table: FilePaths, location_id: int, location_path: str, sub_path: str = "",
            chunks_per_step: int = 64, ctx=None) -> IdentifierRunMetadata:
    """file_identifier::shallow (shallow.rs:26-119): the light scan of one
    directory -- only its direct children (materialized_path equal to the
    directory's children path, :121-139), all steps at once, outside the job
    system; no orphans is not an error (:65-67)."""
    d = "/" + sub_path.strip("/") + "/" if sub_path.strip("/") else "/"
    job = FileIdentifierJob(table, location_id, location_path, None, chunks_per_step, ctx,
                            _shallow_dir=d)
    try:
        job.init()
    except EarlyFinish:
        return IdentifierRunMetadata()
    try:
        return job.run()
    finally:
        job.close()


__all__ = ["FileMetadata", "file_metadata", "identify", "identifier_job", "IdentifyResult",
           "JobResult", "SdgpuError", "FilePaths", "FileIdentifierJob", "IdentifierRunMetadata",
           "EarlyFinish", "shallow"]
