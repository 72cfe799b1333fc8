"""ctypes wrapper of the C oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (spacedrive_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "sd_oracle.c"))):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_blake3.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_blake3_mt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.orc_blake3_incremental.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                             ctypes.c_void_p]
        L.orc_blake3_derive_key.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_void_p]
        L.orc_blake3_keyed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p]
        L.orc_cas_msg_len.argtypes = [ctypes.c_uint64]
        L.orc_cas_msg_len.restype = ctypes.c_uint32
        L.orc_cas_build_message.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_void_p]
        L.orc_cas_build_message.restype = ctypes.c_int64
        L.orc_cas_id_of_message.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_cas_id_path.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.orc_cas_id_path.restype = ctypes.c_int
        L.orc_file_checksum_path.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.orc_file_checksum_path.restype = ctypes.c_int
        L.orc_cas_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        L.orc_cas_batch_simd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        L.orc_synth_file_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_void_p]
        L.orc_synth_cas_message.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.orc_synth_cas_message.restype = ctypes.c_uint32
        L.orc_synth_arena_layout.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_void_p]
        L.orc_synth_arena_layout.restype = ctypes.c_uint64
        L.orc_synth_arena_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        L.orc_group_reps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_void_p]
        L.orc_group_reps.restype = ctypes.c_int
        L.orc_synth_dedup_rows.argtypes = [ctypes.c_uint64] * 5 + [ctypes.c_void_p] * 3
        L.orc_balloon_blake3.argtypes = [ctypes.c_void_p, ctypes.c_size_t] * 3 + [
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_balloon_blake3.restype = ctypes.c_int
        L.orc_balloon_blake3_trace.argtypes = [ctypes.c_void_p, ctypes.c_size_t] * 3 + [
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_balloon_blake3_trace.restype = ctypes.c_int64
        L.orc_cas_paths_simd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_blake3_simd.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_checksum_simd_mt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
        del u8p
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _buf(data: bytes | np.ndarray) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def blake3(data, threads: int = 1) -> bytes:
    a = _buf(data)
    out = np.zeros(32, np.uint8)
    if threads > 1:
        lib().orc_blake3_mt(_ptr(a), a.size, threads, _ptr(out))
    else:
        lib().orc_blake3(_ptr(a), a.size, _ptr(out))
    return out.tobytes()


def blake3_incremental(data, piece: int) -> bytes:
    a = _buf(data)
    out = np.zeros(32, np.uint8)
    lib().orc_blake3_incremental(_ptr(a), a.size, piece, _ptr(out))
    return out.tobytes()


def derive_key(context: str, material: bytes) -> bytes:
    a = _buf(material)
    out = np.zeros(32, np.uint8)
    c = context.encode()
    lib().orc_blake3_derive_key(c, len(c), _ptr(a), a.size, _ptr(out))
    return out.tobytes()


def balloon_blake3(pwd: bytes, salt: bytes, secret: bytes, s_cost: int, t_cost: int) -> bytes:
    """Balloon (balloon-hash 0.4.0) over BLAKE3 hash mode, orc_balloon_blake3."""
    bufs = [_buf(x if x else b"\0") for x in (pwd, salt, secret)]
    out = np.zeros(32, np.uint8)
    rc = lib().orc_balloon_blake3(_ptr(bufs[0]), len(pwd), _ptr(bufs[1]), len(salt),
                                  _ptr(bufs[2]), len(secret), s_cost, t_cost, _ptr(out))
    if rc:
        raise OSError(-rc, os.strerror(-rc))
    return out.tobytes()


def balloon_blake3_trace(pwd: bytes, salt: bytes, secret: bytes, s_cost: int, t_cost: int,
                         stride: int, cap: int):
    """(digest, [(message, blake3 digest)...]) recording every stride-th BLAKE3
    message the Balloon run hashes (replayable through another hasher)."""
    bufs = [_buf(x if x else b"\0") for x in (pwd, salt, secret)]
    out = np.zeros(32, np.uint8)
    msg = np.zeros((cap, 128), np.uint8)
    ln = np.zeros(cap, np.uint32)
    dig = np.zeros((cap, 32), np.uint8)
    k = lib().orc_balloon_blake3_trace(_ptr(bufs[0]), len(pwd), _ptr(bufs[1]), len(salt),
                                       _ptr(bufs[2]), len(secret), s_cost, t_cost, _ptr(out),
                                       stride, cap, _ptr(msg), _ptr(ln), _ptr(dig))
    if k < 0:
        raise OSError(-k, os.strerror(-k))
    return out.tobytes(), [(msg[i, :ln[i]].tobytes(), dig[i].tobytes()) for i in range(k)]


def keyed_hash(key32: bytes, data) -> bytes:
    k = _buf(key32)
    a = _buf(data)
    out = np.zeros(32, np.uint8)
    lib().orc_blake3_keyed(_ptr(k), _ptr(a), a.size, _ptr(out))
    return out.tobytes()


def cas_msg_len(size: int) -> int:
    return int(lib().orc_cas_msg_len(size))


def cas_build_message(file: bytes, size: int | None = None) -> bytes | None:
    f = _buf(file)
    if size is None:
        size = f.size
    out = np.zeros(max(8 + f.size, 57352), np.uint8)
    n = lib().orc_cas_build_message(_ptr(f), f.size, size, _ptr(out))
    return None if n < 0 else out[:n].tobytes()


def cas_id_of_message(msg) -> str:
    a = _buf(msg)
    out = ctypes.create_string_buffer(17)
    lib().orc_cas_id_of_message(_ptr(a), a.size, out)
    return out.value.decode()


def cas_id_of_file_bytes(file: bytes, size: int | None = None) -> str:
    msg = cas_build_message(file, size)
    if msg is None:
        raise EOFError("read_exact: UnexpectedEof")
    return cas_id_of_message(msg)


def cas_id_path(path: str, size: int) -> str:
    out = ctypes.create_string_buffer(17)
    rc = lib().orc_cas_id_path(os.fsencode(path), size, out)
    if rc:
        raise OSError(-rc, os.strerror(-rc), path)
    return out.value.decode()


def file_checksum_path(path: str) -> str:
    out = ctypes.create_string_buffer(65)
    rc = lib().orc_file_checksum_path(os.fsencode(path), out)
    if rc:
        raise OSError(-rc, os.strerror(-rc), path)
    return out.value.decode()


def cas_batch(arena: np.ndarray, off: np.ndarray, length: np.ndarray, threads: int = 1) -> np.ndarray:
    off = np.ascontiguousarray(off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    out = np.zeros((off.size, 8), np.uint8)
    lib().orc_cas_batch(_ptr(arena), _ptr(off), _ptr(length), off.size, _ptr(out), threads)
    return out


def simd_isa() -> str:
    """The SIMD hashers' width on this host: "AVX-512 16-way" or "AVX2 8-way"
    (ORC_SIMD_WIDTH=8 forces the latter)."""
    return "AVX-512 16-way" if lib().orc_simd_width() == 16 else "AVX2 8-way"


def cas_batch_simd(arena: np.ndarray, off: np.ndarray, length: np.ndarray,
                   threads: int = 1) -> np.ndarray:
    """cas bytes (n x 8) with the SIMD chunk/parent hashing -- AVX-512 16-way
    on hosts that have it, else AVX2 8-way, as the reference crate's
    hash_many picks (CPU baseline: the multi-chunk SIMD idea, restated)."""
    arena = np.ascontiguousarray(arena, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    out = np.zeros((off.size, 8), np.uint8)
    lib().orc_cas_batch_simd(_ptr(arena), _ptr(off), _ptr(length), off.size, _ptr(out), threads)
    return out


def blake3_simd(data: np.ndarray) -> bytes:
    """BLAKE3 of a buffer with the SIMD subtree hasher (CPU baseline of
    file_checksum, hash.rs:10-24)."""
    data = np.ascontiguousarray(data, np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_blake3_simd(_ptr(data), data.size, _ptr(out))
    return out.tobytes()


def checksum_simd_mt(data: np.ndarray, threads: int, reps: int) -> bytes:
    """`threads` threads each hash `data` `reps` times with the SIMD hasher
    (one file per thread); returns thread 0's digest."""
    data = np.ascontiguousarray(data, np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_checksum_simd_mt(_ptr(data), data.size, threads, reps, _ptr(out))
    return out.tobytes()


def cas_paths_simd(paths, sizes, threads: int = 1):
    """(cas bytes [n, 8], status [n]) of real files: the reference's reads per
    file (cas.rs:23-62) + the SIMD hasher, `threads` C threads (CPU
    baseline of the config-1 directory)."""
    n = len(paths)
    arr = getattr(paths, "c_paths", None)  # pre-encoded (file_identifier.PathList)
    if arr is None:
        enc = [os.fsencode(os.fspath(p)) for p in paths]
        arr = (ctypes.c_char_p * n)(*enc)
    sizes = np.ascontiguousarray(sizes, np.uint64)
    out = np.zeros((n, 8), np.uint8)
    st = np.zeros(n, np.int32)
    lib().orc_cas_paths_simd(arr, _ptr(sizes), n, _ptr(out), _ptr(st), threads)
    return out, st


def synth_file_bytes(seed: int, offset: int, n: int) -> bytes:
    out = np.zeros(n, np.uint8)
    lib().orc_synth_file_bytes(seed, offset, n, _ptr(out))
    return out.tobytes()


def synth_cas_message(size: int, seed: int) -> bytes:
    out = np.zeros(57352 if size > 102400 else 8 + size, np.uint8)
    n = lib().orc_synth_cas_message(size, seed, _ptr(out))
    return out[:n].tobytes()


def synth_arena(sizes: np.ndarray, seeds: np.ndarray, threads: int = 8):
    """(arena, off, len) of synthetic cas messages packed at 128-B offsets."""
    sizes = np.ascontiguousarray(sizes, np.uint64)
    seeds = np.ascontiguousarray(seeds, np.uint64)
    off = np.zeros(sizes.size, np.uint64)
    ln = np.zeros(sizes.size, np.uint32)
    total = lib().orc_synth_arena_layout(_ptr(sizes), sizes.size, _ptr(off), _ptr(ln))
    arena = np.zeros(int(total) + 128, np.uint8)
    lib().orc_synth_arena_fill(_ptr(sizes), _ptr(seeds), _ptr(off), sizes.size, _ptr(arena), threads)
    return arena, off, ln


def group_reps(key: np.ndarray, has_key: np.ndarray, chunk_rows: int = 100) -> np.ndarray:
    key = np.ascontiguousarray(key, np.uint64)
    has_key = np.ascontiguousarray(has_key, np.uint8)
    rep = np.zeros(key.size, np.uint32)
    rc = lib().orc_group_reps(_ptr(key), _ptr(has_key), key.size, chunk_rows, _ptr(rep))
    if rc:
        raise OSError(-rc, os.strerror(-rc))
    return rep


REP_EXISTING = 0x80000000


def group_reps_existing(key: np.ndarray, has_key: np.ndarray, chunk_rows: int = 100,
                        existing_key: np.ndarray | None = None,
                        existing_handle: np.ndarray | None = None) -> np.ndarray:
    """The grouping of a whole run of rows (ranks 0..n-1 in id order) when some
    Objects exist before it (/root/reference/core/src/object/file_identifier/
    mod.rs:168-185 finds, library-wide, the Objects owning a file_path with the
    row's cas_id; :189-225 links the row to one of them; only the rest,
    :233-241, follow the in-run rule of orc_group_reps).  A key owned by several
    pre-existing Objects links to the lowest handle (the canonical "first").
    Returns uint32 rep: a rank, or REP_EXISTING | handle."""
    rep = group_reps(key, has_key, chunk_rows).astype(np.uint32)
    if existing_key is None or len(existing_key) == 0:
        return rep
    ek = np.asarray(existing_key, np.uint64)
    eh = np.asarray(existing_handle, np.uint32) & np.uint32(0x7FFFFFFF)
    order = np.lexsort((eh, ek))                # by key, then handle
    ek, eh = ek[order], eh[order]
    first = np.concatenate([[True], ek[1:] != ek[:-1]])
    ek, eh = ek[first], eh[first]               # lowest handle per key
    key = np.asarray(key, np.uint64)
    pos = np.searchsorted(ek, key)
    pos = np.minimum(pos, ek.size - 1)
    hit = (ek[pos] == key) & (np.asarray(has_key) != 0)
    rep[hit] = np.uint32(REP_EXISTING) | eh[pos[hit]]
    return rep


def link_batch(rep: np.ndarray, rank: np.ndarray | None = None, valid: np.ndarray | None = None,
               first_rank: int = 0):
    """Object write set of identifier_job_step for a batch of rows
    (/root/reference/core/src/object/file_identifier/mod.rs:189-333): rows whose
    grouping rep is their own rank get a new Object (create_many, :243-297),
    the others connect to the Object of row rep (:189-225); rows whose metadata
    failed (valid == 0, :113,127) stay orphans.  Returns (create, link_row,
    link_obj) in row order."""
    rep = np.asarray(rep, np.uint32)
    r = (np.arange(rep.size, dtype=np.uint64) + first_rank).astype(np.uint32) if rank is None \
        else np.asarray(rank, np.uint32)
    v = np.ones(rep.size, bool) if valid is None else np.asarray(valid) != 0
    create = r[v & (rep == r)]
    lk = v & (rep != r)
    return create, r[lk], rep[lk]


def synth_dedup_rows(seed: int, total: int, distinct: int, first: int, n: int):
    key = np.zeros(n, np.uint64)
    has = np.zeros(n, np.uint8)
    rank = np.zeros(n, np.uint32)
    lib().orc_synth_dedup_rows(seed, total, distinct, first, n, _ptr(key), _ptr(has), _ptr(rank))
    return key, has, rank


def orphan_objects(object_ids, fp_object_ids) -> np.ndarray:
    """Orphan remover's query (/root/reference/core/src/object/orphan_remover.rs:
    57-90, `object::file_paths::none`): the Objects no file_path references, in
    list order."""
    ref = set(int(x) for x in np.asarray(fp_object_ids) if x >= 0)
    return np.array([o for o in np.asarray(object_ids).tolist() if o not in ref], np.int32)


def thumbnail_shards(cas8: np.ndarray, valid=None):
    """Thumbnail directories (/root/reference/core/src/object/media/thumbnail/
    shard.rs:4-8: cas_id[0..2] = the first digest byte): rows ordered by
    directory, stable; rows per directory."""
    first = np.asarray(cas8)[:, 0].astype(np.int64)
    rows = np.arange(first.size) if valid is None else np.flatnonzero(np.asarray(valid))
    order = rows[np.argsort(first[rows], kind="stable")]
    return order.astype(np.int32), np.bincount(first[rows], minlength=256).astype(np.int32)


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (the bijection csrc/rows_device.hpp uses for row
    hashes and the config-5 key variation)."""
    z = np.asarray(x, np.uint64).copy()
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def vary_keys(key: np.ndarray, vary: np.ndarray, step: int) -> np.ndarray:
    """Keys of step `step` of the bench's config-5 run (synthetic-corpus
    convention, not a reference function): rows marked `vary` stand for files
    with new content, key' = mix64(key ^ step * phi64); step 0 unchanged."""
    key = np.asarray(key, np.uint64)
    if step == 0:
        return key.copy()
    with np.errstate(over="ignore"):
        s = np.uint64((step * 0x9E3779B97F4A7C15) & (2**64 - 1))
    return np.where(np.asarray(vary) != 0, mix64(key ^ s), key)
