"""ctypes binding of libsdgpu.so (the C ABI in include/sdgpu.h).

The product path has no CPU fallback: if the library or a gfx950 device is
missing, the calls below raise instead of computing anything elsewhere.
"""
from __future__ import annotations

import ctypes
import os
import re
import weakref

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsdgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "sdgpu.h")

_lib = None

c_u8p = ctypes.c_void_p
c_vp = ctypes.c_void_p


class SdgpuError(OSError):
    """A negative errno returned by libsdgpu (maps to Rust's io::Error)."""

    def __init__(self, rc: int, what: str = ""):
        msg = load().sdgpu_strerror(rc).decode()
        super().__init__(-rc, f"{what}: {msg}" if what else msg)
        self.rc = rc


def _proto(L):
    P = ctypes.POINTER
    i32, u32, u64, sz = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
    ctx = c_vp
    sig = {
        "sdgpu_abi_version": (i32, []),
        "sdgpu_strerror": (ctypes.c_char_p, [i32]),
        "sdgpu_device_count": (i32, [P(i32)]),
        "sdgpu_open": (i32, [i32, P(c_vp)]),
        "sdgpu_close": (i32, [ctx]),
        "sdgpu_sync": (i32, [ctx]),
        "sdgpu_stream": (c_vp, [ctx]),
        "sdgpu_alloc_pinned": (i32, [ctx, sz, P(c_vp)]),
        "sdgpu_free_pinned": (i32, [ctx, c_vp]),
        "sdgpu_alloc_device": (i32, [ctx, sz, P(c_vp)]),
        "sdgpu_free_device": (i32, [ctx, c_vp]),
        "sdgpu_memcpy_async": (i32, [ctx, c_vp, c_vp, sz, c_vp]),
        "sdgpu_cas_batch": (i32, [ctx, c_vp, c_vp, c_vp, u32, c_vp, c_vp]),
        "sdgpu_cas_batch_device": (i32, [ctx, c_vp, u64, c_vp, c_vp, u32, c_vp, c_vp, c_vp]),
        "sdgpu_cas_stage_pinned": (i32, [ctx, c_vp, c_vp, c_vp, u32, c_vp, c_vp, c_vp]),
        "sdgpu_link_batch_device": (i32, [ctx, c_vp, c_vp, c_vp, u32, u64, c_vp, c_vp, c_vp, c_vp,
                                          c_vp]),
        "sdgpu_group_link_device": (i32, [ctx, c_vp, c_vp, c_vp, c_vp, c_vp, u32, u64, u32, c_vp,
                                          c_vp, c_vp, c_vp]),
        "sdgpu_generate_cas_id": (i32, [ctx, ctypes.c_char_p, u64, ctypes.c_char_p]),
        "sdgpu_identify_files": (i32, [ctx, c_vp, c_vp, u32, c_vp, c_vp, c_vp]),
        "sdgpu_checksum": (i32, [ctx, c_vp, u64, c_vp]),
        "sdgpu_checksum_batch_device": (i32, [ctx, c_vp, c_vp, u32, c_vp, c_vp]),
        "sdgpu_subtree_device": (i32, [ctx, c_vp, u64, u64, i32, c_vp, c_vp]),
        "sdgpu_combine_subtrees_device": (i32, [ctx, c_vp, u64, c_vp, c_vp]),
        "sdgpu_checksum_files": (i32, [ctx, c_vp, u32, c_vp, c_vp]),
        "sdgpu_file_checksum": (i32, [ctx, ctypes.c_char_p, ctypes.c_char_p]),
        "sdgpu_latency_service": (i32, [ctx, i32]),
        "sdgpu_latency_service_diag": (i32, [ctx, c_vp]),
        "sdgpu_dedup": (i32, [ctx, c_vp, c_vp, u32, u32, c_vp]),
        "sdgpu_group_pairs_device": (i32, [ctx, c_vp, c_vp, u64, u32, u32, c_vp, c_vp]),
        "sdgpu_group_rows_device": (i32, [ctx, c_vp, c_vp, c_vp, u64, u32, u32, c_vp, c_vp]),
        "sdgpu_shard_count_device": (i32, [ctx, c_vp, c_vp, u64, u32, c_vp, c_vp]),
        "sdgpu_shard_partition_device": (i32, [ctx, c_vp, c_vp, c_vp, u64, u32, c_vp, c_vp, c_vp,
                                               c_vp]),
        "sdgpu_shard_exchange_device": (i32, [ctx, c_vp, c_vp, c_vp, u64, u32, u32, c_vp, c_vp,
                                              c_vp, c_vp, c_vp]),
        "sdgpu_scatter_rep_device": (i32, [ctx, c_vp, c_vp, u64, c_vp, u64, c_vp, i32, c_vp]),
        "sdgpu_index_create": (i32, [ctx, u64, P(c_vp)]),
        "sdgpu_index_destroy": (i32, [c_vp]),
        "sdgpu_index_clear": (i32, [c_vp, c_vp]),
        "sdgpu_index_count": (i32, [c_vp, P(ctypes.c_uint64)]),
        "sdgpu_index_add_objects_device": (i32, [c_vp, c_vp, c_vp, u64, u32, u32, c_vp]),
        "sdgpu_group_rows_indexed_device": (i32, [ctx, c_vp, c_vp, c_vp, c_vp, u64, u32, c_vp,
                                                  c_vp]),
        "sdgpu_dedup_batch": (i32, [ctx, c_vp, c_vp, c_vp, u32, u32, u32, c_vp]),
        "sdgpu_comm_unique_id": (i32, [c_vp]),
        "sdgpu_comm_set_return": (i32, [c_vp, i32]),
        "sdgpu_comm_set_exchange": (i32, [c_vp, i32, u64]),
        "sdgpu_comm_init_rank": (i32, [ctx, i32, i32, c_vp, P(c_vp)]),
        "sdgpu_comm_init_all": (i32, [c_vp, i32, i32, c_vp]),
        "sdgpu_comm_destroy": (i32, [c_vp]),
        "sdgpu_comm_info": (i32, [c_vp, P(i32), P(i32), P(i32)]),
        "sdgpu_comm_init_rank_timeout": (i32, [ctx, i32, i32, c_vp, i32, P(c_vp)]),
        "sdgpu_comm_set_timeout": (i32, [c_vp, i32]),
        "sdgpu_comm_init_host": (i32, [ctx, i32, i32, ctypes.c_char_p, u64, i32, P(c_vp)]),
        "sdgpu_comm_wait": (i32, [c_vp, c_vp]),
        "sdgpu_comm_stats": (i32, [c_vp, c_vp]),
        "sdgpu_group_sharded_device": (i32, [ctx, c_vp, c_vp, c_vp, c_vp, c_vp, u64, u32, c_vp,
                                             c_vp]),
        "sdgpu_group_sharded_all_device": (i32, [c_vp, c_vp, c_vp, i32, c_vp, c_vp, c_vp, c_vp,
                                                 u32, c_vp, c_vp]),
        "sdgpu_group_link_sharded_device": (i32, [ctx, c_vp, c_vp, c_vp, c_vp, c_vp, u64, u32,
                                                  c_vp, c_vp, u64, c_vp, c_vp]),
        "sdgpu_group_link_sharded_all_device": (i32, [c_vp, c_vp, i32, c_vp, c_vp, c_vp, c_vp,
                                                      c_vp, u32, c_vp, c_vp, c_vp, c_vp, c_vp]),
        "sdgpu_dedup_sharded": (i32, [c_vp, i32, c_vp, c_vp, u32, u32, c_vp]),
        "sdgpu_synth_cas_arena_device": (i32, [ctx, c_vp, c_vp, c_vp, u32, c_vp, c_vp]),
        "sdgpu_synth_file_device": (i32, [ctx, u64, u64, u64, c_vp, c_vp]),
        "sdgpu_synth_dedup_rows_device": (i32, [ctx, u64, u64, u64, u64, u64, c_vp, c_vp, c_vp,
                                                c_vp]),
        "sdgpu_orphan_objects_device": (i32, [ctx, c_vp, u64, c_vp, u64, u32, c_vp, c_vp, c_vp]),
        "sdgpu_thumbnail_shards_device": (i32, [ctx, c_vp, c_vp, u64, c_vp, c_vp, c_vp]),
        "sdgpu_synth_vary_keys_device": (i32, [ctx, c_vp, c_vp, u64, u64, c_vp]),
        "sdgpu_set_timing": (i32, [ctx, i32]),
        "sdgpu_timing_reset": (i32, [ctx]),
        "sdgpu_timing_read": (i32, [ctx, u32, ctypes.c_char_p, P(ctypes.c_double),
                                    P(ctypes.c_uint64)]),
        "sdgpu_valu_probe": (i32, [ctx, P(ctypes.c_double)]),
        "sdgpu_valu_probe_kind": (i32, [ctx, i32, P(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def load():
    """Loads libsdgpu.so from the package directory (raises if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                "there is no CPU fallback for the content-identification path")
        # One HIP/HSA runtime per process: torch bundles its own libamdhip64
        # (SONAME libamdhip64.so.7).  Loading torch first lets the dynamic
        # linker bind libsdgpu's libamdhip64.so.7 dependency to that same copy;
        # loading libsdgpu first would pull /opt/rocm's runtime and torch would
        # then start a second HSA runtime that cannot open the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        _proto(L)
        _lib = L
    return _lib


def declared_symbols() -> list[str]:
    """Function names declared in include/sdgpu.h."""
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(sdgpu_[a-z0-9_]+)\s*\(", text)))


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise SdgpuError(rc, what)


class Context:
    """An open device context (sdgpu_open / sdgpu_close)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.sdgpu_open(device, ctypes.byref(h)), f"sdgpu_open({device})")
        self.h = h
        self.device = device
        # indexes and communicators made on this context: sdgpu_close frees
        # what they point into, so close() destroys them first (a handle
        # outliving its context would otherwise be destroyed after it)
        self._deps = weakref.WeakSet()

    def adopt(self, obj):
        """Registers an object with a close() that must run before sdgpu_close."""
        self._deps.add(obj)

    def close(self):
        if self.h:
            for d in list(self._deps):
                d.close()
            self.lib.sdgpu_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(self.lib.sdgpu_sync(self.h), "sdgpu_sync")

    @property
    def stream(self) -> int:
        return self.lib.sdgpu_stream(self.h) or 0

    def latency_service(self, enable: bool = True):
        """Single-file calls through the resident latency kernel
        (sdgpu_latency_service)."""
        check(self.lib.sdgpu_latency_service(self.h, 1 if enable else 0), "sdgpu_latency_service")

    def latency_service_diag(self) -> dict:
        """Breakdown (us) of the last service request."""
        v = (ctypes.c_double * 4)()
        check(self.lib.sdgpu_latency_service_diag(self.h, v), "sdgpu_latency_service_diag")
        return {"copy_to_lds_us": v[0], "hash_us": v[1], "host_post_to_answer_us": v[2],
                "host_read_us": v[3]}

    def set_timing(self, enable: bool = True):
        check(self.lib.sdgpu_set_timing(self.h, 1 if enable else 0), "sdgpu_set_timing")
        check(self.lib.sdgpu_timing_reset(self.h), "sdgpu_timing_reset")

    def kernel_times(self) -> dict[str, tuple[float, int]]:
        """{kernel name: (total device ms, launches)} since set_timing()."""
        res = {}
        i = 0
        while True:
            name = ctypes.create_string_buffer(32)
            ms = ctypes.c_double()
            n = ctypes.c_uint64()
            rc = self.lib.sdgpu_timing_read(self.h, i, name, ctypes.byref(ms), ctypes.byref(n))
            if rc == -2:
                break
            check(rc, "sdgpu_timing_read")
            res[name.value.decode()] = (ms.value, n.value)
            i += 1
        return res

    def valu_peak(self, kind: int = 0) -> float:
        """Measured int32 VALU lane-ops/s: kind 0 = BLAKE3-G instruction mix,
        1 v_xor_b32, 2 v_add3_u32, 3 v_alignbit_b32, 4 v_add_u32, 5 register-only
        BLAKE3 compressions (680 VALU each: the attainable roof of K1/K2)."""
        v = ctypes.c_double()
        check(self.lib.sdgpu_valu_probe_kind(self.h, kind, ctypes.byref(v)), "sdgpu_valu_probe")
        return v.value


_default: dict[int, Context] = {}


def default_context(device: int | None = None) -> Context:
    """Process-wide context per device (the reference runs one job at a time)."""
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0")) if "LOCAL_RANK" in os.environ else 0
        try:
            import torch
            if torch.cuda.is_available():
                device = torch.cuda.current_device()
        except Exception:
            pass
    if device not in _default:
        _default[device] = Context(device)
    return _default[device]
