"""Downstream consumers of the grouping on the device.

* ``orphan_objects`` -- the orphan remover's query
  (/root/reference/core/src/object/orphan_remover.rs:57-90): Objects no
  file_path points at, found in one pass (sdgpu_orphan_objects_device) instead
  of repeated `find_many(file_paths::none).take(512)` round trips.
* ``thumbnail_shards`` -- rows grouped by thumbnail directory
  (/root/reference/core/src/object/media/thumbnail/shard.rs:4-8, directory =
  cas_id[0..2]) with per-directory counts (sdgpu_thumbnail_shards_device);
  ``get_shard_hex`` is the reference function itself.
"""
from __future__ import annotations

from ._native import check, default_context


def get_shard_hex(cas_id: str) -> str:
    """shard.rs:4-8: the first two hex characters of the cas_id."""
    return cas_id[0:2]


def orphan_objects(object_ids, fp_object_ids, max_object_id: int, ctx=None, trim: bool = True):
    """int32 device tensor of the Object ids (from `object_ids`) that no
    file_path's object_id (`fp_object_ids`, negative = NULL) references, in
    list order.  trim=False: the full-length list and the device count [1],
    no synchronisation."""
    import torch
    dev = object_ids.device
    ctx = ctx or default_context(dev.index)
    out = torch.empty(max(object_ids.numel(), 1), dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_orphan_objects_device(
        ctx.h, object_ids.data_ptr(), object_ids.numel(), fp_object_ids.data_ptr(),
        fp_object_ids.numel(), max_object_id, out.data_ptr(), cnt.data_ptr(), s),
        "sdgpu_orphan_objects_device")
    if not trim:
        return out, cnt
    return out[:int(cnt.item())]


def thumbnail_shards(cas8, valid=None, ctx=None, trim: bool = True):
    """(order, counts): rows with a cas_id ordered by thumbnail directory
    (stable inside a directory), and rows per directory (256).  trim=False:
    the full-length order (its first sum(counts) entries), no
    synchronisation."""
    import torch
    dev = cas8.device
    ctx = ctx or default_context(dev.index)
    n = cas8.shape[0]
    order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.empty(256, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    check(ctx.lib.sdgpu_thumbnail_shards_device(
        ctx.h, cas8.data_ptr(), valid.data_ptr() if valid is not None else None, n,
        order.data_ptr(), counts.data_ptr(), s), "sdgpu_thumbnail_shards_device")
    if not trim:
        return order, counts
    total = int(counts.sum().item())
    return order[:total], counts
