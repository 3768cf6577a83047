"""Frame sharding + detection gather across ranks.

Frames are independent, so a batch shards over ranks with no data-path
exchange (C3); a single frame shards by (level, y) rows of its window grid
(Detector.set_shard, every rank rebuilds the integral table); the only collective is the gather of the raw detection records at
the end: one all_gather of the per-frame counts and one all_gather of a
fixed-capacity record buffer (RCCL over xGMI on GPUs, gloo in CPU tests).
Records (RECORD_DTYPE, 40 B) are unsorted on the device; merge_records()
returns them in canonical (global frame, level, y, x) order.
"""
from __future__ import annotations

import numpy as np

from . import RECORD_DTYPE


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous frame range of `rank` (e.g. 256 frames / 8 GPUs -> 32 each)."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def grid_row_owner(layout, step, world):
    """Owner rank of every (level, y) row under sc_detector_set_shard's rule:
    row i of the canonical row list (level-major, y ascending) goes to rank
    i % world.  layout: [(level, l, lh, nx, ny, base)] (oracle.grid_layout).
    Returns {(level, y): rank}."""
    own, i = {}, 0
    for (lv, _l, _lh, _nx, ny, _b) in layout:
        for r in range(ny):
            own[(lv, r * step)] = i % world
            i += 1
    return own


def gather_detections(counts, recs, group=None):
    """all_gather of counts (int32 [1+B]) and records (uint8 [cap*40])."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    gc = [torch.zeros_like(counts) for _ in range(world)]
    gr = [torch.zeros_like(recs) for _ in range(world)]
    dist.all_gather(gc, counts, group=group)
    dist.all_gather(gr, recs, group=group)
    return gc, gr


def merge_records(gathered_counts, gathered_recs, frame_offsets):
    """Decode every rank's records, shift frames to global indices, sort."""
    out = []
    for c, r, off in zip(gathered_counts, gathered_recs, frame_offsets):
        c = np.asarray(c.cpu() if hasattr(c, "cpu") else c)
        raw = np.asarray(r.cpu() if hasattr(r, "cpu") else r, np.uint8)
        cap = raw.nbytes // RECORD_DTYPE.itemsize
        n = min(int(c[0]), cap)
        a = raw[: n * RECORD_DTYPE.itemsize].view(RECORD_DTYPE).copy()
        a["frame"] += off
        out.append(a)
    a = np.concatenate(out) if out else np.zeros(0, RECORD_DTYPE)
    order = np.lexsort((a["x"], a["y"], a["level"], a["frame"]))
    return a[order]
