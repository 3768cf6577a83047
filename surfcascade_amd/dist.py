"""Frame sharding + detection gather across ranks.

Frames are independent, so a batch shards over ranks with no data-path
exchange (C3); a single frame shards by (level, y) rows of its window grid
(Detector.set_shard, every rank rebuilds the integral table).  The only
collective is the gather of the raw detection records at the end, in the
order SURVEY.md 8e gives: one all_gather of the per-frame counts, then one
all_gather of every rank's records padded to the largest count (RCCL over
xGMI on GPUs, gloo in CPU tests).  A rank whose device buffer overflowed
(count > capacity: sc_enqueue_device dropped records) is an error on every
rank, never a silent truncation; `enqueue_and_gather` re-runs the scan with
a large enough buffer instead.
Records (RECORD_DTYPE, 40 B) are unsorted on the device; merge_records()
returns them in canonical (global frame, level, y, x) order.
"""
from __future__ import annotations

import numpy as np

from . import RECORD_DTYPE


class RecordOverflow(RuntimeError):
    """A rank's detection count exceeds its record buffer's capacity."""

    def __init__(self, rank, count, capacity):
        super().__init__("rank %d found %d detections but its record buffer holds %d"
                         % (rank, count, capacity))
        self.rank, self.count, self.capacity = rank, count, capacity


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


def _capacity(recs):
    return recs.numel() * recs.element_size() // RECORD_DTYPE.itemsize


def _frames_max(counts, group, b_max):
    """Frames per rank (len(counts) - 1) may differ between ranks (e.g. 257
    frames over 8 GPUs): the meta all_gather needs one size on every rank, so
    the ranks always all_gather their (B, b_max) first -- one tiny collective,
    the same on every rank whether or not it passed b_max (a shortcut taken by
    some ranks only would mismatch the collectives and hang).  A b_max below
    some rank's B raises ValueError on EVERY rank (they all see the same
    gathered values)."""
    import torch
    import torch.distributed as dist
    b = counts.numel() - 1
    world = dist.get_world_size(group)
    mine = torch.tensor([b, -1 if b_max is None else int(b_max)], dtype=torch.int64, device=counts.device)
    got = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(got, mine, group=group)
    bs = [tuple(int(v) for v in x.tolist()) for x in got]
    bm = max(x[0] for x in bs)
    for r, (_b, m) in enumerate(bs):
        if m >= 0 and m < bm:
            raise ValueError("rank %d passed b_max %d but a rank has %d frames" % (r, m, bm))
    return bm


def _gather_meta(counts, recs, group, b_max=None):
    """One all_gather of every rank's (B, counts padded to b_max frames,
    capacity) as int64 -> host array [world, 3 + b_max]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bm = _frames_max(counts, group, b_max)
    c = counts.to(torch.int64).reshape(-1)
    pad = torch.zeros(1 + bm - c.numel(), dtype=torch.int64, device=counts.device)
    meta = torch.cat([torch.tensor([c.numel() - 1], dtype=torch.int64, device=counts.device), c, pad,
                      torch.tensor([_capacity(recs)], dtype=torch.int64, device=counts.device)])
    gm = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(gm, meta, group=group)
    return torch.stack(gm).cpu().numpy()  # one device-to-host copy


def _gather_records(gm, counts, recs, group):
    import torch
    import torch.distributed as dist
    ns = [int(m[1]) for m in gm]
    for r, m in enumerate(gm):
        if ns[r] > int(m[-1]):
            raise RecordOverflow(r, ns[r], int(m[-1]))
    nb = max(ns) * RECORD_DTYPE.itemsize  # every rank sends its first max(count) records
    gr = [torch.zeros(nb, dtype=recs.dtype, device=recs.device) for _ in gm]
    if nb > 0:
        send = recs[:nb]
        if send.numel() < nb:  # a smaller buffer than another rank's count: pad (sizes must match)
            send = torch.cat([send, torch.zeros(nb - send.numel(), dtype=recs.dtype, device=recs.device)])
        dist.all_gather(gr, send.contiguous(), group=group)
    # each rank's own counts: [total, frame 0 .. B_r - 1]
    gc = [m[1:2 + int(m[0])].astype(np.int32) for m in gm]
    return gc, gr


def gather_detections(counts, recs, group=None, b_max=None):
    """counts: int32 [1+B] (counts[0] = this rank's total), recs: uint8
    [cap*40] record buffer (sc_enqueue_device's outputs).  B may differ
    between ranks; b_max (optional, the largest B as a caller knows it) is
    checked against the gathered sizes on every rank.

    1) all_gather of the counts (and capacities); 2) all_gather of every
    rank's first max(count) records (padded).  Raises RecordOverflow on every
    rank when any rank's count exceeds its capacity (its buffer lost records).
    Returns (per-rank counts, per-rank record bytes)."""
    return _gather_records(_gather_meta(counts, recs, group, b_max), counts, recs, group)


def enqueue_and_gather(det, frames, recs, counts, group=None, b_max=None):
    """One detect step of a rank followed by the gather: scans `frames` into
    `recs` / `counts` (sc_enqueue_device); when some rank's detections
    overflowed its buffer, every rank grows its buffer to the largest count
    and scans again.  Returns (per-rank counts, per-rank records, recs)."""
    import torch
    det.enqueue_device(frames, recs, counts)
    det.synchronize()
    gm = _gather_meta(counts, recs, group, b_max)
    need = int(gm[:, 1].max())
    if (gm[:, 1] > gm[:, -1]).any():
        if need > _capacity(recs):
            recs = torch.zeros(need * RECORD_DTYPE.itemsize, dtype=torch.uint8, device=recs.device)
        det.enqueue_device(frames, recs, counts)
        det.synchronize()
        gm = _gather_meta(counts, recs, group, b_max)
    gc, gr = _gather_records(gm, counts, recs, group)
    return gc, gr, recs


class StreamGather:
    """The gather for a steady stream of equal steps, with no host round trip
    per step.  A rank's counts and records share one device buffer
    (`recs` | `counts`, a fixed size agreed by every rank at construction),
    sc_enqueue_device writes both, and one all_gather of the whole buffer
    follows on the current stream (RCCL orders it after the scan, the next
    scan after it).  The step never reads a count on the host, so the GPU runs
    scan, gather, scan, ... back to back; `result()` syncs once, then raises
    RecordOverflow for a rank whose count exceeded the capacity (its buffer
    lost records: re-run that step with `enqueue_and_gather`, which grows the
    buffers).  `enqueue_and_gather` remains the checked per-step form.
    b: frames per rank (the same on every rank); capacity: records."""

    def __init__(self, b, capacity, device, group=None):
        import torch
        import torch.distributed as dist
        self.group, self.b, self.capacity = group, int(b), int(capacity)
        self.world = dist.get_world_size(group)
        self.cap_bytes = self.capacity * RECORD_DTYPE.itemsize
        n = self.cap_bytes + 4 * (1 + self.b)
        self.buf = torch.zeros(n, dtype=torch.uint8, device=device)
        self.recs = self.buf[: self.cap_bytes]
        self.counts = self.buf[self.cap_bytes:].view(torch.int32)
        self.out = torch.zeros(self.world, n, dtype=torch.uint8, device=device)
        mine = torch.tensor([self.b, self.capacity], dtype=torch.int64, device=device)
        got = [torch.zeros_like(mine) for _ in range(self.world)]
        dist.all_gather(got, mine, group=group)
        for r, g in enumerate(got):
            if g.tolist() != [self.b, self.capacity]:
                raise ValueError("StreamGather needs one layout on every rank: rank %d has (frames, capacity) %s, "
                                 "this rank (%d, %d)" % (r, g.tolist(), self.b, self.capacity))

    def step(self, det, frames):
        import torch.distributed as dist
        det.enqueue_device(frames, self.recs, self.counts)
        dist.all_gather(list(self.out.unbind(0)), self.buf, group=self.group)

    def result(self):
        """(per-rank counts [1+b] int32, per-rank record bytes) of the last step."""
        host = self.out.cpu().numpy()
        gc, gr = [], []
        for r in range(self.world):
            c = host[r, self.cap_bytes:].view(np.int32).copy()
            if int(c[0]) > self.capacity:
                raise RecordOverflow(r, int(c[0]), self.capacity)
            gc.append(c)
            gr.append(host[r, : self.cap_bytes].copy())
        return gc, gr


def merge_records(gathered_counts, gathered_recs, frame_offsets):
    """Decode every rank's records, shift frames to global indices, sort.
    A rank whose count exceeds the records it sent raises RecordOverflow."""
    out = []
    for r, (c, raw, off) in enumerate(zip(gathered_counts, gathered_recs, frame_offsets)):
        c = np.asarray(c.cpu() if hasattr(c, "cpu") else c)
        raw = np.asarray(raw.cpu() if hasattr(raw, "cpu") else raw, np.uint8)
        cap = raw.nbytes // RECORD_DTYPE.itemsize
        n = int(c[0])
        if n > cap:
            raise RecordOverflow(r, n, cap)
        a = raw[: n * RECORD_DTYPE.itemsize].view(RECORD_DTYPE).copy()
        a["frame"] += off
        out.append(a)
    a = np.concatenate(out) if out else np.zeros(0, RECORD_DTYPE)
    order = np.lexsort((a["x"], a["y"], a["level"], a["frame"]))
    return a[order]
