"""Multi-rank path on CPU (gloo, world_size 2): frame sharding + the gather of
detection records must reproduce the single-process result exactly."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import FACE_CFG, ROOT


def _records_for(oracle, casc, frames, params, frame0, rng):
    """Per-rank device-style record buffer (unsorted, like the GPU's atomics)."""
    from surfcascade_amd import RECORD_DTYPE
    recs = []
    for f in range(len(frames)):
        T = oracle.integral(frames[f])
        d, _ = oracle.detect(T, casc, params, nthreads=1)
        for r in d:
            recs.append((f, r["level"], r["x"], r["y"], r["w"], r["h"], r["stage"], 0, r["score"]))
    a = np.array(recs, RECORD_DTYPE)
    rng.shuffle(a)
    return a


def _worker(rank, world, port, n_frames, out_q, tight=False, own_b=False):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import gather_detections, merge_records, shard_range
    casc = O.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45)  # permissive: plenty of detections
    params = O.Params(n_levels=2)
    start, cnt = shard_range(n_frames, world, rank)
    frames = np.stack([synth.make_frame(320, 240, 500 + start + k) for k in range(cnt)])
    a = _records_for(O, casc, frames, params, start, np.random.default_rng(rank))
    # tight: each rank's buffer holds exactly its own records, so the rank
    # with fewer detections sends a buffer shorter than the largest count
    cap = len(a) if tight else 1 << 15
    buf = np.zeros(cap, RECORD_DTYPE)
    buf[:len(a)] = a
    # own_b: each rank's counts hold its own frames only (uneven shards: 5
    # frames over 2 ranks -> 3 and 2; the gather exchanges the sizes first)
    B = cnt if own_b else max(shard_range(n_frames, world, r)[1] for r in range(world))
    counts = np.zeros(1 + B, np.int32)
    counts[0] = len(a)
    for f in range(cnt):
        counts[1 + f] = int((a["frame"] == f).sum())
    gc, gr = gather_detections(torch.from_numpy(counts), torch.from_numpy(buf.view(np.uint8).copy()))
    offs = [shard_range(n_frames, world, r)[0] for r in range(world)]
    merged = merge_records(gc, gr, offs)
    if rank == 0:
        out_q.put(merged.tobytes())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_all():
    from surfcascade_amd.dist import shard_range
    for n, w in ((256, 8), (10, 3), (3, 4)):
        seen = []
        for r in range(w):
            s, c = shard_range(n, w, r)
            seen += list(range(s, s + c))
        assert seen == list(range(n))


@pytest.mark.parametrize("world,tight,own_b", [(2, False, False), (2, True, False), (2, False, True),
                                                 (4, False, True)])
def test_gloo_gather_equals_single_process(oracle, world, tight, own_b):
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import merge_records
    n_frames = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + (7 if tight else 0) + (13 if own_b else 0) + (29 if world > 2 else 0)
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, q, tight, own_b))
             for r in range(world)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=120), RECORD_DTYPE)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process reference
    casc = oracle.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45)
    params = oracle.Params(n_levels=2)
    frames = np.stack([synth.make_frame(320, 240, 500 + k) for k in range(n_frames)])
    a = _records_for(oracle, casc, frames, params, 0, np.random.default_rng(9))
    ref = merge_records([np.array([len(a)])], [a.view(np.uint8)], [0])
    assert len(ref) > 50
    assert got.tobytes() == ref.tobytes()


def _grid_worker(rank, world, port, n_frames, out_q):
    """Grid sharding: every rank scans the same frames, its own rows only."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import gather_detections, grid_row_owner, merge_records
    casc = O.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45)
    params = O.Params(n_levels=3)
    frames = np.stack([synth.make_frame(320, 240, 500 + k) for k in range(n_frames)])
    layout, step = O.grid_layout(320, 240, params)
    own = grid_row_owner(layout, step, world)
    a = _records_for(O, casc, frames, params, 0, np.random.default_rng(rank))
    a = a[[own[(int(r["level"]), int(r["y"]))] == rank for r in a]]  # this rank's rows
    cap = 1 << 15
    buf = np.zeros(cap, RECORD_DTYPE)
    buf[:len(a)] = a
    counts = np.zeros(1 + n_frames, np.int32)
    counts[0] = len(a)
    gc, gr = gather_detections(torch.from_numpy(counts), torch.from_numpy(buf.view(np.uint8).copy()))
    merged = merge_records(gc, gr, [0] * world)  # same frames on every rank
    if rank == 0:
        out_q.put(merged.tobytes())
    dist.barrier()
    dist.destroy_process_group()


def test_grid_row_owner_partitions_rows(oracle):
    from surfcascade_amd.dist import grid_row_owner
    layout, step = oracle.grid_layout(1920, 1080, oracle.Params(n_levels=24))
    for world in (1, 2, 8):
        own = grid_row_owner(layout, step, world)
        assert len(own) == sum(e[4] for e in layout)
        # grid windows per rank balance to within one row of each level
        per = np.zeros(world, np.int64)
        for (lv, _l, _lh, nx, ny, _b) in layout:
            for r in range(ny):
                per[own[(lv, r * step)]] += nx
        assert per.max() - per.min() <= max(e[3] for e in layout) * len(layout)


def test_gloo_grid_shard_gather_equals_single_process(oracle):
    from surfcascade_amd import RECORD_DTYPE
    from surfcascade_amd.dist import merge_records
    world, n_frames = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 500) % 1000
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=120), RECORD_DTYPE)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    casc = oracle.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45)
    from surfcascade_amd import synth
    frames = np.stack([synth.make_frame(320, 240, 500 + k) for k in range(n_frames)])
    a = _records_for(oracle, casc, frames, oracle.Params(n_levels=3), 0, np.random.default_rng(9))
    ref = merge_records([np.array([len(a)])], [a.view(np.uint8)], [0])
    assert len(ref) > 20
    assert got.tobytes() == ref.tobytes()


class _FakeDetector:
    """Stands in for a GPU Detector in the gloo test: enqueue_device writes a
    precomputed (oracle-made, shuffled like the device's atomics) record list
    into the caller's buffer up to its capacity and the full counts, exactly
    as sc_enqueue_device does when its capacity is too small."""

    def __init__(self, records, n_frames):
        from surfcascade_amd import RECORD_DTYPE
        self.a, self.n_frames, self.calls = records, n_frames, 0
        self.itemsize = RECORD_DTYPE.itemsize

    def enqueue_device(self, frames, recs, counts):
        self.calls += 1
        cap = recs.numel() // self.itemsize
        k = min(cap, len(self.a))
        raw = recs.numpy()
        raw[:k * self.itemsize] = self.a[:k].view(np.uint8)
        counts.zero_()
        counts[0] = len(self.a)
        for f in range(self.n_frames):
            counts[1 + f] = int((self.a["frame"] == f).sum())

    def synchronize(self):
        pass


def _overflow_worker(rank, world, port, n_frames, out_q):
    """Rank 0 finds more detections than its first record buffer holds."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import (RecordOverflow, enqueue_and_gather, gather_detections,
                                      merge_records, shard_range)
    casc = O.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45 if rank == 0 else 0.6)  # rank 0: many detections
    params = O.Params(n_levels=2)
    start, cnt = shard_range(n_frames, world, rank)
    frames = np.stack([synth.make_frame(320, 240, 500 + start + k) for k in range(cnt)])
    a = _records_for(O, casc, frames, params, start, np.random.default_rng(rank))
    fake = _FakeDetector(a, cnt)
    cap = 8  # far below rank 0's count
    recs = torch.zeros(cap * RECORD_DTYPE.itemsize, dtype=torch.uint8)
    counts = torch.zeros(1 + cnt, dtype=torch.int32)
    # the plain gather refuses (on every rank) instead of dropping records
    fake.enqueue_device(None, recs, counts)
    raised = False
    try:
        gather_detections(counts, recs)
    except RecordOverflow as e:
        raised = e.rank == 0 and e.capacity == cap
    # enqueue_and_gather grows every rank's buffer and scans again
    gc, gr, recs2 = enqueue_and_gather(fake, None, recs, counts)
    offs = [shard_range(n_frames, world, r)[0] for r in range(world)]
    merged = merge_records(gc, gr, offs)
    out_q.put((rank, raised, fake.calls, len(a), recs2.numel() // RECORD_DTYPE.itemsize,
               merged.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_overflow_grows_not_truncates(oracle):
    """counts first, records padded to the largest count; a rank
    whose record buffer overflowed is an error on every rank (RecordOverflow),
    and enqueue_and_gather re-scans with a large enough buffer, so the merged
    result equals the single-process one."""
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import merge_records
    world, n_frames = 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 250) % 1000
    procs = [ctx.Process(target=_overflow_worker, args=(r, world, port, n_frames, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, raised0, calls0, n0, cap0, m0), (_, raised1, calls1, n1, cap1, m1) = res
    assert raised0 and raised1  # both ranks learn of rank 0's overflow
    assert n0 > 8 and calls0 == calls1 == 3  # first scan, enqueue_and_gather's scan + rescan
    assert cap0 == cap1 == max(n0, n1)
    assert m0 == m1
    # single-process reference
    ref = []
    for r in range(world):
        casc = oracle.cascade_from_cfg(open(FACE_CFG).read())
        casc.theta[:] = np.float32(0.45 if r == 0 else 0.6)
        from surfcascade_amd.dist import shard_range
        start, cnt = shard_range(n_frames, world, r)
        frames = np.stack([synth.make_frame(320, 240, 500 + start + k) for k in range(cnt)])
        a = _records_for(oracle, casc, frames, oracle.Params(n_levels=2), start,
                         np.random.default_rng(9))
        ref.append(merge_records([np.array([len(a)])], [a.view(np.uint8)], [start]))
    ref = np.concatenate(ref)
    ref = ref[np.lexsort((ref["x"], ref["y"], ref["level"], ref["frame"]))]
    assert np.frombuffer(m0, RECORD_DTYPE).tobytes() == ref.tobytes()
    assert len(ref) == n0 + n1


class _FixedDet:
    """Fills the record buffer like sc_enqueue_device (records up to the
    capacity, the full count even when it exceeds it)."""

    def __init__(self, a, b):
        self.a, self.b = a, b

    def enqueue_device(self, frames, recs, counts):
        from surfcascade_amd import RECORD_DTYPE
        cap = recs.numel() // RECORD_DTYPE.itemsize
        k = min(cap, len(self.a))
        recs.numpy()[:k * RECORD_DTYPE.itemsize] = self.a[:k].view(np.uint8)
        counts.zero_()
        counts[0] = len(self.a)
        for f in range(self.b):
            counts[1 + f] = int((self.a["frame"] == f).sum())


def _stream_worker(rank, world, port, cap, out_q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import RecordOverflow, StreamGather, gather_detections, merge_records, shard_range
    casc = O.cascade_from_cfg(open(FACE_CFG).read())
    casc.theta[:] = np.float32(0.45)
    params = O.Params(n_levels=2)
    B = 2
    start, _ = shard_range(B * world, world, rank)
    frames = np.stack([synth.make_frame(320, 240, 700 + start + k) for k in range(B)])
    a = _records_for(O, casc, frames, params, start, np.random.default_rng(rank))
    sg = StreamGather(B, cap, "cpu")
    det = _FixedDet(a, B)
    res = None
    for _ in range(3):  # steps reuse the buffers
        sg.step(det, torch.from_numpy(frames))
    try:
        gc, gr = sg.result()
        offs = [shard_range(B * world, world, r)[0] for r in range(world)]
        merged = merge_records(gc, gr, offs)
        # the checked per-step form gives the same records
        buf = np.zeros(max(cap, len(a)), RECORD_DTYPE)
        buf[:len(a)] = a
        counts = np.zeros(1 + B, np.int32)
        counts[0] = len(a)
        for f in range(B):
            counts[1 + f] = int((a["frame"] == f).sum())
        gc2, gr2 = gather_detections(torch.from_numpy(counts), torch.from_numpy(buf.view(np.uint8).copy()))
        res = ("ok", merged.tobytes() == merge_records(gc2, gr2, offs).tobytes(), len(merged))
    except RecordOverflow as e:
        res = ("overflow", e.rank, e.count)
    if rank == 0:
        out_q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cap", [1 << 12, 3])
def test_gloo_stream_gather(cap):
    """dist.StreamGather (bench.py's timed N > 1 steps: counts and records in
    one buffer, one all_gather per step, no host round trip) returns the same
    merged records as the checked gather_detections; a capacity below a
    rank's count raises RecordOverflow on every rank instead of truncating."""
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + random.randint(0, 900)
    ps = [ctx.Process(target=_stream_worker, args=(r, 2, port, cap, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=180)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    if cap == 3:
        assert res[0] == "overflow" and res[2] > 3
    else:
        assert res[0] == "ok" and res[1] and res[2] > 0


def _bmax_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from surfcascade_amd.dist import gather_detections
    # rank 0: 3 frames and an advisory b_max that is too small for rank 1's
    # 4 frames; rank 1 passes none.  Every rank must raise (no collective
    # mismatch, no hang); then a consistent call still works.
    B = 3 + rank
    counts = torch.zeros(1 + B, dtype=torch.int32)
    recs = torch.zeros(40 * 4, dtype=torch.uint8)
    res = []
    try:
        gather_detections(counts, recs, b_max=3 if rank == 0 else None)
        res.append("ok")
    except ValueError as e:
        res.append("raised" if "b_max" in str(e) else "other")
    gc, _ = gather_detections(counts, recs, b_max=4 if rank == 1 else None)
    res.append([len(c) for c in gc])
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_b_max_mismatch_raises_on_every_rank():
    """b_max passed by some ranks only must not desynchronise the
    collectives; a b_max below another rank's frame count raises everywhere."""
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + random.randint(0, 900)
    ps = [ctx.Process(target=_bmax_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert got[r] == ["raised", [4, 5]]
