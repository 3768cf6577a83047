"""Benchmark: detection windows/s on the 1080p 24-level pyramid (BASELINE.json
metric, config C2 on one GPU; C3-style frame sharding for --gpus N).  --config
C4 (4K, 32 levels) and C5 (64x128 pedestrian cascade) measure the other
single-GPU configs the same way.

A step = one pass of the detect path over one batch of synthetic 1080p frames
already resident in HBM: gradient+integral (rowscan, colscan), prefilter +
cascade + adaptive-stride walk (windows), and the gather of the raw detection
records (RCCL all_gather when N > 1).  value = stride-3 grid windows of all
frames of all ranks / max-over-ranks wall time.  Prints one JSON line (rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C4|C5] [--batch B]

--gpus N > 1 without a torch.distributed environment (WORLD_SIZE unset)
starts the N ranks itself -- `python -m torch.distributed.run --nproc-per-node
N --master-addr 127.0.0.1 bench.py ...` as a child process, before anything
touches a GPU -- and exits with its status; a rank that finds WORLD_SIZE !=
--gpus, or fewer visible GPUs than ranks, exits non-zero instead of measuring
fewer GPUs.  (--stub: a CPU stand-in for the detector, gloo backend -- the
CPU test of this launcher, tests/test_bench_launch.py; never a measurement.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue ceiling: 256 CUs x 4 SIMDs, a wave64 VALU instruction every 2
# cycles per SIMD (SIMD-32), 2.4 GHz (MI355X_MICROARCH.md: wave scheduling)
VALU_ISSUE_PEAK = 1024 * 0.5 * 2.4e9
# the texture data path (TD): one per CU, 64 B/clk, so a 16-B-per-lane wave
# load returns its 1 KiB in 16 cycles whatever its active lanes (DESIGN.md
# 5a, calibrated against TD_TD_BUSY)
TD_CYCLES_PER_LOAD = 16
N_CUS = 256
CSRC = os.path.join(ROOT, "surfcascade_amd", "csrc")


def source_build_id(extra="", arch="gfx950", san=""):
    """The build id the Makefile gives a library built from the current tree
    with EXTRA flags `extra`, ARCH `arch` and SAN `san` (sc_build_info
    "build_id"): sha256 over every csrc/*.hip, *.hpp, *.cpp (sorted), the
    Makefile, include/surfcascade.h and "extra|arch|san" -- kernels, the launch
    schedule in sc_api.cpp, every -D knob, the target and a sanitizer build
    alike."""
    import hashlib
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".cpp")))
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in names] + [os.path.join(CSRC, "Makefile"),
                                                            os.path.join(ROOT, "include", "surfcascade.h")]:
        with open(path, "rb") as fh:
            h.update(fh.read())
    h.update(("%s|%s|%s" % (extra, arch, san)).encode())
    return h.hexdigest()[:16]


def pmc_is_stale(pmc, build_id):
    """A PMC entry describes the binary it was collected on: stale unless its
    build id is the loaded library's."""
    return bool(pmc) and pmc.get("build_id") != build_id


MODELS = os.path.join(ROOT, "surfcascade_amd", "models")
# BASELINE.json configs measured on one GPU (C1 is the CPU-only plumbing case;
# C3 = C2 frame-sharded over --gpus N).  C2's batch is C3's per-GPU shard
# (256 frames / 8 GPUs = 32), so `--gpus 8` runs exactly C3; the chain
# kernel's per-launch fill and drain cost 4.5 % more per frame at 16
# (the single-frame time is reported beside).  C4 runs
# 8 4K frames per step for the same reason (6.49 vs 6.18 G windows/s at 4),
# C5 32 like C2 (3.81 vs 3.58 at 16).
CONFIGS = {
    # C1: the reference's CPU plumbing case -- no GPU; bench.py --config C1
    # prints the CPU restatement's line alone (the cpu_baseline legs)
    "C1": dict(width=640, height=480, levels=1, batch=8, model="face40_synth.cfg",
               pedestrian=False,
               metric="detection windows/sec, 640x480 single scale, CPU reference path",
               desc="C1: %dx%d frames, %d level (l=70..%d), 40x40 face cascade 10 stages / 190 weak LR; "
                    "%d seeded frames, CPU only"),
    "C2": dict(width=1920, height=1080, levels=24, batch=32, model="face40_synth.cfg",
               pedestrian=False,
               metric="detection windows/sec on 1080p 24-scale pyramid",
               desc="C2: %dx%d frames, %d-level window pyramid (l=70..%d), 40x40 face cascade "
                    "10 stages / 190 weak LR"),
    "C4": dict(width=3840, height=2160, levels=32, batch=8, model="face40_synth.cfg",
               pedestrian=False,
               metric="detection windows/sec on 4K 32-scale pyramid",
               desc="C4: %dx%d frames, %d-level window pyramid (l=70..%d), 40x40 face cascade "
                    "10 stages / 190 weak LR"),
    "C5": dict(width=1920, height=1080, levels=23, batch=32, model="ped64x128_synth.cfg",
               pedestrian=True,
               metric="detection windows/sec, 64x128 pedestrian cascade on 1080p 23-scale pyramid",
               desc="C5: %dx%d frames, %d-level window pyramid (l=64..%d, h=2l), 64x128 pedestrian "
                    "cascade 10 stages / 380 weak LR"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, help="frames per GPU per step (config default; 1 with "
                    "--shard grid)")
    ap.add_argument("--shard", default="frames", choices=("frames", "grid"),
                    help="frames: each rank scans its own frames (C3, weak scaling); grid: every "
                         "rank scans the same frames, its (level, y) rows only (SURVEY 8e "
                         "single-frame runs, strong scaling)")
    ap.add_argument("--width", type=int)
    ap.add_argument("--height", type=int)
    ap.add_argument("--levels", type=int)
    ap.add_argument("--model")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--host-steps", type=int, default=5,
                    help="steps of the host-buffer boundary leg (PCIe-inclusive rate; 0: skip)")
    ap.add_argument("--latency-steps", type=int, default=20,
                    help="steps of the batch-1 (single-frame) latency leg (0: skip)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="sc_detector_set_option (tuning / A-B runs; never changes results)")
    ap.add_argument("--detector-stream", default="torch", choices=("torch", "own"),
                    help="launch on torch's current stream (default) or the detector's own (events per call)")
    ap.add_argument("--stub", action="store_true",
                    help="test only: CPU stand-in detector + gloo (launcher test, not a measurement)")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    if a.batch is None and a.shard == "grid":
        a.batch = 1
    for k in ("batch", "width", "height", "levels"):
        if getattr(a, k) is None:
            setattr(a, k, c[k])
    if a.model is None:
        a.model = os.path.join(MODELS, c["model"])
    a.pedestrian = c["pedestrian"]
    return a


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs granted by the cgroup quota (cpu.max), or None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(frames, model_path, levels, seconds, pedestrian=False):
    """The CPU restatement (oracle/, OpenMP over levels like ObjDetector.cpp:177)
    on a bounded sample of the same frames: in-memory u8 frame -> raw detections.
    Timed at every host core this process may run on (sched_getaffinity, no
    cap: SURVEY.md 8d / BASELINE.md 2), at the cgroup CPU quota when that is
    smaller, and at 1 thread."""
    from oracle import oracle as O
    O.build()
    if pedestrian:
        casc = O.cascade_from_cfg(open(model_path).read(), tmpl_w=64, tmpl_h=128)
        params = O.Params(base_len=64, aspect_h=2, n_levels=levels)
    else:
        casc = O.cascade_from_cfg(open(model_path).read())
        params = O.Params(n_levels=levels)
    H, W = frames.shape[1:]
    grid = O.grid_count(W, H, params)
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    # every host core this process may run on (no cap), and -- when a cgroup
    # quota grants fewer CPUs than that -- the quota's worth of threads too:
    # the faster of the two is the baseline, `cores` the threads it used
    quota = cpu_quota()
    legs = [max(1, ncpu)]
    if quota is not None and int(quota) < ncpu:
        legs.append(max(1, int(quota)))
    scratch = np.zeros((H + 1) * (W + 1) * 8, np.float32)
    res = {}
    for nt in legs + [1]:
        done, t0 = 0, time.perf_counter()
        while True:
            O.detect_frame(frames[done % len(frames)], casc, params, nthreads=nt, scratch=scratch)
            done += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = time.perf_counter() - t0
        res[nt] = (done * grid / dt, done, dt)
    # the fastest leg is the baseline (C1's single level gives OpenMP over
    # levels one level to share: one thread wins there)
    threads = max(res, key=lambda nt: res[nt][0])
    v, done, dt = res[threads]
    v1, done1, dt1 = res[1]
    return {"value": v, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": "%d x %dx%d frames (%d levels, %d grid windows each), integral + adaptive-stride "
                      "detect, %.1f s at %d threads; 1 thread: %.4g windows/s (%d frames, %.1f s)"
                      % (done, W, H, levels, grid, dt, threads, v1, done1, dt1),
            "value_1thread": v1,
            "by_threads": {str(nt): res[nt][0] for nt in res},
            "nproc": os.cpu_count(), "affinity": ncpu,
            "cgroup_cpu_quota": quota, "cpu_model": cpu_model()}


def launch_ranks(args):
    """--gpus N > 1 outside torch.distributed: run N ranks of this script under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a
    child process -- nothing here has touched a GPU -- and return its exit
    status (non-zero when any rank failed or fewer than N came up)."""
    import socket
    import subprocess
    with socket.socket() as so:  # a free port for the rendezvous
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    return subprocess.call(cmd, env=env)


class StubDetector:
    """Test only (--stub): a CPU stand-in with the Detector calls bench.py
    makes.  Each frame yields a fixed set of records derived from its pixels,
    so every rank's gather and the merged count are checkable; no timing of
    it is ever a measurement."""

    def __init__(self, W, H, levels, params):
        self.W, self.H = W, H
        self.grid = sum(((W - params.level_len(i)) // 3 + 1) * ((H - params.level_len(i)) // 3 + 1)
                        for i in range(levels) if params.level_len(i) <= min(W, H))
        self.rank, self.world, self.t = 0, 1, {}

    def set_options(self, **kw):
        pass

    def set_shard(self, rank, world):
        self.rank, self.world = rank, world

    def _records(self, frames):
        import surfcascade_amd as sc
        out = []
        for f in range(frames.shape[0]):
            v = int(frames[f].sum()) % 7 + 2  # 2..8 records per frame
            for k in range(v):
                if k % self.world == self.rank:  # grid sharding: this rank's rows only
                    out.append((f, k % 3, 3 * k, 3 * k, 70, 70, 10, 0, 0.5 + k / 64))
        return np.array(out, sc.RECORD_DTYPE)

    def enqueue_device(self, frames, recs, counts):
        import surfcascade_amd as sc
        a = self._records(frames.numpy())
        cap = recs.numel() // sc.RECORD_DTYPE.itemsize
        k = min(cap, len(a))
        recs.numpy()[:k * sc.RECORD_DTYPE.itemsize] = a[:k].view(np.uint8)
        counts.zero_()
        counts[0] = len(a)
        for f in range(frames.shape[0]):
            counts[1 + f] = int((a["frame"] == f).sum())
        self.t.setdefault("windows", [0.0, 0])[1] += 1
        self.t["windows"][0] += 1.0

    def synchronize(self):
        pass

    def info(self, key):
        return self.grid if key == "grid_windows" else 0

    def set_timing(self, on=True):
        pass

    def get_timing(self):
        t, self.t = self.t, {}
        return {k: tuple(v) for k, v in t.items()} or {"windows": (0.0, 0)}

    def detect_batch(self, frames):
        return []


def cpu_only_line(args):
    """--config C1: the CPU plumbing case (BASELINE.json configs[0]) -- the
    oracle's reference loop on in-memory frames (ObjDetector.cpp:157-158,
    246-250 bracket, decode and I/O excluded), all host cores, the cgroup
    quota and 1 thread; no GPU is touched."""
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    W, H, B = args.width, args.height, args.batch
    frames = synth.make_frames(W, H, B, seed0=1000)
    params = sc.ScanParams(n_levels=args.levels)
    cb = cpu_baseline(frames, args.model, args.levels, args.cpu_seconds)
    line = {"metric": CONFIGS[args.config]["metric"], "value": cb["value"], "unit": "windows/s",
            "n_gpus": 0, "higher_is_better": True, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded %dx%d frames, seeded 10-stage 40x40 cascade)" % (W, H),
            "config": {"workload": CONFIGS[args.config]["desc"] % (W, H, args.levels,
                                                                   params.level_len(args.levels - 1), B),
                       "name": args.config, "levels": args.levels},
            "cpu_baseline": cb}
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.config == "C1":
        return cpu_only_line(args)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("error: --gpus %d but WORLD_SIZE %d: refusing to measure a different GPU count"
              % (args.gpus, world), file=sys.stderr)
        sys.exit(2)

    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    from surfcascade_amd.dist import StreamGather, enqueue_and_gather, merge_records, shard_range

    stub = args.stub
    if stub:
        dev = torch.device("cpu")
    else:
        if torch.cuda.device_count() < world:
            print("error: %d ranks but %d visible GPUs" % (world, torch.cuda.device_count()),
                  file=sys.stderr)
            sys.exit(2)
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if stub:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            print("error: process group of %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus),
                  file=sys.stderr)
            sys.exit(2)

    def sync():
        if not stub:
            det.synchronize()  # (also raises on a chain-kernel hand-off timeout)
            torch.cuda.synchronize()

    W, H, B = args.width, args.height, args.batch
    # frame sharding: rank r owns frames 1000 + r*B .. (seeds) -- C3 layout;
    # grid sharding: every rank holds frames 1000 .. and scans its rows of them
    grid_shard = args.shard == "grid"
    start = 0 if grid_shard else shard_range(B * world, world, rank)[0]
    host_frames = synth.make_frames(W, H, B, seed0=1000 + start)
    frames = torch.from_numpy(host_frames).to(dev)
    params = (sc.ScanParams.pedestrian(n_levels=args.levels) if args.pedestrian
              else sc.ScanParams(n_levels=args.levels))
    det = (StubDetector(W, H, args.levels, params) if stub
           else sc.Detector(args.model, params, device=local_rank))
    opts = {}
    for o in args.opt:
        k, v = o.split("=", 1)
        opts[k] = int(v)
    det.set_options(**opts)
    if not stub and args.detector_stream == "torch":  # stream-ordered with the bench's tensors, no event pair per call
        det.set_stream(torch.cuda.current_stream(dev))
    if grid_shard:
        det.set_shard(rank, world)
    # record buffers: grown (every rank, same size) whenever a scan finds more
    # detections than they hold -- never truncated (dist.enqueue_and_gather)
    counts = torch.zeros(1 + B, dtype=torch.int32, device=dev)
    state = {"recs": torch.zeros(256 * B * sc.RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev)}
    gathered = {}

    def step():
        if dist is not None:  # RCCL gather: counts + capacities, then records padded to the max
            gc, gr, state["recs"] = enqueue_and_gather(det, frames, state["recs"], counts, b_max=B)
            gathered["counts"], gathered["recs"] = gc, gr
        else:  # stream-ordered: the next step's launches queue behind this one, no host sync per step
            det.enqueue_device(frames, state["recs"], counts)

    def check_capacity():  # N = 1: the same frames every step -> checked around the timed loop
        n = int(counts[0].item())
        if n * sc.RECORD_DTYPE.itemsize > state["recs"].numel():
            state["recs"] = torch.zeros(n * sc.RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            step()
        gathered["counts"], gathered["recs"] = [counts.cpu().numpy()], [state["recs"].cpu()]

    for _ in range(max(1, args.warmup)):
        step()
    if dist is None:
        check_capacity()
    # N > 1, timed steps: counts and records in one buffer, one all_gather per
    # step on the stream, no host round trip (dist.StreamGather); the warm-up
    # above sized the buffers (every rank alike), one more warm step runs
    # through it, and its overflow check runs after the timed loop
    sg = None
    if dist is not None:
        sg = StreamGather(B, state["recs"].numel() // sc.RECORD_DTYPE.itemsize, dev)
        sg.step(det, frames)
        sync()
        sg.result()
    grid = det.info("grid_windows")
    det.get_timing()  # discard
    det.set_timing(True)
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if sg is not None:
            sg.step(det, frames)
        else:
            step()
    sync()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    det.set_timing(False)
    kt = det.get_timing()
    visited = det.info("visited")
    fused_frames = det.info("fused_frames")  # (before the latency / host legs replace the last call)
    # the launch shape of the timed step: chain-kernel waves per CU, and the
    # item form (1 split cells, one lane per item; 2 interleaved cells, lane pairs)
    shape = {"chain_waves": det.info("chain_waves"), "item_form": det.info("item_form")}
    if dist is None:
        check_capacity()
    else:  # the last timed step's gather (raises if any rank's buffer overflowed)
        gathered["counts"], gathered["recs"] = sg.result()
    # single-frame latency (C2 names "1080p frame"): batch-1 steps, device-resident
    lat = None
    if args.latency_steps > 0 and not grid_shard and not stub:
        one = frames[:1]
        c1 = torch.zeros(2, dtype=torch.int32, device=dev)
        r1 = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        for _ in range(3):
            det.enqueue_device(one, r1, c1)
            det.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.latency_steps):
            det.enqueue_device(one, r1, c1)
            det.synchronize()
        lat = (time.perf_counter() - t1) / args.latency_steps
        if int(c1[0].item()) * sc.RECORD_DTYPE.itemsize > r1.numel():  # (never truncates silently)
            raise RuntimeError("latency leg: %d detections overflow its record buffer" % int(c1[0]))
    # the host-buffer boundary (sc_detect_batch: pageable u8 frames in, raw
    # windows out, H2D + D2H over PCIe inside): reported beside, never `value`
    host_dt = None
    if args.host_steps > 0 and not grid_shard and not stub:
        det.detect_batch(host_frames)
        t1 = time.perf_counter()
        for _ in range(args.host_steps):
            det.detect_batch(host_frames)
        host_dt = (time.perf_counter() - t1) / args.host_steps
    rccl_world = None
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        rccl_world = dist.get_world_size()
    merged = merge_records(gathered["counts"], gathered["recs"],
                           [0 if grid_shard else shard_range(B * world, world, r)[0]
                            for r in range(world)])
    total_det = len(merged)

    if rank == 0:
        windows = grid * B * args.steps * (1 if grid_shard else world)
        value = windows / dt
        # roofline of the dominant kernel (windows): its compulsory bytes per
        # launch = the integral table read once (32 B x (W+1)(H+1) per frame)
        # and, for the frames whose integral ran inside it (fused column
        # walks), the table written once, the frame read and its strip carries
        tab_bytes = 32 * (W + 1) * (H + 1)
        ms_win, n_win = kt["windows"]
        avg_win_s = ms_win / 1e3 / max(n_win, 1)
        launches = max(n_win // max(args.steps, 1), 1)  # chain launches per step
        fused = fused_frames / launches
        win_bytes = tab_bytes * B + fused * (tab_bytes + W * H + H * ((W + 31) // 32) * 32)
        achieved = win_bytes / max(avg_win_s, 1e-12) / 1e9
        # whole pipeline (SURVEY.md 8d per-unit figure: W*H + 64 (W+1)(H+1) per frame)
        pipe_bytes = W * H + 64 * (W + 1) * (H + 1)
        pipe_s = max(sum(v[0] for v in kt.values()) / 1e3 / max(n_win, 1), 1e-12)
        pmc = pmc_for(args, B, W) if not opts and not stub else {}
        binfo = {"build_id": None} if stub else sc.build_info()
        if pmc_is_stale(pmc, binfo["build_id"]):  # collected on another build: its counters describe another binary
            pmc = {"source": pmc.get("source"), "stale": True}
        traffic, valu_insts = pmc.get("hbm_bytes_per_launch"), pmc.get("valu_insts_per_launch")
        line = {
            "metric": CONFIGS[args.config]["metric"],
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if grid_shard else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded %dx%d frames, seeded 10-stage %s cascade, thetas calibrated "
                    "on held-out frames)" % (W, H, "64x128" if args.pedestrian else "40x40"),
            "config": {"workload": (CONFIGS[args.config]["desc"] + (
                           "; window grid sharded by rows over the GPUs, %d frame(s) per step"
                           if grid_shard else "; frame-sharded, %d frames per GPU per step"))
                           % (W, H, args.levels, params.level_len(args.levels - 1), B),
                       "name": args.config,
                       "frames_per_gpu_per_step": B, "grid_windows_per_frame": grid,
                       "levels": args.levels,
                       "parallelism": ("grid-row-sharded x%d" if grid_shard else "frame-sharded dp%d")
                       % world, **shape},
            "roofline": roofline(achieved, traffic, valu_insts, avg_win_s, win_bytes, pipe_bytes * B,
                                 pipe_s, pmc, opts, fused),
            "kernel_ms_per_launch": {k: v[0] / max(v[1], 1) for k, v in kt.items()},
            "build": binfo,
            "visited_windows_last_step": visited,
            "detections_last_step": total_det,
        }
        if rccl_world is not None:
            line["process_group"] = {"backend": "gloo" if stub else "nccl (RCCL)", "world_size": rccl_world}
        if stub:
            line["stub"] = "CPU stand-in detector (launcher test): not a measurement"
        if lat is not None:
            line["latency_batch1"] = {
                "ms_per_frame": lat * 1e3, "value": grid / lat, "unit": "windows/s",
                "steps": args.latency_steps,
                "path": "one device-resident frame per step (sc_enqueue_device + synchronize)"}
        if opts:
            line["options"] = opts
        if host_dt is not None:
            line["pcie_inclusive"] = {
                "value": grid * B / host_dt, "unit": "windows/s", "ms_per_step": host_dt * 1e3,
                "steps": args.host_steps, "per": "GPU",
                "path": "sc_detect_batch: %d pageable host frames in (H2D), raw windows out (D2H)" % B}
        if not args.no_cpu and world == 1 and not stub:
            line["cpu_baseline"] = cpu_baseline(host_frames, args.model, args.levels, args.cpu_seconds,
                                                args.pedestrian)
            line["vs_cpu"] = value / world / line["cpu_baseline"]["value"]
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def pmc_for(args, B, W):
    """PMC per launch of the window kernel for this workload (profiles/
    pmc_windows.json, keyed per config; written by profiles/pmc_summary.py from
    the committed rocprofv3 passes), or {}.  The table's measured ceilings
    (top-level "ceilings") are merged into the entry."""
    pmc_path = os.path.join(ROOT, "profiles", "pmc_windows.json")
    if not os.path.exists(pmc_path):
        return {}
    with open(pmc_path) as f:
        pm = json.load(f)
    entries = pm.get("configs", {}).values() if "configs" in pm else [pm]
    for e in entries:
        if (e.get("batch") == B and e.get("width") == W and e.get("levels") == args.levels
                and e.get("config", "C2") == args.config):
            return dict(e, **{k: v for k, v in pm.get("ceilings", {}).items() if k not in e})
    return {}


def roofline(achieved, traffic, valu_insts, avg_win_s, bytes_launch, pipe_bytes, pipe_s, pmc, opts,
             fused=0):
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
         "kernel": "cascade_kernel" if opts.get("full_grid") else "chain_kernel",
         "avg_launch_ms": avg_win_s * 1e3,
         "bytes_per_launch": bytes_launch,
         "fused_integral_frames_per_launch": fused,
         "pipeline_achieved": pipe_bytes / pipe_s / 1e9,
         "pipeline_frac": pipe_bytes / pipe_s / 1e9 / HBM_PEAK_GBS,
         # beyond-L2 bytes per compulsory byte: re-reads of the table
         "traffic_ratio": traffic / bytes_launch if traffic else None,
         # compute side: VALU wave-instructions per launch (PMC SQ_INSTS_VALU)
         # over the chip's issue rate (1024 SIMDs x 0.5 wave-instr/cycle x
         # 2.4 GHz, MI355X_MICROARCH.md) x this launch's time
         "valu": (valu_insts / VALU_ISSUE_PEAK / avg_win_s) if valu_insts else None,
         "valu_insts_per_launch": valu_insts, "valu_peak_per_s": VALU_ISSUE_PEAK,
         "pmc_source": pmc.get("source")}
    if pmc.get("stale"):
        r["pmc_stale"] = ("profiles/pmc_windows.json was collected on another build (its build_id is not "
                          "the loaded library's): traffic, valu, fabric and TD fields omitted")
        return r
    c = pmc.get("counters_per_launch", {})
    # the level the kernel actually stresses: L2 misses (128-B lines from the
    # Infinity Cache / HBM, TCC_MISS) per second over the beyond-L2 gather
    # ceiling: the guide's best gather into LDS (8.6 TB/s) or the best our
    # calibration kernels measured, whichever is higher (profiles/calib)
    miss = c.get("TCC_MISS_sum")
    ceil = pmc.get("fabric_ceiling_lines_per_s")
    if miss and ceil:
        r["fabric_lines_per_s"] = miss / avg_win_s
        r["fabric_ceiling_lines_per_s"] = ceil
        r["fabric_ceiling_source"] = pmc.get("fabric_ceiling_source")
        r["fabric_frac"] = miss / avg_win_s / ceil
        hit = c.get("TCC_HIT_sum")
        r["l2_hit"] = hit / (hit + miss) if hit else None
        if pmc.get("fabric_ceiling_measured_lines_per_s"):
            r["fabric_ceiling_measured_lines_per_s"] = pmc["fabric_ceiling_measured_lines_per_s"]
    # the texture data path: busy cycles (transfer + waits for data) and the
    # transfer alone (16 cycles per load instruction) over the launch's cycles
    # (GRBM_GUI_ACTIVE summed over the 8 XCDs), per CU
    cyc = c.get("GRBM_GUI_ACTIVE")
    if cyc and c.get("SQ_INSTS_VMEM_RD"):
        cyc_xcd = cyc / 8.0
        r["td_frac"] = c["SQ_INSTS_VMEM_RD"] * TD_CYCLES_PER_LOAD / (N_CUS * cyc_xcd)
        if c.get("TD_TD_BUSY_sum"):
            r["td_busy_frac"] = c["TD_TD_BUSY_sum"] / (N_CUS * cyc_xcd)
        r["clock_ghz_from_grbm"] = cyc_xcd / (pmc.get("avg_launch_ms_pmc") or avg_win_s * 1e3) / 1e6
    return r


if __name__ == "__main__":
    main()
