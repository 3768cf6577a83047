"""One-frame call cost split (round 5): interleaved legs of 300 device-resident
1080p frames each, the detector on torch's current stream (bench.py's form):
  api    Detector.enqueue_device + Detector.synchronize (bench.py's latency leg)
  raw    sc_enqueue_device + sc_synchronize through ctypes with precomputed
         arguments (the C ABI alone: no Python validation)
  queued 300 enqueue_device calls, one synchronize (no host round trip per
         frame: the GPU's time per frame, launch gaps included)
  kern   the kernels' own time (HIP events, Detector timing)"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import surfcascade_amd as sc  # noqa: E402
from surfcascade_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
frames = torch.from_numpy(synth.make_frames(1920, 1080, 1, seed0=1000)).to(dev)
model = os.path.join(os.path.dirname(sc.__file__), "models", "face40_synth.cfg")
det = sc.Detector(model, sc.ScanParams(n_levels=24), device=0)
det.set_stream(torch.cuda.current_stream(dev))
c1 = torch.zeros(2, dtype=torch.int32, device=dev)
r1 = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
lib = sc.load_library()
n, H, W, rs = det._device_frames(frames)
args = (det._h, frames.data_ptr(), n, W, H, rs, r1.data_ptr(), (1 << 20) // 40, c1.data_ptr())
N = 300


def api():
    for _ in range(N):
        det.enqueue_device(frames, r1, c1)
        det.synchronize()


def raw():
    for _ in range(N):
        lib.sc_enqueue_device(*args)
        lib.sc_synchronize(det._h)


def queued():
    for _ in range(N):
        det.enqueue_device(frames, r1, c1)
    det.synchronize()


legs = {"api": api, "raw": raw, "queued": queued}
for f in legs.values():
    f()
res = {k: [] for k in legs}
for _ in range(3):
    for k, f in legs.items():
        t0 = time.perf_counter()
        f()
        res[k].append((time.perf_counter() - t0) / N * 1e3)
det.get_timing()
det.set_timing(True)
for _ in range(100):
    det.enqueue_device(frames, r1, c1)
    det.synchronize()
det.set_timing(False)
kt = det.get_timing()
out = {k: {"min_ms": min(v), "median_ms": statistics.median(v)} for k, v in res.items()}
out["kernels_ms_per_call"] = {k: v[0] / max(v[1], 1) for k, v in kt.items() if v[1]}
out["build"] = sc.build_info()
print(json.dumps(out))
