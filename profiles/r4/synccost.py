"""One-frame call overhead: where the ~0.04 ms between the kernels' sum and
bench.py's latency_batch1 goes.  Interleaved legs of 200 device-resident
1080p frames each:
  api    enqueue_device + Detector.synchronize (bench.py's latency leg)
  torch  enqueue_device + torch.cuda.synchronize (no watchdog-word read)
  raw    sc_enqueue_device alone (no stream-order events) + sc_synchronize
  null_stream / side_stream  the api leg with the detector on torch's null
         stream / a side stream made current (sc_detector_set_stream: no events)
  kern   the kernels' own time (HIP events, Detector timing)"""
import ctypes, json, os, statistics, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import surfcascade_amd as sc
from surfcascade_amd import synth

dev = torch.device("cuda", 0)
frames = torch.from_numpy(synth.make_frames(1920, 1080, 1, seed0=1000)).to(dev)
import os
import bench
det = sc.Detector(os.path.join(bench.MODELS, "face40_synth.cfg"), sc.ScanParams(n_levels=24), device=0)
c1 = torch.zeros(2, dtype=torch.int32, device=dev)
r1 = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
lib = sc.load_library()
n, H, W, rs = det._device_frames(frames)

def api():
    det.enqueue_device(frames, r1, c1); det.synchronize()

def tsync():
    det.enqueue_device(frames, r1, c1); torch.cuda.synchronize()

def raw():
    sc._check(lib.sc_enqueue_device(det._h, frames.data_ptr(), n, W, H, rs, r1.data_ptr(), 1 << 14, c1.data_ptr()))
    sc._check(lib.sc_synchronize(det._h))

side = torch.cuda.Stream(device=dev)
own = det.stream_ptr

def on(stream):  # the detector on torch's stream `stream`, made current
    def leg():
        with torch.cuda.stream(stream):
            det.set_stream(stream)
            det.enqueue_device(frames, r1, c1); det.synchronize()
            det.set_stream(None)
    return leg

legs = {"api": api, "torch": tsync, "raw": raw}
if hasattr(det, "set_stream"):
    legs["null_stream"] = on(torch.cuda.default_stream(dev))
    legs["side_stream"] = on(side)
res = {k: [] for k in legs}
for f in legs.values():
    for _ in range(10): f()
for rnd in range(3):
    for k, f in legs.items():
        if k.endswith("_stream"):  # the switch outside the timed loop
            st = torch.cuda.default_stream(dev) if k == "null_stream" else side
            with torch.cuda.stream(st):
                det.set_stream(st)
                t0 = time.perf_counter()
                for _ in range(200):
                    det.enqueue_device(frames, r1, c1); det.synchronize()
                res[k].append((time.perf_counter() - t0) / 200 * 1e3)
                det.set_stream(None)
            continue
        t0 = time.perf_counter()
        for _ in range(200): f()
        res[k].append((time.perf_counter() - t0) / 200 * 1e3)
det.get_timing(); det.set_timing(True)
for _ in range(50): api()
kt = det.get_timing(); det.set_timing(False)
out = {k: {"min_ms": min(v), "median_ms": statistics.median(v)} for k, v in res.items()}
out["kernels"] = kt
print(json.dumps(out))
