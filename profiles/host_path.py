"""Where the host-boundary call (sc_detect_batch) spends its time, C2 batch of
16 x 1080p frames: device-resident enqueue+sync, sc_detect_device (host
records out), sc_detect_batch (pageable frames in), and the H2D copy alone.
Run on the GPU box:  python3 profiles/host_path.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import surfcascade_amd as sc  # noqa: E402
from surfcascade_amd import synth  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    B = int(os.environ.get("B", "16"))
    host = synth.make_frames(1920, 1080, B)
    dev = torch.from_numpy(host).cuda()
    det = sc.Detector(os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg"),
                      sc.ScanParams(n_levels=24), device=0)
    recs = torch.zeros(256 * B * sc.RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    counts = torch.zeros(1 + B, dtype=torch.int32, device="cuda")
    pinned = torch.from_numpy(host).pin_memory()
    if os.environ.get("MODE") == "batch":  # API-trace runs: the host-buffer call only
        print(json.dumps({"detect_batch_ms": timed(lambda: det.detect_batch(host))}), flush=True)
        return
    res = {
        "enqueue_sync_ms": timed(lambda: (det.enqueue_device(dev, recs, counts), det.synchronize())),
        "detect_device_ms": timed(lambda: det.detect_device(dev)),
        "detect_batch_ms": timed(lambda: det.detect_batch(host)),
        "h2d_pinned_torch_ms": timed(lambda: dev.copy_(pinned, non_blocking=True)),
        "h2d_pageable_torch_ms": timed(lambda: dev.copy_(torch.from_numpy(host))),
        "np_zeros_out_ms": timed(lambda: np.zeros(1 << 18, sc.WINDOW_DTYPE)),
        "host_memcpy_ms": timed(lambda: np.copyto(pinned.numpy(), host)),
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
