"""Probe: do two detectors on their own streams overlap one batch's integral
and chain-kernel fill with the previous batch's chain-kernel drain?

Modes (C2: 32 device-resident 1080p frames per step, face cascade):
  single  one detector, enqueue + synchronize per step (bench.py's N=1 step)
  queued  one detector, K enqueues back to back, one synchronize
  dual    detectors A/B alternate, each on its own torch stream; step k+1 is
          enqueued before step k is synchronized

usage (GPU box): python profiles/r2/overlap/overlap_probe.py [--steps 12] [--frames 32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth

    cfg = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
    frames = torch.from_numpy(np.stack(synth.make_frames(1920, 1080, a.frames, seed0=1000))).to("cuda:0")
    n = a.frames
    cap = 1 << 20

    def mk():
        d = sc.Detector(cfg, sc.ScanParams())
        s = torch.cuda.Stream()
        recs = torch.empty(cap * 40, dtype=torch.uint8, device="cuda:0")
        counts = torch.zeros(1 + n, dtype=torch.int32, device="cuda:0")
        return d, s, recs, counts

    A, B = mk(), mk()

    def enq(X):
        d, s, recs, counts = X
        with torch.cuda.stream(s):
            d.enqueue_device(frames, recs, counts)

    def single(K):
        for _ in range(K):
            enq(A)
            A[0].synchronize()

    def queued(K):
        for _ in range(K):
            enq(A)
        A[0].synchronize()

    def dual(K):
        X = [A, B]
        enq(X[0])
        for k in range(1, K):
            enq(X[k & 1])
            X[(k - 1) & 1][0].synchronize()
        X[(K - 1) & 1][0].synchronize()

    for f in (single, queued, dual):
        f(2)  # warm-up: geometry, buffers
    torch.cuda.synchronize()
    c0 = A[3].clone()
    out = {}
    for name, f in (("single", single), ("queued", queued), ("dual", dual)):
        best = 1e30
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f(a.steps)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / a.steps)
        out[name] = best * 1e3
        print(name, "ms/step %.3f" % (best * 1e3), flush=True)
    assert torch.equal(A[3], c0) and torch.equal(B[3], c0), "counts differ between detectors / runs"
    g = 3729192 * n
    out.update({"frames_per_step": n, "G_windows_per_s": {k: g / v / 1e6 for k, v in out.items()
                                                          if isinstance(v, float)}})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
