"""Measurements for the SURVEY.md 8f rows built after the hot path (one JSON line each).

  f1 groupRectangles: host C++ (sc_group_rectangles) vs the oracle's all-pairs
     restatement, on clustered synthetic detections of a 1080p frame.
  f3 hard-negative mining (FillNegSamples scan): stride-10 windows/s on 1080p
     frames through the miner (integral + cascade + selection), and descriptor
     throughput (608 x 32 floats per candidate) -- next to the oracle on the host.

    python profiles/bench_next_rows.py [--frames 8] [--cpu-seconds 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def clustered_rects(rng, n_clusters, per, W=1920, H=1080):
    import surfcascade_amd as sc
    rows = []
    for _ in range(n_clusters):
        l = int(rng.integers(70, 500))
        cx, cy = int(rng.integers(0, W - l)), int(rng.integers(0, H - l))
        for _ in range(int(rng.integers(1, per + 1))):
            d = int(rng.integers(-6, 7))
            rows.append((cx + int(rng.integers(-8, 9)), cy + int(rng.integers(-8, 9)), l + d, l + d,
                         float(rng.random())))
    r = np.zeros(len(rows), sc.RECT_DTYPE)
    for i, t in enumerate(rows):
        r[i] = t
    return r


def timed(fn, min_s=1.0):
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            return dt / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    a = ap.parse_args()
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    from oracle import oracle as O
    O.build()

    # f1: groupRectangles
    rng = np.random.default_rng(0)
    r = clustered_rects(rng, 400, 12)
    assert sc.groupRectangles(r).tobytes() == O.group_rectangles(r).tobytes()
    t_sc = timed(lambda: sc.groupRectangles(r))
    t_or = timed(lambda: O.group_rectangles(r), min_s=a.cpu_seconds)
    print(json.dumps({"row": "f1 groupRectangles", "rects": len(r), "ms_product": t_sc * 1e3,
                      "ms_oracle_all_pairs": t_or * 1e3, "speedup": t_or / t_sc,
                      "groups": int(len(sc.groupRectangles(r)))}), flush=True)

    # f3: mining scan on 1080p frames
    import torch  # noqa: F401  (one HIP runtime: torch first)
    frames = synth.make_frames(1920, 1080, a.frames, seed0=1000)
    c = O.cascade_from_cfg(open(os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")).read())
    for label, model, cap, feats in (("first round (no stage), 4096 descriptors", None, 4096, True),
                                     ("face40 cascade, candidates only", "face", 1 << 20, False)):
        m = sc.Miner(os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
                     if model else None)
        m.mine(frames[0], cap, features=feats)  # warm-up
        t0 = time.perf_counter()
        tot = 0
        for f in frames:
            w, ft, n = m.mine(f, cap, features=feats)
            tot += n
        dt = (time.perf_counter() - t0) / len(frames)
        T = O.integral(frames[0])
        casc = c if model else O.empty_cascade()
        t1 = time.perf_counter()
        _, _, n_or = O.mine(T, casc, cap if feats else 0, features=feats, nthreads=16)
        dt_or = time.perf_counter() - t1
        grid = O.grid_count(1920, 1080, O.Params(base_len=40, step=10, n_levels=-1))
        print(json.dumps({"row": "f3 FillNegSamples scan", "case": label, "frame": "1920x1080",
                          "grid_windows": grid, "candidates_per_frame": tot / len(frames),
                          "ms_per_frame_gpu_incl_host_copies": dt * 1e3,
                          "windows_per_s_gpu": grid / dt,
                          "descriptors_per_s_gpu": (min(tot / len(frames), cap) / dt) if feats else None,
                          "ms_per_frame_oracle_16thr": dt_or * 1e3,
                          "speedup_vs_oracle": dt_or / dt}), flush=True)


if __name__ == "__main__":
    main()
