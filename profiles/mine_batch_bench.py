"""Row f3 (FillNegSamples scan) throughput: the batched miner against the
one-image-per-call form, 1080p frames, face cascade (candidates only) and
the first round (every window, descriptors kept on the device).

usage (GPU box): python profiles/mine_batch_bench.py [--frames 16] [--reps 5]
Prints one JSON line per case; windows/s counts the stride-10 grid windows
of every scanned image (the scan's own unit, DenseSURFFeatureExtractor.cpp:
132-190)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    from oracle import oracle as O

    cfg = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
    frames = synth.make_frames(1920, 1080, a.frames, seed0=1000)
    dev = torch.from_numpy(np.stack(frames)).to("cuda:0")
    grid = O.grid_count(1920, 1080, O.Params(base_len=40, step=10, n_levels=-1))

    def best(fn):
        fn()  # warm-up (geometry, buffers)
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        return min(ts), r

    out = []
    m = sc.Miner(cfg)
    t_dev, (w, counts) = best(lambda: m.mine_batch_device(dev, 1 << 20))
    t_host, _ = best(lambda: m.mine_batch(frames, 1 << 20, features=False))
    t_loop, _ = best(lambda: [m.mine(f, 1 << 20, features=False) for f in frames])
    n = a.frames
    out.append({"row": "f3 FillNegSamples scan", "case": "face40 cascade, candidates only",
                "frame": "1920x1080", "images": n, "grid_windows_per_image": grid,
                "candidates": int(counts.sum()),
                "batch_device": {"ms_per_image": t_dev / n * 1e3, "windows_per_s": grid * n / t_dev},
                "batch_host_frames": {"ms_per_image": t_host / n * 1e3, "windows_per_s": grid * n / t_host},
                "one_image_per_call": {"ms_per_image": t_loop / n * 1e3, "windows_per_s": grid * n / t_loop}})
    m0 = sc.Miner(None)
    cap = 4096 * n
    feats = torch.empty(cap * m0.n_patches * 32, dtype=torch.float32, device="cuda:0")
    t_fr, (w, counts) = best(lambda: m0.mine_batch_device(dev, cap, feats))
    out.append({"row": "f3 FillNegSamples scan", "case": "first round, %d descriptors kept on the device" % cap,
                "frame": "1920x1080", "images": n, "candidates": int(counts.sum()),
                "ms_per_image": t_fr / n * 1e3, "windows_per_s": grid * n / t_fr,
                "descriptors_per_s": min(int(counts.sum()), cap) / t_fr})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
