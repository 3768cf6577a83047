"""Round 6 experiment (not the bench): C2 steps on ONE detector and stream
against steps alternating between TWO detectors on two streams, so a call's
chain kernel can start on the CUs the previous call's kernel frees in its
drain (and its pre-integrated frames' kernels run inside that drain).
Prints one JSON line: ms per step of each form (interleaved repeats) and the
last step's detection counts of every detector (they must agree).

    python3 profiles/r6/overlap.py [--steps 20] [--repeats 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--repeats", type=int, default=3)
    a = ap.parse_args()
    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    W, H, B, L = 1920, 1080, 32, 24
    dev = torch.device("cuda", 0)
    frames = torch.from_numpy(synth.make_frames(W, H, B, seed0=1000)).to(dev)
    model = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    dets, recs, counts = [], [], []
    for i in range(2):
        d = sc.Detector(model, sc.ScanParams(n_levels=L), device=0)
        d.set_stream(streams[i])
        dets.append(d)
        recs.append(torch.zeros(4096 * B * sc.RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev))
        counts.append(torch.zeros(1 + B, dtype=torch.int32, device=dev))

    def run(n_det, steps):
        for s in range(steps):
            k = s % n_det
            dets[k].enqueue_device(frames, recs[k], counts[k])

    def sync():
        for d in dets:
            d.synchronize()
        torch.cuda.synchronize()

    run(2, 4)
    sync()
    res = {"one": [], "two": []}
    for _ in range(a.repeats):
        for form, nd in (("one", 1), ("two", 2)):
            sync()
            t0 = time.perf_counter()
            run(nd, a.steps)
            sync()
            res[form].append((time.perf_counter() - t0) * 1e3 / a.steps)
    n = [int(c[0].item()) for c in counts]
    grid = dets[0].info("grid_windows")
    out = {"ms_per_step": res, "detections": n, "grid_windows_per_step": grid,
           "g_windows_s": {f: grid / (min(v) * 1e-3) / 1e9 for f, v in res.items()},
           "build": sc.build_info()["build_id"]}
    print(json.dumps(out))
    if len(set(n)) != 1:
        sys.exit(1)


if __name__ == "__main__":
    main()
