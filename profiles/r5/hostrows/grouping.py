"""Row f1 measured (round 5): cv::groupRectangles(wins, 0s, scores, 2, 0.2)
(ObjDetector.cpp:223-225) on real detection sets -- the raw windows the
detect path returns for synthetic 1080p frames x 24 levels under the
calibrated model and under permissive thetas (many overlapping windows) --
timed for the product's host C++ (sc_group_rectangles: x-sorted sweep +
union-find) against the oracle's all-pairs restatement (sc_oracle_group.c),
results compared byte for byte.  CPU only (the detections come from the
oracle's detect, so no GPU is needed).

    python profiles/r5/hostrows/grouping.py [--frames 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def best_time(f, reps):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4)
    a = ap.parse_args()
    from oracle import oracle as O
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    with open(os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")) as f:
        text = f.read()
    base = O.cascade_from_cfg(text)
    out = {"frames": a.frames, "sets": []}
    for label, theta in (("model", None), ("permissive 0.45", 0.45)):
        t = base.theta if theta is None else np.full(base.n_stages, theta, np.float32)
        casc = O.cascade_from_cfg(synth.write_cfg(synth.cascade_tree(base.n_weak, t, base.patch_index, base.w,
                                                                     base.bias)))
        prm = O.Params(n_levels=24)
        for k in range(a.frames):
            img = synth.make_frame(1920, 1080, 1000 + k)
            wins, _ = O.detect(O.integral(img), casc, prm)
            r = sc._as_rects(wins)
            mine = sc.groupRectangles(r)
            ref = O.group_rectangles(r)
            same = mine.tobytes() == ref.tobytes()
            reps = 5 if len(r) < 20000 else 2
            t_sc = best_time(lambda: sc.groupRectangles(r), reps)
            t_or = best_time(lambda: O.group_rectangles(r), reps if len(r) < 5000 else 1)
            row = {"thetas": label, "frame": 1000 + k, "windows": int(len(r)), "groups": int(len(mine)),
                   "equal": bool(same), "product_ms": t_sc * 1e3, "all_pairs_ms": t_or * 1e3}
            out["sets"].append(row)
            print(json.dumps(row), flush=True)
            assert same
    print(json.dumps(out))


if __name__ == "__main__":
    main()
