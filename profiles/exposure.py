"""Exposure of the C2 bench frames to the unpinned third-party arithmetic
(VERDICT r1 Next #6): over the windows the reference visits on
the 16 bench frames (seeds 1000..1015, 24 levels, the synthetic face cascade),
count the weak evaluations whose f64 sigmoid lies within 2 / 16 ulp of an f32
rounding boundary (MSVC CRT exp vs glibc / OCML, LogisticRegression.cpp:65),
the stage decisions within one f32 ulp of theta (ObjDetector.cpp:197), the
final scores within one f32 ulp of 0.5 (:214), and the integral values above
2^24 (cv::integral's order-sensitive regime).  CPU only (oracle).

    python profiles/exposure.py [--frames 16] [--out profiles/r2/exposure.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--out")
    a = ap.parse_args()
    from oracle import oracle as O
    from surfcascade_amd import synth
    casc = O.cascade_from_cfg(open(os.path.join(ROOT, "surfcascade_amd/models/face40_synth.cfg")).read())
    tot = np.zeros(8, np.int64)
    for f in range(a.frames):
        img = synth.make_frame(1920, 1080, 1000 + f)
        tot += O.exposure(O.integral(img), casc, O.Params(n_levels=24))
    keys = ["weak_evals", "sigmoid_within_2ulp_of_f32_boundary", "sigmoid_within_16ulp_of_f32_boundary",
            "stage_decisions", "stage_score_within_1ulp_of_theta", "final_scores",
            "final_score_within_1ulp_of_0.5", "integral_values_above_2^24"]
    res = {k: int(v) for k, v in zip(keys, tot)}
    res["integral_values"] = a.frames * 1921 * 1081 * 8
    res["frames"] = a.frames
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
