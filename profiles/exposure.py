"""Exposure of the C2 bench frames to the unpinned third-party arithmetic
(VERDICT r1 Next #6): over the windows the reference visits on
the 16 bench frames (seeds 1000..1015, 24 levels, the synthetic face cascade),
count the weak evaluations whose f64 sigmoid lies within 2 / 16 ulp of an f32
rounding boundary (MSVC CRT exp vs glibc / OCML, LogisticRegression.cpp:65),
the stage decisions within one f32 ulp of theta (ObjDetector.cpp:197), the
final scores within one f32 ulp of 0.5 (:214), and the integral values above
2^24 (cv::integral's order-sensitive regime).  CPU only (oracle).

With --exp (VERDICT r2 Next 6) it also runs the exact exp() sensitivity
(oracle sco_exp_sensitivity): every visited window's weak evaluations
recomputed with exp(-z) one f64 ulp below / above glibc's, the windows whose
result changes re-evaluated, their rows' x chains re-walked; and it checks with
mpmath (50 digits) that the glibc-based f32 sigmoid of every flipping
evaluation equals the correctly rounded one.

    python profiles/exposure.py [--frames 16] [--exp] [--out profiles/r3/exposure.json]
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
    ap.add_argument("--exp", action="store_true", help="exact exp() sensitivity + mpmath check")
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
    if a.exp:
        res["exp_sensitivity"] = exp_sensitivity(O, casc, synth, a.frames)
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


def f32_round(mpmath, x):
    """Correctly rounded f32 of the mpmath value x (no double rounding through
    f64: these values sit next to f32 midpoints by selection)."""
    f = np.float32(float(x))
    for _ in range(2):
        lo, hi = np.nextafter(f, np.float32(-np.inf)), np.nextafter(f, np.float32(np.inf))
        m_lo = (mpmath.mpf(float(lo)) + mpmath.mpf(float(f))) / 2
        m_hi = (mpmath.mpf(float(hi)) + mpmath.mpf(float(f))) / 2
        if x < m_lo:
            f = lo
        elif x > m_hi:
            f = hi
        elif x == m_lo or x == m_hi:
            raise AssertionError("exact f32 tie at %r" % x)
        else:
            return f
    raise AssertionError("f32 rounding did not settle at %r" % x)


def exp_sensitivity(O, casc, synth, frames):
    """Exact bound of what an exp() one f64 ulp off glibc's changes."""
    import math

    import mpmath
    mpmath.mp.dps = 50
    keys = ["weak_evals", "evals_with_flipping_alternative", "flipping_alternatives",
            "alternatives_flipping_a_stage_decision", "alternatives_changing_window_result",
            "alternatives_changing_stride", "detections_appearing_or_vanishing",
            "windows_with_two_or_more_flips", "detections_with_other_score_bits"]
    tot = np.zeros(9, np.int64)
    zs = []
    for f in range(frames):
        img = synth.make_frame(1920, 1080, 1000 + f)
        st, z = O.exp_sensitivity(O.integral(img), casc, O.Params(n_levels=24))
        tot += st
        zs.extend(z.tolist())
    out = {k: int(v) for k, v in zip(keys, tot)}
    # mpmath: correctly rounded f32 of the exact sigmoid vs the glibc path
    glibc_ne_exact, exp_not_cr = 0, 0
    for z in zs:
        e = math.exp(-z)
        f_glibc = np.float32(1.0 / (1.0 + e))
        ex = 1 / (1 + mpmath.exp(-mpmath.mpf(z)))
        f_exact = f32_round(mpmath, ex)
        glibc_ne_exact += int(f_glibc != f_exact)
        exp_not_cr += int(mpmath.mpf(e) != mpmath.mpf(float(mpmath.nstr(mpmath.exp(-mpmath.mpf(z)), 40))))
    out["mpmath_checked_evals"] = len(zs)
    out["glibc_f32_sigmoid_not_correctly_rounded"] = glibc_ne_exact
    out["glibc_exp_not_correctly_rounded"] = exp_not_cr
    out["model"] = ("MSVC CRT exp within one f64 ulp of glibc's (both faithful); each weak "
                    "evaluation's alternatives exp(-z) -/+ 1 ulp through 1.0/(1.0 + e) in f64 "
                    "(LogisticRegression.cpp:65), one alternative at a time, rows re-walked")
    return out


if __name__ == "__main__":
    main()
