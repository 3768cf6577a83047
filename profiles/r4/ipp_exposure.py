"""How much could an IPP-routed cv::integral change the detections?
(DenseSURFFeatureExtractor.cpp:75; SURVEY.md 8c: OpenCV 3.0.0's Windows build
may route integral 8U->32F through IPP, whose summation order is not
published -- the one part of row (c) still unpinned.)

The oracle follows OpenCV's scalar integral_: S[y+1][x] = fl32(S[y][x] +
(float)R_y[x]), sequential in y (App. A.2).  Two plausible alternative orders
are checked: "exact" -- the exact integer sum rounded once to f32 (any order
that accumulates exactly, e.g. in 32-bit integers, then converts) -- and
"columns_first" -- the transposed recurrence, exact column prefixes added
along x in f32: S[y][x+1] = fl32(S[y][x] + (float)C_x[y]).  All agree
wherever the sums stay below 2^24.  For the C2 bench frames this script builds
both tables, runs the reference's detect loop on each (oracle, same
cascade), and counts what differs: table values, per-window stage
decisions, visited windows, detections and their scores.
Writes profiles/r4/ipp_exposure.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from surfcascade_amd import synth  # noqa: E402

O.build()
casc = O.cascade_from_cfg(open(os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")).read())
W, H, L = 1920, 1080, 24
params = O.Params(n_levels=L)
layout, _ = O.grid_layout(W, H, params)


def exact_then_round(img):
    g = O.gradients(img).astype(np.int64)          # [8, H, W] planes (T2bFilter)
    S = np.zeros((H + 1, W + 1, 8), np.float32)
    c = g.cumsum(axis=2).cumsum(axis=1)             # exact 2-D prefix sums
    S[1:, 1:, :] = np.moveaxis(c, 0, -1).astype(np.float32)  # one RNE rounding per value
    return S


def columns_first(img):
    g = O.gradients(img).astype(np.int64)
    C = np.moveaxis(g.cumsum(axis=1), 0, -1).astype(np.float32)  # [H, W, 8] exact column prefixes (< 2^24)
    S = np.zeros((H + 1, W + 1, 8), np.float32)
    acc = np.zeros((H, 8), np.float32)
    for x in range(W):
        acc = acc + C[:, x, :]  # f32, sequential in x
        S[1:, x + 1, :] = acc
    return S


def key(d):
    return sorted((int(r["level"]), int(r["y"]), int(r["x"]), float(r["score"])) for r in d)


ALTS = {"exact": exact_then_round, "columns_first": columns_first}
tot = {}
for name in ALTS:
    tot[name] = {"frames": 0, "table_values": 0, "values_differ": 0, "values_above_2_24": 0, "grid_windows": 0,
                 "stage_decisions_differ": 0, "last_scores_differ": 0, "visited_differ": 0, "detections_ref": 0,
                 "detections_alt": 0, "detections_differ": 0, "detection_windows_differ": 0,
                 "max_score_diff_common": 0.0}
for seed in range(1000, 1016):
    img = synth.make_frame(W, H, seed)
    T = O.integral(img)
    p, s = O.eval_grid(T, casc, params)
    v, _ = O.walk_grid(p, s, layout, casc.n_stages, 0.5)
    d, _ = O.detect(T, casc, params)
    kd = set(key(d))
    for name, fn in ALTS.items():
        t = tot[name]
        A = fn(img)
        t["frames"] += 1
        t["table_values"] += T.size
        t["values_differ"] += int((T.view(np.uint32) != A.view(np.uint32)).sum())
        t["values_above_2_24"] += int((T >= 2 ** 24).sum())
        pa, sa = O.eval_grid(A, casc, params)
        t["grid_windows"] += len(p)
        t["stage_decisions_differ"] += int((p != pa).sum())
        t["last_scores_differ"] += int((s.view(np.uint32) != sa.view(np.uint32)).sum())
        va, _ = O.walk_grid(pa, sa, layout, casc.n_stages, 0.5)
        t["visited_differ"] += int((v != va).sum())
        da, _ = O.detect(A, casc, params)
        t["detections_ref"] += len(d)
        t["detections_alt"] += len(da)
        ka = set(key(da))
        t["detections_differ"] += len(kd ^ ka)  # window or score bits differ
        wd = {k[:3]: k[3] for k in kd}
        wa = {k[:3]: k[3] for k in ka}
        t["detection_windows_differ"] += len(set(wd) ^ set(wa))  # a window detected under one order only
        common = set(wd) & set(wa)
        if common:
            t["max_score_diff_common"] = max(t["max_score_diff_common"], max(abs(wd[k] - wa[k]) for k in common))
    print(seed, {n: (tot[n]["values_differ"], tot[n]["stage_decisions_differ"], tot[n]["detection_windows_differ"],
                     tot[n]["max_score_diff_common"]) for n in ALTS}, flush=True)
json.dump(tot, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ipp_exposure.json"), "w"), indent=1)
print(json.dumps(tot, indent=1))
