"""Generate the seeded synthetic cascades (SURVEY.md 8d "Models").

Weights are random (w ~ N(0,1), w[32] ~ N(0,0.5), bias 1.0, patch_index
uniform over the template's dense patches); each stage's theta is calibrated
on calibration frames (seeds 9000+, never benchmarked) so that a target
fraction of the windows reaching that stage survives it.  Scores come from the
CPU restatement (oracle/), i.e. this is fixture generation, not product code.

    python tests/golden/make_models.py      # rewrites surfcascade_amd/models/*.cfg
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from surfcascade_amd import synth  # noqa: E402

MODELS = {
    "face40_synth": dict(tmpl=(40, 40), base_len=70, aspect_h=1, n_levels=24,
                         n_weak=[4, 6, 8, 12, 16, 20, 24, 28, 32, 40], seed=42),
    "ped64x128_synth": dict(tmpl=(64, 128), base_len=64, aspect_h=2, n_levels=23,
                            n_weak=[8, 12, 16, 24, 32, 40, 48, 56, 64, 80], seed=43),
}
SURVIVAL = [0.5, 0.4] + [0.3] * 8
CAL_SEEDS = [9000, 9001, 9002, 9003]
MAX_WINDOWS = 600_000


def calibrate(spec, rng):
    tw, th = spec["tmpl"]
    n_patch = len(O.extract_patches(tw, th))
    K = sum(spec["n_weak"])
    pidx = rng.integers(0, n_patch, size=K).astype(np.int32)
    w = rng.normal(0, 1, size=(K, 33)).astype(np.float32)
    w[:, 32] = rng.normal(0, 0.5, size=K).astype(np.float32)
    bias = np.ones(K, np.float64)
    S = len(spec["n_weak"])
    theta = np.full(S, -1.0, np.float32)
    casc = O.Cascade(tw, th, np.array(spec["n_weak"], np.int32), theta, pidx, w, bias)
    params = O.Params(base_len=spec["base_len"], aspect_h=spec["aspect_h"],
                      n_levels=spec["n_levels"])
    for s in range(S):
        scores_all = []
        for seed in CAL_SEEDS:
            img = synth.make_frame(1920, 1080, seed)
            T = O.integral(img)
            layout, st = O.grid_layout(1920, 1080, params)
            pm = O.prefilter_mask(T, params)
            idx = np.nonzero(pm)[0]
            sub = np.random.default_rng(seed).choice(idx, size=min(len(idx), MAX_WINDOWS // len(CAL_SEEDS)),
                                                     replace=False)
            sub.sort()
            L, X, Y = [], [], []
            for (_i, l, lh, nx, ny, b) in layout:
                sel = sub[(sub >= b) & (sub < b + nx * ny)] - b
                L.append(np.full(len(sel), l)); Y.append((sel // nx) * st); X.append((sel % nx) * st)
            L, X, Y = np.concatenate(L), np.concatenate(X), np.concatenate(Y)
            alive = np.ones(len(L), bool)
            for q in range(s):
                sc = O.stage_score_batch(T, casc, L[alive], X[alive], Y[alive], q)
                keep = sc.astype(np.float64) >= np.float64(casc.theta[q])
                a = np.nonzero(alive)[0]
                alive[a[~keep]] = False
            scores_all.append(O.stage_score_batch(T, casc, L[alive], X[alive], Y[alive], s))
        sc = np.concatenate(scores_all)
        casc.theta[s] = np.float32(np.quantile(sc, 1.0 - SURVIVAL[s]))
        print("  stage %d: %d windows reach it, theta=%.7g" % (s, len(sc), casc.theta[s]), flush=True)
    return casc


def main():
    outdir = os.path.join(ROOT, "surfcascade_amd", "models")
    os.makedirs(outdir, exist_ok=True)
    for name, spec in MODELS.items():
        print(name, flush=True)
        casc = calibrate(spec, np.random.default_rng(spec["seed"]))
        tree = synth.cascade_tree(casc.n_weak, casc.theta, casc.patch_index, casc.w, casc.bias,
                                  meta={"stage_fpr": SURVIVAL})
        with open(os.path.join(outdir, name + ".cfg"), "w") as f:
            f.write(synth.write_cfg(tree))


if __name__ == "__main__":
    main()
