"""Round 5 parity soak (beyond the suite's seeded sweep): N random cases
through the C ABI against the oracle -- frame size, frames per call, levels,
base window, step, prefilter factor, stride threshold, permissive or model
thetas, face or pedestrian model, and the schedule options that must never
change a bit (chain waves, dequeue sub-queues, integral fusion and prebuilt
frames, the cell layout, task slots per wave, speculation depth); about one
case in ten is a single large frame (2048-4200 px wide).  Every frame: visited count, visited set and detections (f64 scores);
every 4th case also the integral table and per-window stage / score bits.

    python tests/soak_parity.py [--cases 300] [--seed 9000] [--out F]

(Not collected by pytest: a GPU soak run by hand; results in profiles/r5/soak/.)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def det_set(arr):
    return sorted((int(r["level"]), int(r["y"]), int(r["x"]), int(r["w"]), int(r["h"]),
                   int(r["stage"]), float(r["score"])) for r in arr)


def load_models(O):
    models = {}
    for name, tw, th in (("face40_synth.cfg", 40, 40), ("ped64x128_synth.cfg", 64, 128)):
        with open(os.path.join(ROOT, "surfcascade_amd", "models", name)) as f:
            models[name] = O.cascade_from_cfg(f.read(), tw, th)
    return models


def run_case(sc, O, synth, models, case, seed, stats, big_frames=True):
    """One random case; returns None, or the case's description with the error.
    big_frames: about 1 case in 10 is one frame of 2048-4200 x 700-2200 px."""
    rng = np.random.default_rng(seed + case)
    ped = rng.random() < 0.25
    c = models["ped64x128_synth.cfg" if ped else "face40_synth.cfg"]
    W, H = int(rng.integers(70, 900)), int(rng.integers(140 if ped else 70, 700))
    base = int(rng.choice([64, 72])) if ped else int(rng.choice([40, 48, 56, 70]))
    step = int(rng.choice([0, 1, 2, 3, 4, 5]))
    pk = float(rng.choice([2.0, 4.0, 6.0, 9.0]))
    ss = float(rng.choice([0.3, 0.5, 0.7]))
    n = int(rng.integers(1, 9))
    levels = int(rng.choice([-1, 1, 2, 4, 8]))
    theta = c.theta if rng.random() < 0.5 else np.full(c.n_stages, float(rng.choice([0.35, 0.4, 0.45])),
                                                             np.float32)
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, np.asarray(theta, np.float32), c.patch_index, c.w,
                                              c.bias))
    casc = O.cascade_from_cfg(text, c.tmpl_w, c.tmpl_h)
    kw = dict(base_len=base, step=step, prefilter_k=pk, stride_score=ss, n_levels=levels)
    prm_sc = sc.ScanParams.pedestrian(**kw) if ped else sc.ScanParams(**kw)
    prm_or = O.Params(aspect_h=2 if ped else 1, **kw)
    opts = {"chain_waves": int(rng.choice([0, 8, 10, 12, 14, 16])),
            "chain_subq": int(rng.choice([0, 1, 2, 3, 4, 8])),
            "integral_fuse": int(rng.choice([0, 1, 2])),
            "integral_pre": int(rng.choice([0, 1, 2, 3])),
            "table_layout": int(rng.choice([0, 1])),  # 1: interleaved cells, the lane-pair item form
            "chain_slots": int(rng.choice([0, 1, 2])),
            "chain_spec": int(rng.choice([0, 1, 2, 64]))}
    if rng.random() < 0.1 and big_frames:  # one large frame: multi-chunk one-frame block sums, odd widths, tables > 128 MiB
        W, H, n = int(rng.integers(2048, 4200)), int(rng.integers(700, 2200)), 1
    frames = np.stack([synth.make_frame(W, H, 20000 + 17 * case + k) for k in range(n)])
    desc = dict(case=case, W=W, H=H, n=n, ped=ped, base=base, step=step, pk=pk, ss=ss, levels=levels,
                permissive=bool(theta is not c.theta), **opts)
    try:
        det = sc.Detector(sc.Model.parse(text), prm_sc).set_options(**opts)
        full = case % 4 == 0
        det.set_debug(full)
        try:
            batch = det.detect_batch(frames, capacity=1 << 20)
        except sc.SurfCascadeError as e:  # the API refuses to truncate: retry at the count it names
            if "SC_ERR_CAPACITY" not in str(e):
                raise
            need = int(str(e).split("<")[-1].strip(" ')\""))
            stats["capacity_retries"] = stats.get("capacity_retries", 0) + 1
            batch = det.detect_batch(frames, capacity=need)
        layout = O.grid_layout(W, H, prm_or)[0] if full else None
        nvis_all = 0
        for k in range(n):
            T = O.integral(frames[k])
            ref, nvis = O.detect(T, casc, prm_or)
            assert det_set(batch[k]) == det_set(ref), "detections frame %d" % k
            nvis_all += nvis
            stats["detections"] += len(ref)
            if full:
                assert det.dump_integral(W, H, frame=k).view(np.uint32).tobytes() == \
                    T.view(np.uint32).tobytes(), "table frame %d" % k
                p, s, v = det.dump_grid(frame=k)
                rp, rs = O.eval_grid(T, casc, prm_or)
                ev = p != -2
                assert np.array_equal(p[ev], rp[ev]), "stages frame %d" % k
                assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes(), "scores %d" % k
                rv, _ = O.walk_grid(rp, rs, layout, casc.n_stages, prm_or.stride_score)
                assert np.array_equal(v, rv), "visited set frame %d" % k
                stats["bits_checked"] += int(ev.sum())
        assert det.info("visited") == nvis_all, "visited count"
        stats["frames"] += n
        stats["visited"] += nvis_all
        det.close()
    except Exception as e:  # noqa: BLE001 -- recorded, the soak goes on
        return dict(desc, error=repr(e)[:300])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=300)
    ap.add_argument("--seed", type=int, default=9000)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="comma-separated case numbers (re-runs)")
    a = ap.parse_args()
    from oracle import oracle as O
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    models = load_models(O)
    fails, t0 = [], time.time()
    stats = {"frames": 0, "visited": 0, "detections": 0, "bits_checked": 0}
    only = {int(x) for x in a.only.split(",") if x}
    for case in range(a.cases):
        if only and case not in only:
            continue
        f = run_case(sc, O, synth, models, case, a.seed, stats)
        if f:
            fails.append(f)
        if case % 10 == 9:
            print("soak %d/%d cases, %d failures, %.0f s" % (case + 1, a.cases, len(fails), time.time() - t0),
                  flush=True)
    out = {"cases": a.cases, "seed": a.seed, "failures": fails, "elapsed_s": time.time() - t0,
           "build": sc.build_info(), **stats}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
