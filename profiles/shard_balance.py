"""Balance of the single-frame window-grid split (bench.py --shard grid,
sc_detector_set_shard) measured on ONE GPU: rank r of world W is
run alone, one after the other, on the same device-resident frame, and its
kernels are timed (HIP events on the detector's stream).  Not a scaling
curve (the 1-8 GPU curve is the driver's): it gives each rank's chain-kernel
and integral time, max / mean over the ranks, and the strong-scaling
efficiency the split implies, T(1) / (W * max_r T_r), with every rank
recomputing the whole integral as the multi-GPU path does (VERDICT r4 #7;
the reference's own split is static by level, ObjDetector.cpp:177).

    python profiles/shard_balance.py [--config C2|C4] [--worlds 1,2,4,8] [--steps 20] [--opt k=v]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"C2": (1920, 1080, 24), "C4": (3840, 2160, 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1, help="frames per call (1: the single-frame split)")
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth

    W, H, levels = CONFIGS[a.config]
    frames = torch.from_numpy(synth.make_frames(W, H, a.frames, seed0=1000)).cuda()
    model = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
    params = sc.ScanParams(n_levels=levels)
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in a.opt)}
    out = {"config": a.config, "frames_per_call": a.frames, "steps": a.steps, "build": sc.build_info(),
           "worlds": {}}
    t1 = None
    for world in [int(x) for x in a.worlds.split(",")]:
        ranks = []
        for rank in range(world):
            det = sc.Detector(model, params, device=0)
            det.set_options(**opts)
            det.set_stream(torch.cuda.current_stream())
            det.set_shard(rank, world)
            counts = torch.zeros(1 + a.frames, dtype=torch.int32, device=frames.device)
            recs = torch.zeros(1 << 22, dtype=torch.uint8, device=frames.device)
            for _ in range(3):
                det.enqueue_device(frames, recs, counts)
            det.synchronize()
            det.get_timing()
            det.set_timing(True)
            for _ in range(a.steps):
                det.enqueue_device(frames, recs, counts)
                det.synchronize()  # one call at a time, as a rank of a single-frame run
            det.set_timing(False)
            kt = det.get_timing()
            per = {k: v[0] / max(v[1], 1) for k, v in kt.items() if v[1]}
            integral = per.get("rowscan", 0.0) + per.get("colscan", 0.0)
            ranks.append({"rank": rank, "chain_ms": per.get("windows", 0.0), "integral_ms": integral,
                          "kernels_ms": sum(per.values()), "visited": det.info("visited"),
                          "rows": det.info("rows"), "detections": int(counts[0].item())})
            det.set_stream(None)
            det.close()
        tot = [r["kernels_ms"] for r in ranks]
        ch = [r["chain_ms"] for r in ranks]
        if world == 1:
            t1 = tot[0]
        w = {"ranks": ranks,
             "chain_max_over_mean": max(ch) / statistics.mean(ch),
             "kernels_max_ms": max(tot), "kernels_max_over_mean": max(tot) / statistics.mean(tot),
             "visited_sum": sum(r["visited"] for r in ranks)}
        if t1:
            w["implied_strong_efficiency"] = t1 / (world * max(tot))
            w["implied_strong_efficiency_chain_only"] = (
                out["worlds"]["1"]["ranks"][0]["chain_ms"] / (world * max(ch)) if "1" in out["worlds"] else None)
        out["worlds"][str(world)] = w
        print(json.dumps({"world": world, "chain_ms": [round(x, 4) for x in ch],
                          "integral_ms": round(ranks[0]["integral_ms"], 4),
                          "max_over_mean": round(w["chain_max_over_mean"], 4),
                          "eff": round(w.get("implied_strong_efficiency", 0), 4)}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
