"""Chain-kernel time and work split by level group (VERDICT r2 Next 1: "split
L2 hit and chain-kernel time per level group").

Runs the C2 workload (32 device-resident 1080p frames, 24 levels, face
cascade) with the scan restricted to level ranges (SC_OPT_LEVEL_LO/_HI) and
prints one JSON line per range: chain-kernel ms per launch, the range's grid
and visited windows, ns per grid window.  Under rocprofv3 --pmc each range is
one kernel name's dispatches in order (ranges run in the order printed).

    python profiles/level_split.py [--ranges 0:13,13:24,0:24] [--steps 5]
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
    ap.add_argument("--ranges", default="0:13,13:24,0:24")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--levels", type=int, default=24)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch
    import surfcascade_amd as sc
    from surfcascade_amd import synth

    W, H, B = a.width, a.height, a.batch
    frames = torch.from_numpy(synth.make_frames(W, H, B, seed0=1000)).cuda()
    params = sc.ScanParams(n_levels=a.levels)
    model = os.path.join(ROOT, "surfcascade_amd", "models", "face40_synth.cfg")
    step = 3

    def grid_of(lo, hi):
        n = 0
        for i in range(lo, hi):
            l = params.level_len(i)
            if l <= W and l <= H:
                n += ((W - l) // step + 1) * ((H - l) // step + 1)
        return n

    extra = dict(o.split("=", 1) for o in a.opt)
    for rg in a.ranges.split(","):
        lo, hi = (int(v) for v in rg.split(":"))
        det = sc.Detector(model, params, device=0)
        det.set_options(level_lo=lo, level_hi=hi, **{k: int(v) for k, v in extra.items()})
        counts = torch.zeros(1 + B, dtype=torch.int32, device=frames.device)
        recs = torch.zeros(1 << 24, dtype=torch.uint8, device=frames.device)
        det.enqueue_device(frames, recs, counts)
        det.synchronize()
        det.get_timing()
        det.set_timing(True)
        for _ in range(a.steps):
            det.enqueue_device(frames, recs, counts)
        det.synchronize()
        det.set_timing(False)
        kt = det.get_timing()
        ms, n = kt["windows"]
        g = grid_of(lo, hi) * B
        vis = det.info("visited")
        print(json.dumps({"levels": [lo, hi], "chain_ms": ms / max(n, 1), "launches": n,
                          "grid_windows": g, "visited_last_step": vis,
                          "ns_per_grid_window": ms / max(n, 1) * 1e6 / g,
                          "ns_per_visited_window": ms / max(n, 1) * 1e6 / max(vis, 1),
                          "detections": int(counts[0].item())}), flush=True)
        det.close()


if __name__ == "__main__":
    main()
