"""How much of the chain kernel's table traffic could an LDS-staged tile serve?
(VERDICT r3 "Next" 1: stage the table band a workgroup's tasks need into LDS
with coalesced loads, read corners with ds_read_b128.)

For the C2 frame (1080p, 24 levels, the face cascade) and the reference's
visited windows (ObjDetector.cpp:182-217), take tiles of windows the way a
workgroup would own them -- R consecutive window rows (stride 3) x one row
segment (1/8 of the row's windows, the chain kernel's XCD segment) of one
level -- and count, for the early stages 0..2 (84 % of the L2 misses, DESIGN
5d) and for all stages:
  staged  = distinct 16-B table cells (one channel half) the tile's items read
            = the bytes a perfect staging pass must load per half,
  read    = cells the items read (10 corner slots per half per item, the
            kernel's uniform corner set; 9 distinct for 2x2 patches),
  reuse   = read / staged: LDS reads served per staged byte.
A tile is stageable only if staged * 16 B per half fits the LDS left beside
the model (~60 KiB per channel half at 12 waves, less at 16).
Staging goes through the same texture path (TA/TD) as the gathers it
replaces, so with reuse ~1 it cannot be cheaper than the gathers themselves.
Writes profiles/r4/lds_reuse.json."""
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
patches = O.extract_patches(40, 40)
rects = patches[casc.patch_index]          # per global weak: x, y, w, h (template)
cum = np.concatenate([[0], np.cumsum(casc.n_weak)])
W, H, L = 1920, 1080, 24
params = O.Params(n_levels=L)
img = synth.make_frame(W, H, 1000)
T = O.integral(img)
p, s = O.eval_grid(T, casc, params)
layout, _ = O.grid_layout(W, H, params)
vis, _ = O.walk_grid(p, s, layout, casc.n_stages, 0.5)
vis = vis.astype(bool)


def corners(k, l, x, y):
    """Corner cells (row, col) of weak k's projected patch at window (x, y), level length l
    (ProjectPatches :459-484, GetRectsFromPatch :360-377)."""
    sc = np.float32(l) / np.float32(40)
    px, py, pw, ph = (int(v) for v in rects[k])
    xp, yp = int(np.float32(px) * sc) + x, int(np.float32(py) * sc) + y
    if pw >= ph:
        hh = int(np.float32(ph) * sc); ww = hh * (pw // ph)
    else:
        ww = int(np.float32(pw) * sc); hh = ww * (ph // pw)
    if ww == hh:
        c, gw, gh = ww // 2, 2, 2
    else:
        c = min(ww, hh); gw, gh = ww // c, hh // c
    return [(yp + j * c, xp + i * c) for j in range(gh + 1) for i in range(gw + 1)]


rng = np.random.default_rng(3)
out = {"frame": "C2 1080p seed 1000, face40 cascade", "levels": []}
for (lv, l, lh, nx, ny, base) in layout:
    seg = (nx + 7) // 8
    rec = {"level": lv, "l": l, "segment_windows": seg, "tiles": {}}
    for R in (1, 4, 16):
        for stages, tag in ((3, "stages0-2"), (casc.n_stages, "all")):
            st_l, rd_l = [], []
            for _t in range(6):  # sample tiles
                r0 = int(rng.integers(0, max(1, ny - R + 1)))
                s0 = int(rng.integers(0, 8)) * seg
                cells, reads = set(), 0
                for r in range(r0, min(ny, r0 + R)):
                    for j in range(s0, min(nx, s0 + seg)):
                        gi = base + r * nx + j
                        if not vis[gi] or p[gi] < 0:
                            continue
                        last = min(int(p[gi]), casc.n_stages - 1, stages - 1)
                        for k in range(cum[0], cum[last + 1]):
                            cs = corners(k, l, 3 * j, 3 * r)
                            cells.update(cs)
                            reads += 10  # uniform corner slots per half
                st_l.append(len(cells))
                rd_l.append(reads)
            st, rd = float(np.mean(st_l)), float(np.mean(rd_l))
            rec["tiles"]["R%d_%s" % (R, tag)] = {"staged_KiB_per_half": st * 16 / 1024,
                                                 "read_KiB_per_half": rd * 16 / 1024,
                                                 "reuse": rd / st if st else None}
    out["levels"].append(rec)
    t = rec["tiles"]
    print("level %2d l %3d: R1 early staged %6.1f KiB reuse %.2f | R4 early %6.1f KiB %.2f | R16 early %7.1f KiB %.2f"
          " | R16 all %7.1f KiB %.2f" % (lv, l, t["R1_stages0-2"]["staged_KiB_per_half"], t["R1_stages0-2"]["reuse"],
                                         t["R4_stages0-2"]["staged_KiB_per_half"], t["R4_stages0-2"]["reuse"],
                                         t["R16_stages0-2"]["staged_KiB_per_half"], t["R16_stages0-2"]["reuse"],
                                         t["R16_all"]["staged_KiB_per_half"], t["R16_all"]["reuse"]), flush=True)
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lds_reuse.json"), "w"), indent=1)
