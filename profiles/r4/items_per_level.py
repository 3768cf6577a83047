"""Work per grid window by level, C2 vs C4 (reference semantics, oracle):
the weak evaluations ("items") the reference's x chain performs
(ObjDetector.cpp:182-217: visited windows, prefilter, stages until the first
reject) per level, per grid window.  Used to separate the work the
configurations ask for from the kernel's cost per unit of work."""
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
n_s = np.array([len(k) for k in np.split(np.arange(casc.n_weak.sum()), np.cumsum(casc.n_weak)[:-1])]) \
    if hasattr(casc, "n_weak") else None
cum = np.concatenate([[0], np.cumsum(casc.n_weak)])  # items through stage s = cum[s + 1]
out = {}
for name, W, H, L, seeds in (("C2", 1920, 1080, 24, [1000, 1001]), ("C4", 3840, 2160, 32, [4000])):
    params = O.Params(n_levels=L)
    layout, _ = O.grid_layout(W, H, params)
    per = np.zeros((L, 4))  # grid windows, visited, prefilter-passed visited, items
    for sd in seeds:
        img = synth.make_frame(W, H, sd)
        T = O.integral(img)
        p, s = O.eval_grid(T, casc, params)
        v, _ = O.walk_grid(p, s, layout, casc.n_stages, 0.5)
        v = v.astype(bool)
        items = np.where(p >= 0, cum[np.minimum(p + 1, casc.n_stages)], 0)
        for (lv, l, lh, nx, ny, base) in layout:
            sl = slice(base, base + nx * ny)
            per[lv] += (nx * ny, v[sl].sum(), (v[sl] & (p[sl] >= 0)).sum(), items[sl][v[sl]].sum())
    per /= len(seeds)
    lens = [int(70 * 1.1 ** i) for i in range(L)]
    out[name] = {"levels": [{"l": lens[i], "grid": int(per[i, 0]), "visited": int(per[i, 1]),
                             "items": int(per[i, 3]), "items_per_grid": per[i, 3] / per[i, 0]}
                            for i in range(L)],
                 "items_per_grid_window": per[:, 3].sum() / per[:, 0].sum(),
                 "visited_frac": per[:, 1].sum() / per[:, 0].sum(),
                 "wide_items_frac": per[[i for i in range(L) if lens[i] > 240], 3].sum() / per[:, 3].sum()}
    print(name, "items per grid window %.3f, visited %.3f, items at l > 240: %.3f"
          % (out[name]["items_per_grid_window"], out[name]["visited_frac"], out[name]["wide_items_frac"]))
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "items_per_level.json"), "w"), indent=1)
