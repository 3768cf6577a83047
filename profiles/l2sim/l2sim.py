"""Trace-driven L1 / L2 model of the chain kernel (profiles/l2sim/l2sim.c):
the C2 frame's item stream (oracle: evaluated grid + the reference's visited
windows) under a task order / XCD assignment, L2 hit rate per level group.
Validated against the measured PMC split (profiles/r3/g1: L2 hit 83.7 % for
levels 0-12 alone, 39.5 % for 13-23 alone, 72.6 % for all).

    python profiles/l2sim/l2sim.py [--order blocks] [--row-block 32] [--levels 0:24]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


class Geom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("W", "H", "step", "ph", "Qp", "rowp", "hs", "cs")]


def lib():
    so = os.path.join(HERE, "libl2sim.so")
    src = os.path.join(HERE, "l2sim.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src])
    L = ctypes.CDLL(so)
    L.l2sim_run.argtypes = [ctypes.POINTER(Geom), ctypes.c_int] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int] + \
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    return L


def geometry(W, H, step=3, layout="split"):
    ph = 2 * step
    Q = (W + 1 + ph - 1) // ph
    Qp = (Q + 15) & ~15
    rowp = 2 * ph * Qp
    if layout == "split":
        return Geom(W, H, step, ph, Qp, rowp, ph * Qp, 1)
    return Geom(W, H, step, ph, Qp, rowp, 1, 2)


def build_tasks(O, casc, img, n_levels, lo, hi, row_block, nseg, order, big_split=None, big_from=13,
                xcd_split=None):
    H, W = img.shape
    P = O.Params(n_levels=n_levels)
    T = O.integral(img)
    p, s = O.eval_grid(T, casc, P)
    layout, step = O.grid_layout(W, H, P)
    vis, _ = O.walk_grid(p, s, layout, casc.n_stages)
    vis = vis.astype(bool)
    patches = O.extract_patches(casc.tmpl_w, casc.tmpl_h)
    rects = patches[casc.patch_index]
    shape = np.where(rects[:, 2] == rects[:, 3], 0, np.where(rects[:, 2] < rects[:, 3], 1, 2))
    off = np.concatenate([[0], np.cumsum(casc.n_weak)])
    order_w = [off[st] + np.argsort(shape[off[st]:off[st + 1]], kind="stable") for st in range(casc.n_stages)]
    rows = [(lv, r * step, nx, base + r * nx) for (lv, l, lh, nx, ny, base) in layout
            if lo <= lv < hi for r in range(ny)]
    blk = row_block * step
    if order == "blocks":
        rows.sort(key=lambda t: t[1] // blk)
    elif order == "bigsep":  # small levels in blocks, then the big levels in blocks
        rows.sort(key=lambda t: (t[0] >= 13, t[1] // blk))
    elif order == "levelmajor":
        pass
    tasks, xcd, chunks = [], [], []
    for (lv, y, nx, gb) in rows:
        ns, rc = nseg, 1
        if big_split and lv >= big_from:  # big levels: ns column segments x rc row classes
            ns, rc = big_split
        if xcd_split:  # small levels on XCDs [0, n_small), big ones on [n_small, 8)
            ns = xcd_split if lv < big_from else 8 - xcd_split
        nxs = (nx + ns - 1) // ns
        for sg in range(ns):
            j0, j1 = min(nx, sg * nxs), min(nx, (sg + 1) * nxs)
            js = np.arange(j0, j1)
            js = js[vis[gb + js]]
            pj = p[gb + js]
            parts = []
            for st in range(casc.n_stages):
                surv = js[pj >= st]
                if len(surv) == 0:
                    break
                ks = order_w[st]
                it = np.empty((len(surv) * len(ks), 4), np.int32)
                it[:, 0] = lv
                it[:, 1] = y
                it[:, 2] = np.tile(surv, len(ks))
                it[:, 3] = np.repeat(ks, len(surv))
                parts.append(it)
            if parts:
                chunks.append(np.concatenate(parts))
                if xcd_split:
                    xcd.append(sg if lv < big_from else xcd_split + sg)
                else:
                    xcd.append(sg * 8 // ns + ((y // step) % rc) * (8 // ns // rc) if rc > 1 else sg * 8 // ns)
    lens = np.array([len(c) for c in chunks], np.int64)
    it_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    items = np.ascontiguousarray(np.concatenate(chunks))
    return items, it_off, np.array(xcd, np.int32), layout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--levels", default="0:24")
    ap.add_argument("--order", default="blocks", choices=("blocks", "bigsep", "levelmajor"))
    ap.add_argument("--row-block", type=int, default=32)
    ap.add_argument("--nseg", type=int, default=8)
    ap.add_argument("--conc", type=int, default=768, help="tasks in flight per XCD (32 CUs x waves x 2)")
    ap.add_argument("--layout", default="split", choices=("split", "inter"))
    ap.add_argument("--l2-mib", type=float, default=4.0)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--big-split", help="big levels: SEGS:ROWCLASSES (e.g. 4:2)")
    ap.add_argument("--big-from", type=int, default=13)
    ap.add_argument("--xcd-split", type=int, help="small levels on this many XCDs, big on the rest")
    ap.add_argument("--cell-bytes", type=int, default=16, help="bytes per half cell (12: u24 packing)")
    ap.add_argument("--group", default="level", choices=("level", "stage"))
    ap.add_argument("--alt-from", type=int, default=-1,
                    help="stages >= this read a second table copy in --alt-layout (hybrid layouts)")
    ap.add_argument("--alt-layout", default="inter", choices=("split", "inter", "pix"))
    ap.add_argument("--pair", action="store_true", help="two lanes per item, one per channel half (use with --layout inter)")
    ap.add_argument("--cu-chunk", type=int, default=0,
                    help="a CU takes this many consecutive queue tasks at a time (per-workgroup sub-queue)")
    ap.add_argument("--big-slots", type=int, default=-1,
                    help="two queues: only this many of the conc slots take big-level tasks")
    a = ap.parse_args()
    from oracle import oracle as O
    from surfcascade_amd import synth
    casc = O.cascade_from_cfg(open(os.path.join(ROOT, "surfcascade_amd/models/face40_synth.cfg")).read())
    img = synth.make_frame(1920, 1080, a.seed)
    lo, hi = (int(v) for v in a.levels.split(":"))
    t0 = time.time()
    bs = tuple(int(v) for v in a.big_split.split(":")) if a.big_split else None
    items, it_off, xcd, layout = build_tasks(O, casc, img, 24, lo, hi, a.row_block, a.nseg, a.order, bs,
                                             a.big_from, a.xcd_split)
    t1 = time.time()
    patches = O.extract_patches(casc.tmpl_w, casc.tmpl_h)
    rects = patches[casc.patch_index]
    wide = rects[:, 2] >= rects[:, 3]
    ratio = np.where(wide, rects[:, 2] // rects[:, 3], rects[:, 3] // rects[:, 2])
    rec = np.zeros((len(rects), 4), np.int32)
    rec[:, 0], rec[:, 1] = rects[:, 0], rects[:, 1]
    rec[:, 2] = np.where(wide, rects[:, 3], rects[:, 2])
    rec[:, 3] = np.where(ratio == 1, 0, np.where(wide, 2, 1))
    scale = np.array([np.float32(O.level_len(70, i)) / np.float32(40) for i in range(24)], np.float32)
    grp = np.array([0 if i < a.big_from else 1 for i in range(24)], np.int32)
    g = geometry(1920, 1080, 3, a.layout)
    off = np.concatenate([[0], np.cumsum(casc.n_weak)])
    stage_of = np.zeros(len(rects), np.int32)
    for st in range(casc.n_stages):
        stage_of[off[st]:off[st + 1]] = st
    if a.group == "stage":
        gw, names = stage_of, ["stage %d" % st for st in range(casc.n_stages)]
    else:
        gw, names = None, ["levels 0-12", "levels 13-23"]
    ng = len(names)
    alt = (stage_of >= a.alt_from).astype(np.int32) if a.alt_from >= 0 else None
    if a.alt_layout == "pix":  # one plane, 32-B pixels: cell(y, x, h) = y*rowp + 2x + h
        Q = 1921
        g2 = Geom(1920, 1080, 3, 1, Q, 2 * Q, 1, 2)
    else:
        g2 = geometry(1920, 1080, 3, a.alt_layout)
    alt_base = 1082 * g.rowp + 4096
    stats = np.zeros((ng, 4), np.int64)
    L = lib()
    L.l2sim_set_cell_bytes(a.cell_bytes)
    L.l2sim_set_cu_chunk(a.cu_chunk)
    L.l2sim_set_pair(1 if a.pair else 0)
    L.l2sim_run(ctypes.byref(g), len(it_off) - 1, it_off.ctypes.data, items.ctypes.data, rec.ctypes.data,
                scale.ctypes.data, a.conc, 32, 256, int(a.l2_mib * 8192), xcd.ctypes.data, grp.ctypes.data, ng,
                stats.ctypes.data, a.big_slots, gw.ctypes.data if gw is not None else None,
                alt.ctypes.data if alt is not None else None, ctypes.byref(g2), alt_base)
    out = {"args": vars(a), "items": int(len(items)), "build_s": t1 - t0, "sim_s": time.time() - t1}
    for gi, name in enumerate(names):
        acc, m1, h2, m2 = (int(v) for v in stats[gi])
        if acc:
            out[name] = {"l1_accesses": acc, "l1_miss": round(m1 / acc, 4), "l2_hit": round(h2 / max(m1, 1), 4),
                         "l2_misses": m2}
    tot = stats.sum(0)
    out["all"] = {"l1_accesses": int(tot[0]), "l1_miss": tot[1] / tot[0], "l2_hit": tot[2] / max(tot[1], 1),
                  "l2_misses": int(tot[3])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
