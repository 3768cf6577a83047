"""Drive itembench.hip: the C2 frame's real item stream, timed per variant.

Items: the visited windows of frame 1000 (C2, 24 levels) in the chain
kernel's order -- row blocks of 32 grid rows (level-major inside), each row
cut into 8 segments, segment x -> XCD x's queue -- and per (row segment,
stage) the (survivor, weak) items k-major in shape-sorted weak order, as the
chain kernel's item loop runs them.  Every variant's outputs are compared bit
for bit with variant 0 (the production weak_eval).

    python profiles/itembench/run.py [--reps 5] [--variants 0:12,0:16,1:12]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


class TableGeom(ctypes.Structure):
    _fields_ = [("W", ctypes.c_int), ("H", ctypes.c_int), ("step", ctypes.c_int), ("ph", ctypes.c_int),
                ("Qp", ctypes.c_int), ("rowp", ctypes.c_int), ("cs", ctypes.c_int), ("hs", ctypes.c_int),
                ("frame4", ctypes.c_longlong), ("phm", ctypes.c_uint)]


class Args(ctypes.Structure):
    _fields_ = [("table", ctypes.c_void_p), ("g", TableGeom), ("items", ctypes.c_void_p),
                ("n_items", ctypes.c_void_p), ("cap", ctypes.c_longlong), ("w", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("rects", ctypes.c_void_p), ("scale", ctypes.c_void_p),
                ("K", ctypes.c_int), ("n_levels", ctypes.c_int), ("out", ctypes.c_void_p),
                ("tickets", ctypes.c_void_p), ("omask", ctypes.c_uint), ("fold", ctypes.c_uint)]


ITEM = np.dtype([("origin", "<u4"), ("k", "<u2"), ("level", "u1"), ("parity", "u1")])


def geometry(W, H, step=3):
    ph = 2 * step
    Q = (W + 1 + ph - 1) // ph
    Qp = (Q + 15) & ~15
    rowp = 2 * ph * Qp
    g = TableGeom(W, H, step, ph, Qp, rowp, 1, ph * Qp, (H + 1) * rowp,
                  ((1 << 32) + ph - 1) // ph)
    return g


def geometry_inter(W, H, step=3):
    """interleaved 32-B cells (TableGeom cs 2, hs 1): float4 (y, x, h) =
    y*rowp + 2*((x % ph)*Qp + x // ph) + h"""
    g = geometry(W, H, step)
    g.cs, g.hs = 2, 1
    return g


def inter_table(T, g):
    H1, W1, _ = T.shape
    out = np.zeros((H1, g.rowp, 4), np.float32)
    x = np.arange(W1)
    cell = 2 * ((x % g.ph) * g.Qp + x // g.ph)
    out[:, cell, :] = T[:, :, :4]
    out[:, cell + 1, :] = T[:, :, 4:]
    return out


def split_table(T, g):
    """Reference interleaved (H+1, W+1, 8) table -> phase-split float4 cells."""
    H1, W1, _ = T.shape
    out = np.zeros((H1, g.rowp, 4), np.float32)
    x = np.arange(W1)
    cell = (x % g.ph) * g.Qp + x // g.ph
    out[:, cell, :] = T[:, :, :4]
    out[:, cell + g.hs, :] = T[:, :, 4:]
    return out


def build_items(O, casc, img, n_levels=24, row_block=32, order="seg", nseg=8, level_group=0):
    H, W = img.shape
    P = O.Params(n_levels=n_levels)
    T = O.integral(img)
    p, s = O.eval_grid(T, casc, P)
    layout, step = O.grid_layout(W, H, P)
    vis, _ = O.walk_grid(p, s, layout, casc.n_stages)
    g = geometry(W, H, step)
    patches = O.extract_patches(casc.tmpl_w, casc.tmpl_h)
    rects = patches[casc.patch_index]
    shape = np.where(rects[:, 2] == rects[:, 3], 0, np.where(rects[:, 2] < rects[:, 3], 1, 2))
    off = np.concatenate([[0], np.cumsum(casc.n_weak)])
    order_w = [off[s_] + np.argsort(shape[off[s_]:off[s_ + 1]], kind="stable") for s_ in range(casc.n_stages)]
    rows = []
    for (lv, l, lh, nx, ny, base) in layout:
        for r in range(ny):
            rows.append((lv, r * step, nx, base + r * nx))
    blk = row_block * step
    if level_group:  # groups of levels, each swept in row blocks
        rows.sort(key=lambda t: (t[0] // level_group, t[1] // blk))
    elif row_block > 0:
        rows.sort(key=lambda t: t[1] // blk)  # stable: level-major inside a block
    queues = [[] for _ in range(8)]

    def emit(q, lv, y, js, pj):
        for st in range(casc.n_stages):
            surv = js[pj >= st]
            if len(surv) == 0:
                break
            ks = order_[st]
            it = np.zeros(len(surv) * len(ks), ITEM)
            jj = np.tile(surv, len(ks))
            it["k"] = np.repeat(ks, len(surv))
            it["parity"] = jj & 1
            it["level"] = lv
            it["origin"] = y * g.rowp + (jj & 1) * step * g.Qp + (jj >> 1)
            queues[q].append(it)

    order_ = order_w
    for ri, (lv, y, nx, gb) in enumerate(rows):
        if order == "row":  # whole rows, row blocks dealt to the XCD queues
            js = np.arange(nx)
            js = js[vis[gb + js]]
            for par in (0, 1):
                jp = js[(js & 1) == par]
                emit((y // blk) % 8, lv, y, jp, p[gb + jp])
            continue
        nxs = (nx + nseg - 1) // nseg
        for sg in range(nseg):
            j0, j1 = min(nx, sg * nxs), min(nx, (sg + 1) * nxs)
            js = np.arange(j0, j1)
            js = js[vis[gb + js]]
            emit(sg * 8 // nseg, lv, y, js, p[gb + js])
    queues = [np.concatenate(qq) for qq in queues]
    return T, g, queues


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0:12,0:16,1:12,1:8")
    ap.add_argument("--out")
    ap.add_argument("--order", default="seg", choices=("seg", "row"))
    ap.add_argument("--row-block", type=int, default=32, help="grid rows per block (0: level-major)")
    ap.add_argument("--nseg", type=int, default=8)
    ap.add_argument("--level-group", type=int, default=0)
    ap.add_argument("--omask", type=lambda x: int(x, 0), default=0xFFFFFFFF,
                    help="ablation, variant 2 only: lane offset mask (0: every lane reads lane 0's item)")
    ap.add_argument("--fold", type=lambda x: int(x, 0), default=0xFFFFFFFF,
                    help="ablation, variant 3 only: table rows &= fold (a 2^k - 1 band the L2 holds)")
    a = ap.parse_args()
    import torch
    from oracle import oracle as O
    from surfcascade_amd import synth
    casc = O.cascade_from_cfg(open(os.path.join(ROOT, "surfcascade_amd/models/face40_synth.cfg")).read())
    img = synth.make_frame(1920, 1080, 1000)
    t0 = time.time()
    T, g, queues = build_items(O, casc, img, order=a.order, row_block=a.row_block, nseg=a.nseg,
                               level_group=a.level_group)
    n_items = sum(len(q) for q in queues)
    print("items %d (per XCD %s), built in %.1f s" % (n_items, [len(q) for q in queues], time.time() - t0),
          flush=True)
    dev = "cuda:0"
    tab = torch.from_numpy(split_table(T, g)).to(dev)
    cap = max(len(q) for q in queues)
    items = np.zeros((8, cap), ITEM)
    for i, q in enumerate(queues):
        items[i, :len(q)] = q
    d_items = torch.from_numpy(items.view(np.uint8)).to(dev)
    d_n = torch.tensor([len(q) for q in queues], dtype=torch.int32, device=dev)
    K = int(casc.n_weak.sum())
    w = np.zeros((K, 36), np.float32)
    w[:, :33] = casc.w
    patches = O.extract_patches(casc.tmpl_w, casc.tmpl_h)
    rects = patches[casc.patch_index]
    rec = np.zeros((K, 4), np.int32)
    wide = rects[:, 2] >= rects[:, 3]
    ratio = np.where(wide, rects[:, 2] // rects[:, 3], rects[:, 3] // rects[:, 2])
    rec[:, 0], rec[:, 1] = rects[:, 0], rects[:, 1]
    rec[:, 2] = np.where(wide, rects[:, 3], rects[:, 2])
    rec[:, 3] = np.where(ratio == 1, 0, np.where(wide, 2, 1))
    scale = np.array([np.float32(O.level_len(70, i)) / np.float32(40) for i in range(24)], np.float32)
    d_w = torch.from_numpy(w).to(dev)
    d_b = torch.from_numpy(np.ascontiguousarray(casc.bias, np.float64)).to(dev)
    d_r = torch.from_numpy(rec).to(dev)
    d_s = torch.from_numpy(scale).to(dev)
    d_out = torch.zeros(8 * cap, dtype=torch.float32, device=dev)
    d_t = torch.zeros(8 * 64, dtype=torch.int32, device=dev)
    L = ctypes.CDLL(os.path.join(HERE, "libitembench.so"))
    L.ib_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Args), ctypes.c_void_p]
    assert L.ib_args_size() == ctypes.sizeof(Args), (L.ib_args_size(), ctypes.sizeof(Args))
    args = Args(tab.data_ptr(), g, d_items.data_ptr(), d_n.data_ptr(), cap, d_w.data_ptr(),
                d_b.data_ptr(), d_r.data_ptr(), d_s.data_ptr(), K, 24, d_out.data_ptr(), d_t.data_ptr(), a.omask, a.fold)
    # variant 4: the same items on the interleaved-cell table (origin = y*rowp + 2*col)
    gi = geometry_inter(T.shape[1] - 1, T.shape[0] - 1)
    tab_i = torch.from_numpy(inter_table(T, gi)).to(dev)
    items_i = items.copy()
    yy = items_i["origin"] // g.rowp
    items_i["origin"] = yy * g.rowp + 2 * (items_i["origin"] - yy * g.rowp)
    d_items_i = torch.from_numpy(items_i.view(np.uint8)).to(dev)
    args_i = Args(tab_i.data_ptr(), gi, d_items_i.data_ptr(), d_n.data_ptr(), cap, d_w.data_ptr(),
                  d_b.data_ptr(), d_r.data_ptr(), d_s.data_ptr(), K, 24, d_out.data_ptr(), d_t.data_ptr(), a.omask,
                  a.fold)
    stream = torch.cuda.current_stream().cuda_stream
    ref = None
    res = {}
    for spec in a.variants.split(","):
        v, wv = (int(x) for x in spec.split(":"))
        d_out.zero_()
        av = args_i if v in (4, 9, 12, 13) else args
        assert L.ib_run(v, wv, ctypes.byref(av), stream) == 0
        torch.cuda.synchronize()
        o = d_out.cpu().numpy().copy()
        if ref is None:
            ref = o
        same = np.array_equal(o.view(np.uint32), ref.view(np.uint32)) if v in (0, 1, 3, 4, 8, 9, 10, 11, 12, 13, 15, 16) else None
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.ib_run(v, wv, ctypes.byref(av), stream)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = min(ts)
        res[spec] = {"ms": ms, "med_ms": float(np.median(ts)), "Gitems_s": n_items / ms / 1e6, "bitexact": bool(same)}
        print("variant %-5s %.4f ms (med %.4f)  %.2f G items/s  bit-exact vs v0: %s"
              % (spec, ms, np.median(ts), n_items / ms / 1e6, same), flush=True)
    if a.out:
        json.dump({"items": n_items, "variants": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
