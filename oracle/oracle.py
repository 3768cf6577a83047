"""ctypes front-end of the CPU restatement (oracle/sc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as
the product path.  Also holds an independent libconfig-subset reader
(`parse_cfg`) so the product's C++ model parser is checked against a second
implementation.  Parity status: see sc_oracle.h ("parity unpinned" for the
OpenCV integral order and MSVC exp; everything else restated from source).
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsc_oracle.so")

_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i16p = ctypes.POINTER(ctypes.c_int16)
_i64p = ctypes.POINTER(ctypes.c_int64)


class ScoModel(ctypes.Structure):
    _fields_ = [("n_stages", ctypes.c_int), ("n_weak", _i32p), ("theta", _f32p),
                ("patch", _i32p), ("w", _f32p), ("bias", _f64p),
                ("tmpl_w", ctypes.c_int), ("tmpl_h", ctypes.c_int)]


class ScoParams(ctypes.Structure):
    _fields_ = [("base_len", ctypes.c_int), ("aspect_h", ctypes.c_int),
                ("n_levels", ctypes.c_int), ("step", ctypes.c_int),
                ("prefilter_k", ctypes.c_float), ("stride_score", ctypes.c_double)]


WINDOW_DTYPE = np.dtype([("level", "<i4"), ("x", "<i4"), ("y", "<i4"), ("w", "<i4"),
                         ("h", "<i4"), ("stage", "<i4"), ("score", "<f8")])


# OpenMP threads of the checker: the host's share (at most 16, the GPU box's
# per-GPU CPU share), overridable per call
DEFAULT_THREADS = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                             else (os.cpu_count() or 1)))


def _nt(n):
    return DEFAULT_THREADS if n is None else n


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.sco_level_len.restype = ctypes.c_int
        L.sco_num_levels.restype = ctypes.c_int
        L.sco_grid_count.restype = ctypes.c_int64
        L.sco_grid_count.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoParams)]
        L.sco_effective_levels.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoParams)]
        L.sco_extract_patches.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, ctypes.c_int]
        L.sco_gradients.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        L.sco_integral.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p]
        L.sco_prefilter.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_float, _f32p]
        L.sco_project.argtypes = [_i32p, ctypes.c_float, ctypes.c_int, ctypes.c_int, _i32p]
        L.sco_normalize.argtypes = [_f32p]
        L.sco_calc_feature.argtypes = [_f32p, ctypes.c_int, _i32p, _f32p]
        L.sco_lr_predict.argtypes = [_f32p, ctypes.c_double, _f32p]
        L.sco_lr_predict.restype = ctypes.c_float
        L.sco_eval_window.argtypes = [_f32p, ctypes.c_int, ctypes.POINTER(ScoModel), ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                      _f32p, _f32p]
        L.sco_all_stage_scores.argtypes = [_f32p, ctypes.c_int, ctypes.POINTER(ScoModel),
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p]
        L.sco_stage_score_batch.argtypes = [_f32p, ctypes.c_int, ctypes.POINTER(ScoModel), _i32p,
                                            _i32p, _i32p, ctypes.c_int64, ctypes.c_int, _f32p,
                                            ctypes.c_int]
        L.sco_eval_grid.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoModel),
                                    ctypes.POINTER(ScoParams), _i16p, _f32p, ctypes.c_int]
        L.sco_eval_grid.restype = ctypes.c_int64
        L.sco_detect.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoModel),
                                 ctypes.POINTER(ScoParams), ctypes.c_void_p, ctypes.c_int64,
                                 _i64p, ctypes.c_int]
        L.sco_detect.restype = ctypes.c_int64
        L.sco_detect_frame.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ScoModel), ctypes.POINTER(ScoParams),
                                       ctypes.c_void_p, ctypes.c_int64, _i64p, ctypes.c_int, _f32p]
        L.sco_detect_frame.restype = ctypes.c_int64
        L.sco_exposure.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoModel),
                                   ctypes.POINTER(ScoParams), _i64p, ctypes.c_int]
        L.sco_exp_sensitivity.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoModel),
                                          ctypes.POINTER(ScoParams), _i64p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int]
        L.sco_walk_grid.argtypes = [_i16p, _f32p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_double, _u8p]
        L.sco_walk_grid.restype = ctypes.c_int64
        L.sco_mine.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ScoModel), _i32p,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_int]
        L.sco_mine.restype = ctypes.c_int64
        L.sco_group_rectangles.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_double, ctypes.c_void_p]
        L.sco_fddb_format.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_char_p, ctypes.c_long]
        L.sco_fddb_format.restype = ctypes.c_long
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


RECT_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("width", "<i4"), ("height", "<i4"),
                       ("score", "<f8")])


def group_rectangles(rects, group_threshold=2, eps=0.2):
    """cv::groupRectangles restated (sc_oracle_group.c); rects: RECT_DTYPE."""
    r = np.ascontiguousarray(rects, RECT_DTYPE)
    out = np.zeros(max(len(r), 1), RECT_DTYPE)
    n = lib().sco_group_rectangles(r.ctypes.data if len(r) else None, len(r), group_threshold,
                                   eps, out.ctypes.data)
    return out[:n].copy()


def fast_nms(rects, overlap_th=0.7):
    """fast_nms restated line by line in Python (ObjDetector.cpp:275-383):
    exchange sort ascending by score (:275-288), pick the last, suppress by
    float inverse +1 area (:334-365), compact with sort_stable (:290-313).
    rects: RECT_DTYPE; returns the picked rows in pick order."""
    r = np.ascontiguousarray(rects, RECT_DTYPE)
    n = len(r)
    sc = [float(v) for v in r["score"]]
    idx = list(range(n))
    for i in range(n):
        for j in range(i + 1, n):
            ti, tj = idx[i], idx[j]
            if sc[tj] < sc[ti]:
                idx[i], idx[j] = tj, ti
    inv = [0.0] * n
    for i in range(n):
        w, h = int(r["width"][idx[i]]), int(r["height"][idx[i]])
        inv[idx[i]] = np.float32(1.0) / np.float32((w + 1) * (h + 1))

    def sort_stable(cnt):
        i = j = 0
        while i < cnt:
            if idx[i] == -1:
                if j < i + 1:
                    j = i + 1
                while j < cnt:
                    if idx[j] == -1:
                        j += 1
                    else:
                        idx[i], idx[j] = idx[j], -1
                        j += 1
                        break
                if j == cnt:
                    return i
            i += 1
        return i

    pick, count = [], n
    X, Y, W, H = (r[k].astype(np.int64) for k in ("x", "y", "width", "height"))
    while count > 0:
        last = idx[count - 1]
        pick.append(last)
        x0, y0, x1, y1 = X[last], Y[last], X[last] + W[last], Y[last] + H[last]
        idx[count - 1] = -1
        for i in range(count - 2, -1, -1):
            q = idx[i]
            tx0, ty0 = max(x0, X[q]), max(y0, Y[q])
            tx1, ty1 = min(x1, X[q] + W[q]), min(y1, Y[q] + H[q])
            tx0, ty0 = tx1 - tx0 + 1, ty1 - ty0 + 1
            if tx0 > 0 and ty0 > 0 and float(np.float32(tx0 * ty0) * inv[q]) > overlap_th:
                idx[i] = -1
        count = sort_stable(count)
    return r[pick].copy()


def fddb_format(name, rects):
    r = np.ascontiguousarray(rects, RECT_DTYPE)
    data = r.ctypes.data if len(r) else None
    need = lib().sco_fddb_format(name.encode(), data, len(r), None, 0)
    buf = ctypes.create_string_buffer(need + 1)
    lib().sco_fddb_format(name.encode(), data, len(r), buf, need + 1)
    return buf.value.decode()


# --------------------------------------------------------------------------
# geometry
# --------------------------------------------------------------------------

def level_len(base, i):
    return lib().sco_level_len(base, i)


def num_levels(W, H, base_w, base_h):
    return lib().sco_num_levels(W, H, base_w, base_h)


def extract_patches(tw, th):
    n = lib().sco_extract_patches(tw, th, None, 0)
    r = np.zeros((n, 4), np.int32)
    lib().sco_extract_patches(tw, th, _p(r, _i32p), n)
    return r


@dataclass
class Params:
    base_len: int = 70
    aspect_h: int = 1
    n_levels: int = -1
    step: int = 0
    prefilter_k: float = 6.0
    stride_score: float = 0.5

    def c(self):
        return ScoParams(self.base_len, self.aspect_h, self.n_levels, self.step,
                         self.prefilter_k, self.stride_score)


def grid_count(W, H, params: Params):
    return lib().sco_grid_count(W, H, ctypes.byref(params.c()))


def effective_levels(W, H, params: Params):
    return lib().sco_effective_levels(W, H, ctypes.byref(params.c()))


def grid_layout(W, H, params: Params):
    """[(level, l, lh, nx, ny, base_index)] in canonical (level, y, x) order."""
    st = params.step if params.step > 0 else (params.base_len // 20 if params.base_len > 20 else 1)
    out, base = [], 0
    for i in range(effective_levels(W, H, params)):
        l = level_len(params.base_len, i)
        lh = l * params.aspect_h
        if l > W or lh > H:
            out.append((i, l, lh, 0, 0, base))
            continue
        nx, ny = (W - l) // st + 1, (H - lh) // st + 1
        out.append((i, l, lh, nx, ny, base))
        base += nx * ny
    return out, st


# --------------------------------------------------------------------------
# image side
# --------------------------------------------------------------------------

def gradients(img):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    g = np.zeros((8, H, W), np.uint8)
    lib().sco_gradients(_p(img, _u8p), W, H, W, _p(g, _u8p))
    return g


def integral(img):
    """(H+1, W+1, 8) f32 table (the reference's interleaved F256Dat layout)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    T = np.zeros((H + 1, W + 1, 8), np.float32)
    lib().sco_integral(_p(img, _u8p), W, H, W, _p(T, _f32p))
    return T


# --------------------------------------------------------------------------
# model side
# --------------------------------------------------------------------------

@dataclass
class Cascade:
    """Flattened cascade (the fields the detect path consumes)."""
    tmpl_w: int
    tmpl_h: int
    n_weak: np.ndarray          # int32 [S]
    theta: np.ndarray           # float32 [S]
    patch_index: np.ndarray     # int32 [K]
    w: np.ndarray               # float32 [K, 33]
    bias: np.ndarray            # float64 [K]
    meta: dict = field(default_factory=dict)
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_stages(self):
        return int(len(self.n_weak))

    def c(self):
        patches = extract_patches(self.tmpl_w, self.tmpl_h)
        rects = np.ascontiguousarray(patches[self.patch_index], np.int32)
        arrs = [np.ascontiguousarray(self.n_weak, np.int32), np.ascontiguousarray(self.theta, np.float32),
                rects, np.ascontiguousarray(self.w, np.float32), np.ascontiguousarray(self.bias, np.float64)]
        self._keep = arrs
        return ScoModel(self.n_stages, _p(arrs[0], _i32p), _p(arrs[1], _f32p), _p(arrs[2], _i32p),
                        _p(arrs[3], _f32p), _p(arrs[4], _f64p), self.tmpl_w, self.tmpl_h)


def empty_cascade(tmpl_w=40, tmpl_h=40):
    """A cascade with no stage yet: FillNegSamples' first round (first == true)."""
    return Cascade(tmpl_w, tmpl_h, np.zeros(0, np.int32), np.zeros(0, np.float32),
                   np.zeros(0, np.int32), np.zeros((0, 33), np.float32), np.zeros(0, np.float64))


def mine(T, cascade: Cascade, cap, features=True, nthreads=None):
    """FillNegSamples' scan of one image (sc_oracle.c sco_mine): (candidate
    windows in (level, y, x) order -- the first cap --, their descriptors
    [n, n_patches, 32] over all template patches, total candidate count)."""
    T = np.ascontiguousarray(T, np.float32)
    H, W = T.shape[0] - 1, T.shape[1] - 1
    patches = np.ascontiguousarray(extract_patches(cascade.tmpl_w, cascade.tmpl_h), np.int32)
    P = len(patches)
    out = np.zeros(max(cap, 1), WINDOW_DTYPE)
    feat = np.zeros((max(cap, 1), P, 32), np.float32) if features else None
    m = cascade.c()
    n = lib().sco_mine(_p(T, _f32p), W, H, ctypes.byref(m), _p(patches, _i32p), P, out.ctypes.data,
                       feat.ctypes.data if features else None, cap, _nt(nthreads))
    k = min(n, cap)
    return out[:k].copy(), (feat[:k].copy() if features else None), int(n)


def eval_grid(T, cascade: Cascade, params: Params, nthreads=None):
    T = np.ascontiguousarray(T, np.float32)
    H, W = T.shape[0] - 1, T.shape[1] - 1
    n = grid_count(W, H, params)
    p = np.zeros(n, np.int16)
    s = np.zeros(n, np.float32)
    m = cascade.c()
    lib().sco_eval_grid(_p(T, _f32p), W, H, ctypes.byref(m), ctypes.byref(params.c()),
                        _p(p, _i16p), _p(s, _f32p), _nt(nthreads))
    return p, s


def detect(T, cascade: Cascade, params: Params, nthreads=None):
    """Reference loop (adaptive stride).  Returns (sorted windows, n_visited)."""
    T = np.ascontiguousarray(T, np.float32)
    H, W = T.shape[0] - 1, T.shape[1] - 1
    m = cascade.c()
    nv = ctypes.c_int64(0)
    n = lib().sco_detect(_p(T, _f32p), W, H, ctypes.byref(m), ctypes.byref(params.c()), None, 0,
                         ctypes.byref(nv), _nt(nthreads))
    out = np.zeros(max(n, 1), WINDOW_DTYPE)
    lib().sco_detect(_p(T, _f32p), W, H, ctypes.byref(m), ctypes.byref(params.c()),
                     out.ctypes.data, n, ctypes.byref(nv), _nt(nthreads))
    return out[:n], nv.value


def detect_frame(img, cascade: Cascade, params: Params, nthreads=None, cap=1 << 16, scratch=None):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    m = cascade.c()
    nv = ctypes.c_int64(0)
    out = np.zeros(cap, WINDOW_DTYPE)
    sp = _p(scratch, _f32p) if scratch is not None else None
    n = lib().sco_detect_frame(_p(img, _u8p), W, H, W, ctypes.byref(m), ctypes.byref(params.c()),
                               out.ctypes.data, cap, ctypes.byref(nv), _nt(nthreads), sp)
    return out[:min(n, cap)], n, nv.value


def all_stage_scores(T, cascade: Cascade, l, x, y):
    T = np.ascontiguousarray(T, np.float32)
    W = T.shape[1] - 1
    m = cascade.c()
    out = np.zeros(cascade.n_stages, np.float32)
    lib().sco_all_stage_scores(_p(T, _f32p), W, ctypes.byref(m), l, x, y, _p(out, _f32p))
    return out


def stage_score_batch(T, cascade: Cascade, l, x, y, stage, nthreads=None):
    T = np.ascontiguousarray(T, np.float32)
    W = T.shape[1] - 1
    l = np.ascontiguousarray(l, np.int32)
    x = np.ascontiguousarray(x, np.int32)
    y = np.ascontiguousarray(y, np.int32)
    out = np.zeros(len(l), np.float32)
    m = cascade.c()
    lib().sco_stage_score_batch(_p(T, _f32p), W, ctypes.byref(m), _p(l, _i32p), _p(x, _i32p),
                                _p(y, _i32p), len(l), stage, _p(out, _f32p), _nt(nthreads))
    return out


def prefilter_mask(T, params: Params):
    """Prefilter pass for every grid window (vectorised restatement of
    DenseSURFFeatureExtractor.cpp:351-358 / ObjDetector.cpp:188), canonical
    order.  Same f32 operation order as the C oracle."""
    T = np.asarray(T, np.float32)
    H, W = T.shape[0] - 1, T.shape[1] - 1
    layout, st = grid_layout(W, H, params)
    out = []
    for (_i, l, lh, nx, ny, _b) in layout:
        if nx == 0:
            continue
        ys = np.arange(ny) * st
        xs = np.arange(nx) * st
        Y, X = np.meshgrid(ys, xs, indexing="ij")
        tl = T[Y, X, :4]; br = T[Y + lh, X + l, :4]
        tr = T[Y, X + l, :4]; bl = T[Y + lh, X, :4]
        v = (tl + br) - (tr + bl)
        m = (((v[..., 0] + v[..., 1]) + v[..., 2]) + v[..., 3]) / np.float32(2)
        out.append((m > np.float32(l * lh) * np.float32(params.prefilter_k)).ravel())
    return np.concatenate(out) if out else np.zeros(0, bool)


def exposure(T, cascade: Cascade, params: Params, nthreads=None):
    """sco_exposure counters (see sc_oracle.c) for one frame's table."""
    H, W = T.shape[0] - 1, T.shape[1] - 1
    st = np.zeros(8, np.int64)
    m = cascade.c()
    lib().sco_exposure(_p(T, _f32p), W, H, ctypes.byref(m), ctypes.byref(params.c()), _p(st, _i64p),
                       _nt(nthreads))
    return st


def exp_sensitivity(T, cascade: Cascade, params: Params, zcap=4096, nthreads=None):
    """sco_exp_sensitivity counters (see sc_oracle.c) for one frame's table
    -> (int64[9], z values of the flipping evaluations)."""
    H, W = T.shape[0] - 1, T.shape[1] - 1
    st = np.zeros(9, np.int64)
    zd = np.zeros(zcap, np.float64)
    m = cascade.c()
    lib().sco_exp_sensitivity(_p(T, _f32p), W, H, ctypes.byref(m), ctypes.byref(params.c()),
                              _p(st, _i64p), zd.ctypes.data, zcap, _nt(nthreads))
    return st, zd[:min(int(st[1]), zcap)]


def walk_grid(p_grid, s_grid, layout, n_stages, stride_score=0.5):
    """walk_rows in C (sco_walk_grid): the visited mask for large grids."""
    p = np.ascontiguousarray(p_grid, np.int16)
    s = np.ascontiguousarray(s_grid, np.float32)
    lay = np.array([(e[3], e[4], e[5]) for e in layout], np.int64).reshape(-1)
    vis = np.zeros(len(p), np.uint8)
    lib().sco_walk_grid(_p(p, _i16p), _p(s, _f32p), lay.ctypes.data, len(layout), n_stages,
                        stride_score, _p(vis, _u8p))
    return vis.astype(bool), vis.astype(bool) & (p == n_stages)


def walk_rows(p_grid, s_grid, layout, n_stages, stride_score=0.5):
    """Adaptive-stride walk over full-grid records (ObjDetector.cpp:185-217):
    returns (visited mask, detection mask) in canonical grid order."""
    visited = np.zeros(len(p_grid), bool)
    for (_lvl, _l, _lh, nx, ny, base) in layout:
        for r in range(ny):
            o = base + r * nx
            j = 0
            while j < nx:
                visited[o + j] = True
                pr = int(p_grid[o + j])
                if pr < 0:
                    j += 2
                    continue
                final = (float(np.float64(s_grid[o + j])) + pr + 1) / n_stages
                j += 2 if final < stride_score else 1
    det = visited & (p_grid == n_stages)
    return visited, det


# --------------------------------------------------------------------------
# independent libconfig-subset reader (checks the product's C++ parser)
# --------------------------------------------------------------------------

_TOK = re.compile(r"""
    (?P<ws>\s+|\#[^\n]*|//[^\n]*|/\*.*?\*/)
  | (?P<float>[-+]?(?:[0-9]*\.[0-9]*(?:[eE][-+]?[0-9]+)?|[0-9]+(?:\.[0-9]*)?[eE][-+]?[0-9]+))
  | (?P<hex>0[xX][0-9A-Fa-f]+L{0,2})
  | (?P<int>[-+]?[0-9]+L{0,2})
  | (?P<bool>(?i:true|false)\b)
  | (?P<name>[A-Za-z*][-A-Za-z0-9_*]*)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<p>[=:;,\[\]\(\)\{\}])
""", re.S | re.X)


class CfgFloat(float):
    pass


def _tokens(text):
    pos = 0
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m:
            raise ValueError("cfg: bad token at %d" % pos)
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        yield kind, m.group(kind)


def parse_cfg(text):
    """Parse libconfig text into nested dict/list; floats are CfgFloat."""
    toks = list(_tokens(text))
    i = 0

    def value():
        nonlocal i
        k, v = toks[i]
        i += 1
        if k == "float":
            return CfgFloat(float(v))
        if k == "int":
            return int(v.rstrip("L"))
        if k == "hex":
            return int(v.rstrip("L"), 16)
        if k == "bool":
            return v.lower() == "true"
        if k == "str":
            return bytes(v[1:-1], "utf-8").decode("unicode_escape")
        if v == "{":
            return group("}")
        if v in "[(":
            close = "]" if v == "[" else ")"
            items = []
            while toks[i][1] != close:
                items.append(value())
                if toks[i][1] == ",":
                    i += 1
            i += 1
            return items
        raise ValueError("cfg: unexpected %r" % v)

    def group(close):
        nonlocal i
        d = {}
        while i < len(toks) and toks[i][1] != close:
            k, name = toks[i]
            if k != "name":
                raise ValueError("cfg: expected name, got %r" % name)
            i += 1
            if toks[i][1] not in "=:":
                raise ValueError("cfg: expected = or :")
            i += 1
            d[name] = value()
            if i < len(toks) and toks[i][1] in ";,":
                i += 1
        if close:
            i += 1
        return d

    return group(None)


def _f(x):
    if not isinstance(x, CfgFloat):
        raise TypeError("cfg: float setting expected, got %r" % (x,))
    return float(x)


def cascade_from_cfg(text, tmpl_w=40, tmpl_h=40):
    """Model::Load semantics (Model.cpp:97-194), strict."""
    root = parse_cfg(text)["cascade_classifier"]
    n_weak, theta, pidx, w, bias = [], [], [], [], []
    for st in root["stage_classifiers"]:
        theta.append(np.float32(_f(st["theta"])))
        ws = st["weak_classifiers"]
        n_weak.append(len(ws))
        for wk in ws:
            pidx.append(int(wk["patch_index"]))
            w.append(np.array([np.float32(_f(v)) for v in wk["w"]], np.float32))
            bias.append(_f(wk["bias"]))
    return Cascade(tmpl_w, tmpl_h, np.array(n_weak, np.int32), np.array(theta, np.float32),
                   np.array(pidx, np.int32), np.stack(w).astype(np.float32),
                   np.array(bias, np.float64))
