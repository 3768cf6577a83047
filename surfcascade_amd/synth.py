"""Seeded synthetic inputs for the detect path.

* frames: u8 grayscale; low-frequency background + sharp-edged filled
  rectangles / ellipses (some textured) + Gaussian noise, clipped to [0, 255].
  Frame k of a benchmark batch uses seed 1000 + k; theta calibration uses
  seeds 9000+ (never benchmarked).
* model files: `write_cfg` emits the exact text layout of the reference's
  `Model::Save` (ObjDetector/Model.cpp:21-95) through libconfig's writer
  (libconfig.c:168-243, 631-653: `%.10g` floats with ".0" appended when no
  '.', groups on their own lines, tab width 2).
"""
from __future__ import annotations

import numpy as np


def make_frame(W: int, H: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    # low-frequency background: coarse random grid, bilinear upsample
    gy, gx = max(2, H // 96 + 2), max(2, W // 96 + 2)
    coarse = rng.uniform(50, 200, size=(gy, gx)).astype(np.float32)
    yy = np.linspace(0, gy - 1, H, dtype=np.float32)
    xx = np.linspace(0, gx - 1, W, dtype=np.float32)
    y0 = np.minimum(yy.astype(np.int32), gy - 2)
    x0 = np.minimum(xx.astype(np.int32), gx - 2)
    fy = (yy - y0)[:, None]
    fx = (xx - x0)[None, :]
    a = coarse[y0][:, x0]
    b = coarse[y0][:, x0 + 1]
    c = coarse[y0 + 1][:, x0]
    d = coarse[y0 + 1][:, x0 + 1]
    img = (a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + c * fy * (1 - fx) + d * fy * fx)
    # sharp-edged shapes, some carrying strong texture
    n_shapes = max(8, (W * H) // 16000)
    for _ in range(n_shapes):
        w = int(rng.integers(12, max(13, W // 6)))
        h = int(rng.integers(12, max(13, H // 6)))
        x = int(rng.integers(-w // 2, W - w // 2))
        y = int(rng.integers(-h // 2, H - h // 2))
        xa, xb = max(0, x), min(W, x + w)
        ya, yb = max(0, y), min(H, y + h)
        if xa >= xb or ya >= yb:
            continue
        val = float(rng.uniform(0, 255))
        if rng.random() < 0.5:
            mask = np.ones((yb - ya, xb - xa), bool)
        else:
            cy, cx = y + h / 2.0, x + w / 2.0
            Y, X = np.ogrid[ya:yb, xa:xb]
            mask = ((Y + 0.5 - cy) / (h / 2.0)) ** 2 + ((X + 0.5 - cx) / (w / 2.0)) ** 2 <= 1.0
        patch = img[ya:yb, xa:xb]
        if rng.random() < 0.3:
            tex = val + rng.normal(0, 90, size=patch.shape).astype(np.float32)
            patch[mask] = tex[mask]
        else:
            patch[mask] = val
    img += rng.normal(0, 3.0, size=img.shape).astype(np.float32)
    # row-major like every frame the C ABI takes (the bilinear broadcast above
    # leaves img column-major; a column-major batch costs a full copy per call)
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))


def make_frames(W: int, H: int, n: int, seed0: int = 1000) -> np.ndarray:
    return np.stack([make_frame(W, H, seed0 + k) for k in range(n)])


# --------------------------------------------------------------------------
# libconfig writer (Model::Save layout)
# --------------------------------------------------------------------------

def fmt_float(v) -> str:
    """libconfig.c:216-239: "%.10g", ".0" appended when no '.' and no 'e'."""
    s = "%.10g" % float(v)
    if "e" not in s:
        if "." not in s:
            s += ".0"
        else:
            s = s.rstrip("0") if not s.endswith(".") else s
    return s


class F(float):
    """Marks a value as a libconfig float setting."""


def _write_value(v, depth, out):
    if isinstance(v, bool):
        out.append("true" if v else "false")
    elif isinstance(v, F) or isinstance(v, np.floating):
        out.append(fmt_float(v))
    elif isinstance(v, (int, np.integer)):
        out.append("%d" % int(v))
    elif isinstance(v, tuple):  # list
        out.append("( ")
        for i, e in enumerate(v):
            _write_value(e, depth + 1, out)
            if i + 1 < len(v):
                out.append(",")
            out.append(" ")
        out.append(")")
    elif isinstance(v, list):  # array
        out.append("[ ")
        for i, e in enumerate(v):
            _write_value(e, depth + 1, out)
            if i + 1 < len(v):
                out.append(",")
            out.append(" ")
        out.append("]")
    elif isinstance(v, dict):  # group
        if depth > 0:
            out.append("\n")
            if depth > 1:
                out.append(" " * ((depth - 1) * 2))
            out.append("{\n")
        for k, e in v.items():
            _write_setting(k, e, depth + 1, out)
        if depth > 1:
            out.append(" " * ((depth - 1) * 2))
        if depth > 0:
            out.append("}")
    else:
        raise TypeError(type(v))


def _write_setting(name, v, depth, out):
    if depth > 1:
        out.append(" " * ((depth - 1) * 2))
    if name is not None:
        out.append(name)
        out.append(" : " if isinstance(v, dict) else " = ")
    _write_value(v, depth, out)
    if depth > 0:
        out.append(";\n")


def write_cfg(root: dict) -> str:
    out: list[str] = []
    _write_value(root, 0, out)
    return "".join(out)


def cascade_tree(n_weak, theta, patch_index, w, bias, meta=None) -> dict:
    """Build the Model::Save settings tree (Model.cpp:26-83)."""
    meta = meta or {}
    stages = []
    o = 0
    for s, n in enumerate(n_weak):
        weaks = []
        for k in range(n):
            weaks.append({
                "patch_index": int(patch_index[o + k]),
                "eps": F(0.01), "C": F(0.1), "nr_class": 2, "nr_feature": 32,
                "bias": F(float(bias[o + k])),
                "w": [F(float(np.float32(x))) for x in w[o + k]],
                "label": [1, -1],
            })
        o += n
        stages.append({
            "search_step": F(float(np.float32(0.01))), "auc_step": F(float(np.float32(0.05))),
            "TPR_min": F(float(np.float32(0.995))), "n_total": 1920, "n_pos": 960, "n_neg": 960,
            "FPR": F(float(np.float32(meta.get("stage_fpr", [0.5] * len(n_weak))[s]))),
            "TPR": F(float(np.float32(0.995))),
            "theta": F(float(np.float32(theta[s]))),
            "total_AUC_score": F(float(np.float32(0.0))), "sample_num": 960, "max_iters": 100,
            "weak_classifiers": tuple(weaks),
        })
    return {"cascade_classifier": {
        "max_stages_num": len(n_weak),
        "FPR_target": F(float(np.float32(1e-6))),
        "TPR_min_perstage": F(float(np.float32(0.995))),
        "FPR": F(float(np.float32(meta.get("fpr", 1e-6)))),
        "TPR": F(float(np.float32(meta.get("tpr", 0.95)))),
        "stage_classifiers": tuple(stages),
    }}
