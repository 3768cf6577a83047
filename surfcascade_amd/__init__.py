"""surfcascade_amd -- MI355X-native SURF-cascade detect path.

Python mirror of the reference's in-process API (ObjDetector/Model.h,
CascadeClassifier/*.h) over the C ABI in include/surfcascade.h; the work
happens in libsurfcascade.so (hand-written gfx950 HIP kernels).  There is no
CPU fallback: if the library is missing, importing the binding raises.

    casc = CascadeClassifier()
    Model("model.cfg").Load(casc)                # Model.cpp:97-194
    det = Detector(casc, ScanParams(n_levels=24))
    wins = det.detect(gray_u8)                   # ObjDetector.cpp:165-220
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

__all__ = ["ScanParams", "Model", "CascadeClassifier", "StageClassifier", "LogisticRegression",
           "Detector", "SurfCascadeError", "WINDOW_DTYPE", "RECORD_DTYPE", "library_path",
           "load_library", "extract_patches", "RECT_DTYPE", "groupRectangles", "group_detections",
           "fddb_format", "Miner"]

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

SC_OK = 0
ERRORS = {-1: "SC_ERR_INVALID", -2: "SC_ERR_IO", -3: "SC_ERR_PARSE", -4: "SC_ERR_MODEL",
          -5: "SC_ERR_DEVICE", -6: "SC_ERR_CAPACITY", -7: "SC_ERR_NOMEM"}
EXIT_SUCCESS, EXIT_FAILURE = 0, 1

WINDOW_DTYPE = np.dtype([("level", "<i4"), ("x", "<i4"), ("y", "<i4"), ("w", "<i4"),
                         ("h", "<i4"), ("stage", "<i4"), ("score", "<f8")])
RECORD_DTYPE = np.dtype([("frame", "<i4"), ("level", "<i4"), ("x", "<i4"), ("y", "<i4"),
                         ("w", "<i4"), ("h", "<i4"), ("stage", "<i4"), ("pad", "<i4"),
                         ("score", "<f8")])

RECT_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("width", "<i4"), ("height", "<i4"),
                       ("score", "<f8")])

KERNELS = ("rowscan", "colscan", "windows", "walk")

# sc_detector_set_option keys (include/surfcascade.h SC_OPT_*): 1-14, 17-19
# and 21 are schedule and layout choices that never change a result bit;
# level_lo / level_hi restrict the scan to the levels [lo, hi) (level-group
# profiling); 20 and 22 are test hooks (test-hook build only)
OPTIONS = {"full_grid": 1, "chunk_min": 2, "table_layout": 3, "phases": 4, "substrips": 5,
           "band_rows": 6, "row_order": 7, "row_block": 8, "chain_chunk": 9, "lds_weights": 10,
           "wgs_per_cu": 11, "profile": 12, "chain_segs": 13, "integral_passes": 14,
           "level_lo": 15, "level_hi": 16, "chain_waves": 17,
           "integral_fuse": 18, "integral_pre": 19,
           "test_drop_handoff": 20, "chain_subq": 21, "test_drop_walk": 22,
           "chain_spec": 23, "chain_slots": 24}

# every symbol include/surfcascade.h declares
EXPORTS = ("sc_scan_params_default", "sc_model_load", "sc_model_parse", "sc_model_save",
           "sc_model_num_stages", "sc_model_stage", "sc_model_weak", "sc_model_free",
           "sc_extract_patches", "sc_detector_create", "sc_detector_create_from_model",
           "sc_detector_destroy", "sc_detect", "sc_detect_batch", "sc_detect_device",
           "sc_enqueue_device", "sc_synchronize", "sc_detector_stream", "sc_detector_wait_stream",
           "sc_stream_wait_detector", "sc_detector_set_stream", "sc_detector_info",
           "sc_detector_set_shard", "sc_detector_set_option", "sc_detector_set_debug", "sc_debug_dump", "sc_set_timing", "sc_get_timing",
           "sc_group_rectangles", "sc_group_detections", "sc_fddb_format",
           "sc_miner_create", "sc_mine", "sc_mine_device", "sc_mine_batch", "sc_mine_batch_device", "sc_fast_nms", "sc_decode_jpeg_gray", "sc_imread_gray",
           "sc_selftest_rn", "sc_normalize_operand_range", "sc_last_error", "sc_version",
           "sc_build_info")


class SurfCascadeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(code, "SC_ERR"), code, msg))
        self.code = code


class ScanParams(ctypes.Structure):
    """sc_scan_params; defaults = the reference's constants (ObjDetector.cpp)."""
    _fields_ = [("base_len", ctypes.c_int), ("scale_factor", ctypes.c_double),
                ("n_levels", ctypes.c_int), ("step", ctypes.c_int),
                ("prefilter_k", ctypes.c_float), ("stride_score", ctypes.c_double),
                ("tmpl_w", ctypes.c_int), ("tmpl_h", ctypes.c_int), ("aspect_h", ctypes.c_int)]

    def __init__(self, **kw):
        super().__init__()
        d = dict(base_len=70, scale_factor=1.1, n_levels=-1, step=0, prefilter_k=6.0,
                 stride_score=0.5, tmpl_w=40, tmpl_h=40, aspect_h=1)
        d.update(kw)
        for k, v in d.items():
            setattr(self, k, v)

    def level_len(self, i):
        """Window side of level i: (int)(base_len * scale_factor^i) (ObjDetector.cpp:180)."""
        return int(self.base_len * self.scale_factor ** i)

    @classmethod
    def pedestrian(cls, **kw):
        """64x128 extension (hard part 7): window (l, 2l)."""
        d = dict(base_len=64, tmpl_w=64, tmpl_h=128, aspect_h=2)
        d.update(kw)
        return cls(**d)


def library_path():
    return os.environ.get("SURFCASCADE_LIB", os.path.join(HERE, "lib", "libsurfcascade.so"))


_lib = None


def load_library():
    """Load libsurfcascade.so; raises (never falls back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    # One HIP runtime per process: torch bundles its own libamdhip64 (soname
    # libamdhip64.so.7, NEEDED as "libamdhip64.so").  Loading torch first lets
    # our NEEDED libamdhip64.so.7 bind to that copy instead of pulling in a
    # second runtime from /opt/rocm (two runtimes hide the GPU from torch).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise ImportError("libsurfcascade.so not built (%s); run __graft_entry__.build()" % path)
    L = ctypes.CDLL(path)
    vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
    P = ctypes.POINTER
    L.sc_last_error.restype = ctypes.c_char_p
    L.sc_version.restype = ctypes.c_char_p
    L.sc_build_info.restype = ctypes.c_char_p
    L.sc_scan_params_default.argtypes = [P(ScanParams)]
    L.sc_model_load.argtypes = [ctypes.c_char_p, P(vp)]
    L.sc_model_parse.argtypes = [ctypes.c_char_p, sz, P(vp)]
    L.sc_model_save.argtypes = [vp, ctypes.c_char_p]
    L.sc_model_num_stages.argtypes = [vp]
    L.sc_model_stage.argtypes = [vp, i32, P(ctypes.c_float), P(i32)]
    L.sc_model_weak.argtypes = [vp, i32, i32, P(i32), P(ctypes.c_float), P(ctypes.c_double)]
    L.sc_model_free.argtypes = [vp]
    L.sc_model_free.restype = None
    L.sc_extract_patches.argtypes = [i32, i32, P(ctypes.c_int32), i32]
    L.sc_detector_create.argtypes = [ctypes.c_char_p, P(ScanParams), i32, P(vp)]
    L.sc_detector_create_from_model.argtypes = [vp, P(ScanParams), i32, P(vp)]
    L.sc_detector_destroy.argtypes = [vp]
    L.sc_detector_destroy.restype = None
    L.sc_detect.argtypes = [vp, vp, i32, i32, i32, vp, i32, P(i32)]
    L.sc_detect_batch.argtypes = [vp, P(vp), i32, i32, i32, i32, vp, i32, P(i32)]
    L.sc_detect_device.argtypes = [vp, vp, i32, i32, i32, i32, vp, i32, P(i32)]
    L.sc_enqueue_device.argtypes = [vp, vp, i32, i32, i32, i32, vp, i32, vp]
    L.sc_synchronize.argtypes = [vp]
    L.sc_detector_stream.argtypes = [vp]
    L.sc_detector_stream.restype = vp
    L.sc_detector_wait_stream.argtypes = [vp, vp]
    L.sc_stream_wait_detector.argtypes = [vp, vp]
    L.sc_detector_set_stream.argtypes = [vp, vp, ctypes.c_int]
    L.sc_detector_info.argtypes = [vp, i32, P(i64)]
    L.sc_detector_set_debug.argtypes = [vp, i32]
    L.sc_detector_set_shard.argtypes = [vp, i32, i32]
    L.sc_detector_set_option.argtypes = [vp, i32, i64]
    L.sc_debug_dump.argtypes = [vp, i32, i32, vp, sz]
    L.sc_set_timing.argtypes = [vp, i32]
    L.sc_get_timing.argtypes = [vp, P(ctypes.c_double), P(i64)]
    L.sc_miner_create.argtypes = [vp, i32, i32, i32, P(vp)]
    L.sc_mine.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32, P(i32)]
    L.sc_mine_device.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32, P(i32)]
    L.sc_mine_batch.argtypes = [vp, P(vp), i32, i32, i32, i32, vp, vp, i32, vp]
    L.sc_mine_batch_device.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, i32, vp]
    L.sc_group_rectangles.argtypes = [vp, i32, i32, ctypes.c_double, vp, i32, P(i32)]
    L.sc_group_detections.argtypes = [vp, i32, i32, i32, ctypes.c_double, vp, i32, vp, P(i32)]
    L.sc_fddb_format.argtypes = [ctypes.c_char_p, vp, i32, ctypes.c_char_p, sz, P(sz)]
    L.sc_fast_nms.argtypes = [vp, i32, ctypes.c_double, vp, i32, P(i32)]
    L.sc_decode_jpeg_gray.argtypes = [vp, sz, vp, sz, P(i32), P(i32)]
    L.sc_imread_gray.argtypes = [ctypes.c_char_p, vp, sz, P(i32), P(i32)]
    L.sc_selftest_rn.argtypes = [i32, i32, ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint64)]
    L.sc_normalize_operand_range.argtypes = [i32, i32, P(ctypes.c_double), P(ctypes.c_double)]
    L.sc_normalize_operand_range.restype = None
    _lib = L
    return L


def build_info():
    """sc_build_info of the loaded library: {"build_id", "flags", "arch",
    "ablation", "test_hooks", "profiling"} (include/surfcascade.h)."""
    import json
    return json.loads(load_library().sc_build_info().decode())


def _check(rc):
    if rc < 0:
        raise SurfCascadeError(rc, load_library().sc_last_error().decode(errors="replace"))
    return rc


def selftest_rn(op, lo_bits, hi_bits, device=0):
    """Exhaustive device check of the short IEEE sqrt (op 0) / reciprocal
    (op 1) Normalize uses (sc_selftest_rn): every f32 pattern in
    [lo_bits, hi_bits].  Returns (differs_from_full, differs_from_f64,
    checked, first_bad or None)."""
    L = load_library()
    out = (ctypes.c_uint64 * 4)()
    _check(L.sc_selftest_rn(device, op, lo_bits, hi_bits, out))
    return int(out[0]), int(out[1]), int(out[2]), (None if out[3] == 2**64 - 1 else int(out[3]))


def normalize_operand_range(max_w, max_h):
    """((ss_lo, ss_hi), (d_lo, d_hi)): Normalize's sqrt / reciprocal operand
    bounds for frames up to max_w x max_h (sc_normalize_operand_range)."""
    L = load_library()
    ss = (ctypes.c_double * 2)()
    d = (ctypes.c_double * 2)()
    L.sc_normalize_operand_range(max_w, max_h, ss, d)
    return (ss[0], ss[1]), (d[0], d[1])


def extract_patches(tmpl_w=40, tmpl_h=40):
    """DenseSURFFeatureExtractor::ExtractPatches (x, y, w, h rows)."""
    L = load_library()
    n = _check(L.sc_extract_patches(tmpl_w, tmpl_h, None, 0))
    r = np.zeros((n, 4), np.int32)
    L.sc_extract_patches(tmpl_w, tmpl_h, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n)
    return r


# ---------------------------------------------------------------------------
# post-processing (ObjDetector.cpp:223-231)
# ---------------------------------------------------------------------------

def _as_rects(rects):
    """RECT_DTYPE array from a RECT_DTYPE / WINDOW_DTYPE / RECORD_DTYPE array."""
    a = np.asarray(rects)
    if a.dtype == RECT_DTYPE:
        return np.ascontiguousarray(a)
    r = np.zeros(len(a), RECT_DTYPE)
    r["x"], r["y"], r["score"] = a["x"], a["y"], a["score"]
    r["width"], r["height"] = a["w"], a["h"]
    return r


def groupRectangles(rects, groupThreshold=2, eps=0.2):
    """cv::groupRectangles(wins, weights = 0s, levelWeights = scores, 2, 0.2) as the
    reference calls it (ObjDetector.cpp:224-225): mean rectangle and best score of
    each SimilarRects cluster with more than groupThreshold members."""
    L = load_library()
    r = _as_rects(rects)
    out = np.zeros(max(len(r), 1), RECT_DTYPE)
    n = ctypes.c_int32(0)
    _check(L.sc_group_rectangles(r.ctypes.data if len(r) else None, len(r), int(groupThreshold),
                                 float(eps), out.ctypes.data, len(out), ctypes.byref(n)))
    return out[:n.value].copy()


def group_detections(records, n_frames, groupThreshold=2, eps=0.2):
    """groupRectangles per frame over RECORD_DTYPE detections -> list of RECT_DTYPE arrays."""
    L = load_library()
    rec = np.ascontiguousarray(records, RECORD_DTYPE)
    out = np.zeros(max(len(rec), 1), RECT_DTYPE)
    counts = np.zeros(max(n_frames, 1), np.int32)
    n = ctypes.c_int32(0)
    _check(L.sc_group_detections(rec.ctypes.data if len(rec) else None, len(rec), n_frames,
                                 int(groupThreshold), float(eps), out.ctypes.data, len(out),
                                 counts.ctypes.data, ctypes.byref(n)))
    offs = np.concatenate([[0], np.cumsum(counts[:n_frames])])
    return [out[offs[f]:offs[f + 1]].copy() for f in range(n_frames)]


def fddb_format(name, rects):
    """The per-image block of the reference's surf.txt (ObjDetector.cpp:228-231)."""
    L = load_library()
    r = _as_rects(rects)
    need = ctypes.c_size_t(0)
    data = r.ctypes.data if len(r) else None
    rc = L.sc_fddb_format(name.encode(), data, len(r), None, 0, ctypes.byref(need))
    if rc < 0 and rc != -6:
        _check(rc)
    buf = ctypes.create_string_buffer(need.value + 1)
    _check(L.sc_fddb_format(name.encode(), data, len(r), buf, need.value + 1, ctypes.byref(need)))
    return buf.value.decode()


def fast_nms(rects, overlap_th=0.7):
    """fast_nms (ObjDetector.cpp:318-383; the reference calls it with 0.7 in the
    commented-out line :223): the picked rectangles in pick order."""
    L = load_library()
    r = _as_rects(rects)
    out = np.zeros(max(len(r), 1), RECT_DTYPE)
    n = ctypes.c_int32(0)
    _check(L.sc_fast_nms(r.ctypes.data if len(r) else None, len(r), float(overlap_th),
                         out.ctypes.data, len(out), ctypes.byref(n)))
    return out[:n.value].copy()


# ---------------------------------------------------------------------------
# input side (ObjDetector.cpp:164): cv::imread(path, IMREAD_GRAYSCALE) for JPEG
# ---------------------------------------------------------------------------

def _decode(call):
    w, h = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = call(None, 0, ctypes.byref(w), ctypes.byref(h))
    if rc != -6:
        _check(rc)
    img = np.zeros((h.value, w.value), np.uint8)
    _check(call(img.ctypes.data, img.nbytes, ctypes.byref(w), ctypes.byref(h)))
    return img


def decode_jpeg_gray(data: bytes):
    """JPEG bytes -> (H, W) uint8 luma plane (libjpeg JCS_GRAYSCALE, JDCT_ISLOW)."""
    L = load_library()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return _decode(lambda o, c, w, h: L.sc_decode_jpeg_gray(buf, len(data), o, c, w, h))


def imread_gray(path):
    """cv::imread(path, cv::IMREAD_GRAYSCALE) for a JPEG file."""
    L = load_library()
    p = os.fsencode(path)
    return _decode(lambda o, c, w, h: L.sc_imread_gray(p, o, c, w, h))


# ---------------------------------------------------------------------------
# model objects (CascadeClassifier.h, StageClassifier.h, LogisticRegression.h)
# ---------------------------------------------------------------------------

class LogisticRegression:
    def __init__(self, patch_index, w, bias):
        self.patch_index = int(patch_index)
        self.w = np.asarray(w, np.float32)
        self.bias = float(bias)


class StageClassifier:
    def __init__(self, theta, weak_classifiers):
        self.theta = np.float32(theta)
        self.weak_classifiers = weak_classifiers

    def GetFittedPatchIndexes(self):
        return [wk.patch_index for wk in self.weak_classifiers]


class CascadeClassifier:
    def __init__(self):
        self.stage_classifiers: list[StageClassifier] = []
        self._handle = None

    def GetFittedPatchIndexes(self):
        """CascadeClassifier::GetFittedPatchIndexes (CascadeClassifier.cpp:83-91)."""
        return [s.GetFittedPatchIndexes() for s in self.stage_classifiers]

    def _adopt(self, handle):
        L = load_library()
        if self._handle:
            L.sc_model_free(self._handle)
        self._handle = handle
        self.stage_classifiers = []
        for s in range(L.sc_model_num_stages(handle)):
            th, nw = ctypes.c_float(), ctypes.c_int()
            _check(L.sc_model_stage(handle, s, ctypes.byref(th), ctypes.byref(nw)))
            weaks = []
            for k in range(nw.value):
                pi, b = ctypes.c_int(), ctypes.c_double()
                w = (ctypes.c_float * 33)()
                _check(L.sc_model_weak(handle, s, k, ctypes.byref(pi), w, ctypes.byref(b)))
                weaks.append(LogisticRegression(pi.value, np.frombuffer(w, np.float32).copy(), b.value))
            self.stage_classifiers.append(StageClassifier(th.value, weaks))

    def __del__(self):
        if getattr(self, "_handle", None) and _lib is not None:
            _lib.sc_model_free(self._handle)
            self._handle = None


class Model:
    """Model(string cfg) with Load/Save returning EXIT_SUCCESS/EXIT_FAILURE
    (Model.h:15-18).  Unlike the reference, Load is strict: a missing key or
    a type mismatch fails (the message is in `last_error`)."""

    def __init__(self, model_cfg):
        self.model_cfg = str(model_cfg)
        self.last_error = ""

    def Load(self, cascade: CascadeClassifier):
        L = load_library()
        h = ctypes.c_void_p()
        rc = L.sc_model_load(self.model_cfg.encode(), ctypes.byref(h))
        if rc != SC_OK:
            self.last_error = L.sc_last_error().decode(errors="replace")
            self.last_code = rc
            return EXIT_FAILURE
        cascade._adopt(h.value)
        return EXIT_SUCCESS

    def Save(self, cascade: CascadeClassifier):
        L = load_library()
        if not cascade._handle:
            self.last_error = "cascade has no loaded model"
            return EXIT_FAILURE
        rc = L.sc_model_save(cascade._handle, self.model_cfg.encode())
        if rc != SC_OK:
            self.last_error = L.sc_last_error().decode(errors="replace")
            return EXIT_FAILURE
        return EXIT_SUCCESS

    @staticmethod
    def parse(text: str) -> CascadeClassifier:
        L = load_library()
        h = ctypes.c_void_p()
        b = text.encode()
        _check(L.sc_model_parse(b, len(b), ctypes.byref(h)))
        c = CascadeClassifier()
        c._adopt(h.value)
        return c


# ---------------------------------------------------------------------------
# detector
# ---------------------------------------------------------------------------

class Detector:
    """Owns device model + buffers + one HIP stream (sc_detector)."""

    _stream = None  # the stream object set_stream launches on (kept alive while in use)
    _sp_cache = None  # the detector's stream handle (refreshed by set_stream)

    def __init__(self, cascade, params: ScanParams | None = None, device: int = 0):
        L = load_library()
        self.params = params or ScanParams()
        h = ctypes.c_void_p()
        if isinstance(cascade, CascadeClassifier):
            _check(L.sc_detector_create_from_model(cascade._handle, ctypes.byref(self.params),
                                                   device, ctypes.byref(h)))
        else:
            _check(L.sc_detector_create(str(cascade).encode(), ctypes.byref(self.params), device,
                                        ctypes.byref(h)))
        self._h = h.value
        self.device = device

    def close(self):
        if self._h:
            load_library().sc_detector_destroy(self._h)
            self._h = None
        self._stream = None

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.sc_detector_destroy(self._h)
            self._h = None

    # -- host frames --------------------------------------------------------
    def detect(self, img, capacity=1 << 16):
        img = np.ascontiguousarray(img, np.uint8)
        H, W = img.shape
        out = np.zeros(capacity, WINDOW_DTYPE)
        n = ctypes.c_int()
        _check(load_library().sc_detect(self._h, img.ctypes.data, W, H, W, out.ctypes.data,
                                        capacity, ctypes.byref(n)))
        return out[:n.value]

    def detect_batch(self, frames, capacity=1 << 18):
        # frames go in as they lie when their rows are unit-stride (per-frame
        # pointers + row stride, as sc_detect_batch takes them); other layouts
        # are made row-major first
        frames = np.asarray(frames)
        if frames.dtype != np.uint8 or frames.ndim != 3 or frames.strides[2] != 1 \
                or frames.strides[1] < frames.shape[2]:
            frames = np.ascontiguousarray(frames, np.uint8)
        nf, H, W = frames.shape
        ptrs = (ctypes.c_void_p * nf)(*[frames[i].ctypes.data for i in range(nf)])
        out = np.zeros(capacity, WINDOW_DTYPE)
        counts = (ctypes.c_int * nf)()
        _check(load_library().sc_detect_batch(self._h, ptrs, nf, W, H, frames.strides[1], out.ctypes.data,
                                              capacity, counts))
        res, o = [], 0
        for c in counts:
            res.append(out[o:o + c].copy())
            o += c
        return res

    # -- device frames (torch uint8 tensor [n, H, W] on this device) --------
    @staticmethod
    def _device_frames(frames):
        """(n, H, W, row stride) of a uint8 [n, H, W] device tensor whose
        frames sit at data_ptr + f*H*stride with unit-stride rows (the C ABI's
        layout, sc_detect_device); anything else is refused, not copied."""
        if frames.dim() != 3 or frames.element_size() != 1 or not frames.is_cuda:
            raise ValueError("frames must be a uint8 [n, H, W] device tensor")
        n, H, W = frames.shape
        s0, s1, s2 = frames.stride()
        if s2 != 1 or s1 < W or (n > 1 and s0 != H * s1):
            raise ValueError("frames must be row-major [n, H, W] (strides %s)" % (frames.stride(),))
        return n, H, W, s1

    def _cur_stream(self):
        """torch's current stream on this device (raw handle; the Stream
        object torch.cuda.current_stream builds costs microseconds per call,
        which a one-frame call pays before its first kernel launches)."""
        import torch
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        return raw(self.device) if raw is not None else torch.cuda.current_stream(self.device).cuda_stream

    def _after_torch(self, *tensors):
        """Order the detector's stream after the work torch has queued on the
        current stream of this device (producers of `tensors`, earlier frees):
        sc_detector_wait_stream, no host sync.  Every tensor must live on the
        detector's GPU.  Returns torch's current stream (raw handle)."""
        for t in tensors:
            if t is not None and t.get_device() != self.device:
                raise ValueError("tensor on %s, detector on cuda:%d" % (t.device, self.device))
        s = self._cur_stream()
        if s != self._sp:  # (a detector on torch's current stream is ordered already)
            _check(load_library().sc_detector_wait_stream(self._h, s))
        return s

    def _before_torch(self, s=None):
        """Order torch's current stream (raw handle s, or looked up) after the
        detector's queued work."""
        if s is None:
            s = self._cur_stream()
        if s != self._sp:
            _check(load_library().sc_stream_wait_detector(self._h, s))

    def detect_device(self, frames, capacity=1 << 18):
        n, H, W, rs = self._device_frames(frames)
        self._after_torch(frames)
        out = np.zeros(capacity, WINDOW_DTYPE)
        counts = (ctypes.c_int * n)()
        _check(load_library().sc_detect_device(self._h, frames.data_ptr(), n, W, H, rs,
                                               out.ctypes.data, capacity, counts))
        res, o = [], 0
        for c in counts:
            res.append(out[o:o + c].copy())
            o += c
        return res

    def enqueue_device(self, frames, out_records, counts):
        """Async: out_records = torch uint8 [cap*40] (RECORD_DTYPE), counts = int32 [1+n].
        Stream-ordered like a torch op on the current stream: the scan waits for
        the work already queued there, and later work there waits for the scan."""
        n, H, W, rs = self._device_frames(frames)
        if counts.dtype != __import__("torch").int32 or counts.numel() < 1 + n:
            raise ValueError("counts must be an int32 tensor of at least 1 + n values")
        s = self._after_torch(frames, out_records, counts)
        cap = out_records.numel() * out_records.element_size() // RECORD_DTYPE.itemsize
        _check(load_library().sc_enqueue_device(self._h, frames.data_ptr(), n, W, H, rs,
                                                out_records.data_ptr(), cap, counts.data_ptr()))
        self._before_torch(s)

    def synchronize(self):
        _check(load_library().sc_synchronize(self._h))

    @property
    def stream_ptr(self):
        return load_library().sc_detector_stream(self._h)

    @property
    def _sp(self):  # the detector's stream as a raw int (0: the null stream), cached
        if self._sp_cache is None:
            self._sp_cache = self.stream_ptr or 0
        return self._sp_cache

    def set_stream(self, stream=None):
        """Launch on `stream` (a torch.cuda.Stream, or a raw hipStream_t of the
        detector's GPU, 0 = the null stream; None: the detector's own stream).
        On torch's current stream, enqueue_device needs no stream-order events
        (sc_detector_set_stream).  Lifetime: the detector keeps a reference to
        the stream object until set_stream(None) or close(), because it
        synchronises that stream when destroyed; a raw handle must stay valid
        for as long itself (the caller owns it)."""
        self._sp_cache = None
        if stream is None:
            _check(load_library().sc_detector_set_stream(self._h, None, 1))
            self._stream = None
        else:
            ptr = int(getattr(stream, "cuda_stream", stream))
            _check(load_library().sc_detector_set_stream(self._h, ptr or None, 0))
            self._stream = stream

    # -- introspection ---------------------------------------------------------
    def info(self, key):
        keys = {"levels": 1, "grid_windows": 2, "rows": 3, "table_pitch": 4, "visited": 5, "fused_frames": 6,
                "chain_waves": 7, "column_pass": 8, "spec_rounds": 9, "chain_subq": 10,
                "item_form": 11}
        v = ctypes.c_int64()
        _check(load_library().sc_detector_info(self._h, keys[key], ctypes.byref(v)))
        return v.value

    def set_debug(self, on=True):
        _check(load_library().sc_detector_set_debug(self._h, int(on)))

    def set_option(self, name, value):
        """sc_detector_set_option: a tuning / test choice (OPTIONS) for this detector."""
        _check(load_library().sc_detector_set_option(self._h, OPTIONS[name], int(value)))
        return self

    def set_options(self, **kw):
        for k, v in kw.items():
            self.set_option(k, v)
        return self

    def set_shard(self, rank, world):
        """Window-grid sharding (sc_detector_set_shard): evaluate only the
        (level, y) rows i with i % world == rank of every frame."""
        _check(load_library().sc_detector_set_shard(self._h, int(rank), int(world)))

    def dump_integral(self, W, H, frame=0):
        T = np.zeros((H + 1, W + 1, 8), np.float32)
        _check(load_library().sc_debug_dump(self._h, 1, frame, T.ctypes.data, T.nbytes))
        return T

    def dump_grid(self, frame=0):
        n = self.info("grid_windows")
        p = np.zeros(n, np.int16)
        s = np.zeros(n, np.float32)
        v = np.zeros(n, np.uint8)
        L = load_library()
        _check(L.sc_debug_dump(self._h, 2, frame, p.ctypes.data, p.nbytes))
        _check(L.sc_debug_dump(self._h, 3, frame, s.ctypes.data, s.nbytes))
        _check(L.sc_debug_dump(self._h, 4, frame, v.ctypes.data, v.nbytes))
        return p, s, v.astype(bool)

    def set_timing(self, on=True):
        _check(load_library().sc_set_timing(self._h, int(on)))

    def get_timing(self):
        ms = (ctypes.c_double * len(KERNELS))()
        n = (ctypes.c_int64 * len(KERNELS))()
        _check(load_library().sc_get_timing(self._h, ms, n))
        return {k: (ms[i], n[i]) for i, k in enumerate(KERNELS)}


class Miner(Detector):
    """DenseSURFFeatureExtractor::FillNegSamples' scan (hard-negative mining):
    every stride-10 window of levels tmpl_w * 1.1^k that the cascade accepts --
    or every window when there is no cascade yet (the first round)."""

    def __init__(self, cascade=None, tmpl_w=40, tmpl_h=40, device: int = 0):
        L = load_library()
        self.params = None
        self.tmpl_w, self.tmpl_h = tmpl_w, tmpl_h
        self._own = None
        if cascade is not None and not isinstance(cascade, CascadeClassifier):
            self._own = CascadeClassifier()
            if Model(str(cascade)).Load(self._own) != EXIT_SUCCESS:
                raise SurfCascadeError(-4, "cannot load model %s" % cascade)
            cascade = self._own
        h = ctypes.c_void_p()
        _check(L.sc_miner_create(cascade._handle if cascade is not None else None, tmpl_w, tmpl_h,
                                 device, ctypes.byref(h)))
        self._h = h.value
        self.device = device
        self.n_patches = len(extract_patches(tmpl_w, tmpl_h))

    def mine(self, img, capacity, features=True):
        """-> (windows WINDOW_DTYPE in (level, y, x) order, descriptors
        float32 [n, n_patches, 32] or None, total candidate count)."""
        img = np.ascontiguousarray(img, np.uint8)
        H, W = img.shape
        wins = np.zeros(max(capacity, 1), WINDOW_DTYPE)
        feat = np.zeros((max(capacity, 1), self.n_patches, 32), np.float32) if features else None
        n = ctypes.c_int()
        rc = load_library().sc_mine(self._h, img.ctypes.data, W, H, W, wins.ctypes.data,
                                    feat.ctypes.data if features else None, capacity,
                                    ctypes.byref(n))
        if rc != -6:
            _check(rc)
        k = min(n.value, capacity)
        return wins[:k].copy(), (feat[:k].copy() if features else None), n.value

    def mine_batch(self, imgs, capacity, features=True):
        """FillNegSamples over a list of same-size negative images in one pass
        -> (windows in (image, level, y, x) order, descriptors or None,
        per-image candidate counts int32 [n]); the first `capacity` windows of
        the batch are kept (an image's windows follow the previous image's)."""
        imgs = [np.ascontiguousarray(im, np.uint8) for im in imgs]
        H, W = imgs[0].shape
        if any(im.shape != (H, W) for im in imgs):
            raise ValueError("images of one size")
        ptrs = (ctypes.c_void_p * len(imgs))(*[im.ctypes.data for im in imgs])
        wins = np.zeros(max(capacity, 1), WINDOW_DTYPE)
        feat = np.zeros((max(capacity, 1), self.n_patches, 32), np.float32) if features else None
        counts = np.zeros(len(imgs), np.int32)
        rc = load_library().sc_mine_batch(self._h, ptrs, len(imgs), W, H, W, wins.ctypes.data,
                                          feat.ctypes.data if features else None, capacity,
                                          counts.ctypes.data)
        if rc != -6:
            _check(rc)
        k = min(int(counts.sum()), capacity)
        return wins[:k].copy(), (feat[:k].copy() if features else None), counts

    def mine_batch_device(self, frames, capacity, features=None):
        """Device frames (uint8 [n, H, W] tensor, rows contiguous) -> (windows,
        per-image counts); descriptors into `features` (device) when given."""
        if frames.dim() != 3 or frames.element_size() != 1 or not frames.is_cuda or frames.stride(2) != 1 \
                or frames.stride(0) != frames.shape[1] * frames.stride(1):
            raise ValueError("frames must be a uint8 [n, H, W] device tensor, frames back to back")
        n, H, W = frames.shape
        if features is not None and (not features.is_cuda or features.element_size() != 4
                                     or not features.is_contiguous()
                                     or features.numel() < capacity * self.n_patches * 32):
            raise ValueError("features must be a contiguous float32 device tensor of "
                             "capacity * n_patches * 32 values")
        self._after_torch(frames, features)
        wins = np.zeros(max(capacity, 1), WINDOW_DTYPE)
        counts = np.zeros(n, np.int32)
        rc = load_library().sc_mine_batch_device(self._h, frames.data_ptr(), n, W, H, frames.stride(1),
                                                 wins.ctypes.data,
                                                 features.data_ptr() if features is not None else None,
                                                 capacity, counts.ctypes.data)
        if rc != -6:
            _check(rc)
        return wins[:min(int(counts.sum()), capacity)].copy(), counts

    def mine_device(self, frame, capacity, features=None):
        """Device frame (uint8 [H, W] tensor) -> (windows, total); the
        descriptors go into `features` (float32 device tensor holding at least
        capacity * n_patches * 32 values) when given, never through the host."""
        if frame.dim() != 2 or frame.element_size() != 1 or not frame.is_cuda or frame.stride(1) != 1:
            raise ValueError("frame must be a row-major uint8 [H, W] device tensor")
        H, W = frame.shape
        if features is not None and (not features.is_cuda or features.element_size() != 4
                                     or not features.is_contiguous()
                                     or features.numel() < capacity * self.n_patches * 32):
            raise ValueError("features must be a contiguous float32 device tensor of "
                             "capacity * n_patches * 32 values")
        self._after_torch(frame, features)
        wins = np.zeros(max(capacity, 1), WINDOW_DTYPE)
        n = ctypes.c_int()
        rc = load_library().sc_mine_device(self._h, frame.data_ptr(), W, H, frame.stride(0),
                                           wins.ctypes.data,
                                           features.data_ptr() if features is not None else None,
                                           capacity, ctypes.byref(n))
        if rc != -6:
            _check(rc)
        return wins[:min(n.value, capacity)].copy(), n.value
