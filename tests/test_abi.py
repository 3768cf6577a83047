"""The C-ABI library loads, exports every symbol include/surfcascade.h declares,
and reports errors through status codes (CPU only: no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import FACE_CFG, ROOT


@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


def _declared():
    text = open(os.path.join(ROOT, "include", "surfcascade.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sc_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(sc):
    L = sc.load_library()
    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(sc.EXPORTS)


def test_no_oracle_in_product_library(sc):
    """The product library must not link or embed the CPU restatement."""
    data = open(sc.library_path(), "rb").read()
    assert b"sco_" not in data
    assert b"sc_oracle" not in data


def test_version_and_defaults(sc):
    L = sc.load_library()
    assert b"gfx950" in L.sc_version()
    p = sc.ScanParams()
    q = sc.ScanParams()
    L.sc_scan_params_default(ctypes.byref(q))
    for f, _t in sc.ScanParams._fields_:
        assert getattr(p, f) == getattr(q, f), f
    assert (q.base_len, q.n_levels, q.step, q.tmpl_w, q.aspect_h) == (70, -1, 0, 40, 1)


def test_extract_patches_matches_oracle(sc, oracle):
    for tw, th in ((40, 40), (64, 128), (24, 24)):
        np.testing.assert_array_equal(sc.extract_patches(tw, th), oracle.extract_patches(tw, th))


def test_errors_are_status_codes(sc):
    L = sc.load_library()
    h = ctypes.c_void_p()
    rc = L.sc_detector_create(b"/nonexistent/model.cfg", None, 0, ctypes.byref(h))
    assert rc == -2 and b"nonexistent" in L.sc_last_error()
    assert L.sc_detect(None, None, 0, 0, 0, None, 0, None) == -1
    assert L.sc_model_stage(None, 0, None, None) == -1


def test_bad_scan_params_rejected(sc):
    c = sc.CascadeClassifier()
    sc.Model(FACE_CFG).Load(c)
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.Detector(c, sc.ScanParams(scale_factor=1.0))
    assert e.value.code == -1


def test_no_gpu_is_a_device_error_not_a_crash(sc):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    c = sc.CascadeClassifier()
    sc.Model(FACE_CFG).Load(c)
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.Detector(c)
    assert e.value.code == -5


def test_frame_layouts(sc):
    # synthetic frames are row-major (a column-major batch costs the host
    # boundary a full copy per call); device wrappers refuse what the C ABI
    # would misread
    import torch
    from surfcascade_amd import synth
    assert synth.make_frames(64, 48, 2).flags["C_CONTIGUOUS"]
    with pytest.raises(ValueError):
        sc.Detector._device_frames(torch.zeros(2, 48, 64, dtype=torch.uint8))  # host tensor


def test_option_keys_match_header():
    """surfcascade_amd.OPTIONS names exactly the header's SC_OPT_* values."""
    import re
    import surfcascade_amd as sc
    hdr = open(os.path.join(ROOT, "include", "surfcascade.h")).read()
    defs = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define SC_OPT_(\w+) (\d+)", hdr)}
    assert defs == sc.OPTIONS
