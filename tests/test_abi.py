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


def test_product_library_build_info(sc):
    """sc_build_info: the product library is no ablation, test-hook or
    profiling build, was built with no extra -D knobs, and its build id is the
    one the current sources give (bench.py stamps its line and checks the PMC
    table against it: a schedule change in sc_api.cpp makes the PMC stale)."""
    import importlib.util
    info = sc.build_info()
    assert info["arch"] == "gfx950"
    assert info["flags"] == "" and info["sanitizer"] == ""
    assert info["ablation"] is False and info["test_hooks"] is False and info["profiling"] is False
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert info["build_id"] == b.source_build_id(), "library older than its sources: rebuild"
    assert b.source_build_id("-DSC_TEST_HOOKS=1") != info["build_id"]


def test_test_hook_library_says_so():
    """The test-hook build (lib/testhooks) reports itself as one."""
    import json
    import subprocess
    import sys
    lib = os.path.join(ROOT, "surfcascade_amd", "lib", "testhooks", "libsurfcascade.so")
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); L.sc_build_info.restype=ctypes.c_char_p; "
            "print(L.sc_build_info().decode())")
    out = subprocess.run([sys.executable, "-c", "import torch; " + code, lib], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info["test_hooks"] is True and info["ablation"] is False
    assert info["flags"] == "-DSC_TEST_HOOKS=1"


def test_ablation_flags_refuse_to_build(tmp_path):
    """Every wrong-result timing ablation is an #error unless the build says
    it is an ablation build (SC_ABLATION_BUILD)."""
    import subprocess
    csrc = os.path.join(ROOT, "surfcascade_amd", "csrc")
    src = tmp_path / "probe.cpp"
    src.write_text('#include "sc_kernels.hpp"\nint main() { return 0; }\n')
    for flag in ("-DSC_ABL_NOWAIT=1", "-DSC_WALK_STORE=0", "-DSC_NO_WALK", "-DSC_ABL_EXTRA_RT=2",
                 "-DSC_ABL_EXTRA_EXP=1"):
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-fsyntax-only", "-I" + csrc,
               "-I" + os.path.join(ROOT, "include"), flag, str(src)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode != 0 and "timing ablation" in r.stderr, flag
        r = subprocess.run(cmd + ["-DSC_ABLATION_BUILD"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (flag, r.stderr[-1000:])
