"""Thread safety of the C ABI (include/surfcascade.h: distinct detectors may be
used from different threads; sc_last_error is thread-local).  Two threads run
the host entry points -- and, on a GPU, two detectors -- against the
ThreadSanitizer build of the host code (surfcascade_amd/lib/tsan, built by
__graft_entry__.build(); device code is not sanitised).  Any TSan report or a
result that differs from the single-threaded run fails the test."""
import glob
import os
import subprocess

import numpy as np
import pytest

from conftest import FACE_CFG, GOLDEN, ROOT

TSAN_LIB = os.path.join(ROOT, "surfcascade_amd", "lib", "tsan")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def threads_bin(tmp_path_factory):
    if not os.path.exists(os.path.join(TSAN_LIB, "libsurfcascade.so")):
        pytest.fail("TSan build missing: run __graft_entry__.build()")
    out = str(tmp_path_factory.mktemp("threads") / "threads_main")
    subprocess.check_call([CLANG, "-fsanitize=thread", "-std=c++17", "-O1", "-g",
                           "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "threads_main.cpp"), "-o", out,
                           "-L", TSAN_LIB, "-lsurfcascade", "-Wl,-rpath," + TSAN_LIB])
    return out


def _run(threads_bin, tmp_path, cfg_text):
    from surfcascade_amd import synth
    cfg = tmp_path / "m.cfg"
    cfg.write_text(cfg_text)
    frames = np.stack([synth.make_frame(320, 240, 40 + k) for k in range(3)])
    fp = tmp_path / "frames.u8"
    frames.tofile(fp)
    jpg = sorted(glob.glob(os.path.join(GOLDEN, "*.jpg")))[0]
    supp = os.path.join(ROOT, "tests", "tsan.supp")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 suppressions=" + supp)
    r = subprocess.run([threads_bin, str(cfg), str(fp), "320", "240", "3", jpg],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout.split()


def _permissive_cfg():
    # every theta at 0.45: windows reach the last stage, so the detections
    # the two threads compare are not an empty list
    from oracle import oracle as O
    from surfcascade_amd import synth
    base = O.cascade_from_cfg(open(FACE_CFG).read())
    return synth.write_cfg(synth.cascade_tree(base.n_weak, np.full(base.n_stages, 0.45, np.float32),
                                              base.patch_index, base.w, base.bias))


def test_threads_host_entry_points(threads_bin, tmp_path):
    out = _run(threads_bin, tmp_path, open(FACE_CFG).read())
    assert out[0] == "ok"


@pytest.mark.gpu
def test_threads_two_detectors(threads_bin, tmp_path):
    out = _run(threads_bin, tmp_path, _permissive_cfg())
    assert out[:2] == ["ok", "detect=1"]
    assert int(out[2].split("=")[1]) > 0
