"""Memory and UB safety of the host code that parses untrusted bytes (SURVEY.md
section 5: host ASan / UBSan build), with seeded mutation corpora.

The reference's boundary is a parse of bytes from disk: Model::Load ->
libconfig (Model.cpp:104-116; scanner.c:1111-1190) and cv::imread
(ObjDetector.cpp:164).  tests/cpp/fuzz_main.cpp mutates seed inputs --
truncation, bit flips, extreme 16-bit fields, marker-segment drops /
duplicates / splices / re-typing for JPEG; dictionary tokens, deep nesting,
huge arrays, long escaped strings, @include loops, NaN / inf / hex / int64
literals for model.cfg; extreme int32 rectangles and NaN / inf scores for
groupRectangles / fast_nms / the FDDB writer; random frames, cascades and
parameters for the CPU restatement (oracle/) -- and calls the C ABI of the
AddressSanitizer + UndefinedBehaviorSanitizer build of the host code
(surfcascade_amd/lib/asan, built by __graft_entry__.build(); device code is
not sanitised).  Every input must return a documented status code; any
sanitizer report (memory error, leak, signed overflow, bad shift, float-cast
overflow, null argument) aborts the run and fails the test.  The bugs these
runs found are fixed, each with a regression case below (against the product
library) or in test_jpeg.py / test_model_io.py.
"""
import glob
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import FACE_CFG, GOLDEN, ROOT

ASAN_LIB = os.path.join(ROOT, "surfcascade_amd", "lib", "asan")
CLANG = "/opt/rocm/lib/llvm/bin/clang"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-O1", "-g"]
N = 5000  # mutations per parser


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if not os.path.exists(os.path.join(ASAN_LIB, "libsurfcascade.so")):
        pytest.fail("ASan/UBSan build missing: run __graft_entry__.build()")
    d = tmp_path_factory.mktemp("fuzz")
    objs = []
    for src in ("sc_oracle.c", "sc_oracle_group.c"):  # the checker, sanitised too
        o = str(d / (src + ".o"))
        subprocess.check_call([CLANG] + SAN + ["-std=c99", "-ffp-contract=off", "-msse3", "-Wno-unknown-pragmas",
                                               "-c", os.path.join(ROOT, "oracle", src), "-o", o])
        objs.append(o)
    out = str(d / "fuzz_main")
    subprocess.check_call([CLANG + "++"] + SAN + ["-std=c++17", "-I", os.path.join(ROOT, "include"),
                                                  os.path.join(ROOT, "tests", "cpp", "fuzz_main.cpp")] + objs +
                          ["-o", out, "-L", ASAN_LIB, "-lsurfcascade", "-Wl,-rpath," + ASAN_LIB, "-lm"])
    return out


def _small_cfg():
    """A 2-stage, 5-weak cascade in Model::Save's text (a fast seed)."""
    from oracle import oracle as O
    from surfcascade_amd import synth
    base = O.cascade_from_cfg(open(FACE_CFG).read())
    return synth.write_cfg(synth.cascade_tree(np.array([2, 3], np.int32), np.array([0.4, 0.5], np.float32),
                                              base.patch_index[:5], base.w[:5], base.bias[:5]))


def _run(fuzz_bin, tmp_path, mode, seed, n, files=()):
    env = dict(os.environ, FUZZ_TMP=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin, mode, str(seed), str(n)] + list(files), capture_output=True, text=True,
                       env=env, timeout=600)
    bad = ("AddressSanitizer", "LeakSanitizer", "runtime error", "FUZZ FAILURE")
    assert r.returncode == 0 and not any(b in r.stderr for b in bad), r.stderr[-4000:]
    m = re.match(r"%s n=(\d+)((?: st-?\d+=\d+)*)" % mode, r.stdout.strip())
    assert m and int(m.group(1)) == n, r.stdout
    return {int(k): int(v) for k, v in re.findall(r"st(-?\d+)=(\d+)", m.group(2))}


def test_fuzz_jpeg(fuzz_bin, tmp_path):
    seeds = sorted(glob.glob(os.path.join(GOLDEN, "*.jpg")))
    assert len(seeds) >= 11
    st = _run(fuzz_bin, tmp_path, "jpeg", 20261018, N, seeds)
    # both outcomes occur: corrupt files refused, decodable mutants decoded
    assert st.get(-3, 0) > N // 10 and st.get(100, 0) > N // 10, st


def test_fuzz_cfg(fuzz_bin, tmp_path):
    seed = tmp_path / "small.cfg"
    seed.write_text(_small_cfg())
    st = _run(fuzz_bin, tmp_path, "cfg", 20261018, N, [str(seed)])
    assert st.get(-3, 0) > N // 2 and st.get(0, 0) > 20, st
    # the full 190-weak face model as the seed (slower per case)
    _run(fuzz_bin, tmp_path, "cfg", 7, 300, [FACE_CFG])


def test_fuzz_group(fuzz_bin, tmp_path):
    st = _run(fuzz_bin, tmp_path, "group", 20261018, N)
    assert st.get(0, 0) > N // 2, st


def test_fuzz_oracle(fuzz_bin, tmp_path):
    _run(fuzz_bin, tmp_path, "oracle", 20261018, 2000)


def test_sanitizer_build_says_so(fuzz_bin):
    """The library under test is the sanitizer build, and its build id is its
    own: the Makefile hashes ARCH and SAN with the sources, so a
    PMC table or bench line stamped with the product id never matches it."""
    import importlib.util
    import json
    r = subprocess.run([fuzz_bin, "info", "0", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout)
    assert "-fsanitize=address,undefined" in info["sanitizer"] and info["arch"] == "gfx950"
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert info["build_id"] == b.source_build_id(san=info["sanitizer"])
    assert info["build_id"] != b.source_build_id()


# ---- regression cases of what the runs found (product library) -----------

@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


def _segment(data, marker):
    i = data.index(bytes([0xFF, marker]))
    return i, int.from_bytes(data[i + 2:i + 4], "big")


def test_jpeg_overfull_huffman_table_is_a_parse_error(sc):
    """A DHT with more codes of some length than that many bits can hold
    (here 5 one-bit codes) used to write past the 512-entry lookahead table;
    it is now refused as libjpeg refuses it (jdhuff.c JERR_BAD_HUFF_TABLE)."""
    data = bytearray(open(os.path.join(GOLDEN, "gray_q60_opt.jpg"), "rb").read())
    i, _ = _segment(data, 0xC4)
    data[i + 5] = 5  # counts[1] (after FF C4, length, Tc/Th)
    with pytest.raises(sc.SurfCascadeError, match="Huffman"):
        sc.decode_jpeg_gray(bytes(data))


def test_jpeg_huge_dimensions_are_refused_before_allocation(sc):
    """A 65535 x 65535 SOF in a few hundred bytes used to allocate the 8.6-GB
    coefficient plane; frames above 2^28 px are refused (twice what a detector
    accepts)."""
    data = bytearray(open(os.path.join(GOLDEN, "gray_q60_opt.jpg"), "rb").read())
    i, _ = _segment(data, 0xC0)
    data[i + 5:i + 9] = b"\xff\xff\xff\xff"  # height, width
    with pytest.raises(sc.SurfCascadeError, match="2\\^28"):
        sc.decode_jpeg_gray(bytes(data))


def test_cfg_nesting_bound(sc):
    """Nesting beyond 1000 aggregates is a parse error (it overflowed the
    stack before); 999 levels still parse (the model is then rejected for
    its missing keys, SC_ERR_MODEL, not for its syntax)."""
    def nested(d):
        return "x = " + "(" * d + "1" + ")" * d + ";\n"
    with pytest.raises(sc.SurfCascadeError, match="nested too deeply") as e:
        sc.Model.parse(nested(200000))
    assert e.value.code == -3
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.Model.parse(nested(999))
    assert e.value.code == -4


def test_group_extreme_rectangles(sc):
    """int32-extreme rectangles (sums past INT32_MAX) group and suppress with
    64-bit coordinate arithmetic: same result as OpenCV's int arithmetic
    wherever that does not overflow, defined everywhere else."""
    big = 2**31 - 1
    rects = np.array([(big - 10, big - 10, 100, 100, 0.9), (big - 12, big - 11, 100, 100, 0.8),
                      (big - 9, big - 10, 100, 100, 0.7), (-big, -big, big, big, 0.5)], sc.RECT_DTYPE)
    g = sc.groupRectangles(rects, 2, 0.2)
    assert len(g) == 1
    kept = sc.fast_nms(rects, 0.7)
    assert len(kept) >= 2
