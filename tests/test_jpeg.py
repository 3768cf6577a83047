"""Input side: cv::imread(path, IMREAD_GRAYSCALE) for
JPEG (ObjDetector.cpp:164) and the reference's fast_nms (:275-383).

JPEG parity is pinned against libjpeg-turbo: the committed fixtures in
tests/golden/ (tests/golden/make_jpeg_fixtures.py wrote them with Pillow) and,
where Pillow is importable, live encodes of many more shapes.  Pillow's
draft('L') asks libjpeg for JCS_GRAYSCALE output, exactly what OpenCV's
grayscale imread asks its bundled IJG libjpeg for; IJG islow and turbo's
islow are the same integer transform.  OpenCV itself is absent: parity with
its build is unpinned beyond that.  fast_nms is checked against the literal
Python restatement oracle.fast_nms and hand-derived cases.
"""
import glob
import io
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


def _pil():
    try:
        from PIL import Image
        return Image
    except ImportError:
        return None


def _pil_gray(data):
    Image = _pil()
    im = Image.open(io.BytesIO(data))
    im.draft("L", im.size)
    assert im.mode == "L"
    return np.asarray(im)


def test_golden_fixtures(sc, tmp_path):
    files = sorted(glob.glob(os.path.join(GOLDEN, "*.jpg")))
    assert len(files) >= 4
    for f in files:
        exp = np.load(f[:-4] + ".gray.npy")
        got = sc.imread_gray(f)
        assert got.shape == exp.shape and np.array_equal(got, exp), f
        with open(f, "rb") as fh:
            assert np.array_equal(sc.decode_jpeg_gray(fh.read()), exp)


def _scene(h, w, seed, mode):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = 128 + 90 * np.sin(x / (3.0 + seed % 5)) * np.cos(y / 9.0)
    rgb = np.stack([base, 255 - base, base * 0.5 + 60], -1) + rng.normal(0, 25, (h, w, 3))
    img = np.clip(rgb, 0, 255).astype(np.uint8)
    return img if mode == "RGB" else img[..., 0]


CASES = []
for i, (h, w) in enumerate([(1, 1), (8, 8), (9, 7), (16, 17), (33, 31), (120, 97), (480, 640)]):
    for mode, kw in [("RGB", dict(subsampling=2)), ("RGB", dict(subsampling=1)),
                     ("RGB", dict(subsampling=0)), ("L", {})]:
        for extra in ({}, {"progressive": True}, {"optimize": True}):
            CASES.append((h, w, i, mode, dict(kw, quality=[95, 75, 40][i % 3], **extra)))


@pytest.mark.parametrize("h,w,seed,mode,kw", CASES)
def test_matches_libjpeg_turbo(sc, h, w, seed, mode, kw):
    Image = _pil()
    if Image is None:
        pytest.skip("Pillow absent: the golden fixtures pin the decoder")
    b = io.BytesIO()
    Image.fromarray(_scene(h, w, seed, mode), mode).save(b, "JPEG", **kw)
    data = b.getvalue()
    got = sc.decode_jpeg_gray(data)
    assert np.array_equal(got, _pil_gray(data))


@pytest.mark.parametrize("kw", [dict(restart_marker_blocks=1), dict(restart_marker_blocks=5),
                                dict(restart_marker_rows=1), dict(restart_marker_rows=2)])
@pytest.mark.parametrize("prog", [False, True])
def test_restart_intervals(sc, kw, prog):
    Image = _pil()
    if Image is None:
        pytest.skip("Pillow absent")
    b = io.BytesIO()
    try:
        Image.fromarray(_scene(70, 83, 3, "RGB"), "RGB").save(b, "JPEG", quality=80,
                                                               progressive=prog, **kw)
    except TypeError:
        pytest.skip("this Pillow cannot write restart markers")
    data = b.getvalue()
    assert b"\xff\xdd" in data  # a DRI segment
    assert np.array_equal(sc.decode_jpeg_gray(data), _pil_gray(data))


def test_large_frame_matches(sc):
    Image = _pil()
    if Image is None:
        pytest.skip("Pillow absent")
    from surfcascade_amd import synth
    g = synth.make_frame(1920, 1080, 1000)
    rgb = np.stack([g, 255 - g, g // 2], -1)
    for prog in (False, True):
        b = io.BytesIO()
        Image.fromarray(rgb, "RGB").save(b, "JPEG", quality=85, progressive=prog)
        assert np.array_equal(sc.decode_jpeg_gray(b.getvalue()), _pil_gray(b.getvalue()))


def test_errors(sc, tmp_path):
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.decode_jpeg_gray(b"not a jpeg at all")
    assert e.value.code == -3
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.imread_gray(str(tmp_path / "missing.jpg"))
    assert e.value.code == -2
    f = sorted(glob.glob(os.path.join(GOLDEN, "*.jpg")))[0]
    data = open(f, "rb").read()
    with pytest.raises(sc.SurfCascadeError):
        sc.decode_jpeg_gray(data[:40])  # header cut inside a marker segment


# ---------------------------------------------------------------------------
# fast_nms (ObjDetector.cpp:318-383)
# ---------------------------------------------------------------------------

def _rects(rows):
    from surfcascade_amd import RECT_DTYPE
    return np.array(rows, RECT_DTYPE)


def test_fast_nms_kat(sc):
    # two heavily overlapping windows + one apart: the better of the pair and
    # the isolated one survive, best score first
    r = _rects([(0, 0, 40, 40, 0.7), (2, 2, 40, 40, 0.9), (100, 100, 40, 40, 0.8)])
    got = sc.fast_nms(r, 0.7)
    assert [tuple(x)[:4] for x in got] == [(2, 2, 40, 40), (100, 100, 40, 40)]
    # overlap 39*39/(41*41) = 0.905 > 0.7 suppresses; a 0.95 threshold keeps both
    assert len(sc.fast_nms(r, 0.95)) == 3
    # the area is normalised by the SUPPRESSED rectangle's (w+1)(h+1): a small
    # window inside a big one is removed, the big one inside a small best is not
    r = _rects([(0, 0, 100, 100, 0.5), (10, 10, 20, 20, 0.9)])
    assert len(sc.fast_nms(r, 0.7)) == 2
    r = _rects([(0, 0, 100, 100, 0.9), (10, 10, 20, 20, 0.5)])
    assert len(sc.fast_nms(r, 0.7)) == 1
    assert len(sc.fast_nms(_rects([]), 0.7)) == 0


def test_fast_nms_matches_restatement(sc, oracle):
    rng = np.random.default_rng(5)
    for trial in range(30):
        n = int(rng.integers(1, 90))
        xy = rng.integers(0, 200, (n, 2))
        s = rng.integers(20, 80, n)
        # coarse scores: many ties exercise the exchange sort's tie order
        score = np.round(rng.random(n) * (3 if trial % 2 else 100)) / 10
        r = _rects([(int(a), int(b), int(c), int(c), float(d)) for (a, b), c, d in zip(xy, s, score)])
        for th in (0.3, 0.7):
            got = sc.fast_nms(r, th)
            exp = oracle.fast_nms(r, th)
            assert got.tobytes() == exp.tobytes()
