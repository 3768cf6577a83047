"""Post-processing: groupRectangles + FDDB block (ObjDetector.cpp:223-231).

cv::groupRectangles is OpenCV 3.0.0 objdetect, not vendored with the
reference and not importable here: the oracle (oracle/sc_oracle_group.c)
restates its published algorithm and is pinned by the hand-derived known
answers below ("parity unpinned" against OpenCV itself).  The product
(surfcascade_amd/csrc/sc_group.cpp, a sweep-based partition) must equal the
oracle exactly, including output order, on random and clustered inputs.
These run on the CPU: the product entry points need no GPU.
"""
import numpy as np
import pytest

import surfcascade_amd as sc
from oracle import oracle as O


def rects(rows):
    r = np.zeros(len(rows), sc.RECT_DTYPE)
    for i, t in enumerate(rows):
        r[i] = t
    return r


def as_tuples(r):
    return [tuple(int(v) for v in (q["x"], q["y"], q["width"], q["height"])) + (float(q["score"]),)
            for q in r]


BOTH = [sc.groupRectangles, O.group_rectangles]


@pytest.mark.parametrize("fn", BOTH)
def test_kat_cluster_of_three_passes_threshold_two(fn):
    r = rects([(10, 10, 40, 40, 0.7), (11, 10, 40, 40, 0.9), (12, 11, 41, 40, 0.8)])
    # sums 33/31/121/120 over 3: 11, 10.333 -> 10, 40.333 -> 40, 40
    assert as_tuples(fn(r)) == [(11, 10, 40, 40, 0.9)]


@pytest.mark.parametrize("fn", BOTH)
def test_kat_two_members_are_dropped(fn):
    r = rects([(10, 10, 40, 40, 0.7), (11, 10, 40, 40, 0.9)])
    assert len(fn(r)) == 0


@pytest.mark.parametrize("fn", BOTH)
def test_kat_mean_rounds_half_to_even(fn):
    # x sums 2 and 6 over 4 members: 0.5 -> 0, 1.5 -> 2 (cvRound, SSE2 ties-to-even)
    a = rects([(0, 0, 40, 40, 0.6), (1, 0, 40, 40, 0.6), (0, 0, 40, 40, 0.6), (1, 0, 40, 40, 0.6)])
    b = rects([(1, 0, 40, 40, 0.6), (2, 0, 40, 40, 0.6), (1, 0, 40, 40, 0.6), (2, 0, 40, 40, 0.6)])
    assert as_tuples(fn(a))[0][0] == 0
    assert as_tuples(fn(b))[0][0] == 2


@pytest.mark.parametrize("fn", BOTH)
def test_kat_similarity_is_transitive_through_chains(fn):
    # delta = 0.2 * (40 + 40) / 2 = 8: consecutive x differ by 8 (similar), ends by 24
    r = rects([(0, 0, 40, 40, 0.5), (8, 0, 40, 40, 0.6), (16, 0, 40, 40, 0.7), (24, 0, 40, 40, 0.8)])
    assert as_tuples(fn(r)) == [(12, 0, 40, 40, 0.8)]
    r2 = rects([(0, 0, 40, 40, 0.5), (9, 0, 40, 40, 0.6), (18, 0, 40, 40, 0.7)])  # 9 > 8
    assert len(fn(r2)) == 0


@pytest.mark.parametrize("fn", BOTH)
def test_kat_small_cluster_inside_big_one(fn):
    big = [(100, 100, 200, 200, 0.6)] * 5
    small = [(150, 150, 50, 50, 0.95)] * 3
    out = as_tuples(fn(rects(big + small)))
    assert out == [(100, 100, 200, 200, 0.6)]  # n2 = 5 > max(3, n1 = 3)
    out = as_tuples(fn(rects([(100, 100, 200, 200, 0.6)] * 3 + small)))
    assert len(out) == 2  # n2 = 3 is not > 3 and n1 is not < 3: both kept


@pytest.mark.parametrize("fn", BOTH)
def test_kat_empty_and_nonpositive_scores(fn):
    assert len(fn(rects([]))) == 0
    out = fn(rects([(5, 5, 30, 30, 0.0)] * 3))
    assert out["score"][0] == np.finfo(np.float64).tiny  # rejectWeights starts at DBL_MIN


def _random_scene(rng, n_clusters, per, spread, W=1920, H=1080):
    rows = []
    for _ in range(n_clusters):
        l = int(rng.integers(40, 400))
        cx, cy = int(rng.integers(0, W - l)), int(rng.integers(0, H - l))
        for _ in range(int(rng.integers(1, per + 1))):
            dl = int(rng.integers(-spread, spread + 1))
            rows.append((cx + int(rng.integers(-spread, spread + 1)),
                         cy + int(rng.integers(-spread, spread + 1)), l + dl, l + dl,
                         float(rng.random())))
    r = rects(rows)
    return r[rng.permutation(len(r))]


@pytest.mark.parametrize("seed", range(12))
def test_product_equals_oracle_random(seed):
    rng = np.random.default_rng(seed)
    r = _random_scene(rng, n_clusters=int(rng.integers(1, 80)), per=12, spread=int(rng.integers(1, 30)))
    for thr, eps in ((2, 0.2), (0, 0.2), (1, 0.1), (3, 0.35)):
        a, b = sc.groupRectangles(r, thr, eps), O.group_rectangles(r, thr, eps)
        assert a.tobytes() == b.tobytes(), (thr, eps)


def test_output_set_is_input_order_independent():
    rng = np.random.default_rng(99)
    r = _random_scene(rng, 60, 10, 12)
    a = sorted(as_tuples(sc.groupRectangles(r)))
    b = sorted(as_tuples(sc.groupRectangles(r[::-1].copy())))
    assert a == b


def test_large_input_matches_oracle():
    rng = np.random.default_rng(5)
    r = _random_scene(rng, 600, 15, 10)
    assert len(r) > 3000
    assert sc.groupRectangles(r).tobytes() == O.group_rectangles(r).tobytes()


def test_group_detections_per_frame():
    rng = np.random.default_rng(3)
    recs, per_frame = [], []
    for f in range(3):
        r = _random_scene(rng, 30, 8, 6)
        per_frame.append(r)
        for q in r:
            recs.append((f, 0, q["x"], q["y"], q["width"], q["height"], 10, 0, q["score"]))
    rec = np.array(recs, sc.RECORD_DTYPE)
    rec = rec[rng.permutation(len(rec))]
    got = sc.group_detections(rec, 3)
    for f in range(3):
        # group_detections feeds each frame in (level, y, x) order
        r = per_frame[f]
        r = r[np.lexsort((r["x"], r["y"]))]
        assert got[f].tobytes() == O.group_rectangles(r).tobytes()


def test_fddb_block_matches_oracle_and_stream_format():
    r = rects([(1, 2, 3, 4, 0.95345123), (10, 20, 30, 40, 1.0), (5, 6, 7, 8, 1.23456789e-5)])
    s = sc.fddb_format("2002/07/19/big/img_130", r)
    assert s == O.fddb_format("2002/07/19/big/img_130", r)
    assert s == ("2002/07/19/big/img_130\n3\n1 2 3 4 0.953451\n10 20 30 40 1\n"
                 "5 6 7 8 1.23457e-05\n")
    assert sc.fddb_format("x", rects([])) == "x\n0\n"
