"""The one-frame column pass in row segments (sc_integral.hip colblock +
colseg) restated in numpy, against the oracle's sequential integral
(DenseSURFFeatureExtractor.cpp:75, cv::integral's S_{y+1} = S_y + R_y in f32).

The rule: segment k = [ya, yb) starts a column from the exact integer sum of
the rows above ya when that sum is <= 2^24 (every partial sum is then an
integer f32 holds exactly); a column whose sum passes 2^24 above yb is walked
on to row H by the same segment; the later segments skip it.  This checks the
rule itself on the CPU (frames whose columns pass 2^24 early, late and never);
the GPU tests check the kernels' bits."""
import numpy as np
import pytest


def _colseg(R, seg):
    """R: (H, C) exact row prefixes (int64) -> (H, C) f32 column sums by the rule."""
    H, C = R.shape
    blk = 32
    nb = (H + blk - 1) // blk
    bs = np.add.reduceat(R, np.arange(0, nb * blk, blk).clip(max=H - 1), axis=0)[:nb]
    bs[-1] = R[(nb - 1) * blk:].sum(axis=0)
    S_out = np.full((H, C), np.nan, np.float32)
    owner = np.full((H, C), -1)
    for k, ya in enumerate(range(0, H, seg)):
        yb = min(H, ya + seg)
        ea = bs[:ya // blk].sum(axis=0)
        eb = ea + (bs[ya // blk:yb // blk].sum(axis=0) if yb < H else 0)
        act = ea <= 2 ** 24
        end = np.where(yb < H, np.where(eb <= 2 ** 24, yb, H), H)
        S = ea.astype(np.float32)  # exact where act
        for y in range(ya, int(end[act].max()) if act.any() else ya):
            w = act & (y < end)
            S = np.where(w, (S + R[y].astype(np.float32)).astype(np.float32), S)
            assert (owner[y, w] == -1).all(), "two segments write one row"
            owner[y, w] = k
            S_out[y, w] = S[w]
    assert (owner >= 0).all(), "a row no segment writes"
    return S_out


def _frames():
    rng = np.random.default_rng(7)
    smooth = (np.add.outer(np.arange(300), np.arange(260)) % 256).astype(np.uint8)
    noise = rng.integers(0, 256, (300, 260), dtype=np.uint8)
    checker = ((np.indices((300, 260)).sum(axis=0) % 2) * 255).astype(np.uint8)
    # period-4 stripes: every pixel's horizontal gradient is 255, so the wide
    # columns pass 2^24 from row ~110 on (the order-sensitive regime)
    stripes = np.tile(np.array([0, 0, 255, 255], np.uint8), (300, 300))
    return {"smooth": smooth, "noise": noise, "checker": checker, "stripes": stripes}


@pytest.mark.parametrize("name", ["smooth", "noise", "checker", "stripes"])
@pytest.mark.parametrize("seg", [32, 96, 160])
def test_colseg_rule_matches_sequential_integral(oracle, name, seg):
    img = _frames()[name]
    G = oracle.gradients(img).astype(np.int64)  # (8, H, W)
    R = np.cumsum(G, axis=2)  # exact row prefixes through column x
    H, W = img.shape
    R2 = R.transpose(1, 2, 0).reshape(H, W * 8)
    T = oracle.integral(img)[1:, 1:, :].reshape(H, W * 8)
    got = _colseg(R2, seg)
    assert got.view(np.uint32).tobytes() == T.view(np.uint32).tobytes()
    if name == "stripes":  # the order-sensitive regime, from the middle rows on
        first = (np.cumsum(R2, axis=0) > 2 ** 24).argmax(axis=0)
        assert (R2.sum(axis=0) > 2 ** 24).any() and 64 < first[first > 0].min() < 200
