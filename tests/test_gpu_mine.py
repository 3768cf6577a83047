"""Hard-negative mining scan (DenseSURFFeatureExtractor::FillNegSamples,
DenseSURFFeatureExtractor.cpp:124-195) through the C ABI against the oracle
(oracle/sc_oracle.c sco_mine): candidate windows in (level, y, x) order and
their 608 x 32 descriptors, bit-exact."""
import numpy as np
import pytest

from conftest import FACE_CFG, PED_CFG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


def _frame(W, H, seed):
    from surfcascade_amd import synth
    return synth.make_frame(W, H, seed)


def _win(a):
    return [(int(r["level"]), int(r["x"]), int(r["y"]), int(r["w"]), int(r["h"])) for r in a]


def _check(got, ref):
    gw, gf, gn = got
    rw, rf, rn = ref
    assert gn == rn
    assert _win(gw) == _win(rw)
    assert gw["score"].astype(np.float32).tobytes() == rw["score"].astype(np.float32).tobytes()
    if rf is not None:
        assert gf.view(np.uint32).tobytes() == rf.view(np.uint32).tobytes()


@pytest.mark.parametrize("W,H,seed", [(320, 240, 3), (401, 233, 8)])
def test_first_round_every_window(sc, oracle, W, H, seed):
    """No stage yet (first == true): every stride-10 window is a candidate."""
    img = _frame(W, H, seed)
    m = sc.Miner(None)
    got = m.mine(img, 96)
    ref = oracle.mine(oracle.integral(img), oracle.empty_cascade(), 96)
    _check(got, ref)
    assert got[2] > 96  # capacity path: the first 96 in order, total reported


def test_with_cascade(sc, oracle, face_cascade):
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.42, np.float32)  # ~1300 candidates
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    img = _frame(480, 360, 17)
    casc_or = oracle.cascade_from_cfg(text)
    m = sc.Miner(sc.Model.parse(text))
    wins, feat, n = m.mine(img, 4096, features=False)
    rw, _, rn = oracle.mine(oracle.integral(img), casc_or, 4096, features=False)
    assert 0 < n == rn < 4096
    assert _win(wins) == _win(rw)
    _check(m.mine(img, 40), oracle.mine(oracle.integral(img), casc_or, 40))


def test_calibrated_model_and_tall_template(sc, oracle, face_cascade):
    img = _frame(360, 300, 23)
    T = oracle.integral(img)
    _check(sc.Miner(FACE_CFG).mine(img, 32), oracle.mine(T, face_cascade, 32))
    # FillNegSamples scans square l x l windows (Rect win(0, 0, l, l), :154): a 64x128
    # template's patches project below such a window (the reference would read past
    # it); the miner rejects that geometry instead of reading out of bounds
    with pytest.raises(sc.SurfCascadeError) as e:
        sc.Miner(PED_CFG, 64, 128).mine(img, 16)
    assert e.value.code == -1 and "leaves the window" in str(e.value)


def test_miner_is_not_a_detector(sc):
    m = sc.Miner(None)
    with pytest.raises(sc.SurfCascadeError):
        m.detect(_frame(200, 200, 1))


def test_mine_device_descriptors_stay_on_gpu(sc, oracle):
    # sc_mine_device: device frame in, descriptors into a device buffer; the
    # same windows and descriptor bits as sc_mine and the oracle
    import torch
    img = _frame(320, 240, 5)
    m = sc.Miner(None)
    cap = 64
    feats = torch.zeros(cap * m.n_patches * 32, dtype=torch.float32, device="cuda:0")
    wins, n = m.mine_device(torch.from_numpy(img).to("cuda:0"), cap, feats)
    hw, hf, hn = m.mine(img, cap)
    assert n == hn and _win(wins) == _win(hw)
    f = feats.view(cap, m.n_patches, 32)[:len(wins)].cpu().numpy()
    assert np.array_equal(f.view(np.uint32), hf.view(np.uint32))
    _check((wins, f, n), oracle.mine(oracle.integral(img), oracle.empty_cascade(), cap))


def _oracle_batch(oracle, imgs, casc, cap):
    """Per-image oracle scans concatenated in image order, the first `cap` kept."""
    ws, fs, counts = [], [], []
    for im in imgs:
        T = oracle.integral(im)
        _, _, n = oracle.mine(T, casc, 1 << 16, features=False)
        w, f, n = oracle.mine(T, casc, max(n, 1))
        w, f = w[:n], f[:n]
        ws.append(w)
        fs.append(f)
        counts.append(n)
    w = np.concatenate(ws)[:cap]
    f = np.concatenate(fs)[:cap]
    return w, f, counts


def test_mine_batch_matches_per_image_oracle(sc, oracle, face_cascade):
    # sc_mine_batch: FillNegSamples over an image list in one pass (the
    # reference's loop over negatives, DenseSURFFeatureExtractor.cpp:132-190);
    # the capacity cut falls inside the third image
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.42, np.float32)
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    casc_or = oracle.cascade_from_cfg(text)
    imgs = [_frame(240, 200, 60 + k) for k in range(5)]
    rw, rf, rc = _oracle_batch(oracle, imgs, casc_or, 1 << 20)
    assert min(rc) > 0
    m = sc.Miner(sc.Model.parse(text))
    cap = rc[0] + rc[1] + rc[2] // 2
    gw, gf, gc = m.mine_batch(imgs, cap)
    assert list(gc) == rc
    _check((gw, gf, sum(rc)), (rw[:cap], rf[:cap], sum(rc)))
    # everything kept, and the single-image entry point is the n = 1 batch
    gw, gf, gc = m.mine_batch(imgs, sum(rc), features=False)
    assert _win(gw) == _win(rw)
    w1, f1, n1 = m.mine(imgs[3], 1 << 12)
    assert n1 == rc[3] and _win(w1) == _win(rw[sum(rc[:3]):sum(rc[:4])])


def test_mine_batch_device_first_round(sc, oracle):
    import torch
    imgs = [_frame(200, 160, 70 + k) for k in range(3)]
    m = sc.Miner(None)
    cap = 700  # first round: every window; the cut falls in the second image
    feats = torch.zeros(cap * m.n_patches * 32, dtype=torch.float32, device="cuda:0")
    d = torch.from_numpy(np.stack(imgs)).to("cuda:0")
    wins, counts = m.mine_batch_device(d, cap, feats)
    rw, rf, rc = _oracle_batch(oracle, imgs, oracle.empty_cascade(), cap)
    assert list(counts) == rc and sum(rc) > cap
    f = feats.view(cap, m.n_patches, 32)[:len(wins)].cpu().numpy()
    _check((wins, f, sum(rc)), (rw, rf, sum(rc)))


@pytest.mark.parametrize("W,H", [(30, 60), (60, 39), (40, 40), (44, 300)])
def test_first_round_small_images(sc, oracle, W, H):
    """Negative images at and below the 40-px template: the scale count
    (int)min(log(W/40f)/log 1.1, log(H/40f)/log 1.1) is negative below 40 px
    and the reference's inclusive scale loop (DenseSURFFeatureExtractor.cpp:
    142-145) runs no scale; at 40 px exactly one window."""
    img = _frame(W, H, 31 + W + H)
    m = sc.Miner(None)
    got = m.mine(img, 64)
    ref = oracle.mine(oracle.integral(img), oracle.empty_cascade(), 64)
    _check(got, ref)
    assert (got[2] == 0) == (min(W, H) < 40)


def test_capacity_far_above_candidates(sc, oracle, face_cascade):
    """A trainer-style capacity (FillNegSamples' n_total) far above the
    candidates found: the descriptors are the oracle's, and the host-output
    path sizes its device descriptor buffer to the kept windows, not to the
    capacity (100 000 x 608 x 32 floats would be 7.8 GB)."""
    import torch
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.42, np.float32)
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    img = _frame(480, 360, 17)
    m = sc.Miner(sc.Model.parse(text))
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    got = m.mine(img, 100000)
    free1 = torch.cuda.mem_get_info(0)[0]
    ref = oracle.mine(oracle.integral(img), oracle.cascade_from_cfg(text), 100000)
    _check(got, ref)
    assert 0 < got[2] < 100000
    assert free0 - free1 < (1 << 30), "descriptor buffer sized to the capacity"
