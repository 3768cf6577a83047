"""Pin the CPU restatement (oracle/) with the hand-derivable known-answer tests
of SURVEY.md 8c and with independent numpy restatements of each step.

The reference ships no golden vectors / fixtures and executing it was denied
(SURVEY.md 8c), so these KATs + the committed fixtures in tests/golden/ are
what pins the oracle.
"""
import math

import numpy as np
import pytest

FLT_EPS = np.float32(2.0 ** -23)


# ---------------------------------------------------------------- geometry
def test_patch_counts_and_index_ranges(oracle):
    r = oracle.extract_patches(40, 40)
    assert len(r) == 608
    sq = (r[:, 2] == r[:, 3])
    tall = r[:, 2] < r[:, 3]
    wide = r[:, 2] > r[:, 3]
    assert sq[:344].all() and tall[344:476].all() and wide[476:].all()
    assert (r[:, 0] + r[:, 2] <= 40).all() and (r[:, 1] + r[:, 3] <= 40).all()
    assert tuple(r[-1]) == (0, 28, 40, 10)  # 4x1 shape, cell 10, last y at stride 4
    r2 = oracle.extract_patches(64, 128)
    assert len(r2) == 11870
    assert (r2[:, 2] == r2[:, 3]).sum() == 4970
    assert (r2[:, 2] < r2[:, 3]).sum() == 4900
    assert (r2[:, 2] > r2[:, 3]).sum() == 2000


def test_first_patches_follow_extract_order(oracle):
    # shape 2x2, cell 6 (12x12), y-major then x at stride 4 (cpp:51-60)
    r = oracle.extract_patches(40, 40)
    assert tuple(r[0]) == (0, 0, 12, 12)
    assert tuple(r[1]) == (4, 0, 12, 12)
    assert tuple(r[7]) == (28, 0, 12, 12)
    assert tuple(r[8]) == (0, 4, 12, 12)


def test_level_lengths(oracle):
    exp = [70, 77, 84, 93, 102, 112, 124, 136, 150, 165, 181, 199, 219, 241, 265, 292, 321, 353, 389,
           428, 470, 518, 569, 626]
    assert [oracle.level_len(70, i) for i in range(24)] == exp
    assert oracle.level_len(70, 31) == 1343
    assert [oracle.level_len(64, i) for i in (0, 22)] == [64, 520]


def test_default_level_counts(oracle):
    assert oracle.num_levels(1920, 1080, 70, 70) == 29
    assert oracle.num_levels(3840, 2160, 70, 70) == 36
    assert oracle.num_levels(640, 480, 70, 70) == 21


@pytest.mark.parametrize("W,H,params,count", [
    (640, 480, dict(n_levels=1), 26167),
    (1920, 1080, dict(n_levels=24), 3729192),
    (3840, 2160, dict(n_levels=32), 21302193),
    (1920, 1080, dict(base_len=64, aspect_h=2, n_levels=23), 2876145),
])
def test_grid_counts(oracle, W, H, params, count):
    assert oracle.grid_count(W, H, oracle.Params(**params)) == count


def test_theta_constant():
    th = np.float32(2) / np.sqrt(np.float32(32))
    assert th.view(np.uint32) == 0x3EB504F3


# ---------------------------------------------------------------- gradients
def _np_gradients(img):
    """Independent restatement of T2bFilter (DenseSURFFeatureExtractor.cpp:199-349)."""
    I = img.astype(np.int32)
    H, W = I.shape
    yy = np.arange(H)
    xx = np.arange(W)
    yu, yd = np.maximum(yy - 1, 0), np.minimum(yy + 1, H - 1)
    xp, xn = np.maximum(xx - 1, 0), np.minimum(xx + 1, W - 1)
    pairs = [(I[:, xn], I[:, xp]), (I[yd, :], I[yu, :]), (I[yd][:, xn], I[yu][:, xp]),
             (I[yu][:, xn], I[yd][:, xp])]
    g = []
    for In, Ip in pairs:
        d = In - Ip
        g.append((np.abs(d) - d) // 2)
        g.append((np.abs(d) + d) // 2)
    return np.stack(g).astype(np.uint8)


@pytest.mark.parametrize("W,H", [(2, 2), (17, 3), (64, 48), (301, 77)])
def test_gradients_match_numpy(oracle, W, H):
    img = np.random.default_rng(W * H).integers(0, 256, (H, W), dtype=np.uint8)
    np.testing.assert_array_equal(oracle.gradients(img), _np_gradients(img))


def test_vertical_step_edge(oracle):
    """KAT 5: step edge at column 10 of height 100: only dx+ (plane 1),
    du+/dv+ are nonzero, exactly at columns 9 and 10."""
    img = np.zeros((20, 30), np.uint8)
    img[:, 10:] = 100
    g = oracle.gradients(img)
    assert g[0].sum() == 0 and g[2].sum() == 0 and g[3].sum() == 0
    np.testing.assert_array_equal(np.nonzero(g[1][5])[0], [9, 10])
    assert (g[1][:, 9] == 100).all() and (g[1][:, 10] == 100).all()
    T = oracle.integral(img)
    # box sum of channel 1 over rows 0..19, columns 0..29 = 2 columns * 20 rows * 100
    assert T[20, 30, 1] == 4000.0


# ---------------------------------------------------------------- integral
def _np_integral(img):
    """Independent restatement of cv::integral(8U->32F) + merge: exact integer
    row prefix, sequential f32 column accumulation."""
    g = _np_gradients(img).astype(np.int64)
    C, H, W = g.shape
    R = np.zeros((C, H, W + 1), np.int64)
    R[:, :, 1:] = np.cumsum(g, axis=2)
    Rf = R.astype(np.float32)
    S = np.zeros((H + 1, W + 1, C), np.float32)
    for y in range(H):
        S[y + 1] = S[y] + Rf[:, y, :].T  # one f32 add per element
    return S


@pytest.mark.parametrize("W,H,seed", [(64, 48, 0), (640, 480, 1), (1920, 1080, 1000)])
def test_integral_matches_numpy(oracle, W, H, seed):
    from surfcascade_amd import synth
    img = synth.make_frame(W, H, seed)
    T = oracle.integral(img)
    assert T.view(np.uint32).tobytes() == _np_integral(img).view(np.uint32).tobytes()


def test_integral_exact_below_2_24(oracle):
    """KAT 6: all sums < 2^24 -> integral equals the exact integer integral."""
    img = np.random.default_rng(5).integers(0, 256, (60, 80), dtype=np.uint8)
    T = oracle.integral(img).astype(np.int64)
    g = _np_gradients(img).astype(np.int64)
    exact = np.zeros((61, 81, 8), np.int64)
    exact[1:, 1:, :] = np.cumsum(np.cumsum(g, axis=1), axis=2).transpose(1, 2, 0)
    np.testing.assert_array_equal(T, exact)


def test_integral_rounds_above_2_24(oracle):
    """1080p synthetic frames push the table past 2^24, where the f32 order matters."""
    from surfcascade_amd import synth
    img = synth.make_frame(1920, 1080, 1000)
    T = oracle.integral(img)
    assert T.max() > 2 ** 24
    g = _np_gradients(img).astype(np.int64)
    exact = np.cumsum(np.cumsum(g, axis=1), axis=2)[:, -1, -1]
    assert not np.array_equal(T[-1, -1].astype(np.int64), exact)  # rounding happened


# ---------------------------------------------------------------- normalize / LR
def _np_normalize(f):
    f = np.asarray(f, np.float32).copy()

    def ss(v):
        acc = FLT_EPS
        for k in range(8):
            q = v[4 * k:4 * k + 4] * v[4 * k:4 * k + 4]
            acc = np.float32(acc + np.float32(np.float32(q[0] + q[1]) + np.float32(q[2] + q[3])))
        return acc
    th = np.float32(0.35355338)
    t = np.float32(np.sqrt(ss(f)) * th)
    f = np.minimum(f, t)
    f = np.maximum(f, -t)
    r = np.float32(np.float32(1) / np.sqrt(ss(f)))
    return (f * r).astype(np.float32)


def _c_normalize(oracle, f):
    import ctypes
    a = np.ascontiguousarray(f, np.float32).copy()
    oracle.lib().sco_normalize(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return a


def test_normalize_unit_vector_clip_active(oracle):
    """KAT 7a: f = a*e_k: the single component is clipped to t, result t/sqrt(eps+t^2)."""
    f = np.zeros(32, np.float32)
    f[5] = 1234.0
    out = _c_normalize(oracle, f)
    exp = _np_normalize(f)
    assert out.view(np.uint32).tobytes() == exp.view(np.uint32).tobytes()
    assert np.count_nonzero(out) == 1 and 0.99 < out[5] <= 1.0


def test_normalize_uniform_vector(oracle):
    """KAT 7b: uniform vector: clip inactive-or-boundary, every entry ~ 1/sqrt(32)."""
    f = np.full(32, 3.0, np.float32)
    out = _c_normalize(oracle, f)
    assert out.view(np.uint32).tobytes() == _np_normalize(f).view(np.uint32).tobytes()
    np.testing.assert_allclose(out, 1 / math.sqrt(32), rtol=1e-6)


def test_normalize_random_matches_numpy(oracle):
    rng = np.random.default_rng(3)
    for _ in range(200):
        f = (rng.normal(0, 1, 32) * 10 ** rng.uniform(-2, 6)).astype(np.float32)
        assert (_c_normalize(oracle, f).view(np.uint32) == _np_normalize(f).view(np.uint32)).all()


def test_lr_zero_weights_is_sigmoid_of_bias(oracle):
    """KAT 8: w = 0, bias weight b -> (float)(1/(1+exp(-b)))."""
    import ctypes
    f = np.random.default_rng(1).normal(0, 1, 32).astype(np.float32)
    for b in (0.0, 0.5, -1.25, 3.0):
        w = np.zeros(33, np.float32)
        w[32] = b
        p = oracle.lib().sco_lr_predict(w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 1.0,
                                        f.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        assert np.float32(p) == np.float32(1.0 / (1.0 + math.exp(-float(np.float32(b)))))


def test_lr_dot_order(oracle):
    """Lane sums over i = 0,4,..,28 then (s0+s1)+(s2+s3) (LogisticRegression.cpp:55-63)."""
    import ctypes
    rng = np.random.default_rng(2)
    for _ in range(100):
        w = rng.normal(0, 1, 33).astype(np.float32)
        f = rng.normal(0, 1, 32).astype(np.float32)
        s = np.zeros(4, np.float32)
        for i in range(0, 32, 4):
            s = (w[i:i + 4] * f[i:i + 4]).astype(np.float32) + s
        z = np.float32(np.float32(s[0] + s[1]) + np.float32(s[2] + s[3]))
        prob = float(z) + float(w[32]) * 1.0
        exp = np.float32(1.0 / (1.0 + math.exp(-prob)))
        got = oracle.lib().sco_lr_predict(w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 1.0,
                                          f.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        assert np.float32(got) == exp


# ---------------------------------------------------------------- windows / detect loop
def _py_window(T, casc, l, x, y, patches):
    """Pure-Python restatement of one window's cascade (small cases only)."""
    scale = np.float32(np.float32(l) / np.float32(casc.tmpl_w))
    off = 0
    score = np.float32(0)
    for s in range(casc.n_stages):
        acc = np.float32(0)
        for k in range(casc.n_weak[s]):
            px, py, pw, ph = patches[casc.patch_index[off + k]]
            X = int(np.float32(px) * scale) + x
            Y = int(np.float32(py) * scale) + y
            if pw >= ph:
                h2 = int(np.float32(ph) * scale); w2 = h2 * (pw // ph)
            else:
                w2 = int(np.float32(pw) * scale); h2 = w2 * (ph // pw)
            ce = w2 // 2 if w2 == h2 else min(w2, h2)
            gw, gh = w2 // ce, h2 // ce
            f = np.zeros(32, np.float32)
            for hh in range(gh):
                for ww in range(gw):
                    x0, y0 = X + ww * ce, Y + hh * ce
                    cell = hh * gw + ww
                    f[8 * cell:8 * cell + 8] = (T[y0, x0] + T[y0 + ce, x0 + ce]) - \
                                               (T[y0, x0 + ce] + T[y0 + ce, x0])
            f = _np_normalize(f)
            w = casc.w[off + k]
            sl = np.zeros(4, np.float32)
            for i in range(0, 32, 4):
                sl = (w[i:i + 4] * f[i:i + 4]).astype(np.float32) + sl
            z = np.float32(np.float32(sl[0] + sl[1]) + np.float32(sl[2] + sl[3]))
            prob = float(z) + float(w[32]) * casc.bias[off + k]
            acc = np.float32(acc + np.float32(1.0 / (1.0 + math.exp(-prob))))
        score = np.float32(acc / np.float32(casc.n_weak[s]))
        off += casc.n_weak[s]
        if float(score) < float(casc.theta[s]):
            return s, score
    return casc.n_stages, score


def test_eval_window_matches_python(oracle, face_cascade):
    from surfcascade_amd import synth
    img = synth.make_frame(400, 300, 4)
    T = oracle.integral(img)
    patches = oracle.extract_patches(40, 40)
    rng = np.random.default_rng(0)
    import ctypes
    m = face_cascade.c()
    checked = 0
    for _ in range(60):
        l = int(rng.choice([70, 77, 84, 102]))
        x = int(rng.integers(0, (400 - l) // 3 + 1)) * 3
        y = int(rng.integers(0, (300 - l) // 3 + 1)) * 3
        s = ctypes.c_float()
        p = oracle.lib().sco_eval_window(T.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 400,
                                         ctypes.byref(m), l, l, x, y, 6.0, ctypes.byref(s), None)
        if p < 0:
            continue
        pp, ss = _py_window(T, face_cascade, l, x, y, patches)
        assert (p, np.float32(s.value).view(np.uint32)) == (pp, np.float32(ss).view(np.uint32))
        checked += 1
    assert checked > 10


def test_constant_image_walks_at_double_stride(oracle, face_cascade):
    """KAT 4: constant image: prefilter fails everywhere, each row visits
    ceil(nx/2) windows, no detections."""
    img = np.full((200, 300), 50, np.uint8)
    T = oracle.integral(img)
    assert not T.any()
    params = oracle.Params()
    dets, nvis = oracle.detect(T, face_cascade, params)
    layout, st = oracle.grid_layout(300, 200, params)
    exp = sum(ny * ((nx + 1) // 2) for (_i, _l, _lh, nx, ny, _b) in layout)
    assert len(dets) == 0 and nvis == exp


def test_single_stage_theta_zero_detects_every_visited(oracle, face_cascade):
    """KAT 10: one stage, theta = 0: every prefilter-passing visited window is a
    detection with score (s+1+1)/1, and such windows are followed at stride 1."""
    c = face_cascade
    one = oracle.Cascade(40, 40, np.array([4], np.int32), np.array([0.0], np.float32),
                         c.patch_index[:4], c.w[:4], c.bias[:4])
    from surfcascade_amd import synth
    img = synth.make_frame(320, 240, 9)
    T = oracle.integral(img)
    params = oracle.Params(n_levels=2)
    dets, nvis = oracle.detect(T, one, params)
    p, s = oracle.eval_grid(T, one, params)
    layout, _ = oracle.grid_layout(320, 240, params)
    vis, det = oracle.walk_rows(p, s, layout, 1)
    assert det.sum() == len(dets) > 0
    assert vis.sum() == nvis
    # every visited prefilter-passing window is a detection
    assert ((p >= 0) & vis).sum() == len(dets)
    sc = np.array([d["score"] for d in dets])
    np.testing.assert_array_equal(sc, s[det].astype(np.float64) + 2.0)


def test_walk_matches_reference_loop(oracle, face_cascade):
    from surfcascade_amd import synth
    img = synth.make_frame(640, 480, 1)
    T = oracle.integral(img)
    params = oracle.Params(n_levels=6)
    p, s = oracle.eval_grid(T, face_cascade, params)
    layout, _ = oracle.grid_layout(640, 480, params)
    vis, det = oracle.walk_rows(p, s, layout, face_cascade.n_stages)
    dets, nvis = oracle.detect(T, face_cascade, params)
    assert vis.sum() == nvis and det.sum() == len(dets)


def test_detect_deterministic_across_threads(oracle, face_cascade):
    from surfcascade_amd import synth
    img = synth.make_frame(640, 480, 2)
    T = oracle.integral(img)
    params = oracle.Params(n_levels=8)
    a, na = oracle.detect(T, face_cascade, params, nthreads=1)
    b, nb = oracle.detect(T, face_cascade, params, nthreads=8)
    assert na == nb and a.tobytes() == b.tobytes()


def test_prefilter_numpy_matches_c(oracle):
    from surfcascade_amd import synth
    img = synth.make_frame(320, 240, 3)
    T = oracle.integral(img)
    params = oracle.Params(n_levels=4)
    import ctypes
    pm = oracle.prefilter_mask(T, params)
    layout, st = oracle.grid_layout(320, 240, params)
    k = 0
    for (_i, l, lh, nx, ny, b) in layout:
        for r in range(ny):
            for j in range(nx):
                got = oracle.lib().sco_prefilter(T.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 320,
                                                 j * st, r * st, l, lh, 6.0, None)
                assert bool(got) == pm[k]
                k += 1


def test_mine_first_round_counts_every_stride10_window(oracle):
    """FillNegSamples (DenseSURFFeatureExtractor.cpp:146-161): with no stage
    every l x l window at stride 10 is a candidate, l = (int)(40 * 1.1^k)."""
    import math
    from surfcascade_amd import synth
    W, H = 333, 251
    T = oracle.integral(synth.make_frame(W, H, 4))
    nl = int(min(math.log(np.float32(W / np.float32(40))) / math.log(1.1),
                 math.log(np.float32(H / np.float32(40))) / math.log(1.1)))
    exp = sum(((H - l) // 10 + 1) * ((W - l) // 10 + 1)
              for l in (int(40 * 1.1 ** k) for k in range(nl + 1)) if l <= min(W, H))
    wins, feat, n = oracle.mine(T, oracle.empty_cascade(), 5)
    assert n == exp
    assert [tuple(w)[:5] for w in wins] == [(0, x, 0, 40, 40) for x in range(0, 50, 10)]
    # descriptor of window 0, patch 0 == CalcFeature of the patch itself
    r = oracle.extract_patches(40, 40)[0]
    f = np.zeros(32, np.float32)
    oracle.lib().sco_calc_feature(oracle._p(T, oracle._f32p), W,
                                  oracle._p(np.ascontiguousarray(r, np.int32), oracle._i32p),
                                  oracle._p(f, oracle._f32p))
    assert feat[0, 0].tobytes() == f.tobytes()


def test_exp_sensitivity_consistent_with_exposure(oracle, face_cascade):
    """The exact exp() sensitivity (VERDICT r2 Next 6) walks the same visited
    windows as the exposure counters: the same weak-evaluation count, and every
    evaluation whose f32 sigmoid an exp one f64 ulp off can flip lies within
    2 f64 ulp of an f32 rounding boundary."""
    from surfcascade_amd import synth
    T = oracle.integral(synth.make_frame(640, 480, 1000))
    params = oracle.Params(n_levels=6)
    ex = oracle.exposure(T, face_cascade, params)
    st, z = oracle.exp_sensitivity(T, face_cascade, params)
    assert st[0] == ex[0] > 0
    assert st[1] <= ex[1] and st[2] >= st[1] and len(z) == min(st[1], 4096)
    assert st[3] <= st[4] and st[5] <= st[4] and st[8] <= st[4]
