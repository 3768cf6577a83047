"""GPU parity: the HIP path (through the C ABI) against the CPU restatement.

Bit-exact: integral tables, per-window stage reached, per-window last stage
score (f32 bits), visited set and detection windows; detection scores
(f64) compared exactly as well (tolerance stated by north_star: 1e-5, the
test demands equality and reports the max |diff| if it ever fails).
"""
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


def _det_set(arr):
    return sorted((int(r["level"]), int(r["y"]), int(r["x"]), int(r["w"]), int(r["h"]),
                   int(r["stage"]), float(r["score"])) for r in arr)


@pytest.mark.parametrize("passes", ["1", "2"])
@pytest.mark.parametrize("layout", ["0", "1"])
@pytest.mark.parametrize("W,H,seed", [(640, 480, 1), (1920, 1080, 1000), (257, 131, 7), (2, 2, 3),
                                      (3000, 67, 5)])
def test_integral_bit_exact(sc, oracle, W, H, seed, layout, passes):
    """Both integral forms (colstrip; rowfull + colsum, the small-batch default)."""
    img = _frame(W, H, seed)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1)).set_option("table_layout", int(layout))
    det.set_option("integral_passes", int(passes))
    det.detect(img)  # frames smaller than the window: no rows, integral still built
    T = det.dump_integral(W, H)
    ref = oracle.integral(img)
    assert T.view(np.uint32).tobytes() == ref.view(np.uint32).tobytes()


def _grid_parity(sc, oracle, cascade, cfg, img, params_sc, params_or, model_text=None, det_out=None, **opts):
    det = sc.Detector(sc.Model.parse(model_text) if model_text else cfg, params_sc).set_options(**opts)
    if det_out is not None:
        det_out.append(det)
    det.set_debug(True)
    wins = det.detect(img)
    p, s, v = det.dump_grid()
    T = oracle.integral(img)
    rp, rs = oracle.eval_grid(T, cascade, params_or)
    assert len(p) == len(rp)
    # lazy grid (default): only windows the x chain reaches are evaluated (-2
    # elsewhere); the full_grid option evaluates all of them
    ev = p != -2
    np.testing.assert_array_equal(p[ev], rp[ev])
    assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
    H, W = img.shape
    layout, _ = oracle.grid_layout(W, H, params_or)
    rv, rdm = oracle.walk_grid(rp, rs, layout, cascade.n_stages, params_or.stride_score)
    np.testing.assert_array_equal(v, rv)
    assert ev[rv.astype(bool)].all()  # every visited window was evaluated
    ref, nvis = oracle.detect(T, cascade, params_or)
    assert det.info("visited") == nvis == int(rv.sum())
    assert _det_set(wins) == _det_set(ref)
    return wins, p


def test_grid_parity_640x480_single_scale(sc, oracle, face_cascade):
    img = _frame(640, 480, 1)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=1),
                 oracle.Params(n_levels=1))


@pytest.mark.parametrize("full", [None, "1"])
def test_grid_parity_1080p_24_levels(sc, oracle, face_cascade, full):
    img = _frame(1920, 1080, 1000)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=24),
                 oracle.Params(n_levels=24), full_grid=int(full or 0))


def test_grid_parity_default_levels_odd_size(sc, oracle, face_cascade):
    img = _frame(803, 611, 11)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(), oracle.Params())


@pytest.mark.parametrize("W,H,n_lv,l_last", [(1920, 1080, 29, 1009), (3840, 2160, 36, 1967)])
def test_grid_parity_reference_level_count(sc, oracle, face_cascade, W, H, n_lv, l_last):
    """The scan the reference itself runs on the headline frame sizes: the
    default ScanParams take the level count from ObjDetector.cpp:174
    ((int)min(log(W/70)/log(1.1), log(H/70)/log(1.1)) + 1: 29 levels at 1080p,
    36 at 4K) and l_i = (int)(70 * 1.1^i) (:180), so the widest level is
    l = 1009 / 1967.  Table, per-window stage / score bits, visited set and
    detections against the oracle."""
    img = _frame(W, H, 4242)
    params = oracle.Params()
    assert oracle.effective_levels(W, H, params) == n_lv
    layout, _ = oracle.grid_layout(W, H, params)
    assert len(layout) == n_lv and layout[-1][1] == l_last and layout[-1][3] > 0
    dets = []
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(), params, det_out=dets)
    assert dets[0].info("levels") == n_lv
    T = dets[0].dump_integral(W, H)
    assert T.view(np.uint32).tobytes() == oracle.integral(img).view(np.uint32).tobytes()


@pytest.mark.parametrize("chunk_min,substrips,band_rows,layout,full", [
    ("1", None, None, None, "1"), ("40", None, "3", "0", "1"), (None, "3", "1", "1", "1"),
    (None, "2", "5", None, "1"), ("1", None, "2", "1", "1"), (None, None, None, "0", None),
    (None, None, None, "1", None), ("1", None, None, None, None), (None, None, None, None, "1")])
def test_grid_parity_kernel_paths(sc, oracle, face_cascade, chunk_min, substrips,
                                  band_rows, layout, full):
    """The one-lane-per-window stage path (used for stages with more weak
    classifiers than the item buffer holds), other strip splits, band heights
    and both table cell formats give the same bits as the defaults."""
    opts = {k: int(v) for k, v in (("chunk_min", chunk_min), ("substrips", substrips),
                                   ("band_rows", band_rows), ("table_layout", layout),
                                   ("full_grid", full)) if v}
    img = _frame(1280, 720, 77)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=8),
                 oracle.Params(n_levels=8), **opts)
    if layout:
        det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1)).set_option("table_layout", int(layout))
        det.detect(img)
        T = det.dump_integral(*img.shape[::-1])
        assert T.view(np.uint32).tobytes() == oracle.integral(img).view(np.uint32).tobytes()


@pytest.mark.parametrize("order,block", [("0", None), ("1", None), ("2", "5"), ("2", None), ("3", "5")])
def test_chain_row_orders(sc, oracle, face_cascade, order, block):
    """The chain kernel's task order (level-major, y-major, row blocks top-down
    or bottom-up; one-frame launches deal the explicitly set order instead of
    their default bottom-up blocks of 8) changes the schedule only, never the
    bits."""
    opts = {"row_order": int(order)}
    if block:
        opts["row_block"] = int(block)
    img = _frame(1280, 720, 78)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=8),
                 oracle.Params(n_levels=8), **opts)


@pytest.mark.parametrize("phases,wgs,full", [("1", None, None), ("1", None, "1"), ("2", None, "1"),
                                              (None, "1", None), (None, "1", "1"), (None, "2", "1")])
def test_phase_planes_and_workgroups(sc, oracle, face_cascade, phases, wgs, full):
    """SC_OPT_PHASES (one or two phase planes per step: the chain kernel's
    per-item column mapping takes the ph == step branch with 1) and
    SC_OPT_WGS_PER_CU, on both window kernels: the schedule and layout
    change, the bits do not."""
    opts = {k: int(v) for k, v in (("phases", phases), ("wgs_per_cu", wgs), ("full_grid", full)) if v}
    img = _frame(1280, 720, 80)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=8),
                 oracle.Params(n_levels=8), **opts)


@pytest.mark.parametrize("waves,lw", [("12", None), ("16", None), ("16", "0"), ("12", "0"), ("8", None), ("8", "0"),
                                     ("10", None), ("14", None)])
def test_chain_waves(sc, oracle, face_cascade, waves, lw):
    """SC_OPT_CHAIN_WAVES: the 8-, 10- and 14-wave (A/B), 12-wave (3 per SIMD) and
    16-wave (4 per SIMD, rematerialised lane values, 128 VGPRs) chain
    kernels, with the weights in LDS or read through the caches, give the
    oracle's bits."""
    opts = {"chain_waves": int(waves)}
    if lw:
        opts["lds_weights"] = int(lw)
    img = _frame(1280, 720, 82)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=8),
                 oracle.Params(n_levels=8), **opts)


@pytest.mark.parametrize("lo,hi", [(2, 5), (6, 0)])
def test_level_range_scan(sc, oracle, face_cascade, lo, hi):
    """SC_OPT_LEVEL_LO / _HI (level-group profiling) scan exactly the levels
    [lo, hi): their windows, visited set and detections are the oracle's, the
    other levels are neither evaluated nor visited."""
    img = _frame(1280, 720, 81)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=8)).set_options(level_lo=lo, level_hi=hi)
    det.set_debug(True)
    wins = det.detect(img)
    p, s, v = det.dump_grid()
    params = oracle.Params(n_levels=8)
    T = oracle.integral(img)
    rp, rs = oracle.eval_grid(T, face_cascade, params)
    layout, _ = oracle.grid_layout(1280, 720, params)
    rv, _ = oracle.walk_grid(rp, rs, layout, face_cascade.n_stages, params.stride_score)
    inr = np.zeros(len(p), bool)
    for (lv, _l, _lh, nx, ny, base) in layout:
        if lv >= lo and (hi == 0 or lv < hi):
            inr[base:base + nx * ny] = True
    assert (p[~inr] == -2).all() and (v[~inr] == 0).all()
    ev = (p != -2) & inr
    np.testing.assert_array_equal(p[ev], rp[ev])
    np.testing.assert_array_equal(v[inr], rv[inr])
    assert det.info("visited") == int(rv[inr].sum())
    ref, _ = oracle.detect(T, face_cascade, params)
    ref = [r for r in ref if r["level"] >= lo and (hi == 0 or r["level"] < hi)]
    assert len(ref) > 0 or hi != 0
    assert _det_set(wins) == _det_set(ref)


@pytest.mark.parametrize("n", [2, 3, 4])
def test_integral_batch_frames(sc, oracle, n):
    """Every frame of a batch: 2 and 3 frames take the two-pass integral
    (rowfull + colsum), 4 take colstrip; odd sizes, so strips and rows end
    ragged."""
    frames = np.stack([_frame(577, 301, 900 + k) for k in range(n)])
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=2))
    det.set_debug(True)
    det.detect_batch(frames)
    for k in range(n):
        T = det.dump_integral(577, 301, frame=k)
        assert T.view(np.uint32).tobytes() == oracle.integral(frames[k]).view(np.uint32).tobytes()


@pytest.mark.parametrize("n,opts", [(2, {"integral_fuse": 2, "integral_pre": 1}), (5, {"integral_pre": 2}),
                                    (7, {"chain_chunk": 3, "integral_fuse": 2}), (4, {}),
                                    (4, {"integral_fuse": 1}), (6, {"integral_pre": 1, "chain_waves": 12}),
                                    (5, {"chain_waves": 8})])
def test_fused_integral(sc, oracle, face_cascade, n, opts):
    """The integral's column walks inside the chain kernel (SC_OPT_INTEGRAL_FUSE,
    the default from 4 frames per launch): every frame's table, evaluated
    windows, visited set and detections are the oracle's -- with 1 or 2
    frames integrated ahead, several launches (chain_chunk 3: 3 + 3 + 1
    frames), both chain-kernel widths and fusion off.  Two batches through one
    detector, so the second reads table lines the first left in the caches."""
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=5)).set_options(**opts)
    det.set_debug(True)
    params = oracle.Params(n_levels=5)
    fuse, pre = opts.get("integral_fuse", 0), opts.get("integral_pre", 0) or 2
    chunk = opts.get("chain_chunk", n)
    launches = [min(chunk, n - f0) for f0 in range(0, n, chunk)]
    fused = sum(nc - pre for nc in launches if fuse != 1 and nc >= (2 if fuse == 2 else 4) and nc > pre)
    for rep in range(2):
        frames = np.stack([_frame(641, 483, 3000 + 37 * rep + k) for k in range(n)])
        batch = det.detect_batch(frames)
        assert det.info("fused_frames") == fused
        layout, _ = oracle.grid_layout(641, 483, params)
        for k in range(n):
            T = oracle.integral(frames[k])
            assert det.dump_integral(641, 483, frame=k).view(np.uint32).tobytes() == T.view(np.uint32).tobytes()
            p, s, v = det.dump_grid(frame=k)
            rp, rs = oracle.eval_grid(T, face_cascade, params)
            ev = p != -2
            np.testing.assert_array_equal(p[ev], rp[ev])
            assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
            rv, _ = oracle.walk_grid(rp, rs, layout, face_cascade.n_stages, params.stride_score)
            np.testing.assert_array_equal(v, rv)
            ref, _ = oracle.detect(T, face_cascade, params)
            assert _det_set(batch[k]) == _det_set(ref)


@pytest.mark.parametrize("segs", ["1", "2", "8"])
def test_chain_segments_per_row(sc, oracle, face_cascade, segs):
    """A single frame with other segment counts than its default 4: the
    evaluated windows, visited set and detections stay the oracle's."""
    img = _frame(1280, 720, 79)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=8),
                 oracle.Params(n_levels=8), chain_segs=int(segs))


@pytest.mark.parametrize("segs", [None, "8"])
def test_speculative_rounds_run_and_match(sc, oracle, face_cascade, segs):
    """One-frame launches (12 waves) speculate: an idle wave evaluates a
    waiting task's first windows, both parities, before its entry arrives;
    the task then enters mid-batch (rel > 0) over bits it did not clear.
    The test asserts the path actually ran (SC_INFO_SPEC_ROUNDS) and that the
    evaluated windows, visited set and detections are still the oracle's
    (ADVICE r3), with the default 4 and with 8 segments per row (more
    hand-offs, more waiting tasks, entries across segment boundaries)."""
    img = _frame(1920, 1080, 1000)
    dets = []
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=24),
                 oracle.Params(n_levels=24), det_out=dets, **({"chain_segs": int(segs)} if segs else {}))
    assert dets[0].info("chain_waves") == 12
    assert dets[0].info("spec_rounds") > 0


@pytest.mark.parametrize("spec", ["2", "64"])
def test_speculation_depth(sc, oracle, face_cascade, spec):
    """SC_OPT_CHAIN_SPEC: a waiting task gets up to `spec` speculative rounds,
    each the next 2 x 128 windows of its segment (both parities), merged into
    its bits at the round's offset; 64 evaluates whole segments ahead of their
    entries.  Speculative rounds run (their count depends on the schedule),
    and every evaluated window, the visited set and the detections stay the
    oracle's."""
    img = _frame(1920, 1080, 1000)
    dets = []
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=24),
                 oracle.Params(n_levels=24), det_out=dets, chain_spec=int(spec))
    assert dets[0].info("spec_rounds") > 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_one_frame_grid_shards_speculate(sc, oracle, face_cascade, world):
    """The single-frame grid split as bench.py --shard grid runs it: rank r of
    W scans rows i % W == r of ONE frame in a one-frame launch, whose idle
    waves speculate whole segments (SC_OPT_CHAIN_SPEC auto for a shard).
    Each rank's evaluated windows are the oracle's; the union of the ranks'
    windows and their visited counts are the unsharded result, W = 2 / 4 / 8."""
    img = _frame(1920, 1080, 1000)
    params = oracle.Params(n_levels=24)
    T = oracle.integral(img)
    ref, nv = oracle.detect(T, face_cascade, params)
    rp, rs = oracle.eval_grid(T, face_cascade, params)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=24))
    det.set_debug(True)
    got, vsum = [], 0
    for rank in range(world):
        det.set_shard(rank, world)
        wins = det.detect(img)
        assert det.info("spec_rounds") > 0
        p, s, _v = det.dump_grid()
        ev = p != -2
        np.testing.assert_array_equal(p[ev], rp[ev])
        assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
        got += _det_set(wins)
        vsum += det.info("visited")
    assert sorted(got) == _det_set(ref)
    assert vsum == nv


@pytest.mark.parametrize("lds_weights", [None, "0"])
def test_pedestrian_64x128(sc, oracle, ped_cascade, lds_weights):
    # lds_weights 0: the cache-read weights variant (models too big for the LDS)
    img = _frame(960, 540, 21)
    _grid_parity(sc, oracle, ped_cascade, PED_CFG, img,
                 sc.ScanParams.pedestrian(n_levels=12),
                 oracle.Params(base_len=64, aspect_h=2, n_levels=12),
                 **({"lds_weights": int(lds_weights)} if lds_weights else {}))


@pytest.mark.parametrize("full", [None, "1"])
def test_permissive_cascade_many_detections(sc, oracle, face_cascade, full):
    """Lowered thetas: many windows reach the last stage (detections + stride 1)."""
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.2, np.float32)
    tree = synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias)
    text = synth.write_cfg(tree)
    casc_sc = sc.Model.parse(text)
    casc_or = oracle.cascade_from_cfg(text)
    img = _frame(640, 480, 2)
    det = sc.Detector(casc_sc, sc.ScanParams(n_levels=3)).set_option("full_grid", int(full or 0))
    wins = det.detect(img)
    T = oracle.integral(img)
    ref, nvis = oracle.detect(T, casc_or, oracle.Params(n_levels=3))
    assert len(ref) > 100
    assert _det_set(wins) == _det_set(ref)
    assert det.info("visited") == nvis


def test_lazy_grid_wide_rows_and_frame_chunks(sc, oracle, face_cascade):
    """Row segments wider than one 64-window batch per parity (several rounds per
    task) and a batch split into several chain-kernel launches (frame chunks)."""
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.3, np.float32)  # many good windows: frequent parity switches
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    casc_or = oracle.cascade_from_cfg(text)
    frames = np.stack([_frame(3000, 160, 700 + k) for k in range(5)])
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=3)).set_option("chain_chunk", 2)
    batch = det.detect_batch(frames)
    vis = 0
    for k in range(5):
        ref, nv = oracle.detect(oracle.integral(frames[k]), casc_or, oracle.Params(n_levels=3))
        assert _det_set(batch[k]) == _det_set(ref)
        vis += nv
    assert det.info("visited") == vis
    assert sum(len(b) for b in batch) > 100


@pytest.mark.parametrize("segs", [None, "1", "2", "4", "8"])
def test_batch_equals_single(sc, oracle, face_cascade, segs):
    """Batches (8 segments per row by default) equal single frames (4 by
    default) and the oracle; forced segment counts change the schedule only."""
    frames = np.stack([_frame(640, 480, 100 + k) for k in range(4)])
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=5))
    if segs:
        det.set_option("chain_segs", int(segs))
    batch = det.detect_batch(frames)
    for k in range(4):
        single = det.detect(frames[k])
        assert _det_set(single) == _det_set(batch[k])
        T = oracle.integral(frames[k])
        ref, _ = oracle.detect(T, face_cascade, oracle.Params(n_levels=5))
        assert _det_set(single) == _det_set(ref)


def test_constant_image_no_windows(sc):
    """KAT 4: constant image -> zero gradients -> prefilter fails everywhere."""
    img = np.full((300, 400), 77, np.uint8)
    det = sc.Detector(FACE_CFG, sc.ScanParams())
    det.set_debug(True)
    assert len(det.detect(img)) == 0
    p, s, v = det.dump_grid()
    ev = p != -2  # lazy grid: with every window rejected the chain stays on one parity
    assert (p[ev] == -1).all()
    # every visited window was evaluated (idle waves of the 12-wave kernel may
    # also evaluate the other parity of a waiting segment ahead of its entry)
    assert ev[v.astype(bool)].all()
    # every row walked at stride 2*step: visited = ceil(nx/2) per row
    assert det.info("visited") == int(v.sum())


def test_device_resident_frames(sc, oracle, face_cascade):
    import torch
    frames = np.stack([_frame(640, 480, 300 + k) for k in range(2)])
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=4))
    dev = torch.from_numpy(frames).to("cuda:0")
    res = det.detect_device(dev)
    for k in range(2):
        T = oracle.integral(frames[k])
        ref, _ = oracle.detect(T, face_cascade, oracle.Params(n_levels=4))
        assert _det_set(res[k]) == _det_set(ref)


def test_strided_frames(sc, oracle, face_cascade):
    # frames handed over as row-strided views (a crop of wider buffers): host
    # batch through per-frame pointers + row stride, device tensor likewise
    import torch
    wide = np.stack([_frame(700, 480, 310 + k) for k in range(2)])
    view = wide[:, :, 30:670]
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=4))
    host = det.detect_batch(view)
    dev = det.detect_device(torch.from_numpy(wide).to("cuda:0")[:, :, 30:670])
    for k in range(2):
        T = oracle.integral(np.ascontiguousarray(view[k]))
        ref, _ = oracle.detect(T, face_cascade, oracle.Params(n_levels=4))
        assert _det_set(host[k]) == _det_set(ref)
        assert _det_set(dev[k]) == _det_set(ref)
    with pytest.raises(ValueError):  # column-major frames are refused, not misread
        det.detect_device(torch.from_numpy(wide).to("cuda:0").transpose(1, 2))


@pytest.mark.parametrize("pitch,off", [(644, 0), (643, 0), (700, 30), (700, 32)])
def test_integral_device_pitch(sc, oracle, pitch, off):
    """Device frames whose rows start 4-B aligned (pitch 644 / 700 at column
    offset 0 / 32) take the dword-load rowcarry4 kernel, the others (pitch
    643, offset 30) the byte-load rowcarry; a 641-px row ends inside a dword.
    Every frame's table is bit-exact either way (3 frames: two-pass column
    pass; 5 frames: colstrip or the fused walks)."""
    import torch
    W, H = 641, 301
    rng = np.random.default_rng(pitch + off)
    for n in (3, 5):
        buf = rng.integers(0, 256, (n, H, pitch), dtype=np.uint8)
        view = buf[:, :, off:off + W]
        det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=2))
        det.set_debug(True)
        det.detect_device(torch.from_numpy(buf).to("cuda:0")[:, :, off:off + W])
        for k in range(n):
            T = det.dump_integral(W, H, frame=k)
            ref = oracle.integral(np.ascontiguousarray(view[k]))
            assert T.view(np.uint32).tobytes() == ref.view(np.uint32).tobytes(), (n, k)


def test_capacity_error_reports_count(sc):
    from surfcascade_amd import synth
    from oracle import oracle as O
    oc = O.cascade_from_cfg(open(FACE_CFG).read())
    text = synth.write_cfg(synth.cascade_tree(oc.n_weak, np.zeros(oc.n_stages, np.float32),
                                              oc.patch_index, oc.w, oc.bias))
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=1))
    img = _frame(640, 480, 1)
    with pytest.raises(sc.SurfCascadeError) as e:
        det.detect(img, capacity=3)
    assert e.value.code == -6


def test_grouped_detections_match_oracle(sc, oracle, face_cascade):
    """Detect (GPU) -> groupRectangles (host) equals the oracle's detect -> group,
    i.e. the reference's surf.txt block for the frame (ObjDetector.cpp:224-231)."""
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.25, np.float32)
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=6))
    frames = np.stack([_frame(640, 480, 500 + k) for k in range(3)])
    got = det.detect_batch(frames)
    casc_or = oracle.cascade_from_cfg(text)
    n_groups = 0
    for k in range(3):
        ref, _ = oracle.detect(oracle.integral(frames[k]), casc_or, oracle.Params(n_levels=6))
        assert _det_set(got[k]) == _det_set(ref)
        a = sc.groupRectangles(got[k])
        b = oracle.group_rectangles(sc._as_rects(ref))
        assert a.tobytes() == b.tobytes()
        assert sc.fddb_format("f%d" % k, a) == oracle.fddb_format("f%d" % k, b)
        n_groups += len(a)
    assert n_groups > 0


@pytest.mark.parametrize("world", [2, 3, 8])
def test_grid_shards_union_equals_whole(sc, oracle, face_cascade, world):
    """Single-frame window-grid sharding: the ranks' row sets
    partition the grid and the union of their raw windows (and visited counts)
    is the unsharded result, which equals the oracle's."""
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.45, np.float32)  # ~10^4 detections per frame
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    frames = np.stack([_frame(1920, 1080, 1000 + k) for k in range(2)])
    casc_or = oracle.cascade_from_cfg(text)
    ref, vis = [], 0
    for k in range(2):
        r, nv = oracle.detect(oracle.integral(frames[k]), casc_or, oracle.Params(n_levels=24))
        ref.append(_det_set(r))
        vis += nv
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=24))
    got = [[], []]
    vsum, nrows = 0, 0
    for rank in range(world):
        det.set_shard(rank, world)
        res = det.detect_batch(frames)
        for k in range(2):
            got[k] += _det_set(res[k])
        vsum += det.info("visited")
        nrows += det.info("rows")
    det.set_shard(0, 1)
    whole = det.detect_batch(frames)
    assert nrows == det.info("rows")
    for k in range(2):
        assert sorted(got[k]) == ref[k] == _det_set(whole[k])
    assert vsum == vis == det.info("visited")
    assert sum(len(r) for r in ref) > 100


def test_jpeg_to_detections(sc, oracle, face_cascade):
    """imread(IMREAD_GRAYSCALE) -> detect, the reference's per-image sequence
    (ObjDetector.cpp:164-220), against the oracle on the same decoded plane."""
    import io
    PIL = pytest.importorskip("PIL.Image")
    from surfcascade_amd import synth
    g = synth.make_frame(640, 480, 77)
    b = io.BytesIO()
    PIL.fromarray(np.stack([g, g // 2, 255 - g], -1), "RGB").save(b, "JPEG", quality=90)
    img = sc.decode_jpeg_gray(b.getvalue())
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=4))
    ref, _ = oracle.detect(oracle.integral(img), face_cascade, oracle.Params(n_levels=4))
    assert _det_set(det.detect(img)) == _det_set(ref)


@pytest.mark.parametrize("W,H", [(60, 50), (70, 70), (71, 400), (400, 71), (76, 90), (69, 1000)])
def test_small_frames_default_levels(sc, oracle, face_cascade, W, H):
    """Frames at and below the base window (ObjDetector.cpp:174-186: the level
    count (int)min(log(W/70)/log 1.1, log(H/70)/log 1.1) + 1 is 0 below 70 px,
    one row / one column of windows at exactly 70): detections, scores and
    visited counts equal the oracle's, with a permissive cascade so windows
    that exist reach the last stage."""
    from surfcascade_amd import synth
    c = face_cascade
    theta = np.full(c.n_stages, 0.3, np.float32)
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    casc_or = oracle.cascade_from_cfg(text)
    img = _frame(W, H, 4242 + W + H)
    ref, nvis = oracle.detect(oracle.integral(img), casc_or, oracle.Params())
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams())
    got = det.detect(img)
    assert _det_set(got) == _det_set(ref)
    assert det.info("visited") == nvis
    if min(W, H) < 70:
        assert nvis == 0 and len(ref) == 0
    else:
        assert nvis > 0 and len(ref) > 0


@pytest.mark.parametrize("base,step,pk,ss,full", [(48, 0, 4.0, 0.6, None), (100, 7, 8.0, 0.4, None),
                                                  (40, 1, 6.0, 0.5, None), (48, 0, 4.0, 0.6, "1")])
def test_grid_parity_scan_parameters(sc, oracle, face_cascade, base, step, pk, ss, full):
    """sc_scan_params beyond the reference's constants (ObjDetector.cpp:104,
    139, 188, 214): window base, row/column step (0 = base/20), prefilter
    factor and the adaptive-stride score threshold, on both window kernels."""
    img = _frame(480, 360, 90 + base + step)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img,
                 sc.ScanParams(base_len=base, step=step, prefilter_k=pk, stride_score=ss, n_levels=6),
                 oracle.Params(base_len=base, step=step, prefilter_k=pk, stride_score=ss, n_levels=6),
                 full_grid=int(full or 0))


@pytest.mark.parametrize("full", [None, "1"])
def test_grid_parity_large_stages(sc, oracle, face_cascade, full):
    """A cascade whose stages outgrow the per-wave item buffer (700 weak
    classifiers: the one-lane-per-window stage path) and whose weights do not
    fit the LDS (2 200 weak: weights read through the caches)."""
    from surfcascade_amd import synth
    c = face_cascade
    n_weak = [700, 1500]
    idx = np.arange(sum(n_weak)) % len(c.patch_index)
    text = synth.write_cfg(synth.cascade_tree(n_weak, np.array([0.5, 0.5], np.float32),
                                              c.patch_index[idx], c.w[idx], c.bias[idx]))
    casc = oracle.cascade_from_cfg(text)
    img = _frame(320, 240, 3)
    det_params = sc.ScanParams(n_levels=2)
    _, p = _grid_parity(sc, oracle, casc, None, img, det_params, oracle.Params(n_levels=2),
                        model_text=text, full_grid=int(full or 0))
    assert (p == 0).any() and (p == 2).any()  # stage 0 rejects some windows, some pass both


@pytest.mark.parametrize("kind", ["checker", "noise", "zeros", "white", "stripes"])
@pytest.mark.parametrize("passes", ["1", "2"])
def test_integral_extreme_content(sc, oracle, kind, passes):
    """Content at the ends of the value range (T2bFilter + integral_,
    DenseSURFFeatureExtractor.cpp:73-76, 199-349): a one-pixel 0/255
    checkerboard gives the largest gradients everywhere (in-strip sums at
    64 x 255, table values near 5e8, far past 2^24), noise, flat frames and
    vertical stripes (every column's dx saturated, dy zero)."""
    W, H = 1920, 1080
    yy, xx = np.mgrid[0:H, 0:W]
    img = {"checker": ((xx + yy) & 1) * 255,
           "noise": np.random.default_rng(7).integers(0, 256, (H, W)),
           "zeros": np.zeros((H, W)),
           "white": np.full((H, W), 255),
           "stripes": (xx & 1) * 255}[kind].astype(np.uint8)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1)).set_option("integral_passes", int(passes))
    det.detect(img)
    T = det.dump_integral(W, H)
    ref = oracle.integral(img)
    assert T.view(np.uint32).tobytes() == ref.view(np.uint32).tobytes()


@pytest.mark.parametrize("W,H,amp", [(1920, 1080, 40), (1000, 517, 160)])
def test_one_frame_column_pass_in_segments(sc, oracle, W, H, amp):
    """One frame's column pass in row segments (colblock + colseg,
    SC_INFO_COLUMN_PASS 3): period-4 stripes of amplitude `amp` make every
    column's sum grow linearly, so the right-hand columns pass 2^24 inside a
    middle segment (that segment walks them on to the bottom, the later ones
    skip them) while the left-hand ones never do; the ragged height ends in a
    short segment.  The table must still be the reference's, bit for bit."""
    xx = np.mgrid[0:H, 0:W][1]
    img = (((xx >> 1) & 1) * amp).astype(np.uint8)
    ref = oracle.integral(img)
    over = ref[1:] > 2 ** 24
    first = np.where(over.any(axis=0), over.argmax(axis=0), H)
    assert 0 < first.min() < H // 2 and (first == H).any()  # crossings mid-frame, and none
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1))
    det.detect(img)
    assert det.info("column_pass") == 3
    T = det.dump_integral(W, H)
    assert T.view(np.uint32).tobytes() == ref.view(np.uint32).tobytes()


@pytest.mark.parametrize("kind", ["noise", "checker"])
@pytest.mark.parametrize("W,H", [(2051, 1000), (4099, 700), (2305, 333)])
def test_one_frame_merged_integral_odd_wide(sc, oracle, W, H, kind):
    """The one-frame merged launch (rowcarry4_colblk: row carries plus the
    exact 32-row column-block sums colseg starts from) at odd widths above
    2048: its block role walks more than 8 passes of 256 columns, so the
    running sum crosses chunks, AND the last pass is partial (lanes past W,
    the byte-wise tail of the dword pixel loads).  ADVICE r5: neither the
    soak (W <= 900) nor the 4K tests (3840 = 15 x 256) combine the two."""
    yy, xx = np.mgrid[0:H, 0:W]
    img = (np.random.default_rng(W + H).integers(0, 256, (H, W)) if kind == "noise"
           else ((xx + yy) & 1) * 255).astype(np.uint8)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1))
    det.detect(img)
    assert det.info("column_pass") == 3
    T = det.dump_integral(W, H)
    assert T.view(np.uint32).tobytes() == oracle.integral(img).view(np.uint32).tobytes()


@pytest.mark.parametrize("layout", ["0", "1"])
@pytest.mark.parametrize("W,H", [(1920, 1080), (257, 131)])
def test_integral_fused_extreme_content(sc, oracle, layout, W, H):
    """The fused integral (column walks inside the chain kernel: frames 1.. of
    the launch with integral_pre 1) on the extreme contents of
    test_integral_extreme_content, at 1080p and at a ragged size whose last
    64-column strip is 1 px wide; both table layouts; every frame bit-exact."""
    yy, xx = np.mgrid[0:H, 0:W]
    frames = np.stack([np.random.default_rng(8).integers(0, 256, (H, W)), ((xx + yy) & 1) * 255,
                       np.random.default_rng(7).integers(0, 256, (H, W)), np.zeros((H, W)),
                       np.full((H, W), 255), (xx & 1) * 255]).astype(np.uint8)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1)).set_options(
        table_layout=int(layout), integral_fuse=2, integral_pre=1)
    det.set_debug(True)
    det.detect_batch(frames)
    for k in range(len(frames)):
        T = det.dump_integral(W, H, frame=k)
        assert T.view(np.uint32).tobytes() == oracle.integral(frames[k]).view(np.uint32).tobytes(), k


@pytest.mark.parametrize("kind", ["checker", "noise"])
def test_grid_parity_extreme_content(sc, oracle, face_cascade, kind):
    """Per-window bits, visited set and detections on frames where every
    window passes the prefilter (noise) or every gradient saturates (checker)."""
    W, H = 640, 480
    yy, xx = np.mgrid[0:H, 0:W]
    img = (((xx + yy) & 1) * 255 if kind == "checker"
           else np.random.default_rng(11).integers(0, 256, (H, W))).astype(np.uint8)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=5),
                 oracle.Params(n_levels=5))


@pytest.mark.parametrize("case", range(12))
def test_random_geometry_sweep(sc, oracle, face_cascade, case):
    """Seeded random sweep over what the chain kernel's segmenting, hand-offs,
    integral forms and speculation depend on: frame size (ragged rows and
    strips), level count, base window, step, prefilter factor, stride
    threshold, thetas (permissive or the model's) and frames per call (1: two
    launches and speculation; 2-3: two-pass; 4-5: fused walks).  Every frame:
    evaluated windows, visited set and detections equal the oracle's."""
    from surfcascade_amd import synth
    rng = np.random.default_rng(700 + case)
    W, H = int(rng.integers(90, 720)), int(rng.integers(90, 540))
    base = int(rng.choice([40, 48, 56, 70]))
    step = int(rng.choice([0, 1, 2, 3, 5]))
    pk = float(rng.choice([3.0, 6.0, 9.0]))
    ss = float(rng.choice([0.3, 0.5, 0.7]))
    n = int(rng.integers(1, 6))
    levels = int(rng.integers(1, 7))
    c = face_cascade
    theta = np.full(c.n_stages, 0.4, np.float32) if case % 2 else c.theta
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, theta, c.patch_index, c.w, c.bias))
    casc = oracle.cascade_from_cfg(text)
    prm_sc = sc.ScanParams(base_len=base, step=step, prefilter_k=pk, stride_score=ss, n_levels=levels)
    prm_or = oracle.Params(base_len=base, step=step, prefilter_k=pk, stride_score=ss, n_levels=levels)
    frames = np.stack([_frame(W, H, 5000 + 13 * case + k) for k in range(n)])
    det = sc.Detector(sc.Model.parse(text), prm_sc)
    det.set_debug(True)
    batch = det.detect_batch(frames, capacity=1 << 18)
    layout, _ = oracle.grid_layout(W, H, prm_or)
    nvis_all = 0
    for k in range(n):
        T = oracle.integral(frames[k])
        assert det.dump_integral(W, H, frame=k).view(np.uint32).tobytes() == T.view(np.uint32).tobytes()
        p, s, v = det.dump_grid(frame=k)
        rp, rs = oracle.eval_grid(T, casc, prm_or)
        ev = p != -2
        np.testing.assert_array_equal(p[ev], rp[ev])
        assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
        rv, _ = oracle.walk_grid(rp, rs, layout, casc.n_stages, prm_or.stride_score)
        np.testing.assert_array_equal(v, rv)
        ref, nvis = oracle.detect(T, casc, prm_or)
        assert _det_set(batch[k]) == _det_set(ref)
        nvis_all += nvis
    assert det.info("visited") == nvis_all
