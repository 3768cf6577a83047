"""GPU parity at the BASELINE.json workload sizes (SURVEY.md 8 config
shorthand), through the C ABI, against the CPU restatement:

  C3  one call with the per-rank shard of the 8-GPU batch: 32 x 1080p frames
      (device-resident, sc_enqueue_device records, as bench.py --gpus 8 runs)
  C4  3840 x 2160, 32 levels (l = 70..1343): integral sums far above 2^24,
      a 265 MB table, chain-kernel frame chunks of 15 frames
  C5  64 x 128 pedestrian cascade on 1920 x 1080, 23 levels (l = 64..520,
      h = 2l up to 1040, ProjectPatches scale up to 8.1)

Bit-exact: integral tables, per-window stage reached and last-stage score
bits of every evaluated window, the visited set, detections with their f64
scores (ObjDetector.cpp:174-220).
"""
import os

import numpy as np
import pytest

from conftest import FACE_CFG, PED_CFG
from test_gpu_parity import _det_set, _frame, _grid_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


def test_c4_integral_bit_exact(sc, oracle):
    img = _frame(3840, 2160, 4000)
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1))
    det.detect(img)
    T = det.dump_integral(3840, 2160)
    ref = oracle.integral(img)
    assert float(ref[-1, -1].max()) > 2 ** 24  # the order-sensitive regime
    assert T.view(np.uint32).tobytes() == ref.view(np.uint32).tobytes()


def test_c4_grid_parity_4k_32_levels(sc, oracle, face_cascade):
    img = _frame(3840, 2160, 4000)
    wins, p = _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=32),
                           oracle.Params(n_levels=32))
    assert len(p) == 21302193  # C4 grid windows per frame
    assert sc.ScanParams().level_len(31) == 1343


def test_c4_permissive_detections_4k(sc, oracle, face_cascade):
    """Many detections at 4K (every level, incl. l = 1343): windows + f64 scores."""
    from surfcascade_amd import synth
    c = face_cascade
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, np.full(c.n_stages, 0.45, np.float32),
                                              c.patch_index, c.w, c.bias))
    img = _frame(3840, 2160, 4001)
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=32))
    wins = det.detect(img, capacity=1 << 20)
    ref, nvis = oracle.detect(oracle.integral(img), oracle.cascade_from_cfg(text),
                              oracle.Params(n_levels=32))
    assert len(ref) > 1000
    assert _det_set(wins) == _det_set(ref)
    assert det.info("visited") == nvis


def test_c5_pedestrian_1080p_23_levels(sc, oracle, ped_cascade):
    img = _frame(1920, 1080, 5000)
    params = sc.ScanParams.pedestrian(n_levels=23)
    assert params.level_len(22) == 520
    _grid_parity(sc, oracle, ped_cascade, PED_CFG, img, params,
                 oracle.Params(base_len=64, aspect_h=2, n_levels=23))


def _batch_parity(sc, oracle, cascade, model, frames, params_sc, params_or, **opts):
    """One detect_batch call: every frame's table, evaluated windows, visited
    set and detections against the oracle; returns the detector."""
    det = sc.Detector(model, params_sc).set_options(**opts)
    det.set_debug(True)
    batch = det.detect_batch(frames, capacity=1 << 20)
    H, W = frames.shape[1:]
    layout, _ = oracle.grid_layout(W, H, params_or)
    nvis_all = 0
    for k in range(len(frames)):
        T = oracle.integral(frames[k])
        assert det.dump_integral(W, H, frame=k).view(np.uint32).tobytes() == T.view(np.uint32).tobytes()
        p, s, v = det.dump_grid(frame=k)
        rp, rs = oracle.eval_grid(T, cascade, params_or)
        ev = p != -2
        np.testing.assert_array_equal(p[ev], rp[ev])
        assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
        rv, _ = oracle.walk_grid(rp, rs, layout, cascade.n_stages, params_or.stride_score)
        np.testing.assert_array_equal(v, rv)
        ref, nvis = oracle.detect(T, cascade, params_or)
        assert nvis == int(rv.sum())
        assert _det_set(batch[k]) == _det_set(ref)
        nvis_all += nvis
    assert det.info("visited") == nvis_all
    return det, batch


def test_c5_bench_form_fused_12_waves(sc, oracle, ped_cascade):
    """C5 exactly as bench.py runs it, in small: a batch of pedestrian 1080p
    frames x 23 levels in one call, so the integral's column walks of frames
    2.. run inside the 12-wave chain kernel (the fused walker + frame_ready
    path of the pedestrian model's LDS-bound kernel)."""
    frames = np.stack([_frame(1920, 1080, 5100 + k) for k in range(4)])
    params = sc.ScanParams.pedestrian(n_levels=23)
    det, batch = _batch_parity(sc, oracle, ped_cascade, PED_CFG, frames, params,
                               oracle.Params(base_len=64, aspect_h=2, n_levels=23))
    assert det.info("fused_frames") == 2  # frames 2, 3: walks inside the chain kernel
    assert det.info("chain_waves") == 12
    assert det.info("column_pass") == 1   # frames 0, 1: rowcarry R rows + colsum


def test_c4_bench_form_colstrip_one_launch(sc, oracle, face_cascade):
    """C4's form below 4 frames per call: several 4K frames x 32 levels in
    ONE chain launch (tables beyond the Infinity Cache: interleaved cells, the
    lane-pair item form at 12 waves; no fusion) whose tables colstrip built
    (VERDICT r3 weak #1).  Lowered thetas so every
    level reaches detections."""
    from surfcascade_amd import synth
    c = face_cascade
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, np.full(c.n_stages, 0.45, np.float32),
                                              c.patch_index, c.w, c.bias))
    frames = np.stack([_frame(3840, 2160, 4100 + k) for k in range(3)])
    det, batch = _batch_parity(sc, oracle, oracle.cascade_from_cfg(text), sc.Model.parse(text), frames,
                               sc.ScanParams(n_levels=32), oracle.Params(n_levels=32), integral_passes=1)
    assert det.info("column_pass") == 2  # colstrip
    assert det.info("fused_frames") == 0
    assert det.info("chain_waves") == 12 and det.info("item_form") == 2  # tables beyond the Infinity Cache
    assert all(len(b) > 100 for b in batch)


def test_c4_bench_form_fused_one_prebuilt(sc, oracle, face_cascade):
    """C4 exactly as bench.py runs it, in small: 4K frames x 32 levels in one
    12-wave lane-pair chain launch whose first frame is integrated before it (two-pass;
    one prebuilt frame since a 4K table is larger than 128 MiB) and whose
    other frames' column walks run inside the chain kernel.  Lowered thetas
    so every level reaches detections."""
    from surfcascade_amd import synth
    c = face_cascade
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, np.full(c.n_stages, 0.45, np.float32),
                                              c.patch_index, c.w, c.bias))
    frames = np.stack([_frame(3840, 2160, 4200 + k) for k in range(4)])
    det, batch = _batch_parity(sc, oracle, oracle.cascade_from_cfg(text), sc.Model.parse(text), frames,
                               sc.ScanParams(n_levels=32), oracle.Params(n_levels=32))
    assert det.info("fused_frames") == 3
    assert det.info("column_pass") == 1  # the prebuilt frame: rowcarry R rows + colsum
    assert det.info("chain_waves") == 12 and det.info("item_form") == 2
    assert all(len(b) > 100 for b in batch)


_WATCHDOG_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import surfcascade_amd as sc
from surfcascade_amd import synth
host = np.stack([synth.make_frame(1280, 720, 700 + k) for k in range(2)])
frames = torch.from_numpy(host).to("cuda:0")
det = sc.Detector(sys.argv[2], sc.ScanParams(n_levels=6))
recs = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
counts = torch.zeros(3, dtype=torch.int32, device="cuda:0")
det.enqueue_device(frames, recs, counts)
det.synchronize()                              # clean
det.set_option("test_drop_handoff", 5)
det.enqueue_device(frames, recs, counts)       # step 1: one hand-off lost
det.set_option("test_drop_handoff", -1)
det.enqueue_device(frames, recs, counts)       # step 2: clean (rowcarry zeroes the per-call words)
try:
    det.synchronize()
    print("NOT RAISED")
except sc.SurfCascadeError as e:
    print("RAISED", "hand-off or table wait" in str(e))
det.enqueue_device(frames, recs, counts)
det.synchronize()                              # reported once, not carried further
print("CLEAN AFTER")
"""


def test_watchdog_error_is_sticky_over_pipelined_steps(sc):
    """A lost segment hand-off (SC_OPT_TEST_DROP_HANDOFF, test-hook build
    lib/testhooks) in the FIRST of two pipelined device steps is still raised
    at the one synchronisation after the second (rowcarry used to
    zero the watchdog word every call); the detector then works again.  The
    product library refuses the hook."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=6))
    with pytest.raises(sc.SurfCascadeError, match="test-hook build"):
        det.set_option("test_drop_handoff", 5)
    lib = os.path.join(ROOT, "surfcascade_amd", "lib", "testhooks", "libsurfcascade.so")
    assert os.path.exists(lib), "test-hook library not built (__graft_entry__.build())"
    env = dict(os.environ, SURFCASCADE_LIB=lib)
    r = subprocess.run([sys.executable, "-c", _WATCHDOG_CHILD, ROOT, FACE_CFG], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "RAISED True" in r.stdout and "CLEAN AFTER" in r.stdout, r.stdout


_WALK_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import surfcascade_amd as sc
from surfcascade_amd import synth
host = np.stack([synth.make_frame(1280, 720, 720 + k) for k in range(5)])
frames = torch.from_numpy(host).to("cuda:0")
det = sc.Detector(sys.argv[2], sc.ScanParams(n_levels=6))
recs = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
counts = torch.zeros(6, dtype=torch.int32, device="cuda:0")
det.enqueue_device(frames, recs, counts)
det.synchronize()                              # clean, fused (frames 2-4 walked inside)
print("FUSED", det.info("fused_frames"))
det.set_option("test_drop_walk", 3)            # frame 2's 4th column walk never counts itself done
det.enqueue_device(frames, recs, counts)
det.set_option("test_drop_walk", -1)
try:
    det.synchronize()
    print("NOT RAISED")
except sc.SurfCascadeError as e:
    print("RAISED", "hand-off or table wait" in str(e))
det.enqueue_device(frames, recs, counts)
det.synchronize()
print("CLEAN AFTER")
"""


def test_watchdog_ends_a_lost_walk_count(sc):
    """A fused column walk whose completion count is lost
    (SC_OPT_TEST_DROP_WALK, test-hook build): the tasks waiting for that
    frame's table must time out and the call raise SC_ERR_DEVICE, not spin
    (after another wave's watchdog fired, the idle clock of a wave
    waiting for a table kept restarting); the detector then works again."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=6))
    with pytest.raises(sc.SurfCascadeError, match="test-hook build"):
        det.set_option("test_drop_walk", 3)
    lib = os.path.join(ROOT, "surfcascade_amd", "lib", "testhooks", "libsurfcascade.so")
    env = dict(os.environ, SURFCASCADE_LIB=lib)
    r = subprocess.run([sys.executable, "-c", _WALK_CHILD, ROOT, FACE_CFG], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "FUSED 3" in r.stdout, r.stdout
    assert "RAISED True" in r.stdout and "CLEAN AFTER" in r.stdout, r.stdout


def _bench_form_exact(sc, oracle, cascade, model, W, H, n, params_sc, params_or, expect, full_frames):
    """One sc_enqueue_device call over bench.py's n device-resident frames
    (seeds 1000..), the detector on torch's stream, the launch shape `expect`
    (SC_INFO values) asserted; tables and per-window stage / score bits of
    `full_frames`, the visited set and the detections of every frame."""
    import torch
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import merge_records
    host = synth.make_frames(W, H, n, seed0=1000)  # bench.py's frames
    frames = torch.from_numpy(host).to("cuda:0")
    det = sc.Detector(model, params_sc)
    det.set_stream(torch.cuda.current_stream())
    det.set_debug(True)
    recs = torch.zeros((1 << 18) * RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0")
    counts = torch.zeros(n + 1, dtype=torch.int32, device="cuda:0")
    det.enqueue_device(frames, recs, counts)
    det.synchronize()
    if os.environ.get("SC_TEST_ANY_ITEM_FORM"):  # A/B variant runs (profiles/r6): the form is the variant's
        expect = {k: v for k, v in expect.items() if k != "item_form"}
    for k, v in expect.items():
        assert det.info(k) == v, (k, det.info(k))
    got = merge_records([counts.cpu().numpy()], [recs.cpu().numpy()], [0])
    layout, _ = oracle.grid_layout(W, H, params_or)
    vis_all, det_all = 0, 0
    for f in range(n):
        T = oracle.integral(host[f])
        if f in full_frames:
            assert det.dump_integral(W, H, frame=f).view(np.uint32).tobytes() == \
                T.view(np.uint32).tobytes(), f
        p, s, v = det.dump_grid(frame=f)
        rp, rs = oracle.eval_grid(T, cascade, params_or)
        if f in full_frames:
            ev = p != -2
            np.testing.assert_array_equal(p[ev], rp[ev])
            assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes(), f
        rv, _ = oracle.walk_grid(rp, rs, layout, cascade.n_stages, params_or.stride_score)
        np.testing.assert_array_equal(v, rv)
        ref, nv = oracle.detect(T, cascade, params_or)
        assert nv == int(rv.sum())
        mine = got[got["frame"] == f]
        assert _det_set(mine) == _det_set(ref), f
        vis_all += nv
        det_all += len(ref)
    assert det.info("visited") == vis_all
    assert int(counts[0].item()) == det_all
    det.set_stream(None)
    return det_all


def test_c2_bench_form_exact(sc, oracle, face_cascade):
    """C2 exactly as bench.py measures it: 32 device-resident 1080p frames x
    24 levels in ONE sc_enqueue_device call, the calibrated model
    (models/face40_synth.cfg, not permissive thetas), the detector on torch's
    stream; the launch must be the bench's (16 waves, 30 of 32 frames
    integrated inside the chain kernel, one dequeue sub-queue).  Tables and
    per-window stage / score bits of frames 0 (prebuilt), 2 and 31 (fused),
    the visited set and the detections of every frame (VERDICT r4 next #2;
    ObjDetector.cpp:188-212)."""
    _bench_form_exact(sc, oracle, face_cascade, FACE_CFG, 1920, 1080, 32, sc.ScanParams(n_levels=24),
                      oracle.Params(n_levels=24),
                      {"fused_frames": 30, "chain_waves": 16, "chain_subq": 1, "column_pass": 1, "item_form": 1}, (0, 2, 31))


def test_c4_bench_form_exact(sc, oracle, face_cascade):
    """C4 exactly as bench.py measures it: 8 device-resident 4K frames x 32
    levels (l up to 1343, sums past 2^24) in ONE call with the calibrated
    model: one frame integrated before the chain kernel (a 4K table is larger
    than 128 MiB), the column walks of the other 7 inside it, 12 waves, lane pairs.
    Tables and per-window bits of frames 0, 1 and 7; visited sets and
    detections of all 8."""
    _bench_form_exact(sc, oracle, face_cascade, FACE_CFG, 3840, 2160, 8, sc.ScanParams(n_levels=32),
                      oracle.Params(n_levels=32),
                      {"fused_frames": 7, "chain_waves": 12, "chain_subq": 1, "item_form": 2}, (0, 1, 7))


def test_c5_bench_form_exact(sc, oracle, ped_cascade):
    """C5 exactly as bench.py measures it: 32 device-resident 1080p frames x
    23 levels of the 64 x 128 pedestrian cascade (windows l x 2l) in ONE call:
    30 frames integrated inside the 12-wave chain kernel (the pedestrian
    model's LDS copy leaves no room for 16 waves).  Tables and per-window bits
    of frames 0, 2 and 31; visited sets and detections of all 32."""
    _bench_form_exact(sc, oracle, ped_cascade, PED_CFG, 1920, 1080, 32, sc.ScanParams.pedestrian(n_levels=23),
                      oracle.Params(base_len=64, aspect_h=2, n_levels=23),
                      {"fused_frames": 30, "chain_waves": 12, "chain_subq": 1, "column_pass": 1, "item_form": 2}, (0, 2, 31))


def test_one_frame_launch_subqueues(sc, oracle, face_cascade):
    """One-frame launches deal their tasks through 4 dequeue sub-queues per
    XCD (SC_INFO_CHAIN_SUBQ; one task per wave, SC_OPT_CHAIN_SLOTS), each of
    the two XCDs of a segment over its own contiguous part of the row list;
    batches through one; results are the oracle's at every sub-queue count
    (SC_OPT_CHAIN_SUBQ) and with two task slots per wave."""
    img = _frame(1920, 1080, 1234)
    params = oracle.Params(n_levels=24)
    T = oracle.integral(img)
    ref, nv = oracle.detect(T, face_cascade, params)
    rp, rs = oracle.eval_grid(T, face_cascade, params)
    for q, slots in ((0, 0), (1, 0), (2, 0), (3, 0), (8, 0), (0, 2), (8, 2)):
        det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=24)).set_options(chain_subq=q, chain_slots=slots)
        det.set_debug(True)
        wins = det.detect(img)
        assert det.info("chain_subq") == (q if q else (8 if slots == 2 else 4))
        p, s, _v = det.dump_grid()
        ev = p != -2
        np.testing.assert_array_equal(p[ev], rp[ev])
        assert s[ev].view(np.uint32).tobytes() == rs[ev].view(np.uint32).tobytes()
        assert det.info("visited") == nv
        assert _det_set(wins) == _det_set(ref)


def test_c3_rank_shard_32_frames_one_call(sc, oracle, face_cascade):
    """The C3 per-rank workload: 32 device-resident 1080p frames in ONE
    sc_enqueue_device call (bench.py --gpus 8 shards 256 frames this way);
    records merged canonically equal the per-frame oracle detections."""
    import torch
    from surfcascade_amd import RECORD_DTYPE, synth
    from surfcascade_amd.dist import merge_records
    c = face_cascade
    # permissive enough that every frame has detections
    text = synth.write_cfg(synth.cascade_tree(c.n_weak, np.full(c.n_stages, 0.45, np.float32),
                                              c.patch_index, c.w, c.bias))
    casc_or = oracle.cascade_from_cfg(text)
    host = synth.make_frames(1920, 1080, 32, seed0=1000 + 7 * 32)  # rank 7's shard
    frames = torch.from_numpy(host).to("cuda:0")
    det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=24))
    recs = torch.zeros((1 << 20) * RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0")
    counts = torch.zeros(33, dtype=torch.int32, device="cuda:0")
    det.enqueue_device(frames, recs, counts)
    det.synchronize()
    got = merge_records([counts.cpu().numpy()], [recs.cpu().numpy()], [0])
    cnt = counts.cpu().numpy()
    vis, total = 0, 0
    for f in range(32):
        ref, nv = oracle.detect(oracle.integral(host[f]), casc_or, oracle.Params(n_levels=24))
        mine = got[got["frame"] == f]
        assert int(cnt[1 + f]) == len(mine) == len(ref)
        assert _det_set(mine) == _det_set(ref)
        vis += nv
        total += len(ref)
    assert int(cnt[0]) == total > 32
    assert det.info("visited") == vis


def test_stream_ordered_device_frames(sc, oracle, face_cascade):
    """Frames produced by a torch kernel immediately before the call (no host
    copy, no sync): the detector's stream waits for torch's current stream
    (sc_detector_wait_stream), and torch reads the records after the scan
    (sc_stream_wait_detector) without a host synchronisation."""
    import torch
    from surfcascade_amd import RECORD_DTYPE
    from surfcascade_amd.dist import merge_records
    host = np.stack([_frame(1280, 720, 900 + k) for k in range(3)])
    base = torch.from_numpy(host).to("cuda:0")
    torch.cuda.synchronize()
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=8))
    recs = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
    counts = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(1)
    for it in range(3):
        # a slow torch producer (chained matmuls) whose last kernel writes the
        # frames the scan reads; no host synchronisation before the scan
        m = torch.randn(2048, 2048, device="cuda:0", generator=g)
        for _k in range(8):
            m = (m @ m.T) / 2048.0
        zero = (m[0, 0] * 0).nan_to_num(0.0).to(torch.int16)
        frames = (base.to(torch.int16) + zero).to(torch.uint8)
        det.enqueue_device(frames, recs, counts)
        c_host = counts.clone().cpu().numpy()  # ordered after the scan on torch's stream
        del frames  # the allocator may hand this memory out again at once
    got = merge_records([c_host], [recs.cpu().numpy()], [0])
    for f in range(3):
        ref, _ = oracle.detect(oracle.integral(host[f]), face_cascade, oracle.Params(n_levels=8))
        assert _det_set(got[got["frame"] == f]) == _det_set(ref)


@pytest.mark.parametrize("which", ["default", "side"])
def test_detector_on_torch_stream(sc, oracle, face_cascade, which):
    """sc_detector_set_stream: the detector launches on torch's stream (the
    null stream, or a side stream made current), so enqueue_device skips the
    event pair; a slow torch producer before the scan and torch's read after
    it are ordered by the stream alone.  Switching back to the detector's own
    stream is ordered too."""
    import torch
    from surfcascade_amd.dist import merge_records
    host = np.stack([_frame(1280, 720, 910 + k) for k in range(2)])
    base = torch.from_numpy(host).to("cuda:0")
    torch.cuda.synchronize()
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=8))
    own = det.stream_ptr
    side = torch.cuda.Stream(device="cuda:0") if which == "side" else torch.cuda.current_stream()
    g = torch.Generator(device="cuda:0").manual_seed(2)
    with torch.cuda.stream(side):
        det.set_stream(side)
        assert (det.stream_ptr or 0) == side.cuda_stream
        recs = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
        counts = torch.zeros(3, dtype=torch.int32, device="cuda:0")
        for it in range(2):
            m = torch.randn(2048, 2048, device="cuda:0", generator=g)
            for _k in range(8):
                m = (m @ m.T) / 2048.0
            zero = (m[0, 0] * 0).nan_to_num(0.0).to(torch.int16)
            frames = (base.to(torch.int16) + zero).to(torch.uint8)
            det.enqueue_device(frames, recs, counts)
            c_host = counts.clone().cpu().numpy()
            r_host = recs.cpu().numpy()
            del frames
        det.synchronize()
    det.set_stream(None)
    assert det.stream_ptr == own
    got = merge_records([c_host], [r_host], [0])
    for f in range(2):
        ref, _ = oracle.detect(oracle.integral(host[f]), face_cascade, oracle.Params(n_levels=8))
        assert _det_set(got[got["frame"] == f]) == _det_set(ref)
    # back on its own stream: the same frames, the same records
    counts2 = torch.zeros(3, dtype=torch.int32, device="cuda:0")
    det.enqueue_device(base, recs, counts2)
    det.synchronize()
    assert np.array_equal(counts2.cpu().numpy(), c_host)


def test_device_entry_points_refuse_host_pointers(sc):
    """A host pointer (or another device's memory) where device memory is
    required is SC_ERR_INVALID, not a kernel fault."""
    import ctypes
    import torch
    L = sc.load_library()
    img = np.zeros((100, 120), np.uint8)
    miner = sc.Miner(None, device=0)
    wins = np.zeros(4, sc.WINDOW_DTYPE)
    n = ctypes.c_int()
    rc = L.sc_mine_device(miner._h, img.ctypes.data, 120, 100, 120, wins.ctypes.data, None, 4,
                          ctypes.byref(n))
    assert rc == -1 and b"not device memory" in L.sc_last_error()
    dev = torch.zeros((100, 120), dtype=torch.uint8, device="cuda:0")
    feat = np.zeros(4 * miner.n_patches * 32, np.float32)
    rc = L.sc_mine_device(miner._h, dev.data_ptr(), 120, 100, 120, wins.ctypes.data,
                          feat.ctypes.data, 4, ctypes.byref(n))
    assert rc == -1 and b"d_features" in L.sc_last_error()
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=1))
    counts = np.zeros(2, np.int32)
    rc = L.sc_enqueue_device(det._h, dev.data_ptr(), 1, 120, 100, 120, None, 0, counts.ctypes.data)
    assert rc == -1 and b"d_counts" in L.sc_last_error()
