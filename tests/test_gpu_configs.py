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
