"""GPU parity of the packed-table gathers (SC_OPT_TABLE_U24): the chain
kernel's items read 12-B half-cells (24-bit integers, the exact f32 values
below 2^24) and fall back to the f32 table for items whose bottom-right
corner holds a value >= 2^24 - 1.  The 1080p frames have values past 2^24
in their bottom-right corner (the fallback runs there); the noise frame has
them over most of the frame; 720p stays below 2^24 everywhere."""
import numpy as np
import pytest

from conftest import FACE_CFG, PED_CFG
from test_gpu_parity import _det_set, _frame, _grid_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    import surfcascade_amd as sc
    return sc


@pytest.mark.parametrize("waves", ["12", "16"])
def test_u24_grid_parity_1080p(sc, oracle, face_cascade, waves):
    img = _frame(1920, 1080, 1000)
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=24),
                 oracle.Params(n_levels=24), table_u24=2, chain_waves=int(waves))


@pytest.mark.parametrize("kind", ["noise", "checker", "stripes"])
def test_u24_extreme_content(sc, oracle, face_cascade, kind):
    W, H = 1920, 1080
    yy, xx = np.mgrid[0:H, 0:W]
    img = {"noise": np.random.default_rng(12).integers(0, 256, (H, W)),
           "checker": ((xx + yy) & 1) * 255, "stripes": (xx & 1) * 255}[kind].astype(np.uint8)
    if kind == "noise":
        assert oracle.integral(img).max() >= 2 ** 24  # the fallback runs
    _grid_parity(sc, oracle, face_cascade, FACE_CFG, img, sc.ScanParams(n_levels=10),
                 oracle.Params(n_levels=10), table_u24=2)


def test_u24_pedestrian(sc, oracle, ped_cascade):
    img = _frame(1920, 1080, 21)
    _grid_parity(sc, oracle, ped_cascade, PED_CFG, img, sc.ScanParams.pedestrian(n_levels=12),
                 oracle.Params(base_len=64, aspect_h=2, n_levels=12), table_u24=2)


@pytest.mark.parametrize("n,opts", [(4, {}), (3, {"chain_chunk": 2}), (5, {"integral_fuse": 2})])
def test_u24_batch(sc, oracle, face_cascade, n, opts):
    """Several frames per launch and several launches (the packed copy's
    per-launch base), 1080p frames: every frame's detections are the
    oracle's, and equal to the unpacked path's."""
    params = oracle.Params(n_levels=24)
    frames = np.stack([_frame(1920, 1080, 4000 + k) for k in range(n)])
    det = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=24)).set_options(table_u24=2, **opts)
    got = det.detect_batch(frames)
    plain = sc.Detector(FACE_CFG, sc.ScanParams(n_levels=24)).set_options(table_u24=1, **opts).detect_batch(frames)
    for k in range(n):
        ref, _ = oracle.detect(oracle.integral(frames[k]), face_cascade, params)
        assert _det_set(got[k]) == _det_set(ref) == _det_set(plain[k]), k
