"""A seeded slice of the parity soak (tests/soak_parity.py; the full 600-case
runs are in profiles/r5/soak/) inside the suite: random frame sizes, frames
per call, levels, scan parameters, model or permissive thetas, the face and
the pedestrian model, and random schedule options that must not change a bit
(chain waves, dequeue sub-queues, integral fusion, prebuilt frames); every
frame's detections and visited count, every 4th case also its table and
per-window stage / score bits, against the oracle (ObjDetector.cpp:174-220)."""
import pytest

import soak_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(oracle):
    import surfcascade_amd as sc
    from surfcascade_amd import synth
    return sc, oracle, synth, soak_parity.load_models(oracle)


@pytest.mark.parametrize("case", range(12))
def test_random_schedule_sweep(env, case):
    sc, O, synth, models = env
    stats = {"frames": 0, "visited": 0, "detections": 0, "bits_checked": 0}
    fail = soak_parity.run_case(sc, O, synth, models, case, 31000, stats, big_frames=False)
    assert fail is None, fail
    assert stats["frames"] > 0
