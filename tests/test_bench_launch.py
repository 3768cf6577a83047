"""bench.py's own multi-rank entry: `--gpus N` without a
torch.distributed environment starts N ranks itself and prints ONE line with
n_gpus N; a WORLD_SIZE that disagrees with --gpus is an error, never a
silent single-GPU measurement.  Runs the launcher with the CPU stand-in
detector (--stub) over gloo, world size 2."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

ARGS = ["--stub", "--steps", "2", "--warmup", "1", "--width", "320", "--height", "240",
        "--levels", "3", "--batch", "2", "--no-cpu", "--host-steps", "0", "--latency-steps", "0"]


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _run(extra, env=None, timeout=240):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS + extra,
                       cwd=ROOT, env=env or _env(), capture_output=True, text=True, timeout=timeout)
    return p, [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def _stub_records(frames, world=1, rank=0):
    n = 0
    for f in frames:
        v = int(f.sum()) % 7 + 2
        n += sum(1 for k in range(v) if k % world == rank)
    return n


@pytest.mark.parametrize("shard", ["frames", "grid"])
def test_launcher_starts_n_ranks(shard):
    from surfcascade_amd import synth
    p, lines = _run(["--gpus", "2", "--shard", shard])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout  # rank 0 prints the one line
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["process_group"]["world_size"] == 2
    assert line["scaling"] == ("strong" if shard == "grid" else "weak")
    if shard == "frames":  # ranks own frames 1000.., 1002..: all four frames' records
        frames = synth.make_frames(320, 240, 4, seed0=1000)
        assert line["detections_last_step"] == _stub_records(frames)
        assert line["config"]["parallelism"] == "frame-sharded dp2"
    else:  # both ranks scan frames 1000, 1001, each its own rows
        frames = synth.make_frames(320, 240, 2, seed0=1000)
        assert line["detections_last_step"] == _stub_records(frames)
    # windows of all ranks: the value is computed over world x frames (frames)
    # or the frames once (grid)
    assert line["steps"] == 2 and line["value"] > 0


def test_world_size_mismatch_is_an_error():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p, lines = _run(["--gpus", "2"], env=env, timeout=120)
    assert p.returncode != 0 and not lines
    assert "refusing" in p.stderr
