"""The RCCL gather on a real GPU: one rank, backend "nccl"
(RCCL), the same code path bench.py takes at N > 1 -- counts + capacities
all_gather, the grow-and-rescan on overflow, the padded record all_gather --
against sc_detect_batch of the same frames, and the stream-ordered
StreamGather of bench.py's timed steps, with the detector on its own stream
and on torch's (bench.py's form).  The multi-rank logic is covered
by the gloo tests (tests/test_dist.py); N > 1 on GPUs runs in the driver's
scaling bench.  Runs in a child process so the process group is torn down
with it."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import FACE_CFG, ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r'''
import sys
sys.path.insert(0, ROOT)
import numpy as np
import torch
import torch.distributed as dist
import surfcascade_amd as sc
from oracle import oracle as O
from surfcascade_amd import synth
from surfcascade_amd.dist import StreamGather, enqueue_and_gather, merge_records

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
base = O.cascade_from_cfg(open(CFG).read())
text = synth.write_cfg(synth.cascade_tree(base.n_weak, np.full(base.n_stages, 0.45, np.float32),
                                          base.patch_index, base.w, base.bias))
frames = np.stack([synth.make_frame(640, 480, 70 + k) for k in range(3)])
det = sc.Detector(sc.Model.parse(text), sc.ScanParams(n_levels=6))
if STREAM == "torch":  # bench.py's form: the detector on torch's current stream
    det.set_stream(torch.cuda.current_stream(0))
dev = torch.from_numpy(frames).to("cuda:0")
counts = torch.zeros(1 + len(frames), dtype=torch.int32, device="cuda:0")
recs = torch.zeros(8 * sc.RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0")  # overflows
gc, gr, recs2 = enqueue_and_gather(det, dev, recs, counts)
assert recs2.numel() > recs.numel(), "the overflow path did not grow the buffer"
merged = merge_records(gc, gr, [0])
ref = det.detect_batch(frames)
key = lambda r: (int(r["frame"]), int(r["level"]), int(r["y"]), int(r["x"]), float(r["score"]))
got = sorted(key(r) for r in merged)
exp = sorted((f,) + (int(r["level"]), int(r["y"]), int(r["x"]), float(r["score"]))
             for f, res in enumerate(ref) for r in res)
assert got == exp and len(got) > 100, (len(got), len(exp))
gc2, gr2, _ = enqueue_and_gather(det, dev, recs2, counts)  # second step: no regrowth
assert [list(c) for c in gc2] == [list(c) for c in gc]
# bench.py's timed steps: counts + records in one buffer, one all_gather per
# step on the stream, no host sync per step (dist.StreamGather)
sg = StreamGather(len(frames), recs2.numel() // sc.RECORD_DTYPE.itemsize, "cuda:0")
for _ in range(3):
    sg.step(det, dev)
det.synchronize()
torch.cuda.synchronize()
gc3, gr3 = sg.result()
assert sorted(key(r) for r in merge_records(gc3, gr3, [0])) == exp
sg_small = StreamGather(len(frames), 8, "cuda:0")  # overflow: raised, never truncated
sg_small.step(det, dev)
torch.cuda.synchronize()
try:
    sg_small.result()
    raise AssertionError("StreamGather overflow not raised")
except sc.dist.RecordOverflow:
    pass
dist.barrier()
dist.destroy_process_group()
print("ok", len(got))
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("stream", ["own", "torch"])
def test_rccl_one_rank_gather_equals_detect_batch(tmp_path, stream):
    script = tmp_path / "rccl_gather.py"
    script.write_text("ROOT = %r\nCFG = %r\nSTREAM = %r\n" % (ROOT, FACE_CFG, stream) + SCRIPT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-4000:]
    last = r.stdout.strip().splitlines()[-1].split()  # (RCCL prints a banner to stdout first)
    assert last[0] == "ok" and int(last[1]) > 100, r.stdout[-2000:]
