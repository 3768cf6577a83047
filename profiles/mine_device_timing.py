"""sc_mine vs sc_mine_device on one 1080p frame, first round (every stride-10
window a candidate), 4096 descriptors kept.  Run on the GPU box."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import surfcascade_amd as sc  # noqa: E402
from surfcascade_amd import synth  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


img = synth.make_frame(1920, 1080, 1000)
m = sc.Miner(None)
cap = 4096
dev = torch.from_numpy(img).cuda()
feats = torch.empty(cap * m.n_patches * 32, dtype=torch.float32, device="cuda")
print(json.dumps({"frame": "1920x1080", "kept": cap, "n_patches": m.n_patches,
                  "mine_host_ms": timed(lambda: m.mine(img, cap)),
                  "mine_device_ms": timed(lambda: m.mine_device(dev, cap, feats))}))
