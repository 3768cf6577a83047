# Analysis only (not product code): builds /tmp/ee/ee.so from profiles/r6/ee/ee.c + oracle/sc_oracle.c:
#   gcc -O2 -fPIC -shared -ffp-contract=off -msse3 -fopenmp -I oracle -o /tmp/ee/ee.so profiles/r6/ee/ee.c oracle/sc_oracle.c -lm
#   python3 profiles/r6/ee/run.py W H n_frames
import ctypes, sys, os, time
import numpy as np
sys.path.insert(0, "/root/repo")
from oracle import oracle as O
from surfcascade_amd import synth
lib = ctypes.CDLL("/tmp/ee/ee.so")
cfg = open("/root/repo/surfcascade_amd/models/face40_synth.cfg").read()
casc = O.cascade_from_cfg(cfg, 40, 40)
print("n_weak", list(casc.n_weak) if hasattr(casc, "n_weak") else None, "theta", getattr(casc, "theta", None))
W, H = int(sys.argv[1]), int(sys.argv[2])
chunks = [1, 4, 8, 16]
tot = np.zeros(2 + len(chunks), np.int64)
for seed in range(1000, 1000 + int(sys.argv[3])):
    img = synth.make_frame(W, H, seed)
    T = np.ascontiguousarray(O.integral(img), np.float32)
    m = casc.c(); prm = O.Params(n_levels=24).c()
    ch = (ctypes.c_int * len(chunks))(*chunks)
    out = np.zeros(2 + len(chunks), np.int64)
    t = time.time()
    lib.ee_stats(T.ctypes.data_as(ctypes.c_void_p), W, H, ctypes.byref(m), ctypes.byref(prm), len(chunks), ch,
                 out.ctypes.data_as(ctypes.c_void_p))
    tot += out
    print(seed, out, "%.1fs" % (time.time() - t), flush=True)
print("full", tot[0], "ideal %.3f" % (tot[1] / tot[0]), " ".join("c%d %.3f" % (c, tot[2 + i] / tot[0]) for i, c in enumerate(chunks)))
