#!/bin/bash
# Round 4: the host-visible watchdog flag (no device copy in sc_synchronize)
# and sc_detector_set_stream: GPU suite, call-overhead legs, A/B vs the
# previous build (old) at C2 and one frame.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/run.sh r4stream "pytest" || exit 1
mkdir -p gpurun_out/r4stream
timeout -k 10 120 python3 profiles/r4/synccost.py > gpurun_out/r4stream/synccost.json 2> gpurun_out/r4stream/synccost.err || { tail -5 gpurun_out/r4stream/synccost.err; exit 1; }
cat gpurun_out/r4stream/synccost.json
bash profiles/run.sh r4stream "ab c2 3 old cur" "ab b1 3 old cur -- --batch 1 --steps 50"
