#!/bin/bash
# Round 4: C4 with the fused integral and one prebuilt frame (tables > 128 MiB):
# the configs tests (incl. the new C4 bench form), a C4 bench line, the
# C4 PMC passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4c4new; mkdir -p $R/$O; cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/run.sh r4c4new "bench bench_C4 --config C4" || exit 1
bash profiles/collect_pmc_cfg.sh $O/pmc/C4 --config C4 || exit 1
echo c4new done
