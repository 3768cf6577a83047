#!/bin/bash
# Round 5: one-frame launches at 8 / 10 / 14 waves per CU with the speculative
# idle rounds compiled into that width (SC_SPEC_NW2, SC_ONEFRAME_WAVES) vs 12;
# parity of one-frame / speculation tests on each; C4 (10-wave batches) on w10s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for v in w10s w14s w8s; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so PYTEST_K="(one_frame or speculative or subq or batch1 or single) and not speculative_rounds_run_and_match" \
    bash profiles/run.sh r5ow_$v "pytest" || exit 1
done
bash profiles/run.sh r5ow "ab b1 3 cur w10s w14s w8s -- --batch 1 --steps 50" "ab c4 2 cur w10s -- --config C4" || exit 1
echo done
