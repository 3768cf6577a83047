#!/bin/bash
# round-end rehearsal: gpu suite, smoke, default bench line
O=gpurun_out/final_check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; j=json.load(open('$O/bench.json')); print(round(j['value']/1e9,3), j['ms_per_step'], j['roofline']['valu'], j['roofline']['traffic_ratio'])"
