#!/bin/bash
# GPU check used while iterating: gpu tests, a C2 bench line, the item-loop variants
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r2b/pytest.log 2>&1 && tail -3 gpurun_out/r2b/pytest.log &&
timeout -k 10 300 python bench.py --no-cpu --latency-steps 0 --host-steps 0 > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err && cat gpurun_out/r2b/bench.json &&
timeout -k 10 150 python profiles/itembench/run.py --reps 5 --variants 0:12,11:12,8:12 > gpurun_out/r2b/ib.txt 2>&1; grep variant gpurun_out/r2b/ib.txt
