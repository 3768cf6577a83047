#!/bin/bash
# batched miner + thread-safety tests on the GPU, then the f3 throughput
O=gpurun_out/mine; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mine.py tests/test_threads.py tests/test_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python profiles/mine_batch_bench.py > $O/mine_batch.json 2> $O/mine_batch.err; rc=$?
cat $O/mine_batch.json; tail -3 $O/mine_batch.err; exit $rc
