set -e
mkdir -p gpurun_out/ib4
run() { n=$1; shift; timeout -k 10 120 python profiles/itembench/run.py --reps 5 "$@" > gpurun_out/ib4/$n.txt 2>&1; grep variant gpurun_out/ib4/$n.txt | sed "s/^/$n /"; }
run base --variants 0:12
run bcast0 --variants 2:12,2:16,2:8 --omask 0
run coal --variants 2:12,2:16 --omask 63
