set -e
mkdir -p gpurun_out/ib3
run() { n=$1; shift; timeout -k 10 120 python profiles/itembench/run.py --variants 0:12 --reps 5 "$@" > gpurun_out/ib3/$n.txt 2>&1; grep variant gpurun_out/ib3/$n.txt | sed "s/^/$n /"; }
run blk32
run blk8 --row-block 8
run blk16 --row-block 16
run blk64 --row-block 64
run lvmajor --row-block 0
run seg16 --nseg 16
run seg32 --nseg 32
run lg4 --level-group 4
run lg1 --level-group 1 --row-block 32
run lg2b8 --level-group 2 --row-block 8
