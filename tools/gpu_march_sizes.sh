#!/bin/bash
# The z-march DV SpMV against the row-parallel ELL kernel (MSPLIT_TUNING 268435456) across mesh sizes,
# interleaved in one process per size (tools/microbench.py, DV storage).
set -o pipefail
O=gpurun_out/${1:-march_sizes}; mkdir -p $O
for n in 64 128 256 384 512; do
  ML=0,1; [ $((n % 256)) = 0 ] && ML=0,1,4   # the four-line tiles need nx % 256 == 0
  timeout -k 10 120 python tools/microbench.py --n $n --storage dv --kernels spmv --tunings 0,268435456 --march-z 0,8,16 --march-lines $ML --reps 20 --rounds 3 > $O/n$n.json 2>> $O/err || exit 1
done
echo "exit 0" > $O/status
