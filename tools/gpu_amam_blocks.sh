#!/bin/bash
# configs[3] / configs[4] per-GPU blocks through bench.py --variant amam on the round-3 build, both minimizations.
set -o pipefail
OUT=gpurun_out/amam_blocks
mkdir -p $OUT
for M in lsqr rtr; do
  timeout -k 10 300 python bench.py --variant amam --minimization $M --steps 2 --warmup 1 > $OUT/configs3_$M.json 2> $OUT/configs3_$M.err || exit 1
  timeout -k 10 300 python bench.py --variant amam --minimization $M --peclet 0.5,0.25,-0.3 --steps 2 --warmup 1 > $OUT/configs4_$M.json 2> $OUT/configs4_$M.err || exit 1
done
echo done > $OUT/status
