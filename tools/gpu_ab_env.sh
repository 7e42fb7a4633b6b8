#!/bin/bash
# Same-box interleaved A/B of MSPLIT_TUNING settings on the N=1 bench: tools/gpu_ab_env.sh OUT "0 64 ..."
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for t in $2; do
    MSPLIT_TUNING=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare ${3:-} > $OUT/bench_t${t}_r${rep}.json 2>> $OUT/bench.err || { echo "exit 1" > $OUT/status; exit 1; }
  done
done
echo "exit 0" > $OUT/status
