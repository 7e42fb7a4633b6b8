#!/bin/bash
set -o pipefail
OUT=gpurun_out/ab3
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/timing_r$rep.json 2>> $OUT/err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare --no-timing > $OUT/notiming_graphs_r$rep.json 2>> $OUT/err || exit 1
  MSPLIT_GRAPHS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare --no-timing > $OUT/notiming_eager_r$rep.json 2>> $OUT/err || exit 1
done
