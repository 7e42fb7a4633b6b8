#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-opfuse}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 &&
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/bench_fused_r$rep.json 2>> $OUT/bench.err &&
  MSPLIT_TUNING=65536 timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/bench_unfused_r$rep.json 2>> $OUT/bench.err || break
done &&
timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/bench_smsm_fused.json 2>> $OUT/bench.err &&
MSPLIT_TUNING=65536 timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/bench_smsm_unfused.json 2>> $OUT/bench.err
echo "exit $?" > $OUT/status
