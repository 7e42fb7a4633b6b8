#!/bin/bash
# DV storage: parity tests, ELL SpMV variants (microbench), bench A/B.
set -o pipefail
OUT=gpurun_out/${1:-dv}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_gmres.py tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python tools/microbench.py --n 256 --kernels spmv --storage dv --tunings 0,16384,8192 > $OUT/mb_dv_256.json 2> $OUT/mb.err &&
timeout -k 10 200 python tools/microbench.py --n 512 --kernels spmv --storage dv --tunings 0,16384,8192 --reps 10 > $OUT/mb_dv_512.json 2>> $OUT/mb.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/bench_dv.json 2> $OUT/bench_dv.err &&
MSPLIT_TUNING=16384 timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/bench_rpl2.json 2>> $OUT/bench_dv.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-csr-compare > $OUT/bench_dv2.json 2>> $OUT/bench_dv.err
echo "exit $?" > $OUT/status
