#!/bin/bash
# DV storage: parity tests, SpMV microbench (ELL rows per lane 4 / 2 / 1, CSR-order codes), bench.
set -o pipefail
OUT=gpurun_out/${1:-dv}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_kernels.py tests/test_gpu_gmres.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python tools/microbench.py --n 256 --kernels spmv --storage dv --tunings 0,16384,8192 > $OUT/mb_dv_256.json 2> $OUT/mb.err &&
MSPLIT_TUNING=32768 timeout -k 10 200 python tools/microbench.py --n 256 --kernels spmv --storage dv --tunings 32768,49152,40960 > $OUT/mb_dvcsr_256.json 2>> $OUT/mb.err &&
timeout -k 10 200 python tools/microbench.py --n 512 --kernels spmv --storage dv --tunings 0,16384,8192 --reps 10 > $OUT/mb_dv_512.json 2>> $OUT/mb.err &&
timeout -k 10 300 python bench.py --storage dv --no-cpu-baseline > $OUT/bench_dv.json 2> $OUT/bench_dv.err &&
MSPLIT_TUNING=16384 timeout -k 10 300 python bench.py --storage dv --no-cpu-baseline > $OUT/bench_dv_rpl2.json 2>> $OUT/bench_dv.err &&
MSPLIT_TUNING=8192 timeout -k 10 300 python bench.py --storage dv --no-cpu-baseline > $OUT/bench_dv_rpl1.json 2>> $OUT/bench_dv.err
echo "exit $?" > $OUT/status
