#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace stats and two PMC passes.
# Every GPU step has its own time limit; steps are chained with && so the
# script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 --no-cpu-baseline --no-csr-compare > $OUT/bench_trace.json 2> $OUT/trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-timing > $OUT/pmc_fetch.out 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-timing > $OUT/pmc_write.out 2>&1 &&
timeout -k 10 300 python tools/microbench.py --n 512 --kernels spmv --storage csr --reps 10 > $OUT/spmv512_csr.json 2> $OUT/mb.err &&
timeout -k 10 300 python tools/microbench.py --n 512 --kernels spmv --storage dv --reps 10 > $OUT/spmv512_dv.json 2>> $OUT/mb.err
echo "exit $?" > $OUT/status
