#!/bin/bash
# The LDS-staged GMRES back-solve (k_build_lds): GMRES / graph / DV / seq / config GPU tests, then the kernel's
# average duration in a kernel-trace profile of the bench step.
set -o pipefail
OUT=gpurun_out/buildlds
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_gmres.py tests/test_gpu_graphs.py tests/test_gpu_dv.py \
  tests/test_gpu_seq.py tests/test_gpu_configs.py tests/test_gpu_kats.py tests/test_gpu_drivers.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 \
  --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-assembled --no-spmv512 > $OUT/bench_trace.json 2> $OUT/trace.err
echo "exit $?" > $OUT/status
