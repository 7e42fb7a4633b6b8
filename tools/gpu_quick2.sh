#!/bin/bash
# Parity of the DV paths and the block drivers (which release A_ii / A_ext CSR), then SMSM on one GPU.
set -o pipefail
OUT=gpurun_out/${1:-q2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/bench_smsm_dv.json 2> $OUT/bench_smsm.err &&
MSPLIT_MAT_STORAGE=csr timeout -k 10 300 python bench.py --variant smsm --storage csr --steps 2 --warmup 1 > $OUT/bench_smsm_csr.json 2>> $OUT/bench_smsm.err
echo "exit $?" > $OUT/status
