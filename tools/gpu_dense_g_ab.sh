#!/bin/bash
# Columns per load group in the LSQR kernels (k_dense_gemv, k_scaled_dot): 4 (default) against 5 and 10
# (MSPLIT_DENSE_G), bitwise LSQR tests under each, the LSQR microbench at the SMSM block size, then the SMSM block.
set -o pipefail
OUT=gpurun_out/dense_g
mkdir -p $OUT
export TMPDIR=/tmp
for G in 5 10; do
  MSPLIT_DENSE_G=$G timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqr.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > $OUT/tests_g$G.log 2>&1 || exit 1
done
for r in 1 2; do
  for G in 0 5 10; do
    MSPLIT_DENSE_G=$G timeout -k 10 200 python tools/microbench.py --n 512 --nz 256 --kernels lsqr --reps 2 --rounds 2 \
      > $OUT/mb_g${G}_$r.json 2> $OUT/mb.err || exit 1
  done
done
for r in 1 2; do
  for G in 0 5 10; do
    MSPLIT_DENSE_G=$G timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_g${G}_$r.json 2>/dev/null || exit 1
  done
done
echo done > $OUT/status
