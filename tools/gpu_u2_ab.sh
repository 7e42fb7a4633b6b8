#!/bin/bash
# The fused MatMult+MDot with its dot groups unrolled by two (MSPLIT_BOXMDOT_UNROLL2=1): bitwise check on the
# GMRES/DV tests, then GMRES step and SMSM block against the default, interleaved.
# (MSPLIT_BOXMDOT_UNROLL2 was an A/B-only knob, removed after this run: profiles/r03/boxmdot/unroll2/)
set -o pipefail
OUT=gpurun_out/u2
mkdir -p $OUT
export TMPDIR=/tmp
MSPLIT_BOXMDOT_UNROLL2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_gmres.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  MSPLIT_BOXMDOT_UNROLL2=1 timeout -k 10 120 python bench.py $B > $OUT/g_u2_$r.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
done
for r in 1 2; do
  MSPLIT_BOXMDOT_UNROLL2=1 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_u2_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_base_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
