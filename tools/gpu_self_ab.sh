#!/bin/bash
# The fused z-march MatMult+MDot taking the dot with x (the basis' last vector) from its registers: the DV/GMRES/
# graph/config GPU tests, then same-box A/B against MSPLIT_BOXMDOT_SELF=0 (the dot streamed), GMRES step and SMSM.
set -o pipefail
OUT=gpurun_out/self
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_gmres.py tests/test_gpu_graphs.py \
  tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $OUT/g_self_$r.json 2>/dev/null || exit 1
  MSPLIT_BOXMDOT_SELF=0 timeout -k 10 120 python bench.py $B > $OUT/g_strm_$r.json 2>/dev/null || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_self_$r.json 2>/dev/null || exit 1
  MSPLIT_BOXMDOT_SELF=0 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_strm_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
