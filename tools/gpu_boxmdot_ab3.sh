#!/bin/bash
# k_box_spmv_mdot_march, default on (MSPLIT_TUNING 1073741824: the separate kernels; 524288: tiles in plane order,
# not XCD-contiguous): bitwise tests, then the configs[1] step and the SMSM block, same box, interleaved.
set -o pipefail
OUT=gpurun_out/boxmdot4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dv.py -k "march or assembled" > $OUT/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  for t in 1073741824 0 524288; do
    MSPLIT_TUNING=$t timeout -k 10 120 python bench.py $B > $OUT/g_t${t}_$r.json 2>/dev/null || exit 1
  done
  MSPLIT_BOXMDOT_ZT=1 timeout -k 10 120 python bench.py $B > $OUT/g_z1_$r.json 2>/dev/null || exit 1
  for t in 1073741824 0 524288; do
    MSPLIT_TUNING=$t timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_t${t}_$r.json 2>/dev/null || exit 1
  done
done
echo done > $OUT/status
