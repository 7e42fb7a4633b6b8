#!/bin/bash
# k_box_spmv_mdot (GMRES MatMult fused with VecMDot on box stencils, MSPLIT_TUNING 1073741824; +32: no z-march):
# bitwise tests, then a same-box A/B of the configs[1] step (z-march depths 2, 4, 8) and the SMSM block, interleaved.
set -o pipefail
OUT=gpurun_out/boxmdot2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dv.py -k "march or assembled" > $OUT/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  MSPLIT_TUNING=0 timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
  for zt in 2 4 8; do
    MSPLIT_BOXMDOT_ZT=$zt MSPLIT_TUNING=1073741824 timeout -k 10 120 python bench.py $B > $OUT/g_z${zt}_$r.json 2>/dev/null || exit 1
  done
done
for r in 1 2; do for t in 0 1073741824; do
MSPLIT_TUNING=$t timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_t${t}_$r.json 2>/dev/null || exit 1
done; done
echo done > $OUT/status
