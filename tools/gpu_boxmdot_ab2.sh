#!/bin/bash
# k_box_spmv_mdot z-march depth 1/2/3 on the configs[1] step, and the SMSM block with and without it (depth 2),
# same box, interleaved.
set -o pipefail
OUT=gpurun_out/boxmdot3
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  MSPLIT_TUNING=0 timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
  for zt in 1 2 3; do
    MSPLIT_BOXMDOT_ZT=$zt MSPLIT_TUNING=1073741824 timeout -k 10 120 python bench.py $B > $OUT/g_z${zt}_$r.json 2>/dev/null || exit 1
  done
  for t in 0 1073741824; do
    MSPLIT_BOXMDOT_ZT=2 MSPLIT_TUNING=$t timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_t${t}_$r.json 2>/dev/null || exit 1
  done
done
echo done > $OUT/status
