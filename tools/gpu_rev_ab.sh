#!/bin/bash
# Same-box A/B: alternating sweep directions so one kernel starts where the previous one ended (the MALL holds
# the last ~256 MB it touched): the fused MatMult+MDot top plane group first (MSPLIT_BOXMDOT_REV), or MAXPY top
# chunk first (MSPLIT_MAXPY_REV), interleaved, GMRES step and SMSM block.
set -o pipefail
OUT=gpurun_out/rev
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
  MSPLIT_BOXMDOT_REV=1 timeout -k 10 120 python bench.py $B > $OUT/g_frev_$r.json 2>/dev/null || exit 1
  MSPLIT_MAXPY_REV=1 timeout -k 10 120 python bench.py $B > $OUT/g_mrev_$r.json 2>/dev/null || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_base_$r.json 2>/dev/null || exit 1
  MSPLIT_BOXMDOT_REV=1 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_frev_$r.json 2>/dev/null || exit 1
  MSPLIT_MAXPY_REV=1 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_mrev_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
