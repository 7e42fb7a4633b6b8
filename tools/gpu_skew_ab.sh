#!/bin/bash
# Same-box A/B: power-of-two strides of the SMSM basis (MSPLIT_BASIS_SKEW) and dense blocks (MSPLIT_DENSE_SKEW),
# and the temporal W store of the fused GMRES kernel (MSPLIT_TUNING 1048576), interleaved.
set -o pipefail
OUT=gpurun_out/skew
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_base_$r.json 2>/dev/null || exit 1
  MSPLIT_BASIS_SKEW=512 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_bskew_$r.json 2>/dev/null || exit 1
  MSPLIT_DENSE_SKEW=512 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_dskew_$r.json 2>/dev/null || exit 1
  MSPLIT_BASIS_SKEW=512 MSPLIT_DENSE_SKEW=512 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_both_$r.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
  MSPLIT_TUNING=1048576 timeout -k 10 120 python bench.py $B > $OUT/g_wtemp_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
