#!/bin/bash
# 256^3 GMRES step: MAXPY's w kept in the MALL (default-policy store, MSPLIT_TUNING 64) with MAXPY top chunk first
# (MSPLIT_MAXPY_REV=1), so the next fused MatMult+MDot, which starts at the bottom, reads x = that w from the MALL;
# against the defaults and each change alone, interleaved.
set -o pipefail
OUT=gpurun_out/wmall
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
  MSPLIT_MAXPY_REV=1 MSPLIT_TUNING=64 timeout -k 10 120 python bench.py $B > $OUT/g_both_$r.json 2>/dev/null || exit 1
  MSPLIT_TUNING=64 timeout -k 10 120 python bench.py $B > $OUT/g_t64_$r.json 2>/dev/null || exit 1
  MSPLIT_MAXPY_REV=1 timeout -k 10 120 python bench.py $B > $OUT/g_rev_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
