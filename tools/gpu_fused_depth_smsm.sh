#!/bin/bash
# Depth of the fused MatMult+MDot march (MSPLIT_BOXMDOT_ZT) at the SMSM block size (512 x 512 planes), interleaved.
set -o pipefail
OUT=gpurun_out/fdepth
mkdir -p $OUT
for r in 1 2; do
  for Z in 1 2 4 8; do
    MSPLIT_BOXMDOT_ZT=$Z timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_z${Z}_$r.json 2>/dev/null || exit 1
  done
done
echo done > $OUT/status
