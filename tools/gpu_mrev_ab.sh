#!/bin/bash
# Same-box A/B of the MAXPY chunk order at the SMSM block size (512x512x256, vectors of 537 MB): top chunk first
# (the default above 2^25 rows) against bottom first (MSPLIT_MAXPY_REV=0), four interleaved pairs.
set -o pipefail
OUT=gpurun_out/mrev
mkdir -p $OUT
for r in 1 2 3 4; do
  MSPLIT_MAXPY_REV=0 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_fwd_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_auto_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
