#!/bin/bash
# Five more interleaved pairs of the GMRES step: x's dot from the march registers against streamed.
set -o pipefail
OUT=gpurun_out/self2
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3 4 5; do
  MSPLIT_BOXMDOT_SELF=0 timeout -k 10 120 python bench.py $B > $OUT/g_strm_$r.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py $B > $OUT/g_self_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
