#!/bin/bash
# Physically contiguous large buffers (MSPLIT_ALLOC_CONTIGUOUS=1) against hipMalloc: GMRES step and SMSM block,
# interleaved (run-to-run spread of the LSQR kernels and the first-run effect).
set -o pipefail
OUT=gpurun_out/contig
mkdir -p $OUT
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  MSPLIT_ALLOC_CONTIGUOUS=1 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_contig_$r.json 2> $OUT/s_contig_$r.err || exit 1
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_base_$r.json 2>/dev/null || exit 1
  MSPLIT_ALLOC_CONTIGUOUS=1 timeout -k 10 120 python bench.py $B > $OUT/g_contig_$r.json 2> $OUT/g_contig_$r.err || exit 1
  timeout -k 10 120 python bench.py $B > $OUT/g_base_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
