#!/bin/bash
# Contiguous matrix arrays too (CSR rowptr/col/val, DV codes, presence bytes): the 512^3 CSR MatMult of the bench
# line and the GMRES step against MSPLIT_ALLOC_CONTIGUOUS=0, interleaved; the DV/kernel GPU tests first.
set -o pipefail
OUT=gpurun_out/contig2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-seq-mode --no-assembled --no-csr-compare --steps 10"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $B > $OUT/g_contig_$r.json 2>/dev/null || exit 1
  MSPLIT_ALLOC_CONTIGUOUS=0 timeout -k 10 200 python bench.py $B > $OUT/g_plain_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
