#!/bin/bash
# The chunk-tile march SpMV (k_box_march_chunk): DV/GMRES/config GPU tests, the microbench of MatMult /
# MatResidual at 256^3 and 512^3 against the line kernels (msk_set_march_lines 4), and the GMRES step / SMSM
# block against MSPLIT_MARCH_CHUNK=0, interleaved.
set -o pipefail
OUT=gpurun_out/chunk
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_gmres.py tests/test_gpu_configs.py \
  tests/test_gpu_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --n 256 --storage dv --kernels spmv --march-lines 0,4,16 --reps 20 --rounds 3 > $OUT/mb256.json 2> $OUT/mb.err || exit 1
timeout -k 10 200 python tools/microbench.py --n 512 --nz 256 --storage dv --kernels spmv --march-lines 0,4,16 --reps 10 --rounds 3 > $OUT/mb512.json 2>> $OUT/mb.err || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2; do
  timeout -k 10 120 python bench.py $B > $OUT/g_chunk_$r.json 2>/dev/null || exit 1
  MSPLIT_MARCH_CHUNK=0 timeout -k 10 120 python bench.py $B > $OUT/g_lines_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
