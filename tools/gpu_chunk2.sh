#!/bin/bash
# The chunk-tile march with its grid-balanced depth: the DV GPU tests, the MatMult microbench (auto = chunk,
# 4 = line tiles) at 256^3 and 512x512x256, then GMRES step and SMSM block against MSPLIT_MARCH_CHUNK=0.
set -o pipefail
OUT=gpurun_out/chunk4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dv.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --n 256 --storage dv --kernels spmv --march-lines 0,4 --reps 20 --rounds 3 > $OUT/mb256.json 2> $OUT/mb.err || exit 1
timeout -k 10 200 python tools/microbench.py --n 512 --nz 256 --storage dv --kernels spmv --march-lines 0,4 --reps 10 --rounds 3 > $OUT/mb512.json 2>> $OUT/mb.err || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $OUT/g_chunk_$r.json 2>/dev/null || exit 1
  MSPLIT_MARCH_CHUNK=0 timeout -k 10 120 python bench.py $B > $OUT/g_lines_$r.json 2>/dev/null || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_chunk_$r.json 2>/dev/null || exit 1
  MSPLIT_MARCH_CHUNK=0 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_lines_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
