#!/bin/bash
# Check of the LDS-staged k_norm_update and the size-chosen MAXPY order: the GMRES/graph/DV/KAT/seq/config
# GPU tests, a kernel-trace stats profile of the bench step (k_norm_update's average duration), then the
# GMRES step and the SMSM block (MAXPY top chunk first at 512x512x256) against MSPLIT_MAXPY_REV=0, interleaved.
set -o pipefail
OUT=gpurun_out/nu
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gmres.py tests/test_gpu_graphs.py tests/test_gpu_dv.py \
  tests/test_gpu_kats.py tests/test_gpu_seq.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 \
  --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-assembled --no-spmv512 > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
B="--no-cpu-baseline --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --no-csr-compare --steps 20"
for r in 1 2; do
  timeout -k 10 120 python bench.py $B > $OUT/g_new_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_auto_$r.json 2>/dev/null || exit 1
  MSPLIT_MAXPY_REV=0 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_fwd_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
