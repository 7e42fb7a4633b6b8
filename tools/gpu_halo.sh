#!/bin/bash
# The chunk-tile march with coupling planes (A_ext: MatMult, MatResidual, R = A S): DV/convdiff/SMSM/driver GPU
# tests, then the SMSM block against MSPLIT_MARCH_CHUNK=0, interleaved.
set -o pipefail
OUT=gpurun_out/halo
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_convdiff.py tests/test_gpu_drivers.py \
  tests/test_gpu_libcomm_mp.py tests/test_gpu_configs.py tests/test_gpu_async.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_chunk_$r.json 2>/dev/null || exit 1
  MSPLIT_MARCH_CHUNK=0 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_ell_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
