#!/bin/bash
# updateLocalRHS over the coupled rows only: kernel / driver / multi-process GPU tests, then the SMSM block
# against MSPLIT_RHS_FULL=1 (the full MatResidual, a copy of b per update), interleaved.
set -o pipefail
OUT=gpurun_out/rhs
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_drivers.py tests/test_gpu_libcomm_mp.py \
  tests/test_gpu_c_drivers.py tests/test_gpu_configs.py tests/test_gpu_seq.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_listed_$r.json 2>/dev/null || exit 1
  MSPLIT_RHS_FULL=1 timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_full_$r.json 2>/dev/null || exit 1
done
echo done > $OUT/status
