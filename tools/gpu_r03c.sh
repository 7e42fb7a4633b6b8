#!/bin/bash
# LSQR deferred U1 scale: the LSQR/SMSM/seq parity tests, then the SMSM block with and without it (same box,
# interleaved), then the round session (tests, smoke, bench, rocprof, PMC).
set -o pipefail
OUT=gpurun_out/lsqrdefer
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lsqr.py tests/test_gpu_seq.py tests/test_gpu_gram.py > $OUT/tests.log 2>&1 || exit 1
for r in 1 2 3; do for w in 1 0; do
  MSPLIT_LSQR_SCALE_WRITE=$w timeout -k 10 200 python bench.py --variant smsm --steps 3 --warmup 1 > $OUT/s_w${w}_$r.json 2>/dev/null || exit 1
done; done
echo done > $OUT/status
bash tools/gpu_r03.sh r03b
