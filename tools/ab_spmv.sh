#!/bin/bash
# Same-box A/B of SpMV variants (tuning flags), then the parity tests.
set -o pipefail
O=gpurun_out/${1:-spmv_ab}; mkdir -p $O
T=${2:-0,8}
timeout -k 10 300 python tools/microbench.py --n 256 --kernels spmv --tunings $T --rounds 5 > $O/mb256.json 2> $O/mb256.err &&
timeout -k 10 300 python tools/microbench.py --n 512 --nz 256 --kernels spmv --tunings $T --rounds 5 > $O/mb512x256.json 2> $O/mb512x256.err &&
timeout -k 10 300 python tools/microbench.py --n 512 --nz 512 --kernels spmv --tunings $T --rounds 3 > $O/mb512.json 2> $O/mb512.err &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/tests.log 2>&1
echo "exit $?" > $O/status
