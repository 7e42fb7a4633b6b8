#!/bin/bash
# CSR SpMV policy/staging A/B inside the library (and the standalone lab on the same box).
set -o pipefail
O=gpurun_out/${1:-spmv_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gmres.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmv or storage_and_store or combination" > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 5 --flags ${FLAGS:-0,2097152,4194304,6291456,2} > $O/lib_ab_torch.json 2> $O/ab.err &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 5 --no-torch --flags ${FLAGS:-0,2097152,4194304,6291456,2} > $O/lib_ab_notorch.json 2>> $O/ab.err &&
timeout -k 10 200 tools/spmv_lab 512 10 0 1 > $O/lab512.json 2> $O/lab.err
echo "exit $?" > $O/status
