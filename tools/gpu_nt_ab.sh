#!/bin/bash
# After the store-policy fix: SpMV tests, CSR policies at 512^3, DV (ELL) non-temporal y on the GMRES step.
set -o pipefail
O=gpurun_out/${1:-nt_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gmres.py tests/test_gpu_dv.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 5 --flags 0,2097152,2,4194304,6291456 > $O/lib_ab_512.json 2> $O/ab.err &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 256 --reps 20 --rounds 5 --flags 0,2097152,2,4194304,6291456 > $O/lib_ab_256.json 2>> $O/ab.err &&
bash tools/ab_bench.sh "0 1048576" 3 --no-smsm-n1 --no-spmv512 --no-csr-compare > $O/ab_ell_nty.txt 2>&1
echo "exit $?" > $O/status
