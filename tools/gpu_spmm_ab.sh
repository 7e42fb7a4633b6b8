set -o pipefail
O=gpurun_out/${1:-spmm_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_lsqr.py -m gpu -x -q --timeout 120 --timeout-method thread -k "matmult_dense or smsm" > $O/tests.log 2>&1 &&
MSPLIT_SPMM_COLS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dv.py tests/test_gpu_lsqr.py -m gpu -x -q --timeout 120 --timeout-method thread -k "matmult_dense or smsm" > $O/tests_cols1.log 2>&1 &&
for c in 0 1 2 4 8 0 4; do MSPLIT_SPMM_COLS=$c timeout -k 10 200 python tools/spmm_ab.py >> $O/ab.jsonl 2>> $O/ab.err || exit 1; done
echo "exit $?" > $O/status
