set -o pipefail
O=gpurun_out/${1:-glds_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gmres.py tests/test_gpu_kats.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmv or storage_and_store or combination or kat" > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 5 --flags 0,4194304,2 > $O/ab512.json 2> $O/ab.err &&
timeout -k 10 300 python tools/spmv_policy_ab.py --n 256 --reps 20 --rounds 5 --flags 0,4194304,2 > $O/ab256.json 2>> $O/ab.err
echo "exit $?" > $O/status
