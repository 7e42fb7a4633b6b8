set -o pipefail
O=gpurun_out/${1:-ellx_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dv.py tests/test_gpu_gmres.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/microbench.py --n 512 --kernels spmv --storage dv --reps 10 --rounds 3 --tunings 0,134217728 > $O/mb512.json 2> $O/mb.err &&
timeout -k 10 300 python tools/microbench.py --n 1024 --nz 128 --kernels spmv --storage dv --reps 10 --rounds 3 --tunings 0,134217728 > $O/mb1024.json 2>> $O/mb.err &&
timeout -k 10 300 python tools/microbench.py --n 256 --kernels spmv --storage dv --reps 20 --rounds 3 --tunings 0,67108864 > $O/mb256.json 2>> $O/mb.err &&
bash tools/ab_bench.sh "0 134217728" 2 --variant smsm --steps 2 > $O/ab_smsm.txt 2>&1
echo "exit $?" > $O/status
