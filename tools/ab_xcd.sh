set -o pipefail
O=gpurun_out/xcd1; mkdir -p $O
timeout -k 10 300 python tools/microbench.py --n 256 --kernels spmv --tunings 0,4 --groups 0,8,16 --rounds 5 > $O/mb256.json 2> $O/mb256.err &&
timeout -k 10 300 python tools/microbench.py --n 512 --nz 256 --kernels spmv --tunings 0,4 --groups 0,32,128 --rounds 5 > $O/mb512x256.json 2> $O/mb512x256.err &&
timeout -k 10 300 python tools/microbench.py --n 512 --nz 512 --kernels spmv --tunings 0,4 --groups 0,32,128 --rounds 3 > $O/mb512.json 2> $O/mb512.err &&
MSPLIT_TUNING=4 timeout -k 10 300 python -m pytest tests/test_gpu_gmres.py tests/test_gpu_kernels.py tests/test_gpu_lsqr.py -x -q > $O/tests_t4.log 2>&1
echo "exit $?" > $O/status
