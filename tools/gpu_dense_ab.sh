set -o pipefail
O=gpurun_out/${1:-dense_ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqr.py tests/test_gpu_seq.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python tools/microbench.py --n 512 --nz 256 --kernels lsqr,maxpy --reps 2 --rounds 3 --tunings 0,8388608,16777216,33554432,41943040 > $O/mb_lsqr.json 2> $O/mb.err &&
bash tools/ab_bench.sh "0 41943040" 2 --variant smsm --steps 2 > $O/ab_smsm.txt 2>&1
echo "exit $?" > $O/status
