set -o pipefail
O=gpurun_out/${1:-glds_ab2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 8 --flags 0,4194304 > $O/ab512.json 2> $O/ab.err &&
bash tools/ab_bench.sh "0 4194304" 2 --storage csr --no-smsm-n1 --no-spmv512 --no-csr-compare > $O/ab_gmres_csr.txt 2>&1
echo "exit $?" > $O/status
