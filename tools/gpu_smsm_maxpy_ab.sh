set -o pipefail
O=gpurun_out/${1:-smsm_maxpy_ab}; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_bench.sh "0 64 131072 256 16" 2 --variant smsm --steps 2 > $O/ab.txt 2>&1
echo "exit $?" > $O/status
