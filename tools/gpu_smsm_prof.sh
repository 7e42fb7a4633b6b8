set -o pipefail
O=gpurun_out/${1:-smsm_prof}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --variant smsm --steps 3 --warmup 1 --timing-every 1 > $O/smsm.json 2> $O/err
echo "exit $?" > $O/status
