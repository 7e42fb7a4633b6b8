set -o pipefail
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 400 python bench.py --variant smsm --steps 2 --warmup 1 > $O/smsm.json 2> $O/smsm.err
echo "exit $?" > $O/status
