set -o pipefail
O=gpurun_out/reentry; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo "exit $?" > $O/status
