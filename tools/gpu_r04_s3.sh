set -o pipefail
OUT=gpurun_out/r04_s3; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python tools/async_bench.py --n 256 --planes 128 --nb 2 --variant am --max-iterations 40 > $OUT/async_bench.json 2> $OUT/async_bench.err
echo "exit $?" > $OUT/status
