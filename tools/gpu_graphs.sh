#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-graphs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_gmres.py tests/test_gpu_dv.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/graph_bench.py > $OUT/graph_bench.json 2> $OUT/graph_bench.err &&
MSPLIT_GRAPHS=0 timeout -k 10 300 python bench.py --variant smsm --smsm-mesh 64 --smsm-planes 32 --steps 3 --warmup 1 --no-timing > $OUT/smsm_small_eager.json 2> $OUT/smsm.err &&
MSPLIT_GRAPHS=1 timeout -k 10 300 python bench.py --variant smsm --smsm-mesh 64 --smsm-planes 32 --steps 3 --warmup 1 --no-timing > $OUT/smsm_small_graph.json 2>> $OUT/smsm.err &&
timeout -k 10 300 python bench.py --no-timing --no-cpu-baseline --no-csr-compare > $OUT/bench_graph.json 2> $OUT/bench.err
echo "exit $?" > $OUT/status
