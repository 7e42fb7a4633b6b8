#!/bin/bash
# SMSM-global on the GPU: parity tests, single-GPU bench (small + configs[2]
# block size) and 2-rank gloo rehearsals (both ranks on the box's one GPU).
set -o pipefail
OUT=gpurun_out/${1:-smsm}
mkdir -p $OUT
export TMPDIR=/tmp
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 300 python -m pytest tests/test_gpu_lsqr.py -x -q > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --variant smsm --smsm-mesh 64 --smsm-planes 32 --steps 2 --warmup 1 > $OUT/bench_small.json 2> $OUT/bench_small.err &&
timeout -k 10 300 $RUN bench.py --gpus 2 --backend gloo --smsm-mesh 64 --smsm-planes 32 --steps 2 --warmup 1 > $OUT/bench_gloo_small.json 2> $OUT/bench_gloo_small.err &&
timeout -k 10 400 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/bench_smsm.json 2> $OUT/bench_smsm.err &&
timeout -k 10 500 $RUN bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 > $OUT/bench_gloo.json 2> $OUT/bench_gloo.err
echo "exit $?" > $OUT/status
