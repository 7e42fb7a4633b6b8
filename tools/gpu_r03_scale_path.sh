#!/bin/bash
# The N > 1 bench path on the final round-3 build, on the one-GPU box:
#  0. tests/test_gpu_bench.py (2- and 3-rank launches whose lines carry the multi-rank check);
#  1. the per-GPU SMSM-global block every N > 1 line runs (bench.py --variant smsm, N = 1), under
#     rocprofv3 --kernel-trace --stats, so the SCALE lines' kernel mix has a profile of its own;
#  2. bench.py at N = 2 through torch.distributed.run (both ranks on the one GPU, gloo + the library's host
#     transport: RCCL refuses two ranks on one GPU), the exact launch the driver uses for SCALE, 512^2 x 128
#     blocks (two blocks of the configs[2] per-GPU size do not fit one card's time budget at full depth).
# Each GPU step has its own time limit; steps are chained with && so the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-scale_path}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $OUT/bench_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $OUT/smsm_trace -o run -f csv -- python3 bench.py --variant smsm --steps 2 --warmup 1 > $OUT/bench_smsm_trace.json 2> $OUT/smsm_trace.err &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --smsm-planes 128 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err
echo "exit $?" > $OUT/status
exit 0
