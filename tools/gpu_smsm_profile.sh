#!/bin/bash
# SMSM-global (the N > 1 per-GPU workload) on one GPU: rocprofv3 kernel stats and FETCH/WRITE PMC passes.
set -o pipefail
O=gpurun_out/${1:-smsm_profile}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run -f csv -- python3 bench.py --variant smsm --steps 2 --warmup 1 --no-timing > $O/bench_trace.json 2> $O/trace.err &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing > $O/pmc_fetch.out 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing > $O/pmc_write.out 2>&1
echo "exit $?" > $O/status
