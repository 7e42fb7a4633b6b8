#!/bin/bash
# rocprofv3 kernel-trace stats + PMC traffic passes of the SMSM bench (1 GPU, configs[2] block).
set -o pipefail
OUT=gpurun_out/${1:-prof_smsm}
mkdir -p $OUT
export TMPDIR=/tmp
A="--variant smsm --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py $A > $OUT/bench_trace.json 2> $OUT/trace.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -f csv -- python3 bench.py $A --no-timing > $OUT/pmc_fetch.out 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -f csv -- python3 bench.py $A --no-timing > $OUT/pmc_write.out 2>&1
echo "exit $?" > $OUT/status
