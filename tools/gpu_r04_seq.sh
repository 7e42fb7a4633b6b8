#!/bin/bash
# Round-4 session for MSP_REDUCE_SEQ's exact parallel engine: the SEQ parity tests, the walk counters of one
# PETSc-order configs[1] step (MSPLIT_SEQ_STATS=1), a kernel-trace stats profile of that step, and the default bench.
# Each GPU step has its own time limit; steps are chained with && so the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-r04_seq}
mkdir -p $OUT
export TMPDIR=/tmp
SEQONLY="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-non-stencil --no-assembled"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_seq_engine.py tests/test_gpu_seq.py > $OUT/tests.txt 2>&1 &&
MSPLIT_SEQ_STATS=1 timeout -k 10 300 python bench.py $SEQONLY > $OUT/stats.json 2> $OUT/stats.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py $SEQONLY > $OUT/trace.json 2> $OUT/trace.err &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "exit $?" > $OUT/status
exit 0
