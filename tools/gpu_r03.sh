#!/bin/bash
# Round-3 GPU session: the whole -m gpu suite, smoke, the default bench, a kernel-trace stats profile of
# the bench and the two PMC traffic passes (the parity-mode seq_mode step is left out of the profiler runs).
# Each GPU step has its own time limit; steps are chained with && so the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-assembled > $OUT/bench_trace.json 2> $OUT/trace.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-timing --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled > $OUT/pmc_fetch.out 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-timing --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled > $OUT/pmc_write.out 2>&1
echo "exit $?" > $OUT/status
exit 0
