#!/bin/bash
# Round-4 GPU session (after the -m gpu suite): smoke, the default bench, a kernel-trace stats profile of it, the
# two PMC traffic passes of the GMRES step, and the same three for the SMSM-global per-GPU block that every N > 1
# line runs (bench.py --variant smsm: 512 x 512 x 256, s 20, inner max_it 20, LSQR 70).
# Each GPU step has its own time limit; steps are chained with && so the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-r04}
mkdir -p $OUT
export TMPDIR=/tmp
NOX="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-assembled --no-non-stencil"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 $NOX > $OUT/bench_trace.json 2> $OUT/trace.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-timing --no-spmv512 $NOX > $OUT/pmc_fetch.out 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-timing --no-spmv512 $NOX > $OUT/pmc_write.out 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/smsm_trace -o run -f csv -- python3 bench.py --variant smsm --steps 2 --warmup 1 --no-cpu-baseline > $OUT/smsm_trace.json 2> $OUT/smsm_trace.err &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/smsm_pmc_fetch -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing --no-cpu-baseline > $OUT/smsm_pmc_fetch.out 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/smsm_pmc_write -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing --no-cpu-baseline > $OUT/smsm_pmc_write.out 2>&1
echo "exit $?" > $OUT/status
exit 0
