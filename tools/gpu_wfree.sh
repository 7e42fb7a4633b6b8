#!/bin/bash
# The W-free GMRES step (k_box_maxpy_march recomputes W; the fused MatMult+MDot does not store it):
#  1. its bitwise tests and the march/GMRES tests of test_gpu_dv.py;
#  2. same-box A/B of the GMRES step (bench.py N = 1, extras off): W-free (default) against MSPLIT_GM_WFREE=0,
#     twice in alternation, then the SMSM block (the N > 1 per-GPU workload) both ways;
#  3. rocprofv3 --kernel-trace --stats of the default bench.
# Each GPU step has its own time limit; steps are chained with && so the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-wfree}
mkdir -p $OUT
export TMPDIR=/tmp
X="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled"
timeout -k 10 600 python -u -m pytest tests/test_gpu_wfree.py tests/test_gpu_dv.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 $X > $OUT/on_1.json 2> $OUT/on_1.err &&
MSPLIT_GM_WFREE=0 timeout -k 10 200 python bench.py --steps 10 $X > $OUT/off_1.json 2> $OUT/off_1.err &&
timeout -k 10 200 python bench.py --steps 10 $X > $OUT/on_2.json 2> $OUT/on_2.err &&
MSPLIT_GM_WFREE=0 timeout -k 10 200 python bench.py --steps 10 $X > $OUT/off_2.json 2> $OUT/off_2.err &&
timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/smsm_on.json 2> $OUT/smsm_on.err &&
MSPLIT_GM_WFREE=0 timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/smsm_off.json 2> $OUT/smsm_off.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 $X > $OUT/bench_trace.json 2> $OUT/trace.err
echo "exit $?" > $OUT/status
exit 0
