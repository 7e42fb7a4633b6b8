#!/bin/bash
# A/B 3 of the W-free MAXPY on the final build: wout stored with the default policy (MSPLIT_TUNING=64, so the next
# step's fused kernel may find VV(it+1) in the MALL) and the group loop unrolled by two (MSPLIT_MAXPY_MARCH_U2=1),
# against the defaults (non-temporal store, one group per iteration), GMRES step and SMSM block, two rounds.
set -o pipefail
OUT=gpurun_out/${1:-wfree_ab3}
mkdir -p $OUT
export TMPDIR=/tmp
X="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --steps 8"
run() { timeout -k 10 200 env $2 python bench.py $X > $OUT/$1.json 2> $OUT/$1.err; }
srun() { timeout -k 10 300 env $2 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/$1.json 2> $OUT/$1.err; }
for r in 1 2; do
  run g_d_$r "A=0" && run g_t_$r "MSPLIT_TUNING=64" && run g_u_$r "MSPLIT_MAXPY_MARCH_U2=1" &&
  srun s_d_$r "A=0" && srun s_t_$r "MSPLIT_TUNING=64" && srun s_u_$r "MSPLIT_MAXPY_MARCH_U2=1" || exit 1
done
echo "exit 0" > $OUT/status
exit 0
