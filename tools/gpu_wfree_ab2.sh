#!/bin/bash
# A/B 2 of the W-free MAXPY (k_box_maxpy_march): one plane per workgroup (MSPLIT_MAXPY_ZT=1) with and without the
# group loop unrolled by two, against the 2-plane default, on the GMRES step and on the SMSM block; two rounds.
set -o pipefail
OUT=gpurun_out/${1:-wfree_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
X="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --steps 8"
run() { timeout -k 10 200 env $2 python bench.py $X > $OUT/$1.json 2> $OUT/$1.err; }
srun() { timeout -k 10 300 env $2 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/$1.json 2> $OUT/$1.err; }
run z1_1 "MSPLIT_MAXPY_ZT=1" && run z1u2_1 "MSPLIT_MAXPY_ZT=1 MSPLIT_MAXPY_MARCH_U2=1" &&
run z1_2 "MSPLIT_MAXPY_ZT=1" && run z1u2_2 "MSPLIT_MAXPY_ZT=1 MSPLIT_MAXPY_MARCH_U2=1" &&
srun s_z2_1 "MSPLIT_MAXPY_ZT=2" && srun s_z1_1 "MSPLIT_MAXPY_ZT=1" && srun s_z1u2_1 "MSPLIT_MAXPY_ZT=1 MSPLIT_MAXPY_MARCH_U2=1" &&
srun s_z2_2 "MSPLIT_MAXPY_ZT=2" && srun s_z1_2 "MSPLIT_MAXPY_ZT=1" && srun s_z1u2_2 "MSPLIT_MAXPY_ZT=1 MSPLIT_MAXPY_MARCH_U2=1"
echo "exit $?" > $OUT/status
exit 0
