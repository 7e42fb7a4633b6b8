#!/bin/bash
# A/B of the W-free MAXPY's launch shape (k_box_maxpy_march), same box, GMRES step (bench.py N = 1, extras off):
# default (2 planes per workgroup, one group of four per loop iteration, plane order) against the group loop
# unrolled by two (MSPLIT_MAXPY_MARCH_U2=1), 1 and 4 planes per workgroup (MSPLIT_MAXPY_ZT), top plane groups
# first (MSPLIT_MAXPY_REV=1); two rounds in alternation; then the SMSM block default / U2 / REV=0.
set -o pipefail
OUT=gpurun_out/${1:-wfree_ab}
mkdir -p $OUT
export TMPDIR=/tmp
X="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --steps 8"
run() { timeout -k 10 200 env $2 python bench.py $X > $OUT/$1.json 2> $OUT/$1.err; }
run d_1 "A=0" && run u2_1 "MSPLIT_MAXPY_MARCH_U2=1" && run z1_1 "MSPLIT_MAXPY_ZT=1" && run z4_1 "MSPLIT_MAXPY_ZT=4" &&
run rev_1 "MSPLIT_MAXPY_REV=1" &&
run d_2 "A=0" && run u2_2 "MSPLIT_MAXPY_MARCH_U2=1" && run z1_2 "MSPLIT_MAXPY_ZT=1" && run z4_2 "MSPLIT_MAXPY_ZT=4" &&
run rev_2 "MSPLIT_MAXPY_REV=1" &&
timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/smsm_d.json 2> $OUT/smsm_d.err &&
MSPLIT_MAXPY_MARCH_U2=1 timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/smsm_u2.json 2> $OUT/smsm_u2.err &&
MSPLIT_MAXPY_REV=0 timeout -k 10 300 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/smsm_rev0.json 2> $OUT/smsm_rev0.err
echo "exit $?" > $OUT/status
exit 0
