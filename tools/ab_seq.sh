#!/bin/bash
# Same-box A/B of two library builds on bench.py's seq_mode leg (one configs[1] step in PETSc's order):
# tools/ab_lib/libmsplit_old.so is the other build (see tools/ab_rv.sh), loaded through MSPLIT_LIB.
set -o pipefail
O=gpurun_out/${1:-r04_seqab}; mkdir -p $O
B="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-non-stencil --no-assembled"
for i in 1 2; do
  MSPLIT_LIB=$PWD/tools/ab_lib/libmsplit_old.so timeout -k 10 200 python bench.py $B > $O/old$i.json 2> $O/old$i.err || exit 1
  timeout -k 10 200 python bench.py $B > $O/new$i.json 2> $O/new$i.err || exit 1
done
