# Same-box A/B of two library builds on bench.py's non_stencil_aij leg: tools/ab_lib/libmsplit_old.so is the other
# build (make it by building the library from the other source and copying libmsplit_hip.so there; MSPLIT_LIB loads it).
set -o pipefail
O=gpurun_out/r04_rvab; mkdir -p $O
B="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled"
for i in 1 2 3; do
  MSPLIT_LIB=$PWD/tools/ab_lib/libmsplit_old.so timeout -k 10 200 python bench.py $B > $O/old$i.json 2> $O/old$i.err || exit 1
  timeout -k 10 200 python bench.py $B > $O/new$i.json 2> $O/new$i.err || exit 1
done
