#!/bin/bash
# Round-5 GPU session 14: the STENCIL storage's GMRES step with the MatMult and the MDot as two kernels (the MDot then
# runs at the occupancy of the plain stage-1 kernel) against the fused one, same process, two runs.
OUT=gpurun_out/${1:-r05_s14}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
NS="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-seq-smsm --no-assembled"
export MSPLIT_BENCH_STENCIL_AB=1
step ns1 300 python bench.py $NS
step ns2 300 python bench.py $NS
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py $NS
echo done >> $OUT/status
