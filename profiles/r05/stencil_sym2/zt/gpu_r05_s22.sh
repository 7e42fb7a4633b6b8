#!/bin/bash
# Round-5 GPU session 22: the STENCIL step's default plane depth 4 (against 8 and 2 by MSPLIT_BOXMDOT_ZT), and the
# STENCIL parity tests at the new default.
OUT=gpurun_out/${1:-r05_s22}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dv.py -k "stencil or variable_coefficient or non_stencil"
NS="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-seq-smsm --no-assembled"
for i in 1 2; do
  step ns_def$i 300 python bench.py $NS
  step ns_zt8_$i 300 env MSPLIT_BOXMDOT_ZT=8 python bench.py $NS
done
echo done >> $OUT/status
