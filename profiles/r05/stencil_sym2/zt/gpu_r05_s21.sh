#!/bin/bash
# Round-5 GPU session 21: plane depth of the fused z-march (MSPLIT_BOXMDOT_ZT = 2 / 3 / 4) for the symmetric STENCIL
# step (and the headline's DV step, which shares the knob), interleaved.
OUT=gpurun_out/${1:-r05_s21}
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
for i in 1 2; do
  for z in 2 3 4; do
    step ns_zt${z}_$i 300 env MSPLIT_BOXMDOT_ZT=$z python bench.py $NS
  done
done
echo done >> $OUT/status
