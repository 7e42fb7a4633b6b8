#!/bin/bash
# Round-5 GPU session 24: plane depth of the DV fused step on the SMSM block (512 x 512 x 256) and the headline:
# MSPLIT_BOXMDOT_ZT = 2 (default) / 4, interleaved.
OUT=gpurun_out/${1:-r05_s24}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
SM="--variant smsm --steps 2 --warmup 1 --no-cpu-baseline"
HD="--steps 5 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-seq-smsm --no-assembled --no-non-stencil"
for i in 1 2; do
  step sm_zt2_$i 300 python bench.py $SM
  step sm_zt4_$i 300 env MSPLIT_BOXMDOT_ZT=4 python bench.py $SM
  step hd_zt2_$i 300 python bench.py $HD
  step hd_zt4_$i 300 env MSPLIT_BOXMDOT_ZT=4 python bench.py $HD
done
echo done >> $OUT/status
