#!/bin/bash
# Round-5 GPU session 26: plane depth of the W-free MAXPY march (MSPLIT_MAXPY_ZT = 1, the default, against 2) on the
# headline and the SMSM block, interleaved, with the fused step at four planes.
OUT=gpurun_out/${1:-r05_s26}
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
  step hd_z1_$i 300 python bench.py $HD
  step hd_z2_$i 300 env MSPLIT_MAXPY_ZT=2 python bench.py $HD
  step sm_z1_$i 300 python bench.py $SM
  step sm_z2_$i 300 env MSPLIT_MAXPY_ZT=2 python bench.py $SM
done
echo done >> $OUT/status
