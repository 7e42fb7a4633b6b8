#!/bin/bash
# Round-5 GPU session 19: the symmetric STENCIL fused step with two threads per DBR lane (k_box_spmv_mdot_march_sym2)
# against the one-thread form (MSPLIT_RV_SYM2=0): STENCIL parity tests, interleaved non_stencil_aij A/B, a trace.
OUT=gpurun_out/${1:-r05_s19}
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
  step ns_two$i 300 python bench.py $NS
  step ns_one$i 300 env MSPLIT_RV_SYM2=0 python bench.py $NS
done
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py $NS
echo done >> $OUT/status
