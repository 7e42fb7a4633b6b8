#!/bin/bash
# Round-5 GPU session 11: the symmetric STENCIL storage's fused step without the legs' LDS windows
# (k_box_spmv_mdot_march_sym, two workgroups a CU): the STENCIL-storage parity tests (every kernel variant bitwise the
# oracle and CSR), an interleaved A/B of bench.py's non_stencil_aij line (default / MSPLIT_RV_SYM_WPE=1 /
# MSPLIT_RV_SYM_LDS=1, the round-5 windowed kernel), and a kernel-trace profile of the default.
OUT=gpurun_out/${1:-r05_s11}
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
  step ns_new$i 300 python bench.py $NS
  step ns_wpe1_$i 300 env MSPLIT_RV_SYM_WPE=1 python bench.py $NS
  step ns_lds$i 300 env MSPLIT_RV_SYM_LDS=1 python bench.py $NS
done
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py $NS
echo done >> $OUT/status
