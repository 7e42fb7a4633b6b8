#!/bin/bash
# Round-5 GPU session 4: the symmetric STENCIL storage (diagonal + upper legs, 32 B/row): its parity tests, a
# same-box A/B against the seven-leg storage (MSPLIT_RV_SYM=0) on bench.py's non_stencil_aij leg, and a kernel
# trace of that leg.
OUT=gpurun_out/${1:-r05_s4}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dv.py -k "stencil or non_stencil or duplicate"
NS="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled"
for i in 1 2; do
  step ns_legs7_$i 200 env MSPLIT_RV_SYM=0 python bench.py $NS
  step ns_sym_$i 200 python bench.py $NS
done
step ns_trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/ns_trace -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-timing $NS
echo done >> $OUT/status
