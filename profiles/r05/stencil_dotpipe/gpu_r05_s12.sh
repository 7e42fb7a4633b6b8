#!/bin/bash
# Round-5 GPU session 12: the STENCIL storage's fused step with its MDot in software-pipelined vector groups
# (MSPLIT_RV_DOTPIPE = 2 / 4): the STENCIL parity tests, then an interleaved A/B of bench.py's non_stencil_aij line,
# and a kernel-trace profile of each variant; then the SEQ parity suites and two seq_mode steps (trans prefetch).
OUT=gpurun_out/${1:-r05_s12}
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
  for d in 0 2 4; do
    step ns_dp${d}_$i 300 env MSPLIT_RV_DOTPIPE=$d python bench.py $NS
  done
done
for d in 0 2 4; do
  export MSPLIT_RV_DOTPIPE=$d
  step trace_dp$d 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace_dp$d -o run -f csv -- python3 bench.py $NS
done
unset MSPLIT_RV_DOTPIPE
# the SEQ transducer build with the next sum's y loaded one sum ahead
step seq_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq_engine.py tests/test_gpu_seq.py
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil --no-seq-smsm"
step seq1 200 python bench.py $SQ
step seq2 200 python bench.py $SQ
echo done >> $OUT/status
