#!/bin/bash
# Round-5 GPU session 7: the SEQ walk with batched segment loads and ripple applies: the SEQ-engine and PETSc-order
# parity suites, bench.py's seq_mode step at ripple widths 0 / 4 / 8 / 16, one statistics run, the SMSM seq line.
OUT=gpurun_out/${1:-r05_s7}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq_engine.py tests/test_gpu_seq.py
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil"
for r in 0 8 4 16 8; do
  step seq_r$r 200 env MSPLIT_SEQ_RIPPLE=$r python bench.py $SQ
done
step seq_stats 200 env MSPLIT_SEQ_STATS=1 python bench.py $SQ
step seq_smsm 400 python bench.py $SQ --no-seq-mode
echo done >> $OUT/status
