#!/bin/bash
# Round-5 GPU session 10: ripple steps of one add and two DPP moves (no parity select without ties, no copy of s):
# SEQ parity suites, bench.py's seq_mode step at ripple widths (segments / after a serial sub), one statistics run,
# the SMSM seq line.
OUT=gpurun_out/${1:-r05_s10}
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
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil --no-seq-smsm"
for c in "16 8" "32 8" "16 16" "32 16" "8 8" "16 4" "16 8"; do
  set -- $c
  step seq_w$1_s$2 200 env MSPLIT_SEQ_RIPPLE_W=$1 MSPLIT_SEQ_RIPPLE=$2 python bench.py $SQ
done
step seq_stats 200 env MSPLIT_SEQ_STATS=1 python bench.py $SQ
step seq_smsm 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil --no-seq-mode
echo done >> $OUT/status
