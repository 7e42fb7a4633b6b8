#!/bin/bash
# Round-5 GPU session 16: the SEQ transducer build refactored into trans_segment: SEQ parity suites, seq_mode steps.
OUT=gpurun_out/${1:-r05_s16}
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
step seq1 400 python bench.py $SQ
step seq2 400 python bench.py $SQ
echo done >> $OUT/status
