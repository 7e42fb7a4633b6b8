#!/bin/bash
# Round-5 GPU session 17: the SEQ transducer kernel held to 3 waves per SIMD (spills) against 2: SEQ engine tests at
# both, then seq_mode steps interleaved.
OUT=gpurun_out/${1:-r05_s17}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests3 600 env MSPLIT_SEQ_TRANS_WPE=3 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq_engine.py
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil"
for i in 1 2; do
  step seq_w2_$i 400 python bench.py $SQ
  step seq_w3_$i 400 env MSPLIT_SEQ_TRANS_WPE=3 python bench.py $SQ
done
echo done >> $OUT/status
