#!/bin/bash
# Round-5 GPU session 9: the ripple walk's predicted-segment prefetch: SEQ parity suites, then bench.py's seq_mode
# step with and without it (MSPLIT_SEQ_PREFETCH=0), interleaved, one statistics run, the SMSM seq line.
OUT=gpurun_out/${1:-r05_s9}
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
for i in 1 2; do
  step seq_pf0_$i 200 env MSPLIT_SEQ_PREFETCH=0 python bench.py $SQ
  step seq_pf1_$i 200 python bench.py $SQ
done
step seq_stats 200 env MSPLIT_SEQ_STATS=1 python bench.py $SQ
step seq_smsm 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil --no-seq-mode
echo done >> $OUT/status
