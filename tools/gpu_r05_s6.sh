#!/bin/bash
# Round-5 GPU session 6: the SMSM per-GPU block in PETSc's reduction order (bench.py smsm_seq_mode), after its
# 48x48x32 golden test; the SEQ walk with its memory waits timed (MSPLIT_SEQ_STATS=1).
OUT=gpurun_out/${1:-r05_s6}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq.py -k "smsm"
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil --no-seq-mode"
step seq_smsm 400 python bench.py $SQ
SM="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil"
step seq_stats 200 env MSPLIT_SEQ_STATS=1 python bench.py $SM
echo done >> $OUT/status
