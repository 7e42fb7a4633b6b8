#!/bin/bash
# Round-5 GPU session 8: the ripple walk (k_seqx_ripwalk): the SEQ-engine and PETSc-order parity suites, bench.py's
# seq_mode step with the scan walk and the ripple walk at several widths, one statistics run, the SMSM seq line.
OUT=gpurun_out/${1:-r05_s8}
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
step seq_scan 200 env MSPLIT_SEQ_WALK=scan python bench.py $SQ
for c in "16 8" "8 8" "32 8" "16 4" "16 16"; do
  set -- $c
  step seq_w$1_s$2 200 env MSPLIT_SEQ_RIPPLE_W=$1 MSPLIT_SEQ_RIPPLE=$2 python bench.py $SQ
done
step seq_stats 200 env MSPLIT_SEQ_STATS=1 python bench.py $SQ
step seq_smsm 400 python bench.py $SQ --no-seq-mode
echo done >> $OUT/status
