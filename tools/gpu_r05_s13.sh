#!/bin/bash
# Round-5 GPU session 13: the SEQ engine chosen by kind (norms parallel from 2^13 terms, dots 2^17, MDots 2^19):
# every test that runs the PETSc-order mode, then two seq_mode steps.
OUT=gpurun_out/${1:-r05_s13}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq_engine.py tests/test_gpu_seq.py tests/test_gpu_lsqr.py tests/test_gpu_gram.py tests/test_gpu_drivers.py tests/test_gpu_c_drivers.py -k "seq or order or petsc or gram or lsqr"
SQ="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-assembled --no-non-stencil"
step seq1 400 python bench.py $SQ
step seq2 400 python bench.py $SQ
echo done >> $OUT/status
