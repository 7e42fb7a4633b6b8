#!/bin/bash
# Round-5 GPU session 15: the one-launch SEQ engine (k_seqx_one): the SEQ-engine parity tests, then the crossover
# measurement with all three engines.
OUT=gpurun_out/${1:-r05_s15}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_seq_engine.py
step xover 500 python tools/seq_crossover.py
echo done >> $OUT/status
