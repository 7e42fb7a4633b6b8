#!/bin/bash
# Round-5: bench.py --variant amam (the configs[3] / configs[4] per-GPU AMAM-global blocks) on the final tree, both
# minimizations.
OUT=gpurun_out/${1:-r05_amam}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step c3_rtr 500 python bench.py --variant amam --minimization rtr --no-cpu-baseline
step c3_lsqr 500 python bench.py --variant amam --minimization lsqr --no-cpu-baseline
step c4_rtr 500 python bench.py --variant amam --minimization rtr --peclet 0.5,0.25,-0.3 --no-cpu-baseline
step c4_lsqr 500 python bench.py --variant amam --minimization lsqr --peclet 0.5,0.25,-0.3 --no-cpu-baseline
echo done >> $OUT/status
