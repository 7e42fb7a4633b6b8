#!/bin/bash
# Round-5 GPU session 20: PMC traffic of the two-thread symmetric STENCIL fused step (FETCH_SIZE / WRITE_SIZE passes of
# bench.py's non_stencil_aij leg).
OUT=gpurun_out/${1:-r05_s20}
mkdir -p $OUT
export TMPDIR=/tmp
pmc() {
  local name=$1 secs=$2; shift 2
  timeout -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -ne 0 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
NS="--steps 1 --warmup 0 --no-timing --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-seq-smsm --no-assembled"
pmc ns_fetch 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/ns_fetch -o run -f csv -- python3 bench.py $NS
pmc ns_write 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/ns_write -o run -f csv -- python3 bench.py $NS
echo done >> $OUT/status
