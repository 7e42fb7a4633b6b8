#!/bin/bash
# Round-5 GPU session 2: the whole -m gpu suite on the tree with the one-pass DBR LSQR step (regenerated
# oracle records), the stream-published R broadcast, stream-ordered comm hops and the optional STENCIL storage;
# then a same-box interleaved A/B of the SMSM-global block with the one-pass LSQR against the two passes
# (MSPLIT_LSQR_ONEPASS=0), and the configs[3] AMAM-global rank footprint (minimization time).  A test failure
# (exit 1) goes on; anything else ends the script.
OUT=gpurun_out/${1:-r05_s2}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
SM="--variant smsm --steps 2 --warmup 1 --no-cpu-baseline"
for i in 1 2; do
  step smsm_two$i 200 env MSPLIT_LSQR_ONEPASS=0 python bench.py $SM
  step smsm_one$i 200 python bench.py $SM
done
step amam_fp 400 python tools/amam_configs.py footprint --minimization lsqr
echo done >> $OUT/status
NS="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled"
for i in 1 2; do
  step ns_soa$i 300 env MSPLIT_RV_LAYOUT=soa python bench.py $NS
  step ns_blocked$i 300 python bench.py $NS
  step ns_blocked_p4_$i 300 env MSPLIT_RV_PREFETCH=4 python bench.py $NS
  step ns_blocked_p2_$i 300 env MSPLIT_RV_PREFETCH=2 python bench.py $NS
done
echo done2 >> $OUT/status
