#!/bin/bash
# Round-5 GPU session 3: the R-broadcast suites after registering only the device-state words of the shared
# region (session 2's configs[3] footprint run pinned the whole region), the LSQR tests, the configs[3]
# AMAM-global rank footprint, and the STENCIL-storage layout / prefetch A/B on the non-stencil AIJ step.
OUT=gpurun_out/${1:-r05_s3}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step tests 600 $PYT tests/test_gpu_lsqr.py tests/test_gpu_async.py tests/test_gpu_async_mp.py tests/test_gpu_amam_configs.py tests/test_gpu_nb8.py -k "lsqr or async or amam or mp"
step amam_fp 400 python tools/amam_configs.py footprint --minimization lsqr
NS="--steps 3 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled"
for i in 1 2; do
  step ns_soa$i 200 env MSPLIT_RV_LAYOUT=soa python bench.py $NS
  step ns_blocked$i 200 python bench.py $NS
  step ns_blocked_p4_$i 200 env MSPLIT_RV_PREFETCH=4 python bench.py $NS
  step ns_blocked_p2_$i 200 env MSPLIT_RV_PREFETCH=2 python bench.py $NS
done
echo done >> $OUT/status
