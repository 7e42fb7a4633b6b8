#!/bin/bash
# Round-5 flake check: the multi-process GPU suites (MPI C hosts, multi-process IPC / LibComm, the bench rehearsals,
# nb = 8) twice more on the final tree.  A test failure (exit 1) goes on; anything else ends the script.
OUT=gpurun_out/${1:-r05_flake}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
MP="tests/test_gpu_async_mp.py tests/test_gpu_libcomm_mp.py tests/test_gpu_bench.py tests/test_gpu_c_host.py tests/test_gpu_c_drivers.py tests/test_gpu_async.py"
for i in 1 2; do
  step mp$i 540 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider $MP
done
echo done >> $OUT/status
