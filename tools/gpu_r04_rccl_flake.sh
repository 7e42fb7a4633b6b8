#!/bin/bash
# Repeat the multi-rank C-host and LibComm cases (MPI host transport and RCCL over its socket transport, ranks sharing
# the one GPU) three times: the check on msp_comm_sum_ordered's host synchronisations.  A test failure (exit 1) is data and the script goes on; any other
# status (a time limit, a signal) ends it.
set -o pipefail
OUT=gpurun_out/${1:-r04_rcclflake}
mkdir -p $OUT
run() {  # $1 tag
  timeout -k 10 330 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_c_drivers.py tests/test_gpu_libcomm_mp.py tests/test_gpu_bench.py -k "mpi_ranks_equal_oracle or rccl" > $OUT/$1.txt 2>&1
  local rc=$?
  echo "$1 exit $rc" >> $OUT/summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run rep1 && run rep2 && run rep3
echo "done $?" >> $OUT/summary.txt
exit 0
