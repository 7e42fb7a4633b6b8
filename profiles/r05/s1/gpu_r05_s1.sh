#!/bin/bash
# Round-5 GPU session 1: the nb = 8 suite (one process, 8 MPI ranks over the host transport and RCCL, AMAM-global
# twin at 8 blocks, configs[4] whole), the stop-agreement fault tests, the 8-rank bench launch; then the comm-fix
# diagnostic (persistent buffers without the host-synchronised hops, MSPLIT_COMM_HOST_SYNC=0) on the serialised
# cases; then one FETCH / WRITE PMC pass of the non-stencil AIJ step.  A test failure (exit 1) goes on to the next
# step; any other exit status (a timeout, an abort, a fault) ends the script there.
OUT=gpurun_out/${1:-r05_s1}
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
step() {  # step NAME SECONDS CMD...: runs, records the status; stops the script on anything but 0 or 1
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
step nb8 1100 $PYT tests/test_gpu_nb8.py
step fault 300 $PYT tests/test_gpu_c_drivers.py -k disagreement
step bench8 600 $PYT tests/test_gpu_bench.py -k "rccl_multi_rank and 8"
step nosync_serial 400 env MSPLIT_COMM_HOST_SYNC=0 $PYT tests/test_gpu_c_drivers.py -k serialized
step nosync_ranks 600 env MSPLIT_COMM_HOST_SYNC=0 $PYT tests/test_gpu_c_drivers.py -k "mpi_ranks_equal_oracle"
NOX="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-assembled --no-spmv512 --no-timing"
step ns_fetch 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/ns_pmc_fetch -o run -f csv -- python3 bench.py --steps 1 --warmup 0 $NOX
step ns_write 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/ns_pmc_write -o run -f csv -- python3 bench.py --steps 1 --warmup 0 $NOX
echo done >> $OUT/status
