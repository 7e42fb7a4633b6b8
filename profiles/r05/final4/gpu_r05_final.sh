#!/bin/bash
# Round-5 measurement session: the whole -m gpu suite, smoke, the default bench (every N = 1 line), a kernel-trace
# stats profile of the headline step, its two PMC traffic passes, and the same three for the SMSM-global per-GPU
# block that every N > 1 line runs (bench.py --variant smsm: 512 x 512 x 256, s 20, inner max_it 20, LSQR 70).
# A test failure (exit 1) goes on; anything else ends the script.
OUT=gpurun_out/${1:-r05_final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -gt 1 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
pmc() {  # a counter pass: SIGKILL at its limit (a pass that asks too much of the hardware ignores SIGTERM)
  local name=$1 secs=$2; shift 2
  timeout -s KILL $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name $rc" >> $OUT/status
  if [ $rc -ne 0 ]; then echo "stopping after $name ($rc)" >> $OUT/status; exit 0; fi
}
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  step suite 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cp $OUT/bench.log $OUT/bench.json
NOX="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-seq-mode --no-seq-smsm --no-assembled --no-non-stencil"
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run -f csv -- python3 bench.py --steps 3 $NOX
pmc pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-timing --no-spmv512 $NOX
pmc pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -f csv -- python3 bench.py --steps 1 --warmup 0 --no-timing --no-spmv512 $NOX
step smsm_trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/smsm_trace -o run -f csv -- python3 bench.py --variant smsm --steps 2 --warmup 1 --no-cpu-baseline
pmc smsm_pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/smsm_pmc_fetch -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing --no-cpu-baseline
pmc smsm_pmc_write 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/smsm_pmc_write -o run -f csv -- python3 bench.py --variant smsm --steps 1 --warmup 0 --no-timing --no-cpu-baseline
echo done >> $OUT/status
