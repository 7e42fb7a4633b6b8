#!/bin/bash
# Round 4: the 2-rank C-host SMSM-global case GPUTEST_r03 caught (5 outer iterations against the oracle's 3).
# Repeats it in one process and over 2 MPI ranks under each transport / runtime setting, printing the transport,
# the outer count and the history of every run, so the failing configuration is named by evidence.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r04_diag
OUT=gpurun_out/r04_diag/runs.txt
: > "$OUT"
echo "HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES-unset} ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES-unset}" | tee -a "$OUT"
timeout -k 10 60 rocm-smi --showid 2>&1 | grep -E "GPU|Device" | head -20 | tee -a "$OUT" || true
make -s -C host || exit 1
INNER="-inner1_ksp_max_it 20 -inner1_ksp_rtol 1e-20 -inner2_ksp_max_it 20 -inner2_ksp_rtol 1e-20"
OUTER=""
for b in 1 2; do
  OUTER="$OUTER -outer${b}_ksp_type lsqr -outer${b}_ksp_convergence_test default -outer${b}_ksp_lsqr_exact_mat_norm"
  OUTER="$OUTER -outer${b}_ksp_max_it 70 -outer${b}_ksp_rtol 1e-15 -outer${b}_ksp_atol 1e-100"
done
ARGS="synchronous-multisplitting-synchronous-minimization-global -dim 3 -m 8 -n 8 -p 8 -s 4 -rtol 1e-6 $INNER $OUTER -json"
MPI="/opt/conda/bin/mpiexec -launcher fork -iface lo -n 2"
run() {  # label, command...
  local label=$1; shift
  local line
  line=$(timeout -k 10 120 "$@" 2>>gpurun_out/r04_diag/stderr.txt | grep '^{' | tail -1)
  local rc=$?
  echo "$label rc=$rc $line" | tee -a "$OUT"
  [ $rc -eq 0 ] || exit 1
}
for i in 1 2; do run "one-process#$i" ./host/msplit_driver $ARGS; done
for i in 1 2 3; do run "mpi2-default#$i" $MPI ./host/msplit_driver_mpi $ARGS; done
for i in 1 2 3 4; do run "mpi2-host#$i" $MPI ./host/msplit_driver_mpi $ARGS -msplit_transport host; done
for i in 1 2; do run "mpi2-host-nographs#$i" env MSPLIT_GRAPHS=0 $MPI ./host/msplit_driver_mpi $ARGS -msplit_transport host; done
for i in 1 2; do run "mpi2-host-coherent#$i" env HIP_HOST_COHERENT=1 $MPI ./host/msplit_driver_mpi $ARGS -msplit_transport host; done
echo done | tee -a "$OUT"
