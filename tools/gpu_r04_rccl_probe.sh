#!/bin/bash
# Can the RCCL transport run two ranks on the box's one GPU?  RCCL refuses two ranks of one host on one device
# ("Duplicate GPU detected"); with a different NCCL_HOSTID per rank it takes them for two hosts and connects them
# over its socket transport on the loopback interface -- enough to run msplit_comm.hip's RCCL branch
# (grouped ncclSend/ncclRecv planes, ncclAllGather of the sums and LSQR partials) multi-rank and compare the
# result with the oracle.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r04_rccl}
mkdir -p $OUT
make -s -C host || exit 1
INNER="-inner1_ksp_max_it 20 -inner1_ksp_rtol 1e-20 -inner2_ksp_max_it 20 -inner2_ksp_rtol 1e-20"
OUTER=""
for b in 1 2; do
  OUTER="$OUTER -outer${b}_ksp_type lsqr -outer${b}_ksp_convergence_test default -outer${b}_ksp_lsqr_exact_mat_norm"
  OUTER="$OUTER -outer${b}_ksp_max_it 70 -outer${b}_ksp_rtol 1e-15 -outer${b}_ksp_atol 1e-100"
done
ARGS="synchronous-multisplitting-synchronous-minimization-global -dim 3 -m 8 -n 8 -p 8 -s 4 -rtol 1e-6 $INNER $OUTER -json -msplit_require_rccl"
ENV="-env NCCL_SOCKET_IFNAME lo -env NCCL_IB_DISABLE 1 -env NCCL_DEBUG WARN"
timeout -k 10 120 /opt/conda/bin/mpiexec -launcher fork -iface lo \
  -n 1 $ENV -env NCCL_HOSTID msplit-rank0 ./host/msplit_driver_mpi $ARGS : \
  -n 1 $ENV -env NCCL_HOSTID msplit-rank1 ./host/msplit_driver_mpi $ARGS > $OUT/smsm_rccl.json 2> $OUT/smsm_rccl.err
echo "rc $?" | tee $OUT/status
tail -c 1500 $OUT/smsm_rccl.json
