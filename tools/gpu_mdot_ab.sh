#!/bin/bash
# Same-box A/B of the MDot variants (MSPLIT_TUNING 262144: two groups of four per loop iteration) on SMSM-global
# (vectors of 537 MB, k <= 20) and the GMRES bench, interleaved.
set -o pipefail
O=gpurun_out/${1:-mdot_ab}; mkdir -p $O
bash tools/ab_bench.sh "0 262144" 2 --variant smsm --steps 2 > $O/smsm.txt 2>&1 &&
bash tools/ab_bench.sh "0 262144" 2 --variant gmres --no-csr-compare --no-smsm-n1 --no-spmv512 > $O/gmres.txt 2>&1
echo "exit $?" > $O/status
