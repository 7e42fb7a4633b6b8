#!/bin/bash
# Same-box A/B of the z-march DV SpMV (default) against the row-parallel ELL kernel (MSPLIT_TUNING 268435456):
# the GMRES bench (256^3), SMSM-global (512 x 512 x 256 block) and AMAM (1024 x 1024 x 128 block), interleaved.
set -o pipefail
O=gpurun_out/${1:-march_ab}; mkdir -p $O
bash tools/ab_bench.sh "0 268435456" 2 --variant gmres --no-csr-compare --no-smsm-n1 --no-spmv512 > $O/gmres.txt 2>&1 &&
bash tools/ab_bench.sh "0 268435456" 2 --variant smsm --steps 2 > $O/smsm.txt 2>&1 &&
bash tools/ab_bench.sh "0 268435456" 1 --variant amam --steps 2 > $O/amam.txt 2>&1
echo "exit $?" > $O/status
