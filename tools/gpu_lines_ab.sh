#!/bin/bash
# Same-box A/B of the DV march tiles inside the GMRES and SMSM benches: MSPLIT_MARCH_LINES=1 (256 plane rows per
# workgroup) against 4 (four y lines, the default for nx % 256 == 0), interleaved.
set -o pipefail
O=gpurun_out/${1:-lines_ab}; mkdir -p $O
for r in 1 2; do
  for l in 1 4; do
    MSPLIT_MARCH_LINES=$l timeout -k 10 240 python bench.py --no-cpu-baseline --variant gmres --no-csr-compare --no-smsm-n1 --no-spmv512 > $O/g_l${l}_r$r.json 2>> $O/err || exit 1
    MSPLIT_MARCH_LINES=$l timeout -k 10 240 python bench.py --no-cpu-baseline --variant smsm --steps 2 > $O/s_l${l}_r$r.json 2>> $O/err || exit 1
  done
done
echo "exit 0" > $O/status
