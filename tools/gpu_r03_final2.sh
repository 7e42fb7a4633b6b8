#!/bin/bash
# Round-3 closing GPU call: the N > 1 bench path (tools/gpu_r03_scale_path.sh: bench tests, SMSM block under rocprof,
# N = 2 through torch.distributed.run over gloo + the host transport) on the W-free build, then the SMSM-block A/B of
# the W-free MAXPY's depth (1 plane, the default, against 2), two rounds.
set -o pipefail
OUT=gpurun_out/${1:-r03_final2}
bash tools/gpu_r03_scale_path.sh ${1:-r03_final2}/scale && grep -q "exit 0" $OUT/scale/status &&
mkdir -p $OUT/ab &&
for r in 1 2; do
  timeout -k 10 300 env MSPLIT_MAXPY_ZT=1 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/ab/s_z1_$r.json 2> $OUT/ab/s_z1_$r.err &&
  timeout -k 10 300 env MSPLIT_MAXPY_ZT=2 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/ab/s_z2_$r.json 2> $OUT/ab/s_z2_$r.err || exit 1
done
echo "exit $?" > $OUT/status
exit 0
