#!/bin/bash
# Round-3 tail GPU call on the W-free build: (1) A/B of the fused MatMult+MDot's depth (MSPLIT_BOXMDOT_ZT 1 against
# the default 2) on the GMRES step and the SMSM block, two rounds; (2) the configs[3] / configs[4] per-GPU AMAM-global
# blocks (tools/gpu_amam_blocks.sh, both minimizations).
set -o pipefail
OUT=gpurun_out/${1:-r03_tail}
mkdir -p $OUT/zt
export TMPDIR=/tmp
X="--no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-seq-mode --no-assembled --steps 8"
for r in 1 2; do
  timeout -k 10 200 env MSPLIT_BOXMDOT_ZT=2 python bench.py $X > $OUT/zt/g_z2_$r.json 2> $OUT/zt/g_z2_$r.err &&
  timeout -k 10 200 env MSPLIT_BOXMDOT_ZT=1 python bench.py $X > $OUT/zt/g_z1_$r.json 2> $OUT/zt/g_z1_$r.err &&
  timeout -k 10 300 env MSPLIT_BOXMDOT_ZT=2 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/zt/s_z2_$r.json 2> $OUT/zt/s_z2_$r.err &&
  timeout -k 10 300 env MSPLIT_BOXMDOT_ZT=1 python bench.py --variant smsm --steps 2 --warmup 1 > $OUT/zt/s_z1_$r.json 2> $OUT/zt/s_z1_$r.err || exit 1
done
bash tools/gpu_amam_blocks.sh && cp -r gpurun_out/amam_blocks $OUT/ &&
echo "exit 0" > $OUT/status
exit 0
