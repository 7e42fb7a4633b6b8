#!/bin/bash
# Same-box A/B of MSPLIT_TUNING settings on the bench workload, interleaved.
#   tools/ab_bench.sh "0 16 80" [rounds] [extra bench args]
set -e
mkdir -p gpurun_out/ab
T=${1:-"0 16"}
R=${2:-2}
shift 2 || true
for r in $(seq 1 $R); do
  for t in $T; do
    MSPLIT_TUNING=$t timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab/t${t}_r${r}.json 2> gpurun_out/ab/t${t}_r${r}.err
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab/t${t}_r${r}.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('t=$t r=$r', '%.4e'%d['value'], '%.1f ms'%d['ms_per_step'], ' '.join('%s=%.0f'%(c,v['GBps']) for c,v in k.items() if v.get('GBps')))"
  done
done
