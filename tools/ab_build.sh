#!/bin/bash
# Same-box A/B of builds of the library (and MSPLIT_TUNING flags) on the bench workload, interleaved.
#   tools/ab_build.sh "base:tools/ab_lib/base.so:0 new::0 new1024::1024" [rounds] [extra bench args]
# spec = name:library:tuning; an empty library means the in-tree build.
set -e
mkdir -p gpurun_out/abb
L=${1:-"base:tools/ab_lib/base.so:0 new::0"}
R=${2:-2}
shift 2 || true
for r in $(seq 1 $R); do
  for spec in $L; do
    IFS=: read -r name lib tun <<< "$spec"
    MSPLIT_LIB=$lib MSPLIT_TUNING=${tun:-0} timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/abb/${name}_r${r}.json 2> gpurun_out/abb/${name}_r${r}.err
    python -c "import json,sys; d=json.loads(open('gpurun_out/abb/${name}_r${r}.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('$name r=$r', '%.4e'%d['value'], '%.1f ms'%d['ms_per_step'], ' '.join('%s=%.0f/%.3f'%(c,v['GBps'],v['share']) for c,v in k.items() if v.get('GBps')))"
  done
done
