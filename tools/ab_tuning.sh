#!/bin/bash
# Same-box A/B of the tuning flags (MSPLIT_TUNING), interleaved.
mkdir -p gpurun_out/abt
for r in 1 2; do for t in 0 1 2 3; do
MSPLIT_TUNING=$t timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/abt/t${t}_$r.json 2>/dev/null || exit 1
done; done
