#!/bin/bash
# 2D box stencils: the march (default) against the row-parallel ELL kernel, back-to-back MatMult
# (tools/microbench.py has no 2D operator; this uses a small inline timing loop).
set -o pipefail
O=gpurun_out/${1:-march2d}; mkdir -p $O
timeout -k 10 200 python tools/march2d_bench.py > $O/march2d.json 2> $O/err
echo "exit $?" > $O/status
