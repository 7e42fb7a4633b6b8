#!/bin/bash
# MDot -> MAXPY Infinity Cache reuse lab (tools/mall_lab.hip) at 256^3 and 512 x 512 x 256-sized vectors.
set -o pipefail
O=gpurun_out/${1:-mall_lab}; mkdir -p $O
timeout -k 10 200 tools/mall_lab 256 10 > $O/n256.json 2> $O/err
echo "exit $?" > $O/status
