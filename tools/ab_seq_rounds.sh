#!/bin/bash
# bench.py seq_mode at several MSPLIT_SEQ_ROUNDS (vector rounds per failing sub-segment; 0 = the f64 adds only).
set -o pipefail
O=gpurun_out/${1:-r04_rounds}; mkdir -p $O
B="--steps 1 --warmup 0 --no-cpu-baseline --no-csr-compare --no-smsm-n1 --no-spmv512 --no-non-stencil --no-assembled"
for r in 0 1 2 4; do
  MSPLIT_SEQ_ROUNDS=$r timeout -k 10 200 python bench.py $B > $O/r$r.json 2> $O/r$r.err || exit 1
done
MSPLIT_SEQ_ROUNDS=1 MSPLIT_SEQ_STATS=1 timeout -k 10 200 python bench.py $B > $O/stats1.json 2> $O/stats1.err || exit 1
MSPLIT_SEQ_ROUNDS=0 MSPLIT_SEQ_STATS=1 timeout -k 10 200 python bench.py $B > $O/stats0.json 2> $O/stats0.err
