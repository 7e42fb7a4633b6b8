#!/bin/bash
# Does torch in the process (its bundled HIP runtime) slow the CSR MatMult?  Alternating processes, same box.
set -o pipefail
O=gpurun_out/${1:-spmv_rt}; mkdir -p $O
export TMPDIR=/tmp
F=${FLAGS:-0,4194304}
for i in 1 2 3; do
timeout -k 10 200 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 3 --no-torch --flags $F > $O/notorch_$i.json 2>> $O/err &&
timeout -k 10 200 python tools/spmv_policy_ab.py --n 512 --reps 10 --rounds 3 --flags $F > $O/torch_$i.json 2>> $O/err || break
done
echo "exit $?" > $O/status
