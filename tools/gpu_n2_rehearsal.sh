set -o pipefail
O=gpurun_out/${1:-n2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --smsm-planes 128 > $O/bench_n2_gloo.json 2> $O/err
echo "exit $?" > $O/status
