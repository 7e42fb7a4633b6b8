set -o pipefail
O=gpurun_out/${1:-lab2}; mkdir -p $O
timeout -k 10 200 tools/spmv_lab 512 10 0 2 > $O/lab512_contig.json 2> $O/err &&
timeout -k 10 200 tools/spmv_lab 512 10 0 2 > $O/lab512_contig_b.json 2>> $O/err
echo "exit $?" > $O/status
