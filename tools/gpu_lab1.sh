set -o pipefail
mkdir -p gpurun_out/lab1
timeout -k 10 200 tools/spmv_lab 512 10 0 1 > gpurun_out/lab1/lab512.json 2> gpurun_out/lab1/err512 &&
timeout -k 10 200 tools/spmv_lab 256 20 0 1 > gpurun_out/lab1/lab256.json 2> gpurun_out/lab1/err256
echo "exit $?" > gpurun_out/lab1/status
