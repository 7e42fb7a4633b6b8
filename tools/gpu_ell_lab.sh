set -o pipefail
O=gpurun_out/${1:-ell_lab}; mkdir -p $O
timeout -k 10 200 tools/ell_lab 256 20 > $O/ell256.json 2> $O/err &&
timeout -k 10 200 tools/ell_lab 512 10 > $O/ell512.json 2>> $O/err
echo "exit $?" > $O/status
