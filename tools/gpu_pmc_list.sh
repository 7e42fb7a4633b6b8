set -o pipefail
O=gpurun_out/${1:-pmc_list}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > $O/avail.txt 2>&1
echo "exit $?" > $O/status
