set -o pipefail
O=gpurun_out/lazy2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 900 bash tools/ab_build.sh "base:tools/ab_lib/base.so:0 new::0 new1024::1024" 3 > $O/ab.log 2>&1
echo "exit $?" > $O/status
