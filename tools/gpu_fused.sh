set -o pipefail
O=gpurun_out/fused; mkdir -p $O
export TMPDIR=/tmp
MSPLIT_TUNING=2048 timeout -k 10 400 python -u -m pytest tests/test_gpu_gmres.py tests/test_gpu_drivers.py -x -q --timeout 200 --timeout-method thread > $O/tests2048.log 2>&1 &&
MSPLIT_TUNING=6144 timeout -k 10 400 python -u -m pytest tests/test_gpu_gmres.py -x -q --timeout 200 --timeout-method thread > $O/tests6144.log 2>&1 &&
timeout -k 10 900 bash tools/ab_build.sh "unf::0 fused4::2048 fused2::6144" 3 > $O/ab.log 2>&1
echo "exit $?" > $O/status
