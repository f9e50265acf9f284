set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
KUBEML_LOG_LEVEL=INFO timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_e2e_gpu.py -k "share_one_gpu or elastic_one_two" > gpurun_out/r4/e2e_packed.log 2>&1
echo "e2e rc=$?"
tail -5 gpurun_out/r4/e2e_packed.log
