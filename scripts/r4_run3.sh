set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_e2e_gpu.py -k "share_one_gpu" > gpurun_out/r4/e2e_packed.log 2>&1
echo "e2e rc=$?"
timeout -k 10 900 python -u tools/convergence_multirank.py --out gpurun_out/r4/convergence_multirank.json > gpurun_out/r4/conv.log 2>&1 || { tail -40 gpurun_out/r4/conv.log; exit 1; }
tail -3 gpurun_out/r4/conv.log
