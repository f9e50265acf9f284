#!/bin/bash
# fused K-AVG peer round: tests, packed timing probe, then the default bench (warm-up check)
set -o pipefail
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_gpu.py \
  tests/test_e2e_gpu.py -k "kavg or peer_allreduce" > gpurun_out/r5/kavg_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/kavg_peer_probe.py --world 2 > gpurun_out/r5/kavg_probe2.json 2> gpurun_out/r5/kavg_probe.err &&
timeout -k 10 200 python -u tools/kavg_peer_probe.py --world 4 > gpurun_out/r5/kavg_probe4.json 2>> gpurun_out/r5/kavg_probe.err &&
timeout -k 10 400 python -u bench.py > gpurun_out/r5/bench_default2.json 2> gpurun_out/r5/bench_default2.err
rc=$?
tail -3 gpurun_out/r5/kavg_tests.log; cat gpurun_out/r5/kavg_probe2.json gpurun_out/r5/kavg_probe4.json 2>/dev/null; cat gpurun_out/r5/bench_default2.json 2>/dev/null
exit $rc
