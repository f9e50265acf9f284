#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python tools/conv_bwd_check.py > $out/convchk.log 2>&1 || { tail -5 $out/convchk.log; exit 1; }
grep -v amdgpu.ids $out/convchk.log
