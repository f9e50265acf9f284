#!/bin/bash
set -o pipefail
out=gpurun_out/gemm_pmc2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "256,256,4" "128,128,2"; do
  tag=$(echo $cfg | tr ',' 'x')
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $out/a_$tag -o run --output-format csv -- python tools/gemm_one.py --tile $cfg > $out/a_$tag.log 2>&1 || { tail -5 $out/a_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/b_$tag -o run --output-format csv -- python tools/gemm_one.py --tile $cfg > $out/b_$tag.log 2>&1 || { tail -5 $out/b_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCP_TCC_READ_REQ_sum -d $out/c_$tag -o run --output-format csv -- python tools/gemm_one.py --tile $cfg > $out/c_$tag.log 2>&1 || { tail -5 $out/c_$tag.log; exit 1; }
done
