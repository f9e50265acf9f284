#!/bin/bash
set -o pipefail
out=gpurun_out/gemm_pmc3
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
args="--layout 2 --M 3072 --N 768 --K 16384 --tile 128,128,2 --splits 2"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/p1 -o run --output-format csv -- python tools/gemm_one.py $args > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/p2 -o run --output-format csv -- python tools/gemm_one.py $args > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $out/p3 -o run --output-format csv -- python tools/gemm_one.py $args > $out/p3.log 2>&1 || { tail -5 $out/p3.log; exit 1; }
args="--layout 0 --M 16384 --N 3072 --K 768 --tile 128,128,2"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/f1 -o run --output-format csv -- python tools/gemm_one.py $args > $out/f1.log 2>&1 || { tail -5 $out/f1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/f2 -o run --output-format csv -- python tools/gemm_one.py $args > $out/f2.log 2>&1 || { tail -5 $out/f2.log; exit 1; }
