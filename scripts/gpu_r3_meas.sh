#!/bin/bash
# Round-3 measurements: convergence parity, framework-path epoch, comm probe, device timelines.
set -o pipefail
out=gpurun_out/r3meas
mkdir -p $out
for v in 1 0 1 0; do
  KUBEML_U22_GATHER=$v timeout -k 10 200 python bench.py --steps 300 --warmup 20 --e2e off --no-epoch > $out/ab_g$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "gather=$v $(python -c "import json;d=json.load(open('$out/ab_g$v.json'));print(d['ms_per_step'])")"
done
timeout -k 10 500 python -u tools/convergence_check.py --steps 1200 --out $out/convergence.json > $out/convergence.log 2>&1 || { tail -20 $out/convergence.log; exit 1; }
tail -1 $out/convergence.log | cut -c1-400
timeout -k 10 500 python -u tools/bench_e2e.py --epochs 4 --validate --trace $out/e2e_trace > $out/e2e.json 2> $out/e2e.err || { tail -20 $out/e2e.err; exit 1; }
cut -c1-700 $out/e2e.json
timeout -k 10 150 python bench.py --steps 5 --warmup 2 --force-comm --comm-plan rccl:overlap:fp32 --no-epoch --e2e off --trace $out/trace_rccl > $out/tl_rccl.json 2> $out/tl_rccl.err || { tail -20 $out/tl_rccl.err; exit 1; }
python tools/trace_table.py $out/trace_rccl > $out/timeline_rccl.md || true
timeout -k 10 600 python -u tools/interference_probe.py --out $out/interference.json --plan-out $out/comm_plan.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
tail -2 $out/probe.log | cut -c1-600
timeout -k 10 150 python bench.py --steps 5 --warmup 2 --force-comm --comm-plan peer:end:fp32:256 --no-epoch --e2e off --trace $out/trace_peer > $out/tl_peer.json 2> $out/tl_peer.err || { tail -20 $out/tl_peer.err; exit 1; }
python tools/trace_table.py $out/trace_peer > $out/timeline_peer.md || true
echo done
