#!/bin/bash
# config 2 (QPPVM) with the inline-repair policy (default), forced off, forced on
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in auto 0 1; do
  if [ $v = auto ]; then e=""; else e="WBQ_INLREP=$v"; fi
  env $e timeout -k 10 300 python bench.py --config 2 --steps 60 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/cfg2_inl_$v.log 2>&1 || exit 1
  tail -n 1 gpurun_out/cfg2_inl_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 inl=$v', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', d['ms_per_step'])"
done
