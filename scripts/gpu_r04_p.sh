#!/bin/bash
# BVLS warm start: last sides kept (qppvm_amd/expK/libwbq.so) vs sides from the gradient at the warm corner
# (the product): the config-0 stress plant and config 4 on one box
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/stress_prod.log 2>&1 || exit 1
tail -n 1 gpurun_out/stress_prod.log
LD_LIBRARY_PATH="$GRAFT_REPO_ROOT/qppvm_amd/expK:${LD_LIBRARY_PATH:-}" timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/stress_keep.log 2>&1 || exit 1
tail -n 1 gpurun_out/stress_keep.log
timeout -k 10 300 python scripts/ab_bench.py qppvm_amd/expK/libwbq.so --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/cfg4_keep.log 2>&1 || exit 1
tail -n 1 gpurun_out/cfg4_keep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 keep', d['value']/1e6, 'M')"
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/cfg4_prod.log 2>&1 || exit 1
tail -n 1 gpurun_out/cfg4_prod.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 prod', d['value']/1e6, 'M')"
