#!/bin/bash
# repair kernel's dual active set behind a call: the GPU suite, the stress plant, the tick diagnostic
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_s.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_s.log; grep -n "^FAILED\|Error" gpurun_out/pytest_s.log | head -5
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_s.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_s.log
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_nominal_s.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_nominal_s.log
DIAG_STRESS=1 DIAG_TICKS=400 timeout -k 10 300 python scripts/diag_plugin_tick.py > gpurun_out/diag_plugin_tick_stress_s.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/diag_plugin_tick_stress_s.log | head -4 | cut -c1-400
timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 3 --no-cpu --no-pmc > gpurun_out/bench_cfg2_s.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg2_s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2', d['value']/1e6, 'M')"
