#!/bin/bash
# contact / KKT tests, then config 4 and the config-0 stress plant (BVLS latency)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_contact_ext.py tests/test_gpu_kkt.py tests/test_gpu_contact.py tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_elbow.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_sel.log; grep -n "E  " gpurun_out/pytest_sel.log | head -5
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/bench_cfg4.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us')"
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress.log
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_nominal.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_nominal.log
timeout -k 10 300 python scripts/ab_rollout.py > gpurun_out/ab_rollout.log 2>&1 || exit 1
cat gpurun_out/ab_rollout.log
timeout -k 10 300 python scripts/diag_phases.py > gpurun_out/diag_phases.log 2>&1 || exit 1
timeout -k 10 300 python scripts/diag_contact.py > gpurun_out/diag_contact.log 2>&1 || exit 1
echo diag done
