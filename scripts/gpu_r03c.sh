#!/bin/bash
# Round-3: W1 = I warm start -- its test, the full suite, config 1 / config 2 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_warmstart.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_warm.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/pytest_warm.log | tail -12; [ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 6 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-variant > gpurun_out/bench_cfg2.log 2>&1 || exit 1
for f in bench bench_cfg2; do python -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e6,2), 'M', d['ms_per_step'], r['kernel_avg_us'], r.get('traffic'), d.get('mean_active_set_steps'), d.get('max_active_set_steps'))"; done
