#!/bin/bash
# Round-3: spill-free n = 39 fast kernel (MR columns, M loads after the task forces) -- full GPU
# suite, n = 39 config-1 line with PMC traffic, config-1 headline, dummy drivers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 4 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --n 39 --no-cpu --no-variant > gpurun_out/bench_n39.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_qppvm.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_qppvm_stress.log 2>&1 || exit 1
tail -n 3 gpurun_out/dummy_*.log
for f in bench bench_n39; do python -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us', r['kernel_avg_us'], r.get('traffic'), r.get('frac'))"; done
exit $rc
