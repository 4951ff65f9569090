#!/bin/bash
# Round-3: warm_extend (contact / W1 = M) -- warm-start tests, the full suite, config-1 contact
# variant and config-2 lines of the three forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_warmstart.py tests/test_gpu_contact.py tests/test_gpu_w1m.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_warm.log 2>&1
rc=$?; tail -n 4 gpurun_out/pytest_warm.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 4 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --form contact --config 2 --steps 100 --warmup 10 --no-cpu --no-pmc > gpurun_out/bench_contact_cfg2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --weight M --config 2 --steps 50 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/bench_w1m_cfg2.log 2>&1 || exit 1
for f in bench bench_contact_cfg2 bench_w1m_cfg2; do python -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']; cv=d.get('contact_variant',{})
print('$f', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us', r['kernel_avg_us'], d.get('mean_active_set_steps'), d.get('max_active_set_steps'), 'contact_variant', cv.get('value'), cv.get('kernel_avg_us'))"; done
