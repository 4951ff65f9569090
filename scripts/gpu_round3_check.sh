set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --no-pmc > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --form contact --config 2 --steps 50 --warmup 5 --no-cpu --no-pmc > gpurun_out/bench_contact_cfg2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --weight M --steps 50 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/bench_w1m.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --weight M --config 2 --steps 30 --warmup 3 --no-cpu --no-pmc --no-variant > gpurun_out/bench_w1m_cfg2.log 2>&1 || exit 1
for f in bench bench_contact_cfg2 bench_w1m bench_w1m_cfg2; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e6,2), 'M', d.get('contact_variant',{}).get('value',0)/1e6, d.get('status_histogram'))"; done
