#!/bin/bash
# hybrid BVLS warm start: GPU suite, stress plant, config 4
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_q.log; grep -n "^FAILED" gpurun_out/pytest_q.log | head -8
[ $rc -ge 2 ] && exit 1
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_q.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_q.log
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_cfg4_q.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value']/1e6, 'M', d['roofline'], 'contact', d.get('contact_variant',{}).get('value',0)/1e6)"
timeout -k 10 300 python scripts/diag_mpc_steps.py > gpurun_out/diag_mpc_steps_q.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_q.log").read(); d = json.loads(s[s.index("{"):])
print("hybrid", [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d["steps_kernel"]][:9])
PY
