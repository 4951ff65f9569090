#!/bin/bash
# DPP reductions: the whole GPU suite, then config 1 (+ contact), config 2, config 4, stress plant
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_m.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_m.log; grep -n "E  " gpurun_out/pytest_m.log | head -5
[ $rc -ge 2 ] && exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc > gpurun_out/bench_cfg1_m.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg1_m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', d['ms_per_step'], 'contact', d['contact_variant']['value']/1e6, d['contact_variant']['kernel_avg_us'])"
timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 3 --no-cpu --no-pmc > gpurun_out/bench_cfg2_m.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg2_m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', 'contact', d.get('contact_variant',{}).get('value',0)/1e6)"
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/bench_cfg4_m.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4_m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', 'contact', d.get('contact_variant',{}).get('value',0)/1e6)"
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_m.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_m.log
timeout -k 10 300 python scripts/diag_mpc_steps.py > gpurun_out/diag_mpc_steps_m.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_m.log").read(); d = json.loads(s[s.index("{"):])
print("steps_kernel", [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d["steps_kernel"]][:9])
PY
timeout -k 10 300 python scripts/diag_mpc_repair.py > gpurun_out/diag_mpc_repair_m.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_repair_m.log").read(); d = json.loads(s[s.index("{"):])
print({k: v for k, v in d.items() if k != "worst"})
PY
