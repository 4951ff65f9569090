#!/bin/bash
# warm dual active set after the level-0 repair: QPPVM parity subset, config-4 A/B and steps, stress plant
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_warmstart.py tests/test_gpu_elbow.py tests/test_gpu_kkt.py tests/test_plugin.py tests/test_gpu_contact.py tests/test_gpu_contact_ext.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_h.log; grep -n "E  " gpurun_out/pytest_h.log | head -5
[ $rc -ge 2 ] && exit $rc
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python scripts/ab_rollout.py > gpurun_out/ab_rollout_h.log 2>&1 || exit 1
grep -A1 '/fused\|/steps' gpurun_out/ab_rollout_h.log | grep ms_per | tr -s ' ' | tr '\n' ' '; echo
timeout -k 10 300 python scripts/diag_mpc_steps.py > gpurun_out/diag_mpc_steps_h.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_h.log").read(); d = json.loads(s[s.index("{"):])
for k in ("steps_kernel", "steps_inline"):
    print(k, [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d[k]])
PY
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_h.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_h.log
timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 3 --no-cpu --no-pmc > gpurun_out/bench_cfg2_h.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg2_h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', 'contact', d.get('contact_variant',{}).get('value',0)/1e6)"
