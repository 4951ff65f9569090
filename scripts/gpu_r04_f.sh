#!/bin/bash
# rollout/INLREP spill fixes: parity subset, A/B of the rollout paths, config-4 steps, repair phases
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_warmstart.py tests/test_gpu_elbow.py tests/test_gpu_contact_ext.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_f.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_f.log; grep -n "E  " gpurun_out/pytest_f.log | head -5
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python scripts/ab_rollout.py > gpurun_out/ab_rollout_f.log 2>&1 || exit 1
cat gpurun_out/ab_rollout_f.log | grep -v amdgpu.ids
timeout -k 10 300 python scripts/diag_mpc_steps.py > gpurun_out/diag_mpc_steps.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps.log").read(); d = json.loads(s[s.index("{"):])
for k in ("steps_kernel", "steps_inline"):
    print(k, [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d[k]])
PY
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/bench_cfg4_f.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4_f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us')"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-pmc > gpurun_out/bench_cfg1_f.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg1_f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', 'contact', d['contact_variant']['value']/1e6)"
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_f.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_f.log
timeout -k 10 300 python scripts/diag_phases.py > gpurun_out/diag_phases_f.log 2>&1 || exit 1
echo done
