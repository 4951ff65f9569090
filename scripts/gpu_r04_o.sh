#!/bin/bash
# LDS column step for the 12-row BVLS: the GPU suite, the stress plant, n = 39, config 4; rocprofv3 CSV stats;
# config-4 steps with the warm start keeping the last sides (expK, the previous build)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_o.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_o.log; grep -n "^FAILED" gpurun_out/pytest_o.log | head -8
[ $rc -ge 2 ] && exit 1
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_stress_o.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_stress_o.log
timeout -k 10 300 qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_nominal_o.log 2>&1 || exit 1
tail -n 1 gpurun_out/dummy_nominal_o.log
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/bench_cfg4_o.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4_o.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', 'contact', d.get('contact_variant',{}).get('value',0)/1e6)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c1.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c4.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
for d in prof_c1 prof_c4; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; cut -c1-160 "$f" | head -6; done
timeout -k 10 300 python scripts/diag_mpc_steps.py qppvm_amd/libwbq_expK.so > gpurun_out/diag_mpc_steps_K.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_K.log").read(); d = json.loads(s[s.index("{"):])
print("keep-sides", [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d["steps_kernel"]][:9])
PY
