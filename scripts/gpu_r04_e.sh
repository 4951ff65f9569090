#!/bin/bash
# friction sweep with the windowed certificate, config-4 per-step diagnostics, config-4 kernel stats
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_contact_ext.py -k friction -m gpu -x -q -s -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_fric.log 2>&1; rc=$?
tail -n 4 gpurun_out/pytest_fric.log; grep -n "E  " gpurun_out/pytest_fric.log | head -5
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python scripts/diag_mpc_steps.py > gpurun_out/diag_mpc_steps.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps.log").read(); d = json.loads(s[s.index("{"):])
for k in ("steps_kernel", "steps_inline"):
    print(k, [(r["ms"].__round__(2), r["iters_max"], r["hint_repair"]) for r in d[k]])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4e" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4e.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"; find gpurun_out/prof_cfg4e -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
