#!/bin/bash
# rocprofv3 kernel stats (config 1, config 4) as CSV; config-4 steps with the BVLS warm start keeping the last sides (expK)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c1.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c4.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
for d in prof_c1 prof_c4; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; cut -c1-160 "$f" | head -8; done
timeout -k 10 300 python scripts/diag_mpc_steps.py qppvm_amd/libwbq_expK.so > gpurun_out/diag_mpc_steps_K.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_K.log").read(); d = json.loads(s[s.index("{"):])
print("keep-sides", [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d["steps_kernel"]][:9])
PY
