#!/bin/bash
# config 4 with a cold BVLS in every repair (expW) vs the warm start; config 1 with the inline-repair variant forced
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/diag_mpc_steps.py qppvm_amd/libwbq_expW.so > gpurun_out/diag_mpc_steps_W.log 2>&1 || exit 1
python - <<'PY'
import json
s = open("gpurun_out/diag_mpc_steps_W.log").read(); d = json.loads(s[s.index("{"):])
for k in ("steps_kernel",):
    print("cold", k, [(round(r["ms"], 2), r["iters_max"], r["hint_repair"]) for r in d[k]])
PY
for v in 0 1; do
WBQ_INLREP=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > gpurun_out/bench_cfg1_inl$v.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg1_inl$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1 inl$v', d['value']/1e6, 'M', d['roofline']['kernel_avg_us'], 'us', d['ms_per_step'])"
done
