#!/bin/bash
# Round-6 config-2 step composition: the bench line (events) and a rocprofv3 kernel trace of the same command.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; ROOT=$(pwd)
timeout -k 10 200 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/c2_line.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/c2_line.log').read().strip().splitlines()[-1]); print('c2', round(d['value']/1e6,2), 'M/s step', round(d['ms_per_step']*1e3,1), 'kernel', round(d['roofline']['kernel_avg_us'],1))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c2" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config 2 --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > "$ROOT/gpurun_out/prof_c2.log" 2>&1
echo "prof rc=$?"
f=$(find "$ROOT/gpurun_out/prof_c2" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-160 "$f"
