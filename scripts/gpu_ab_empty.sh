set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in prod empty prod empty; do
  lib=qppvm_amd/libwbq.so; [ $v = empty ] && lib=qppvm_amd/ab_empty_repair.so
  timeout -k 10 200 python scripts/ab_bench.py $lib --steps 300 --warmup 30 --no-cpu --no-pmc --no-variant > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'])"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_empty" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/ab_bench.py" "$GRAFT_REPO_ROOT/qppvm_amd/ab_empty_repair.so" --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > "$GRAFT_REPO_ROOT/gpurun_out/prof_empty.log" 2>&1 || exit 1
cut -d, -f1-4,6,7 "$GRAFT_REPO_ROOT/gpurun_out/prof_empty/run_kernel_stats.csv" | head -4
