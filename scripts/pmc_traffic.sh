#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters (separate passes for
# FETCH_SIZE and WRITE_SIZE, kernel-trace only, per MI355X_MICROARCH.md's HBM section).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc/$c" -o run -- \
     python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu > "$R/gpurun_out/pmc/$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc/trace" -o run -- \
     python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu > "$R/gpurun_out/pmc/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R" && python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json
