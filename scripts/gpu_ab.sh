#!/bin/bash
# A/B of experiment libraries (abv/*.so) against the product build, configs 1 and 2, then
# one SQ PMC pass over the product's dominant kernel. Each GPU step has its own limit.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS1="--steps 200 --warmup 20 --no-cpu --no-pmc --no-variant"
ARGS2="--config 2 --steps 60 --warmup 10 --no-cpu --no-pmc --no-variant"
for lib in qppvm_amd/libwbq.so abv/*.so; do
  nm=$(basename "$lib" .so)
  timeout -k 10 200 python scripts/ab_bench.py "$lib" $ARGS1 ${EXTRA:-} > gpurun_out/ab_${nm}_c1.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/ab_bench.py "$lib" $ARGS2 ${EXTRA:-} > gpurun_out/ab_${nm}_c2.log 2>&1 || exit 1
  if [ -n "${C4:-}" ]; then
    timeout -k 10 200 python scripts/ab_bench.py "$lib" --config 4 --steps 20 --warmup 3 --no-cpu --no-pmc --no-variant > gpurun_out/ab_${nm}_c4.log 2>&1 || exit 1
  fi
  if [ -n "${W1M:-}" ]; then
    timeout -k 10 200 python scripts/ab_bench.py "$lib" $ARGS1 --weight M > gpurun_out/ab_${nm}_c1m.log 2>&1 || exit 1
  fi
  python - "$nm" <<'PY'
import json, sys
nm = sys.argv[1]
import os
for c in ("c1", "c2", "c4", "c1m"):
    if not os.path.exists(f"gpurun_out/ab_{nm}_{c}.log"): continue
    d = json.loads(open(f"gpurun_out/ab_{nm}_{c}.log").read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f"{nm:24s} {c} {d['value']/1e6:8.2f} M/s  step {d['ms_per_step']*1e3:7.1f} us  kernel {r.get('kernel_avg_us', 0):7.1f} us")
PY
done
if [ -n "${PMC:-}" ]; then
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-include-regex "${PMCK:-qppvm_fast}" -d "$GRAFT_REPO_ROOT/gpurun_out/pmc" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-cpu --no-pmc --no-variant ${EXTRA:-} > "$GRAFT_REPO_ROOT/gpurun_out/pmc.log" 2>&1
  echo "pmc rc=$?"
fi
