#!/bin/bash
# Config-4 WRITE_SIZE per twenty-step rollout launch for the product and abv/inl.so (repair inlined), one pass
# each (kernel trace + one counter), the launch shape of the timed region only (--no-repair-share).
set -u
cd /tmp; export TMPDIR=/tmp
for lib in $GRAFT_REPO_ROOT/qppvm_amd/libwbq.so $GRAFT_REPO_ROOT/abv/inl.so; do
  nm=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex qppvm_rollout -d "$GRAFT_REPO_ROOT/gpurun_out/c4w_$nm" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/scripts/ab_bench.py" $lib --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant --no-repair-share > "$GRAFT_REPO_ROOT/gpurun_out/c4w_$nm.log" 2>&1
  echo "c4w $nm rc=$?"
done
