#!/bin/bash
# Round-6 probe: kernel time vs batch (one box, both libraries) and two SQ PMC passes over the product's fast
# kernel at B = 4096. Each GPU step has its own limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in qppvm_amd/libwbq.so abv/*.so; do
  for B in ${BATCHES:-1024 2048 3072 4096 8192}; do
    timeout -k 10 120 python scripts/ab_bench.py "$lib" --batch $B --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/sw_$(basename $lib .so)_b$B.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['kernel_avg_us'],2), 'us', round(d['value']/1e6,1), 'M/s')" gpurun_out/sw_$(basename $lib .so)_b$B.log
  done
done
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM"
k=0
for P in "$P1" "$P2"; do
  k=$((k+1))
  for lib in $GRAFT_REPO_ROOT/qppvm_amd/libwbq.so $GRAFT_REPO_ROOT/abv/gj.so; do
    nm=$(basename $lib .so)
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex qppvm_fast -d "$GRAFT_REPO_ROOT/gpurun_out/pmc${k}_$nm" -o run --output-format csv -- \
       python3 "$GRAFT_REPO_ROOT/scripts/ab_bench.py" $lib --steps 20 --warmup 2 --no-cpu --no-pmc --no-variant > "$GRAFT_REPO_ROOT/gpurun_out/pmc${k}_$nm.log" 2>&1
    echo "pmc$k $nm rc=$?"
  done
done
