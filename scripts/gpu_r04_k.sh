#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/diag_mpc_repair.py > gpurun_out/diag_mpc_repair.log 2>&1 || { tail -n 5 gpurun_out/diag_mpc_repair.log; exit 1; }
cat gpurun_out/diag_mpc_repair.log | grep -v amdgpu.ids
