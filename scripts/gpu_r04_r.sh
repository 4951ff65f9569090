#!/bin/bash
# where the config-0 stress plant's slow ticks go (stamp build, 400 ticks)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DIAG_STRESS=1 DIAG_TICKS=400 timeout -k 10 300 python scripts/diag_plugin_tick.py > gpurun_out/diag_plugin_tick_stress.log 2>&1 || { tail -n 5 gpurun_out/diag_plugin_tick_stress.log; exit 1; }
grep -v amdgpu.ids gpurun_out/diag_plugin_tick_stress.log | cut -c1-400
