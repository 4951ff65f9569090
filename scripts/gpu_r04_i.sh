#!/bin/bash
# which change broke the W1 = M config-2 level-0 certificate: 40-column repair Gauss-Jordan (libwbq.so)
# vs the full-width one (expD)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/probe_cfg2_cert.py qppvm_amd/libwbq.so 1 > gpurun_out/probe_cert_w1m.log 2>&1 || { tail -n 5 gpurun_out/probe_cert_w1m.log; exit 1; }
tail -n 1 gpurun_out/probe_cert_w1m.log | cut -c1-3000
timeout -k 10 240 python -u scripts/probe_cfg2_cert.py qppvm_amd/libwbq_expD.so 1 > gpurun_out/probe_cert_w1m_D.log 2>&1 || { tail -n 5 gpurun_out/probe_cert_w1m_D.log; exit 1; }
tail -n 1 gpurun_out/probe_cert_w1m_D.log | cut -c1-1500
