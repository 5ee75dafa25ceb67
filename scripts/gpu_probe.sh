#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/probe_gemm.py 2>&1 | tee gpurun_out/probe_gemm.log || exit $?
STEPS=1 bash scripts/gpu_profile.sh
