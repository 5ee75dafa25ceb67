#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
MIOPEN_FIND_MODE=FAST PROBE_BATCHES=16384,32768,65536,131072 timeout -k 10 500 python scripts/probe_perf.py 2>&1 | tee gpurun_out/probe_fast.log
