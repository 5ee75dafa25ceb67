#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PROBE="scripts/probe_h3_planes.py" LOG=probe_planes3 bash scripts/gpu_probe_r05.sh || exit $?
PROBE="scripts/probe_h3_ablate.py 111000 20 42 50 53 47 49" LOG=probe_ablate2 bash scripts/gpu_probe_r05.sh
