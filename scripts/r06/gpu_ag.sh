#!/bin/bash
# round 6 (ag): the plane GEMMs' epilogue / DMA / main-loop split (scripts/probe_epilogue.py on the probe library)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
MERLIN_HIP_LIB="$R/ppo-2dgrid_amd/lib/libmerlin_hip_probe.so" timeout -k 10 300 python -u scripts/probe_epilogue.py \
    > gpurun_out/r06ag_epilogue.log 2>&1; rc=$?
cat gpurun_out/r06ag_epilogue.log; exit $rc
