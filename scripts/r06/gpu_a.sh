#!/bin/bash
# round 6 (a): the DMA kernels after the m0 save/restore, the reference first-step gradient, the weight gradient
# serial vs beside conv3's backward sums, and the device memory of cfg 3's per-rank and single-process shapes
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 200 python -u -m pytest -v -s --timeout 150 --timeout-method thread tests/test_gpu_update_grad.py \
    > gpurun_out/r06a_grad.log 2>&1; rc=$?
tail -30 gpurun_out/r06a_grad.log; crash $rc && exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dz_planes.py \
    tests/test_gpu_h3.py > gpurun_out/r06a_tests.log 2>&1 || { tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
timeout -k 10 300 python -u scripts/ab_update.py 3 5 fast_timers4,fast_wgradmain_timers4,fast_cu3_timers4,fast_cu2_timers4 > gpurun_out/r06a_ab.log 2>&1 \
    || { tail -30 gpurun_out/r06a_ab.log; exit 1; }
tail -40 gpurun_out/r06a_ab.log
timeout -k 10 200 python -u scripts/probe_cfg3.py 4096 256 8 1 > gpurun_out/r06a_cfg3_rank.log 2>&1 \
    || { tail -30 gpurun_out/r06a_cfg3_rank.log; exit 1; }
cat gpurun_out/r06a_cfg3_rank.log
timeout -k 10 300 python -u scripts/probe_cfg3.py 32768 256 8 1 > gpurun_out/r06a_cfg3_single.log 2>&1 \
    || { tail -30 gpurun_out/r06a_cfg3_single.log; exit 1; }
cat gpurun_out/r06a_cfg3_single.log
