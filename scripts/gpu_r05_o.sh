#!/bin/bash
# round 5 (o): per-step timelines (n), then one-setting-per-process A/B (m)
R="$GRAFT_REPO_ROOT"; cd "$R"
AB="fast fast_noa3p" bash scripts/gpu_r05_n.sh || exit $?
AB="${AB2:-fast fast_wgrad_early fast_h3s16 fast_noa3p fast_noa3p_wgrad_early fast_nodzp}" bash scripts/gpu_r05_m.sh
