#!/bin/bash
# round 6 (ah): the input gradient's tile stores non-temporal (k_h3_pq) -- the h3 / update tests on the new library,
# then the bench at the driver's step counts, alternating with the library before the change (lib/libmerlin_hip_base.so)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_h3.py \
    tests/test_gpu_dz_planes.py tests/test_gpu_update_grad.py tests/test_gpu_windows.py > gpurun_out/r06ah_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/r06ah_tests.log)"; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
BASE="$R/ppo-2dgrid_amd/lib/libmerlin_hip_base.so"
for L in new base new base; do
  if [ $L = base ]; then export MERLIN_HIP_LIB="$BASE"; else unset MERLIN_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tiers > gpurun_out/r06ah_bench_$L.log 2>&1; rc=$?
  echo "bench $L: $(tail -1 gpurun_out/r06ah_bench_$L.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], {k: d["kernels"][k]["avg_us"] for k in ("gemm_fc1_fwd","gemm_fc1_dgrad","gemm_wgrad","k_seg_sum_R")})')"
  crash $rc && exit $rc
done
exit 0
