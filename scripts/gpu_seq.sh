#!/bin/bash
# ordered kernel launches of one optimizer step (rocprofv3 --kernel-trace of a short bench run)
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
if [ -n "$TESTS" ]; then
  (cd "$R" && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/pytest_sel.log 2>&1); rc=$?
  tail -5 "$R/gpurun_out/pytest_sel.log"; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/seq" -o run -- python "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-tiers > "$R/gpurun_out/seq.log" 2>&1 || exit $?
cd "$R" && python scripts/kernel_sequence.py gpurun_out/seq/run_kernel_trace.csv gpurun_out/seq_step.md && rm -f gpurun_out/seq/run_kernel_trace.csv
grep -o '"value": [0-9.]*' gpurun_out/seq.log | head -1
