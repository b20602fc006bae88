#!/bin/bash
# RCCL collectives under HIP-graph capture at world size 1, one process per case; the
# all-to-all case (known to crash at capture end / hang at exit) runs LAST under a short limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/rccl_capture_probe.txt
: > $OUT
for c in ar_graph bc_graph rs32_graph rs_graph ag_graph a2a_eager; do
  timeout -k 10 90 python -u scripts/rccl_capture_probe.py $c >> $OUT 2>&1; rc=$?
  echo "$c rc=$rc" >> $OUT; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 60 python -u scripts/rccl_capture_probe.py a2a_graph >> $OUT 2>&1; echo "a2a_graph rc=$?" >> $OUT
grep -v "^\[W\|amdgpu.ids" $OUT | tail -30
