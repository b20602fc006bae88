#!/bin/bash
# RCCL collectives under HIP-graph capture at world size 1, one process per case; the
# all-to-all graph case (round 4: printed ok, then hung at teardown) runs LAST, first with the
# captured graph deleted + the device drained before destroy_process_group (the teardown order
# bench.py / train.py use), then as round 4 ran it, each under a short limit with a faulthandler
# watchdog that dumps the blocking Python frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/rccl_capture_probe.txt
: > $OUT
for c in ar_graph bc_graph rs32_graph rs_graph ag_graph a2a_eager; do
  timeout -k 10 90 python -u scripts/rccl_capture_probe.py $c >> $OUT 2>&1; rc=$?
  echo "$c rc=$rc" >> $OUT; [ $rc -eq 0 ] || exit $rc
done
echo "=== a2a_graph, graph deleted before destroy_process_group" >> $OUT
CMX_PROBE_DEL_GRAPH=1 CMX_PROBE_WATCHDOG_S=15 timeout -k 10 60 python -u scripts/rccl_capture_probe.py a2a_graph >> $OUT 2>&1
rc=$?; echo "a2a_graph (del graph) rc=$rc" >> $OUT
if [ $rc -eq 0 ]; then
  echo "=== a2a_graph, graph alive at destroy_process_group (round-4 order)" >> $OUT
  CMX_PROBE_WATCHDOG_S=15 timeout -k 10 60 python -u scripts/rccl_capture_probe.py a2a_graph >> $OUT 2>&1
  echo "a2a_graph (graph alive) rc=$?" >> $OUT
fi
grep -v "^\[W\|amdgpu.ids" $OUT | tail -60
