#!/bin/bash
# Full GPU suite (minus the bf16-payload capture case, probed separately), the RCCL capture probe, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_b}
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  --deselect "tests/test_gpu_dist.py::test_dp_world1_graph_step_equals_plain_step[bf16]" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
for c in a2a_eager ag_eager rs_eager ag_graph rs_graph a2a_graph; do
  timeout -k 10 120 python -u scripts/rccl_capture_probe.py $c >> gpurun_out/rccl_probe_$TAG.log 2>&1
  rc=$?; echo "probe $c rc=$rc"; [ $rc -eq 0 ] || exit 0
done
