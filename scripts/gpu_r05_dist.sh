#!/bin/bash
# the data-parallel path (RCCL all-reduce of the flat gradient segments, SyncBN, overlap, captured
# in the step graph) at world size 1 under torch.distributed.run, beside the plain one-GPU bench;
# plus the world-1 GPU distributed tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dist_plain.json 2> gpurun_out/dist_plain.err || exit 1
CMX_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dist_force.json 2> gpurun_out/dist_force.err || { tail -20 gpurun_out/dist_force.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dist_plain2.json 2>> gpurun_out/dist_plain.err || exit 1
for f in dist_plain dist_force dist_plain2; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['config'].get('hip_graph_streams'))"; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
