#!/bin/bash
# round-6: parity at every config with the stage-3 fast SRA forward, bench, the world-1 DP
# rehearsal (2 exchange groups), then the GPU_MAX_HW_QUEUES=2 crash probe (last: it aborts)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_gemm.py -k "sra_fwd_kernel_choice or gemm_ln" > gpurun_out/r06/c_sra.log 2>&1
rc=$?; echo "sra/ln rc=$rc"; grep "sra fwd" gpurun_out/r06/c_sra.log | head -8; tail -3 gpurun_out/r06/c_sra.log; [ $rc -le 1 ] || exit $rc
CMX_PARITY_OUT=gpurun_out/r06/parity_c timeout -k 10 1500 python -u -m pytest -v -s --timeout 1200 --timeout-method thread tests/test_config_parity.py > gpurun_out/r06/c_par.log 2>&1
echo "parity rc=$?"; grep -E "PASSED|FAILED|worst" gpurun_out/r06/c_par.log | head -20
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r06/c_bench.json 2> gpurun_out/r06/c_bench.err
echo "bench rc=$?"; cut -c1-150 gpurun_out/r06/c_bench.json
for arm in plain force; do
  if [ $arm = force ]; then export CMX_FORCE_DIST=1; fi
  CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29517 bench.py --no-cpu-baseline > gpurun_out/r06/c_dist_$arm.json 2> gpurun_out/r06/c_dist_$arm.err
  echo "dist $arm rc=$?"; grep -o '"value": [0-9.]*' gpurun_out/r06/c_dist_$arm.json
done
unset CMX_FORCE_DIST
GPU_MAX_HW_QUEUES=2 CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 120 python -u -X faulthandler bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06/c_hwq2.json 2> gpurun_out/r06/c_hwq2.err
echo "hwq2 rc=$?"; tail -40 gpurun_out/r06/c_hwq2.err
