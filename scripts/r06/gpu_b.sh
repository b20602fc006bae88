#!/bin/bash
# round-6 check: new / changed GPU tests, the SRA fast-forward parity question, the bench line's
# in-step roofline, then the GPU_MAX_HW_QUEUES=2 crash probe (last: it may abort)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
P="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 240 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_modules.py -k "frm_channel_one_launch or frm_pool_one_launch" > gpurun_out/r06/b_frm.log 2>&1
rc=$?; echo "frm rc=$rc"; tail -3 gpurun_out/r06/b_frm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $P tests/test_gpu_kernels.py::test_sra_fwd_kernel_choice tests/test_metric_eval.py::test_evaluator_graph_cache_of_one \
  tests/test_gpu_gemm.py tests/test_gpu_modules.py -k "ln or sra or graph_cache or frm" > gpurun_out/r06/b_unit.log 2>&1
echo "unit rc=$?"; tail -3 gpurun_out/r06/b_unit.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_optim.py > gpurun_out/r06/b_optim.log 2>&1
echo "optim rc=$?"; tail -2 gpurun_out/r06/b_optim.log
CMX_PARITY_OUT=gpurun_out/r06/parity timeout -k 10 1000 $P -s tests/test_config_parity.py -k "config4 and not fp16" > gpurun_out/r06/b_par4.log 2>&1
echo "par4 rc=$?"; grep -E "worst|PASS|FAIL|Error" gpurun_out/r06/b_par4.log | tail -4
CMX_SRA_SMALL_FWD_N=600 CMX_PARITY_OUT=gpurun_out/r06/parity600 timeout -k 10 1000 $P -s tests/test_config_parity.py -k "config4 and not fp16" > gpurun_out/r06/b_par4_600.log 2>&1
echo "par4_600 rc=$?"; grep -E "worst|PASS|FAIL|Error" gpurun_out/r06/b_par4_600.log | tail -4
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r06/b_bench.json 2> gpurun_out/r06/b_bench.err
echo "bench rc=$?"; cut -c1-200 gpurun_out/r06/b_bench.json
GPU_MAX_HW_QUEUES=2 timeout -k 10 60 python -u -X faulthandler -c "import torch; x = torch.ones(4, device='cuda'); torch.cuda.synchronize(); print('hwq2 trivial ok', x.sum().item())" > gpurun_out/r06/b_hwq2_trivial.log 2>&1
echo "hwq2 trivial rc=$?"; tail -30 gpurun_out/r06/b_hwq2_trivial.log
