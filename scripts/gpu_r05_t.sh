#!/bin/bash
# caller-owned AdamW / FRM-pool tickets: optimizer, module and train tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_modules.py tests/test_gpu_train.py tests/test_gpu_improved.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_t.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_t.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*'
REPS=2 bash scripts/ab_env.sh base CMX_GEMM_UP_TILE=64 || exit 1
REPS=1 bash scripts/ab_prof.sh "gemm_bf16_kernel<128, 128, false, false|gemm_bf16_kernel<64, 64, false, false, 2, 1, bf16, 0>" base CMX_GEMM_UP_TILE=64
