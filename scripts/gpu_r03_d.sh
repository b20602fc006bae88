#!/bin/bash
# short-sequence SRA kernels: correctness, per-stage timing, step A/B; fp16 fixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py tests/test_gpu_gemm.py -m gpu \
  -v --timeout 120 --timeout-method thread -k "sra or dist or payload or implicit" > gpurun_out/pytest_a_$TAG.log 2>&1
rc=$?; echo "pytest A rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_a_$TAG.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for st in 1 2 3 4; do
  timeout -k 10 120 python -u scripts/bench_sra.py stage $st >> gpurun_out/sra_small_$TAG.log 2>&1 || exit $?
  CMX_SRA_SMALL_N=0 timeout -k 10 120 python -u scripts/bench_sra.py stage $st >> gpurun_out/sra_fast_$TAG.log 2>&1 || exit $?
done
echo "small:"; grep "N=" gpurun_out/sra_small_$TAG.log; echo "fast:"; grep "N=" gpurun_out/sra_fast_$TAG.log
for arm in 0 2048 0 2048; do
  CMX_SRA_SMALL_N=$arm timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_small${arm}_$TAG.json 2>&1 || exit $?
  echo "small_n=$arm $(grep -o '"value": [0-9.]*' gpurun_out/ab_small${arm}_$TAG.json)"
done
timeout -k 10 900 python -u -m pytest tests/test_config_parity.py tests/test_gpu_modules.py -m gpu -v --timeout 120 \
  --timeout-method thread -k "fp16 or float16 or config2" > gpurun_out/pytest_b_$TAG.log 2>&1
rc=$?; echo "pytest B rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_b_$TAG.log | tail -12
