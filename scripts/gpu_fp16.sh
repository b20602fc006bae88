#!/bin/bash
# fp16 (config 5) checks: every fp16 kernel / module / model case, then the config-5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_fp16}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_dist_$TAG.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_dist_$TAG.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py tests/test_gpu_dwconv.py \
  tests/test_gpu_grouped.py tests/test_gpu_modules.py tests/test_config_parity.py -m gpu -v --timeout 120 \
  --timeout-method thread -k "float16 or fp16" > gpurun_out/pytest_fp16_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_fp16_$TAG.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --backbone mit_b5 --height 1024 --width 1024 --batch 1 --classes 19 \
  --dtype float16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_config5_fp16_$TAG.json 2> gpurun_out/bench_config5_fp16_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_config5_fp16_$TAG.json; [ $rc -eq 0 ] || exit $rc
# per-dispatch kernel trace of the B2 bf16 step (scripts/step_trace.py / step_census.py read it)
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 4 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for st in 1 2 3 4; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sra_$TAG/s$st -o run -- python3 scripts/bench_sra.py stage $st \
    > gpurun_out/sra_${TAG}_s$st.log 2>&1 || exit $?
done

for arm in 0 1 0 1; do
  CMX_GEMM_DEEP=$arm timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_deep${arm}_$TAG.json 2>&1 || exit $?
  echo "deep=$arm $(cut -c1-200 gpurun_out/ab_deep${arm}_$TAG.json | grep -o '"value": [0-9.]*')"
done
