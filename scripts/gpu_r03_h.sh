#!/bin/bash
# Round-3 session 2: full GPU suite (HEAD + stream GEMM kernel + batched TrainPre + side-stream
# weight gradients), GEMM stream probe, step A/B, kernel census, config-5 fp16 line, loader rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_augment.py tests/test_gpu_train.py -m gpu \
  -v --timeout 120 --timeout-method thread -k "stream or batch or side or segment" > gpurun_out/pytest_new_$TAG.log 2>&1
rc=$?; echo "pytest new rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_new_$TAG.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/gemm_probe.py GEMM_STREAM=0,1 GEMM_STREAM_NS=2,3,4 > gpurun_out/probe_$TAG.txt 2>&1 || exit $?
cat gpurun_out/probe_$TAG.txt
REPS=2 STEPS=20 bash scripts/ab_env.sh base "CMX_GEMM_STREAM=512" "CMX_WGRAD_SIDE=1" "CMX_GEMM_STREAM=512 CMX_WGRAD_SIDE=1" \
  > gpurun_out/ab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls /tmp/prof_$TAG/*.db /tmp/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -60 gpurun_out/step_census_$TAG.txt
stats=$(ls /tmp/prof_$TAG/*kernel_stats.csv /tmp/prof_$TAG/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$stats" ] && cp "$stats" gpurun_out/kernel_stats_$TAG.csv
timeout -k 10 300 python -u bench.py --backbone mit_b5 --height 1024 --width 1024 --batch 1 --classes 19 \
  --dtype float16 --loss-scaling --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_fp16_$TAG.json \
  2> gpurun_out/bench_c5_fp16_$TAG.err || exit $?
cat gpurun_out/bench_c5_fp16_$TAG.json
timeout -k 10 300 python -u scripts/bench_loader.py > gpurun_out/loader_$TAG.json 2> gpurun_out/loader_$TAG.err || exit $?
cat gpurun_out/loader_$TAG.json
