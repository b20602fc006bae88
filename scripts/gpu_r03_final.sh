#!/bin/bash
# Round-3 record of the committed tree: PMC HBM traffic of the grouped weight-gradient launch
# (two passes), full GPU suite, bench line (with CPU baselines), rocprofv3 kernel-trace summary
# and step census, config-1 / config-4 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out gpurun_out/profiles
TAG=${1:-r03_z}
bash scripts/pmc_pass.sh $TAG "CMX-B2 train step 480x640 bs=2 K=40" gemm_grouped > gpurun_out/pmc_$TAG.out 2>&1 || exit $?
cat gpurun_out/pmc_$TAG.out; cp gpurun_out/pmc_$TAG.json profiles/${TAG}_pmc_gemm_grouped.json
cp gpurun_out/pmc_$TAG.json gpurun_out/profiles/${TAG}_pmc_gemm_grouped.json
rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/prof_summary.py $db 10 > gpurun_out/kernel_stats_$TAG.txt 2>&1
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -30 gpurun_out/kernel_stats_$TAG.txt
rm -f $db
timeout -k 10 300 python -u bench.py --backbone mit_b0 --height 240 --width 320 --batch 1 --classes 9 --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/bench_c1_$TAG.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --backbone mit_b4 --height 480 --width 640 --batch 4 --classes 9 --steps 10 --warmup 3 \
  --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2>&1 || exit $?
grep -h -o '"value": [0-9.]*' gpurun_out/bench_c1_$TAG.json gpurun_out/bench_c4_$TAG.json
timeout -k 10 300 python -u bench.py --backbone mit_b5 --height 1024 --width 1024 --batch 1 --classes 19 \
  --dtype float16 --loss-scaling --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_fp16_$TAG.json \
  2> gpurun_out/bench_c5_fp16_$TAG.err || exit $?
grep -h -o '"value": [0-9.]*' gpurun_out/bench_c5_fp16_$TAG.json
