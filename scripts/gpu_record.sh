#!/bin/bash
# End-of-round record of the committed tree on ONE fresh GPU box, in the driver's order:
#   1. the bench line FIRST (as the driver runs it: the first GPU process of the lease),
#   2. rocprofv3 kernel trace of the same command -> kernel stats, step census, family table,
#   3. PMC HBM traffic of the dominant launch (two passes, FETCH_SIZE / WRITE_SIZE),
#   4. the full GPU suite,
#   5. the other BASELINE configs (1, 4, 5) as bench lines.
# Every GPU step has its own time limit; anything but a clean exit (pytest: 0 or 1) ends it.
# Usage: bash scripts/gpu_record.sh TAG [skip-suite]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out gpurun_out/profiles
TAG=${1:?tag}
SKIP_SUITE=${2:-}
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/prof_summary.py $db 10 > gpurun_out/profiles/${TAG}_kernel_stats.txt 2>&1
python3 scripts/step_census.py $db 200 > gpurun_out/profiles/${TAG}_step_census.txt 2>&1
python3 scripts/step_series.py $db 3 > gpurun_out/profiles/${TAG}_step_series.txt 2>&1
python3 scripts/family_table.py gpurun_out/profiles/${TAG}_step_census.txt --md > gpurun_out/profiles/${TAG}_family_table.md 2>&1
head -12 gpurun_out/profiles/${TAG}_step_census.txt
rm -rf gpurun_out/prof_$TAG
bash scripts/pmc_pass.sh $TAG "CMX-B2 train step 480x640 bs=2 K=40" gemm_grouped > gpurun_out/pmc_$TAG.out 2>&1 || exit $?
cp gpurun_out/pmc_$TAG.json gpurun_out/profiles/${TAG}_pmc_gemm_grouped.json
rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
# the tile-GEMM family (the bench line's roofline kernel): PMC bytes per launch
bash scripts/pmc_pass.sh ${TAG}f "CMX-B2 train step 480x640 bs=2 K=40" "gemm_bf16_kernel|gemm_stream_kernel|gemm_multi_kernel|splitk_reduce_kernel" > gpurun_out/pmc_${TAG}f.out 2>&1 || exit $?
cp gpurun_out/pmc_${TAG}f.json gpurun_out/profiles/${TAG}_pmc_gemm_family.json
rm -rf gpurun_out/pmc_${TAG}f_FETCH_SIZE gpurun_out/pmc_${TAG}f_WRITE_SIZE
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --backbone mit_b0 --height 240 --width 320 --batch 1 --classes 9 --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/profiles/${TAG}_bench_config1.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --backbone mit_b4 --height 480 --width 640 --batch 4 --classes 9 --steps 10 --warmup 3 \
  --no-cpu-baseline > gpurun_out/profiles/${TAG}_bench_config4.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --backbone mit_b5 --height 1024 --width 1024 --batch 1 --classes 19 --dtype float16 \
  --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profiles/${TAG}_bench_config5_fp16.json 2>&1 || exit $?
grep -h -o '"value": [0-9.]*' gpurun_out/profiles/${TAG}_bench_config*.json
