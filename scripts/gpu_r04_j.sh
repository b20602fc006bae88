#!/bin/bash
# pe1 load batching + 4-tile wgrad blocks, SRA 10-wave auto policy, AdamW grid-cap sweep:
# kernel tests, microbenches, bench, step census
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "pe1" -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_r04_j1.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_j1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/bench_adamw.py > gpurun_out/adamw_r04_j.txt 2>&1
rc=$?; cat gpurun_out/adamw_r04_j.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/bench_sra.py > gpurun_out/sra_r04_j.txt 2>&1
rc=$?; cat gpurun_out/sra_r04_j.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 > gpurun_out/bench_r04_j.json 2> gpurun_out/bench_r04_j.err
rc=$?; cut -c1-300 gpurun_out/bench_r04_j.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_j" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_j.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
db=$(ls gpurun_out/prof_r04_j/*.db gpurun_out/prof_r04_j/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/profiles/r04_j_step_census.txt 2>&1
python3 scripts/family_table.py gpurun_out/profiles/r04_j_step_census.txt --md > gpurun_out/profiles/r04_j_family_table.md 2>&1
head -30 gpurun_out/profiles/r04_j_step_census.txt
grep -E "pe1|sra_|adamw" gpurun_out/profiles/r04_j_step_census.txt
rm -rf gpurun_out/prof_r04_j
