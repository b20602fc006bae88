#!/bin/bash
# stage-1 direct patch-embed conv: kernel tests, train / parity tests, bench + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r04_h
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_modules.py -k "pe1 or implicit or frm or ifrm or multi" -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_r04_h1.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_h1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_config_parity.py -m gpu -q --timeout 400 \
  --timeout-method thread > gpurun_out/pytest_r04_h2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_h2.log; grep -E "^FAILED|worst ratios" gpurun_out/pytest_r04_h2.log | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bench_sra.py nw > gpurun_out/sra_nw_r04_h.txt 2>&1
rc=$?; tail -3 gpurun_out/sra_nw_r04_h.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 > gpurun_out/bench_r04_h.json 2> gpurun_out/bench_r04_h.err
rc=$?; tail -c 600 gpurun_out/bench_r04_h.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_h" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_h/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profiles
db=$(ls gpurun_out/prof_r04_h/*.db gpurun_out/prof_r04_h/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/profiles/r04_h_step_census.txt 2>&1
python3 scripts/family_table.py gpurun_out/profiles/r04_h_step_census.txt --md > gpurun_out/profiles/r04_h_family_table.md 2>&1
head -8 gpurun_out/profiles/r04_h_step_census.txt
rm -rf gpurun_out/prof_r04_h
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --kernel-include-regex "ln_bwd|ln_fwd|dw2_bwdg|dw2_fwd" \
    -d gpurun_out/pmc_ln_$C -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_ln_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_dispatch.py $(ls gpurun_out/pmc_ln_FETCH_SIZE/*.db gpurun_out/pmc_ln_FETCH_SIZE/*/*.db 2>/dev/null | head -1) \
  $(ls gpurun_out/pmc_ln_WRITE_SIZE/*.db gpurun_out/pmc_ln_WRITE_SIZE/*/*.db 2>/dev/null | head -1) "ln_bwd|ln_fwd|dw2_bwdg|dw2_fwd" \
  > gpurun_out/profiles/r04_h_pmc_ln_dw.txt 2>&1
tail -3 gpurun_out/profiles/r04_h_pmc_ln_dw.txt
rm -rf gpurun_out/pmc_ln_FETCH_SIZE gpurun_out/pmc_ln_WRITE_SIZE
