#!/bin/bash
# round-5 (session 2) check: Mix-FFN band A/B, a kept kernel trace of the default step (idle gaps),
# PMC HBM traffic of the tile-GEMM family
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles
REPS=3 bash scripts/ab_env.sh base CMX_MIXFFN=0 > gpurun_out/ab_mixffn.txt 2>&1 || { cat gpurun_out/ab_mixffn.txt; exit 1; }
cat gpurun_out/ab_mixffn.txt
KEEP="0" bash scripts/trace_ab.sh r05_b base || exit 1
db=$(ls gpurun_out/tab_r05_b_0/run_results.db gpurun_out/tab_r05_b_0/*/run_results.db 2>/dev/null | head -1)
python3 scripts/step_trace.py $db > gpurun_out/profiles/r05_b_step_trace.txt
python3 scripts/step_trace.py $db --gaps 8 | head -40
bash scripts/pmc_pass.sh r05_b "CMX-B2 train step 480x640 bs=2 K=40" "gemm_bf16_kernel|gemm_multi_kernel|splitk_reduce_kernel" > gpurun_out/pmc_r05_b.out 2>&1 || { tail gpurun_out/pmc_r05_b.out; exit 1; }
cp gpurun_out/pmc_r05_b.json gpurun_out/profiles/r05_b_pmc_gemm_family.json
rm -rf gpurun_out/pmc_r05_b_FETCH_SIZE gpurun_out/pmc_r05_b_WRITE_SIZE
cat gpurun_out/profiles/r05_b_pmc_gemm_family.json
