#!/bin/bash
# End-of-round record on one GPU box: PMC traffic of the grouped weight-gradient launch (copied
# into profiles/ so the bench line's roofline.traffic uses it), then the full GPU suite, the
# bench line and a rocprofv3 kernel trace (scripts/gpu_check.sh).  Usage: bash scripts/final_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
bash scripts/pmc_pass.sh $TAG "CMX-B2 train step 480x640 bs=2 K=40" gemm_grouped > gpurun_out/pmc_$TAG.out 2>&1 || exit $?
cp gpurun_out/pmc_$TAG.json profiles/${TAG}_pmc_gemm_grouped.json
mkdir -p gpurun_out/profiles && cp profiles/${TAG}_pmc_gemm_grouped.json gpurun_out/profiles/
bash scripts/gpu_check.sh $TAG
