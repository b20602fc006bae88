#!/bin/bash
# round-6: CM-FRM combine prologue loads in flight together -- FRM local / config parity tests,
# step A/B and traced census against the previous commit (CMX_LIB_VARIANT=old)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fusion_local.py \
  tests/test_config_parity.py tests/test_gpu_fused.py > gpurun_out/r06/frm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06/frm_tests.log; grep -E "^FAILED" gpurun_out/r06/frm_tests.log | head; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-3} bash scripts/ab_env.sh base "CMX_LIB_VARIANT=old"
