#!/bin/bash
# which change moves the config-4 FRM parity: SRA forward threshold or the LayerNorm-backward fusion
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for arm in CMX_SRA_SMALL_FWD_N=2048 CMX_LN_BWD_FUSE=0; do
  env $arm timeout -k 10 400 python -u -m pytest tests/test_config_parity.py -k "config4 and not fp16" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_g2_$arm.log 2>&1
  echo "[$arm] rc=$?"; grep -E "passed|failed|worst ratios" gpurun_out/pytest_r05_g2_$arm.log | head -3
done
