#!/bin/bash
# config-4 parity under the three numerics variants (default, no multi-GEMM, no multi-GEMM +
# im2col stage 1) with the GPU gradients dumped for an off-box look
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default; do
  case $v in
    default) envs="" ;;
    nomulti) envs="CMX_MULTI_GEMM=0" ;;
    nomulti_nope1) envs="CMX_MULTI_GEMM=0 CMX_PE1_DIRECT=0" ;;
  esac
  env $envs timeout -k 10 400 python -u -m pytest \
    "tests/test_config_parity.py::test_bf16_train_step_vs_fp64_oracle[config4_b4_480x640_bs4]" "tests/test_config_parity.py::test_bf16_train_step_vs_fp64_oracle[config2_b2_480x640_bs2]" -x -q -s --timeout 380 \
    --timeout-method thread > gpurun_out/parity_i_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -E "worst ratios|cpu oracle" gpurun_out/parity_i_$v.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
