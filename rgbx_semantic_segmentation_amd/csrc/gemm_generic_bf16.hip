// bf16 instantiations of the register-staged generic GEMM launchers; see gemm_kernels.h
#include "gemm_kernels.h"
using gemmk::GemmArgs;
CMX_GEMM_GENERIC_SHAPES(CMX_GEMM_GENERIC_INST, bf16)
