// bf16 instantiations of the 16-bit GEMM launchers (LDS-DMA tile kernels); see gemm_kernels.h
#include "gemm_kernels.h"
using gemmk::GemmArgs;
CMX_GEMM_FAST_INST(bf16)
