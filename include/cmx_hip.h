/* cmx_hip.h — C-ABI of libcmx_hip.so, the MI355X (gfx950) kernels of the CMX RGB-X
 * segmentation training step.
 *
 * The reference (ynalcakan/RGBX_Semantic_Segmentation) has no FFI: its hot path is eager
 * PyTorch modules.  Each entry point below replaces the op(s) cited in its comment; the
 * Python host layer (rgbx_semantic_segmentation_amd/) binds them with ctypes and keeps
 * the reference's module API (models.builder.EncoderDecoder, engine.engine.Engine).
 *
 * Conventions
 *  - Return 0 on success, a negative cmx_status on bad shape / dtype / launch failure;
 *    cmx_last_error() returns a thread-local message.
 *  - dtype: 0 = fp32, 1 = bf16 (activations); parameters and statistics are fp32.
 *  - Activations are token-major (rows x channels, channels contiguous; NHWC for images).
 *    G = number of modality groups processed in one launch (RGB and X streams -> G = 2).
 *  - The caller owns every buffer, including workspaces sized by *_workspace(); the
 *    library never allocates, frees or synchronises, so every call is graph-capturable.
 *  - All work is enqueued on `stream`.
 *
 * Every declaration is on one line: the Python binding parses this file.
 */
#ifndef CMX_HIP_H
#define CMX_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
#ifndef __HIP_INCLUDE_HIP_HIP_RUNTIME_API_H
typedef struct ihipStream_t* hipStream_t;
#endif

/* ---- housekeeping ------------------------------------------------------------------ */
int cmx_abi_version(void);
const char* cmx_last_error(void);

/* ---- LayerNorm: nn.LayerNorm in Block.norm1/norm2, stage norms (eps 1e-6,
 *      dual_segformer.py:148,155,257), OverlapPatchEmbed.norm (:198), Attention.norm (:97),
 *      CrossPath.norm1/2 (net_utils.py:270-271), eps 1e-5.  x,y: (G*R, C); gamma,beta (G,C). */
int cmx_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, int64_t R, int G, int C, float eps, int dtype, hipStream_t stream);
size_t cmx_layernorm_bwd_workspace(int64_t R, int G, int C, int dtype);
int cmx_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta, float* workspace, int64_t R, int G, int C, int accumulate, int dtype, hipStream_t stream);

/* ---- elementwise: residual + DropPath (Block.forward, dual_segformer.py:177-178),
 *      activations (CrossPath ReLU net_utils.py:273-274), bias-grad column sums, casts. */
int cmx_residual_add(const void* x, const void* y, const float* sample_scale, void* out, int64_t n_per_sample, int64_t n, int dtype, hipStream_t stream);
int cmx_scale_samples(const void* x, const float* sample_scale, void* out, int64_t n_per_sample, int64_t n, int dtype, hipStream_t stream);
int cmx_act_fwd(const void* x, void* y, int64_t n, int act, int dtype, hipStream_t stream);
int cmx_act_bwd(const void* dy, const void* z, void* dx, int64_t n, int act, int dtype, hipStream_t stream);
int cmx_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t stream);
size_t cmx_colsum_workspace(int64_t M, int G, int N);
int cmx_colsum(const void* x, float* out, float* workspace, int64_t M, int G, int N, int64_t ld, int accumulate, float alpha, int dtype, hipStream_t stream);

/* ---- SRA attention core: softmax(q k^T * scale) v of Attention.forward
 *      (dual_segformer.py:130-134).  q,o: (Bt, N, heads*D) row strides qs/os; k,v: halves of
 *      the kv projection (Bt, Nk, 2*heads*D), row stride kvs; lse (Bt, heads, N) fp32. */
int cmx_sra_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int Bt, int N, int Nk, int heads, int D, int64_t qs, int64_t kvs, int64_t os, float scale, int dtype, hipStream_t stream);
size_t cmx_sra_attn_bwd_workspace(int Bt, int N, int Nk, int heads, int D);
int cmx_sra_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse, void* dq, void* dk, void* dv, float* workspace, int Bt, int N, int Nk, int heads, int D, int64_t qs, int64_t kvs, int64_t os, int64_t dos, int64_t dqs, int64_t dkvs, float scale, int dtype, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
