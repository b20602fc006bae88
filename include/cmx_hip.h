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
/* ABI revision of this header; cmx_abi_version() returns the revision the library was built
 * from, and the Python binding refuses a library whose revision differs (an older .so with the
 * same symbol names but shifted arguments would otherwise corrupt memory silently).  Bump it
 * on every change of an entry point's argument list. */
#define CMX_ABI_VERSION 6
int cmx_abi_version(void);
const char* cmx_last_error(void);
/* pinned host -> device copy of a packed record table on `stream` (see grouped launches) */
int cmx_upload(void* dst, const void* src, size_t nbytes, hipStream_t stream);
/* launch-policy knobs (GEMM_TILES, GEMM_SMALLK, GEMM_T128, GEMM_KW, GEMM_SPLITKW, SRA_SMALL_N,
 * SRA_DKV_DIRECT, SRA_QW, SRA_NW, GROUPED_KT, GROUPED_CHUNK): initialised from the
 * CMX_<NAME> environment variable, changed in-process by cmx_tune for interleaved A/B runs;
 * a knob set before the first launch that reads it keeps the set value.  tune_get: -1 if unset. */
int cmx_tune(const char* name, int value);
int cmx_tune_get(const char* name);

/* ---- LayerNorm: nn.LayerNorm in Block.norm1/norm2, stage norms (eps 1e-6,
 *      dual_segformer.py:148,155,257), OverlapPatchEmbed.norm (:198), Attention.norm (:97),
 *      CrossPath.norm1/2 (net_utils.py:270-271), eps 1e-5.  x,y: (G*R, C); gamma,beta (G,C).
 *      Backward with dgamma = dbeta = NULL leaves the per-block partials (G, nb, 2C) =
 *      [dgamma | dbeta] in the workspace (nb = workspace bytes / (8 G C)) for cmx_reduce_grouped. */
int cmx_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, int64_t R, int G, int C, float eps, int dtype, hipStream_t stream);
size_t cmx_layernorm_bwd_workspace(int64_t R, int G, int C, int dtype);
int cmx_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta, float* workspace, int64_t R, int G, int C, int accumulate, int dtype, hipStream_t stream);
/* backward of a norm whose input also feeds a residual (Block.forward x + drop_path(..), dual_segformer.py:168-169)
 * and whose output has two consumers (Attention.q and .sr, :114-121): upstream gradient dy + dy2,
 * dx = dres + LN_bwd(dy + dy2) and the DropPath-scaled copy dxs = sscale[(g*R+row)/rows_per_sample] * dx (NULLable). */
int cmx_layernorm_bwd_res(const void* dy, const void* dy2, const void* x, const float* gamma, const float* mean, const float* rstd, const void* dres, const float* sscale, void* dxs, void* dx, float* dgamma, float* dbeta, float* workspace, int64_t R, int G, int C, int64_t rows_per_sample, int accumulate, int dtype, hipStream_t stream);

/* ---- elementwise: residual + DropPath (Block.forward, dual_segformer.py:177-178),
 *      activations (CrossPath ReLU net_utils.py:273-274), bias-grad column sums, casts. */
int cmx_residual_add(const void* x, const void* y, const float* sample_scale, void* out, int64_t n_per_sample, int64_t n, int dtype, hipStream_t stream);
int cmx_scale_samples(const void* x, const float* sample_scale, void* out, int64_t n_per_sample, int64_t n, int dtype, hipStream_t stream);
int cmx_act_fwd(const void* x, void* y, int64_t n, int act, int dtype, hipStream_t stream);
int cmx_act_bwd(const void* dy, const void* z, void* dx, int64_t n, int act, int dtype, hipStream_t stream);
int cmx_partials_sum(const float* ws, float* out, int G, int nblk, int W, int accumulate, float alpha, hipStream_t stream);
int cmx_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t stream);
int cmx_cast_f32_h16(const float* src, void* dst, int64_t n, int dtype, hipStream_t stream);
/* All random masks of one training step in one launch (replaces the torch.rand draws of
   timm DropPath, dual_segformer.py:141-180, and Dropout2d, MLPDecoder.py:63, plus
   every BatchNorm2d's num_batches_tracked += 1): dp[i] = floor(keep[i] + u) / keep[i],
   d2[i] = (u >= p) / (1 - p), u = splitmix64(seed, *step, i); *step += 1 on the device. */
int cmx_step_masks(const float* keep, int nkeep, float* dp, int nd2, float p, float* d2, uint64_t seed, uint64_t* step, int64_t* nbt, int nnbt, hipStream_t stream);
/* bf16 gradient payload of the DP exchange (replaces DDP's fp32 bucket all-reduce,
   train.py:145-146 / engine.py:56): the bf16 -> fp32 copy of the all-gathered shard sums
   (cmx_cast_f32_bf16 makes the payload). */
int cmx_cast_bf16_f32(const void* src, float* dst, int64_t n, hipStream_t stream);
size_t cmx_colsum_workspace(int64_t M, int G, int N);
int cmx_colsum(const void* x, float* out, float* workspace, int64_t M, int G, int N, int64_t ld, int accumulate, float alpha, int dtype, hipStream_t stream);

/* ---- SRA attention core: softmax(q k^T * scale) v of Attention.forward
 *      (dual_segformer.py:130-134).  q,o: (Bt, N, heads*D) row strides qs/os; k,v: halves of
 *      the kv projection (Bt, Nk, 2*heads*D), row stride kvs; lse (Bt, heads, N) fp32. */
int cmx_sra_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int Bt, int N, int Nk, int heads, int D, int64_t qs, int64_t kvs, int64_t os, float scale, int dtype, hipStream_t stream);
size_t cmx_sra_attn_bwd_workspace(int Bt, int N, int Nk, int heads, int D);
int cmx_sra_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse, void* dq, void* dk, void* dv, float* workspace, int Bt, int N, int Nk, int heads, int D, int64_t qs, int64_t kvs, int64_t os, int64_t dos, int64_t dqs, int64_t dkvs, float scale, int dtype, hipStream_t stream);

/* ---- depthwise 3x3 + bias + act: Mix-FFN DWConv + GELU (dual_segformer.py:27-33,67-71) and
 *      ChannelEmbed DW3x3 + ReLU (net_utils.py:315-318).  h,out: (NI, H, W, C) NHWC,
 *      image n in group n / imgs_per_group; w (G, C, 9), b (G, C) fp32; act 0/1 gelu/2 relu.
 *      Backward with dw = db = NULL leaves the partials (G, P, C*10) = [9 taps | bias] per channel
 *      in the workspace (P = workspace bytes / (40 G C) - 1) for cmx_reduce_grouped. */
int cmx_dwconv3x3_fwd(const void* h, const float* w, const float* b, void* out, int NI, int imgs_per_group, int H, int W, int C, int act, int dtype, hipStream_t stream);
/* fwd_save also writes gprime = act'(z) (z = the conv + bias pre-activation); bwd_saved then forms dz = da * gprime
 * with no 3x3 recompute (LDS-tiled channel counts only; dw = db = NULL leaves the partials as cmx_dwconv3x3_bwd). */
int cmx_dwconv3x3_fwd_save(const void* h, const float* w, const float* b, void* out, void* gprime, int NI, int imgs_per_group, int H, int W, int C, int act, int dtype, hipStream_t stream);
int cmx_dwconv3x3_bwd_saved_tiles(int imgs_per_group, int H, int W);
int cmx_dwconv3x3_bwd_saved(const void* da, const void* h, const void* gprime, const float* w, void* dh, float* dw, float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int accumulate, int dtype, hipStream_t stream);
size_t cmx_dwconv3x3_bwd_workspace(int NI, int imgs_per_group, int H, int W, int C);
int cmx_dwconv3x3_bwd(const void* da, const void* h, const float* w, const float* b, void* dz, void* dh, float* dw, float* db, float* workspace, int NI, int imgs_per_group, int H, int W, int C, int act, int accumulate, int dtype, hipStream_t stream);

/* ---- conv as im2col + GEMM: OverlapPatchEmbed.proj (dual_segformer.py:196-197) and the SRA
 *      spatial-reduction conv Attention.sr (:95-96).  NHWC cols use (kh, kw, c) order (weights
 *      stored (Cout, kh, kw, Cin)); the NCHW variant takes the fp32 input image. */
int cmx_im2col_nhwc(const void* x, void* cols, int NI, int H, int W, int C, int KH, int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t stream);
int cmx_im2col_nchw_f32(const float* x, void* cols, int NI, int C, int H, int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t stream);
/* the same over two image batches: images n < nsplit from x, the rest from x2 (the RGB and X
 * inputs of EncoderDecoder.forward without the concat, builder.py:240-253) */
int cmx_im2col_nchw2_f32(const float* x, const float* x2, int nsplit, void* cols, int NI, int C, int H, int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t stream);
int cmx_col2im_nhwc(const void* cols, void* dx, int NI, int H, int W, int C, int KH, int KW, int stride, int pad, int Ho, int Wo, int64_t ldc, int dtype, hipStream_t stream);

/* ---- FFM cross attention (CrossAttention.forward, net_utils.py:199-214):
 *      ctx = softmax_{-2}(k^T v * scale) per (g, b, head); out_1 = q_1 ctx_2, out_2 = q_2 ctx_1.
 *      The token contractions are per-head cmx_gemm_h2 calls over (g, b, head) (d x d products,
 *      the reference's MACs); these two kernels sit between them.  Every array is
 *      (G*B, heads, D, D): kv / dctx fp32 GEMM results (k^T v, u^T dout), ctx fp32 (saved);
 *      ctxT[(1-g)*B + b][h][j][i] = ctx_{g,b,h}[i][j] (crossed, transposed) and
 *      da[g*B + b][h][i][j] = scale * softmax_bwd in the compute dtype; dctx is filed under the
 *      modality that consumed the context. */
int cmx_ffm_ctx_fwd(const float* kv, float* ctx, void* ctxT, int G, int B, int heads, int D, float scale, int dtype, hipStream_t stream);
int cmx_ffm_ctx_bwd(const float* ctx, const float* dctx, void* da, int G, int B, int heads, int D, float scale, int dtype, hipStream_t stream);

/* ---- CM-FRM (FeatureRectifyModule, net_utils.py:124-152): ChannelWeights pooling (:22-27)
 *      + tiny-M MLP (:16-20), SpatialWeights 1x1 C->2 + sigmoid (:74-83), rectification. */
size_t cmx_frm_pool_workspace(int B, int N, int C);
/* tickets: cmx_frm_pool_tickets(B, C) zeroed uint32 arrival counters owned by the caller (each launch leaves
 * them zero; launches that may overlap need their own); NULL = the library's device-global set */
size_t cmx_frm_pool_tickets(int B, int C);
int cmx_frm_pool_fwd(const void* x, float* pooled, int* argmax, float* workspace, unsigned* tickets, int B, int N, int C, int dtype, hipStream_t stream);
/* dx += pooling backward; dpooled (B, 4C) given as partial slices dp[b][k] = sum_s part[s*slice_stride + b*4C + k] */
int cmx_frm_pool_bwd(const float* dpooled_part, int nslice, int64_t slice_stride, const int* argmax, void* dx, int B, int N, int C, int dtype, hipStream_t stream);
/* tiny-M linear y = act(x w^T + b) (x (M, K) fp32, M <= 8); backward in one pass over w: dy given as partial slabs
 * dy[m][n] = sum_s part[s*dy_slice_stride + m*dy_row_stride + n]; writes dw / db; dx as cmx_small_linear_nslice()
 * partial slices (nslice, M, K) in dx_part (NULL: skip) */
int cmx_small_linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int K, int Nout, int act, hipStream_t stream);
int cmx_small_linear_nslice(void);
size_t cmx_small_linear_bwd_workspace(int M, int K, int Nout);
int cmx_small_linear_bwd(const float* dy_part, int dy_nslice, int64_t dy_slice_stride, int64_t dy_row_stride, const float* y, const float* x, const float* w, float* dx_part, float* dw, float* db, int M, int K, int Nout, int act, int accumulate, hipStream_t stream);
/* rectification fused with SpatialWeights' C -> 2 conv + sigmoid: h (B*N, C) = the 2C -> C conv output (pre-ReLU),
 * w2 (2, C), b2 (2) fp32; writes sw (B*N, 2) (saved for the backward) and out (2, B, N, C) */
/* ChannelWeights (net_utils.py:11-30) of FeatureRectifyModule (:145) as ONE launch per direction:
 * a grid of one workgroup per CU whose phases (pool partial, pool final, GEMV W1 + relu, GEMV W2 +
 * sigmoid; backward: dcw slab sum * sigmoid', W2 pass, W1 pass, pooling gradient) meet at grid
 * barriers.  x (2,B,N,C); pooled, y1 (B,4C), argmax, cw (B,2C) fp32/int32; W1 (4C,4C), W2 (2C,4C) fp32.
 * Backward: dcw_part = the combine backward's (B, nslab, 2C) partials; dW / db written (not
 * accumulated); the pooling gradient is ADDED into dx.  B <= 8, C % 16 == 0, C <= 512.  One launch
 * of each direction at a time per device.  barrier_timeouts: count of polls that gave up (0 = every
 * grid was co-resident; synchronous, for tests). */
int cmx_frm_combine_fwd(const void* x, const float* cw, const void* h, const float* w2, const float* b2, float* sw, void* out, int B, int N, int C, int dtype, hipStream_t stream);
/* backward: dx direct path (2,B,N,C), dh (B*N, C); workspace = dcw partials (B, nblk, 2C) followed by the
 * [dw2 (2C) | db2 (2)] partials (B*nblk, 2C+2); nblk = cmx_frm_combine_bwd_nblk(N, C, dtype).
 * dout2 (may be NULL): the gradient of the output's second consumer (the next stage beside the FFM),
 * summed on load and rounded to the storage type, as autograd's add of the two would */
int cmx_frm_combine_bwd_nblk(int N, int C, int dtype);
size_t cmx_frm_combine_bwd_workspace(int B, int N, int C, int dtype);
int cmx_frm_combine_bwd(const void* dout, const void* dout2, const void* x, const float* cw, const float* sw, const void* h, const float* w2, void* dx, void* dh, float* workspace, int B, int N, int C, int dtype, hipStream_t stream);

/* ---- BatchNorm (ChannelEmbed BNs net_utils.py:319-329, decoder SyncBN MLPDecoder.py:51-55):
 *      fp64 channel sums -> (all-reduce for SyncBN) -> finalize; fused residual / act / Dropout2d. */
size_t cmx_bn_workspace(int64_t M, int C);
int cmx_bn_stats(const void* x, double* sums, double* workspace, int64_t M, int C, int dtype, hipStream_t stream);
int cmx_bn_stats_finalize(const void* x, double* sums, double* workspace, int64_t M, int C, float eps, float momentum, float* running_mean, float* running_var, float* mean, float* invstd, int dtype, hipStream_t stream);
int cmx_bn_finalize(const double* sums, double count, float eps, float momentum, float* running_mean, float* running_var, float* mean, float* invstd, int C, int training, hipStream_t stream);
int cmx_bn_apply(const void* x, const float* mean, const float* invstd, const float* gamma, const float* beta, const void* res, const float* dscale, void* y, int64_t M, int C, int64_t rows_per_sample, int act, int dtype, hipStream_t stream);
int cmx_bn_bwd_reduce(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma, const float* beta, const void* res, const float* dscale, double* sums, float* dgamma, float* dbeta, double* workspace, int64_t M, int C, int64_t rows_per_sample, int act, int accumulate, int dtype, hipStream_t stream);
int cmx_bn_bwd_apply(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma, const float* beta, const void* res, const float* dscale, const double* sums, double count, void* dx, void* dres, int64_t M, int C, int64_t rows_per_sample, int act, int training, int dtype, hipStream_t stream);
/* Small maps (local statistics, training; the stage-3/4 ChannelEmbed BNs): the forward (sums, finalize incl. running
 * stats, apply) and the backward (both sums, dgamma / dbeta, dx / dres) each in ONE launch of C / 16 workgroups that
 * own 16 channels over all M rows.  C % 16 == 0. */
int cmx_bn_small_fwd(const void* x, const void* res, const float* gamma, const float* beta, const float* dscale, void* y, double* sums, float* mean, float* invstd, float* running_mean, float* running_var, int64_t M, int C, int64_t rows_per_sample, int act, float eps, float momentum, int dtype, hipStream_t stream);
int cmx_bn_small_bwd(const void* dy, const void* x, const float* mean, const float* invstd, const float* gamma, const float* beta, const void* res, const float* dscale, float* dgamma, float* dbeta, void* dx, void* dres, int64_t M, int C, int64_t rows_per_sample, int act, int accumulate, int dtype, hipStream_t stream);

/* ---- bilinear, align_corners=False (F.interpolate in MLPDecoder.py:67-73, builder.py:233)
 *      and its separable 1-D adjoint (backward). */
int cmx_bilinear_fwd_nhwc(const void* in, void* out, int NB, int Hi, int Wi, int Ho, int Wo, int C, int64_t out_pix_stride, int dtype, hipStream_t stream);
int cmx_bilinear_fwd_nchw_f32(const void* in, float* out, int NB, int Hi, int Wi, int Ho, int Wo, int C, int dtype, hipStream_t stream);
/* U (B, H, W, C) = bias + up(z0) + up(z1) + up(z2) (any source NULL: absent; bias fp32 or NULL): DecoderHead's three
 * upsampled branch products summed in one pass (the decoder fold's c1 GEMM adds U as its residual).  C % 64 == 0,
 * the source widths sum to <= 160. */
int cmx_bilinear_up3_add(const void* z0, const void* z1, const void* z2, int B, int h0, int w0, int h1, int w1, int h2, int w2, const float* bias, void* out, int H, int W, int C, int dtype, hipStream_t stream);
/* The backward of up to three upsampled branches from one read of dz (B, H, W, C): y_s (B, h_s, w_s, C) = up_s^T dz
 * (y1 / y2 NULL: absent), through fp32 workspaces t_s (B*H, w_s, C).  Two launches (x pass, y pass); C % 128 == 0 (fp32: C % 64 == 0). */
int cmx_bilinear_adjoint3(const void* dz, float* t0, float* t1, float* t2, void* y0, void* y1, void* y2, int B, int H, int W, int h0, int w0, int h1, int w1, int h2, int w2, int C, int dtype, hipStream_t stream);
int cmx_bilinear_adjoint_1d(const void* in, void* out, int64_t P, int Lo, int Li, int Q, int64_t sp, int64_t so, const float* a1, const float* a2, float alpha0, int in_dtype, int out_dtype, hipStream_t stream);
/* DecoderHead.linear_fuse (MLPDecoder.py:66-77) without the (B, N1, 4E) concat: the 1x1 conv commutes with the
 * bilinear upsample (linear, weights sum to 1), so Z = e1 Wf[:, 3E:]^T + bias + up(z4) + up(z3) + up(z2) with the
 * low-resolution products z_i = e_i Wf[:, slot_i]^T (B, h_i, w_i, E) added by the GEMM epilogue (z_i may be NULL).
 * e1 (B*H1*W1, K) with row stride lda; Wf_c1 (E, K) with row stride ldw (column 3E of linear_fuse's weight: K = E);
 * Z (B*H1*W1, E). */
/* dx of the SRA spatial-reduction conv Attention.sr (kernel = stride = R, pad 0; dual_segformer.py:95-96): the
 * dgrad GEMM dy (G, NIg*Ho*Wo, N) @ W (G, N, R*R*C) with the col2im folded into its epilogue as an address remap
 * (non-overlapping patches).  dx (G*NIg, H, W, C) NHWC; pixels outside the Ho*R x Wo*R window are not written. */
int cmx_conv_patch_dgrad(const void* dy, const void* Wt, void* dx, int G, int NIg, int H, int W, int C, int R, int Ho, int Wo, int N, int64_t sdy, int64_t sW, int64_t sdx, int dtype, hipStream_t stream);

int cmx_decoder_fuse_fwd(const void* e1, const void* Wf_c1, void* Z, const float* bias, const void* z4, const void* z3, const void* z2, int B, int H1, int W1, int h4, int w4, int h3, int w3, int h2, int w2, int E, int K, int64_t lda, int64_t ldw, int dtype, hipStream_t stream);
/* DecoderHead with linear_c{1..4} folded into linear_fuse (MLPDecoder.py:60-77; default path, functions.DecoderFoldF):
 * Z = sum_i up_i(x_i M_i^T) + b with M_i = Wf_i Wc_i, b = bf + sum_i Wf_i bc_i (cmx_decoder_fuse_fwd with e1 = x1,
 * K = C1, Wf_c1 = M_1).  cmx_decoder_fold_bias forms b from Wf (E, ldw) and the four fp32 biases (slot order
 * c4, c3, c2, c1).  cmx_decoder_fold_bwd_prep, after dM_i = dY_i^T x_i and gb = sum_rows dZ are known: dMh = dtype(dM)
 * (n elements; dMh NULL: none), WfT (4E, E) = Wf^T, dWf (E, ldg) = gb bcat^T (the dM_i Wc_i^T GEMMs accumulate onto
 * it), dbc_i = Wf_i^T gb, dbf = gb.  E a multiple of 64. */
int cmx_decoder_fold_bias(const void* Wf, int64_t ldw, const float* bf, const float* bc4, const float* bc3, const float* bc2, const float* bc1, float* b, int E, int dtype, hipStream_t stream);
int cmx_decoder_fold_bwd_prep(const float* dM, void* dMh, int64_t n, const float* gb, const void* Wf, int64_t ldw, void* WfT, float* dWf, int64_t ldg, const float* bc4, const float* bc3, const float* bc2, const float* bc1, float* dbc4, float* dbc3, float* dbc2, float* dbc1, float* dbf, int E, int dtype, hipStream_t stream);

/* ---- fused final upsample + CrossEntropyLoss(mean, ignore_index=255) (builder.py:233,249). */
size_t cmx_upsample_ce_workspace(int B, int H, int W);
/* grad = NULL: loss only (H = 4h, W = 4w, K <= 40), the backward then recomputes the gradient tile by tile:
 * cmx_upsample_ce_bwd writes dlogits (B, h, w, K) = bilinear adjoint of (softmax - onehot) * dloss[0] * stats[1]
 * (stats = the forward's out) without materialising any full-resolution tensor. */
int cmx_upsample_ce_fwd(const void* logits, const int64_t* label, void* grad, float* out, float* workspace, int B, int h, int w, int H, int W, int K, int ignore_index, int dtype, hipStream_t stream);
int cmx_upsample_ce_bwd(const void* logits, const int64_t* label, const float* dloss, const float* stats, void* dlogits, int B, int h, int w, int H, int W, int K, int ignore_index, int dtype, hipStream_t stream);
/* Training form (H = 4h, W = 4w, K <= 40): the loss (out, as cmx_upsample_ce_fwd) and adj (B, h, w, K) fp32 = bilinear
 * adjoint of (softmax - onehot) in one pass over the pixels; the backward is cmx_upsample_ce_bwd_scale:
 * dlogits (n elements, dtype) = adj * dloss[0] * stats[1]. */
int cmx_upsample_ce_fwd_adj(const void* logits, const int64_t* label, float* adj, float* out, float* workspace, int B, int h, int w, int H, int W, int K, int ignore_index, int dtype, hipStream_t stream);
int cmx_upsample_ce_bwd_scale(const float* adj, const float* dloss, const float* stats, void* dlogits, int64_t n, int dtype, hipStream_t stream);

/* ---- dense layers: batched MFMA GEMM with fused epilogues -----------------------------
 * Replaces every nn.Linear and 1x1 Conv2d of the path (dual_segformer.py:42-43, 87-96, 110;
 * net_utils.py:14-17, 72-75, 196-198, 265-269, 316-326; MLPDecoder.py:13-19, 63-70), the
 * im2col'd OverlapPatchEmbed / SR convs (dual_segformer.py:95, 196) and their dgrad / wgrad.
 * C[g](i,j) = epi(sum_k A(i,k) B(j,k)); A(i,k) = A[i*lda+k] (transA=0) or A[k*lda+i] (1); k >= K1
 * reads A2 (cat-free two-input Linear).  epi: v = act(acc + bias[g*sbias+j]); residual R (layout
 * of C): v = R + rscale[(g*M+i)/rows_per_sample]*v; out_mode 0: C = dtype(v), 1: C = fp32(v), 2: C += v.
 * ones_col: B row N-1 is virtual ones and column N-1 of the result goes to dbias (bias gradient).
 * splitk > 1: K split over blocks into a workspace of cmx_gemm_workspace() bytes, then reduced (the
 * reducer applies the epilogue); splitk <= 0: the library's choice, cmx_gemm_splitk(). */
size_t cmx_gemm_workspace(int G, int M, int N, int splitk);
int cmx_gemm_splitk(int G, int M, int N, int K, int ones_col, int dtype);
int cmx_gemm(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R, const float* rscale, const void* mask, float* dbias, float* workspace, int G, int M, int N, int K, int K1, int64_t lda, int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias, int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode, int ones_col, int splitk, int dtype, hipStream_t stream);
/* ---- independent GEMMs in ONE launch: Attention.q beside Attention.kv (dual_segformer.py:114-121, forward and
 *      dgrad) and the decoder's linear_c1..c4 (MLPDecoder.py:66-73).  cmx_gemm_plan takes cmx_gemm's arguments
 *      and fills a plan (host memory of cmx_gemm_plan_size() bytes) instead of launching: > 0 = block count,
 *      0 = not eligible (16-bit 64 x 64-tile problems without split-K / bias-gradient column only; the caller
 *      runs cmx_gemm), < 0 = invalid.  cmx_gemm_multi launches n <= 4 plans of one dtype and B layout. */
size_t cmx_gemm_plan_size(void);
int cmx_gemm_plan(void* plan, const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R, const float* rscale, const void* mask, float* dbias, float* workspace, int G, int M, int N, int K, int K1, int64_t lda, int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias, int64_t sdb, int rows_per_sample, int transA, int transB, int act, int out_mode, int ones_col, int splitk, int dtype);
int cmx_gemm_multi(const void* plans, int n, hipStream_t stream);
/* cmx_gemm_h2: cmx_gemm (no A2 / bias / residual / epilogue extras) over a two-level batch of G = Go * gh
 *      problems: problem g reads / writes at (g / gh) * sX + (g % gh) * sXh -- the per-head k^T v,
 *      u @ ctx and their backward products of the FFM cross attention (net_utils.py:206-212), one
 *      (image x modality, head) pair per problem. */
int cmx_gemm_h2(const void* A, const void* B, void* C, float* workspace, int G, int gh, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sAh, int64_t sB, int64_t sBh, int64_t sC, int64_t sCh, int transA, int transB, int out_mode, int splitk, int dtype, hipStream_t stream);

/* ---- grouped (deferred) launches: the weight gradients of a backward segment in ONE GEMM
 *      launch and every partial-sum reduction (split-K slabs, LayerNorm dgamma/dbeta, DWConv
 *      dW/db partials) in ONE reduce launch, issued when the segment's backward is done.
 *      Replaces the per-layer weight-gradient half of autograd's Linear/Conv2d/LayerNorm
 *      backward (the DDP reducer consumes those gradients, train.py:145-146).  The host packs
 *      records (cmx_*_pack, host memory of cmx_*_record_size() bytes each, blk0 = first block of
 *      the record, returns its block count), copies them to device memory, then launches. */
size_t cmx_gemm_group_record_size(void);
int cmx_gemm_grouped_splitk(int G, int M, int N, int K, int ones_col);
int cmx_gemm_group_pack(void* rec, const void* A, const void* B, void* C, float* dbias, float* workspace, int G, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC, int64_t sdb, int transA, int transB, int out_mode, int ones_col, int splitk, int blk0);
/* cmx_gemm_grouped: dtype = the operands' storage type of every record (1 bf16, 2 fp16) */
/* cmx_gemm_ln: cmx_gemm's forward (A (G,M,K1) [| A2], B (G,N,K), both k-contiguous; bias, residual
 *      R with DropPath scale rscale, activation; 16-bit, no split-K) plus the LayerNorm of its output
 *      rows in the same launch -- the consumer norm of a residual Linear (Block: x + drop_path(proj(.))
 *      -> norm2, x + drop_path(fc2(.)) -> next norm1 / stage norm; dual_segformer.py:168-169,382):
 *      ln_y = LN(C) * ln_gamma[g] + ln_beta[g] (C's dtype and strides), ln_mean / ln_rstd (fp32, g*M + i).
 *      N <= 128, N % 8 == 0: one output tile spans the row and normalises it in the epilogue
 *      (statistics bit-identical to cmx_layernorm_fwd).  CMX_ERR_ARG when not eligible. */
int cmx_gemm_ln(const void* A, const void* A2, const void* B, void* C, const float* bias, const void* R, const float* rscale, int G, int M, int N, int K, int K1, int64_t lda, int64_t lda2, int64_t ldb, int64_t ldc, int64_t sA, int64_t sA2, int64_t sB, int64_t sC, int64_t sbias, int rows_per_sample, int act, const float* ln_gamma, const float* ln_beta, int64_t ln_sg, float ln_eps, void* ln_y, float* ln_mean, float* ln_rstd, int dtype, hipStream_t stream);
/* cmx_gemm_ln_bwd: a Linear's input gradient dy = A (G,M,K) B^T (B (G,N,K) logical, row-contiguous: the
 *      weight W (G,K,N) read transposed, as cmx_gemm's transB = 1 dgrad) fed straight into the backward
 *      of the LayerNorm that produced that Linear's input (Block.norm2 -> fc1, dual_segformer.py:169;
 *      nn.LayerNorm backward): dx = rstd (g - mean(g) - xhat mean(g xhat)) + dres, g = (dy [+ dy2]) * gamma,
 *      xhat = (x - mean) rstd; dxs = sscale[(g*M + i) / rows_per_sample] * dx (may be NULL); partials =
 *      (G, ceil(M/64), 2N) fp32 dgamma | dbeta column sums per 64-row tile (cmx_gemm_ln_bwd_partials
 *      bytes) for cmx_reduce_grouped.  dx, x, dres, dy2, dxs share C's layout (ldc, sC); mean / rstd
 *      (G*M) fp32 as cmx_layernorm_fwd saves them; N <= 128, N % 8 == 0, 16-bit.  dy never reaches HBM. */
int cmx_gemm_ln_bwd(const void* A, const void* B, void* dx, int G, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sA, int64_t sB, int64_t sC, const void* x, const float* gamma, int64_t sg, const float* mean, const float* rstd, const void* dres, const void* dy2, const float* sscale, int rows_per_sample, void* dxs, float* partials, int dtype, hipStream_t stream);
size_t cmx_gemm_ln_bwd_partials(int G, int M, int N);
/* cmx_conv_patch_dgrad_ln_bwd: cmx_conv_patch_dgrad (Attention.sr's input gradient, col2im in the epilogue)
 *      fed straight into the backward of the LayerNorm that produced the conv's input (Block.norm1 ->
 *      Attention.sr, dual_segformer.py:95-96,167): dx = LN'(col2im(dy W) [+ dy2]) + dres as cmx_gemm_ln_bwd,
 *      x / dres / dy2 / dxs / dx NHWC (G*NIg, H, W, C), mean / rstd per pixel (G*NIg*H*W) fp32; exact
 *      patches (H = Ho R, W = Wo R), C 64 or 128, 16-bit.  partials: (G, ceil(NIg Ho Wo / 64) R^2, 2C)
 *      dgamma | dbeta per (64-patch, tap) tile (cmx_conv_patch_dgrad_ln_bwd_partials bytes). */
int cmx_conv_patch_dgrad_ln_bwd(const void* dy, const void* Wt, void* dx, int G, int NIg, int H, int Wd, int C, int R, int Ho, int Wo, int N, int64_t sdy, int64_t sW, int64_t sdx, const void* x, const float* gamma, int64_t sg, const float* mean, const float* rstd, const void* dres, const void* dy2, const float* sscale, int rows_per_sample, void* dxs, float* partials, int dtype, hipStream_t stream);
size_t cmx_conv_patch_dgrad_ln_bwd_partials(int G, int NIg, int Ho, int Wo, int C, int R);
int cmx_gemm_grouped(const void* recs, int nrec, int total_blocks, int dtype, hipStream_t stream);
/* cmx_gemm_grouped_capped: the same launch on a grid of at most max_blocks workgroups (a multiple
 * of 8; <= 0: uncapped), each walking blocks b, b + grid, ...: a grouped weight-gradient launch
 * beside the backward on a side stream keeps to that share of the chip */
int cmx_gemm_grouped_capped(const void* recs, int nrec, int total_blocks, int max_blocks, int dtype, hipStream_t stream);
/* ---- im2col-free convolution on the same GEMM (bf16, NHWC, C % 64 == 0 for the forward): OverlapPatchEmbed.proj
 *      (k3 s2 p1, dual_segformer.py:196-197) and Attention.sr (kR sR, :95-96).  The forward's A operand is DMA'd
 *      tap by tap straight from x (padding = zeros from the buffer range check); the weight gradient is one
 *      grouped-GEMM record per tap whose B operand gathers x at that tap (dW row pitch KH*KW*C). */
int cmx_conv_implicit_fwd(const void* x, const void* Wt, void* y, const float* bias, float* workspace, int G, int NIg, int H, int Wd, int C, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int64_t sx, int64_t sW, int64_t sy, int64_t sbias, int splitk, int dtype, hipStream_t stream);
int cmx_gemm_group_pack_conv_wgrad(void* rec, const void* dy, const void* x, float* dW, float* dbias, float* workspace, int G, int NIg, int H, int Wd, int C, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int tap, int64_t sdy, int64_t sx, int64_t sdW, int64_t sdb, int splitk, int blk0);
/* ---- stage-1 OverlapPatchEmbed.proj (Conv2d 3 -> N, k7 s4 p3, dual_segformer.py:196-197 / :219) straight from
 *      the fp32 NCHW input batches, no im2col columns: img0 feeds group 0 (RGB), img1 group 1 (the X modality;
 *      image_encoder forward, dual_segformer.py:347-350).  Wt = the 16-bit (G, N, Kp) weight shadow, columns in
 *      the reference's (c, kh, kw) flatten order, Kp = 152 (147 zero-padded); y (G, B*Ho*Wo, N) NHWC 16-bit.
 *      cmx_pe1_conv_wgrad writes one fp32 partial slab (N, Kp + 1) per workgroup into ws (G, nblk, N, Kp + 1),
 *      nblk = cmx_pe1_conv_wgrad_nblk(B, Ho, Wo); column Kp is the bias gradient.  The caller sums the slabs
 *      (cmx_reduce_pack with csplit = Kp). */
/*      gamma != NULL: OverlapPatchEmbed.norm (dual_segformer.py:198) fused into the epilogue -- y_ln (same layout as
 *      y) = LayerNorm of the stored y, mean / rstd (G*B*Ho*Wo) as cmx_layernorm_fwd writes them (N 32 or 64). */
int cmx_pe1_conv_fwd(const float* img0, const float* img1, const void* Wt, const float* bias, void* y, int G, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int Kp, int64_t sW, int64_t sbias, int64_t sy, const float* gamma, const float* beta, void* y_ln, float* mean, float* rstd, int64_t sgb, float eps, int dtype, hipStream_t stream);
int cmx_pe1_conv_wgrad_nblk(int B, int Ho, int Wo);
int cmx_pe1_conv_wgrad(const void* dy, const float* img0, const float* img1, float* ws, int G, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int Ho, int Wo, int N, int Kp, int64_t sdy, int dtype, hipStream_t stream);
size_t cmx_reduce_record_size(void);
int cmx_reduce_pack(void* rec, const float* src, float* dst, float* dst2, int G, int nblk, int64_t sg, int64_t sb, int rows, int cols, int csplit, int64_t dg, int ldd, int64_t dg2, int ldd2, int accumulate, int blk0);
int cmx_reduce_grouped(const void* recs, int nrec, int total_blocks, hipStream_t stream);

/* ---- fused AdamW over the flat parameter buffer (train.py:128-129, init_func.py:33-57). */
/* tickets (all three steps): cmx_adamw_tickets() zeroed uint32s owned by the optimizer (the step count's
 * arrival counters; each launch leaves them zero); NULL = the library's device-global set */
size_t cmx_adamw_tickets(void);
int cmx_adamw_step(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype, const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1, double beta2, float eps, double weight_decay, float grad_scale, unsigned* tickets, hipStream_t stream);
/* ---- dynamic loss scaling: torch.cuda.amp.GradScaler of the reference's AMP path (train.py:13,56,185-198, config 5).
 *      The scale, growth tracker and found-inf flag live on the device, so a scaled step replays from a HIP graph:
 *      grad_nonfinite sets found_inf if any gradient is inf/nan; adamw_step_scaled unscales by 1/loss_scale[0] and
 *      skips the whole update (and the step count) when found_inf[0] != 0; loss_scale_update applies backoff /
 *      growth (after growth_interval clean steps) and clears found_inf. */
int cmx_adamw_step_scaled(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype, const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1, double beta2, float eps, double weight_decay, float grad_scale, const float* loss_scale, const float* found_inf, unsigned* tickets, hipStream_t stream);
/* adamw_step_segment: the same update on one contiguous range of the flat buffers (p, g, m, v,
 *      shadow and decay64 offset by the caller; n a multiple of 64), e.g. one backward-completion
 *      segment updated on a side stream while the backward of the earlier stages runs.  Every launch
 *      reads the step count; only the one with store_step = 1 (the step's last) stores t + 1.
 *      max_blocks > 0 caps the grid (the launch then keeps to that share of the chip). */
int cmx_adamw_step_segment(float* p, const float* g, float* m, float* v, void* shadow, int shadow_dtype, const uint8_t* decay64, int64_t n, const float* lr_ptr, float* step_ptr, double beta1, double beta2, float eps, double weight_decay, float grad_scale, int store_step, int max_blocks, unsigned* tickets, hipStream_t stream);
/* grad_nonfinite: flags64 (nullable) = the per-64-element decay flags of adamw_step; blocks flagged 2
 *      (frozen slots, in no optimizer group) are not scanned, as GradScaler.unscale_ checks only the
 *      optimizer's parameters. */
int cmx_grad_nonfinite(const float* g, int64_t n, const uint8_t* flags64, float* found_inf, hipStream_t stream);
int cmx_loss_scale_update(float* scale, int* growth_tracker, float* found_inf, float growth_factor, float backoff_factor, int growth_interval, hipStream_t stream);

/* ---- IFRM (ImprovedFeatureRectifyModule, net_utils.py:155-180; config.py:57 'IFRM').
 *      mul2: out = a * b (fp32; the channel gate y * sigmoid(gate(y)), :61-63), bwd da = d*b, db = d*a.
 *      combine: o1 = x1 + (lc*cw[1] + ls*sw[1]) * x2, o2 = x2 + (lc*cw[0] + ls*sw[0]) * x1 (:174-175);
 *      x / out (2, B, N, C), cw (B, 2C) fp32, sw (B*N, 2) un-squashed spatial logits, lc / ls device scalars.
 *      bwd: dx, dsw directly; part (nblk, 2C) per-block dcw partials (blocks image-major: B x nblk/B),
 *      lpart (2, nblk) per-block dlc / dls partials; nblk = cmx_ifrm_combine_nblk (cmx_partials_sum folds them). */
int cmx_mul2(const float* a, const float* b, float* out, int64_t n, hipStream_t stream);
/* LayerNorm of R fp32 rows of any width C (ImprovedChannelWeights' LN(4C) / LN(2C), :42,45); bwd writes dgamma / dbeta */
int cmx_rowln_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int R, int C, float eps, hipStream_t stream);
int cmx_rowln_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, float* dx, float* dgamma, float* dbeta, int R, int C, hipStream_t stream);
int cmx_mul2_bwd(const float* d, const float* a, const float* b, float* da, float* db, int64_t n, hipStream_t stream);
int cmx_ifrm_combine_nblk(int B, int N);
int cmx_ifrm_combine_fwd(const void* x, const float* cw, const void* sw, const float* lc, const float* ls, void* out, int B, int N, int C, int dtype, hipStream_t stream);
int cmx_ifrm_combine_bwd(const void* dout, const void* x, const float* cw, const void* sw, const float* lc, const float* ls, void* dx, void* dsw, float* part, float* lpart, int B, int N, int C, int dtype, hipStream_t stream);

/* ---- TrainPre augmentation on the GPU (dataloader/dataloader.py:9-112,
 *      utils/transforms.py:182-187, RGBXDataset.py:65-68), uint8 HWC images (BGR as cv2 reads them).
 *      resize: cv2.resize INTER_LINEAR (nearest = 0) / INTER_NEAREST (nearest = 1) of an h x w x C
 *      image to oh x ow, reading the source mirrored (random_mirror, mirror = 1) and clamped to
 *      [0, clip_max] (TrainPre's label clip; clip_max < 0: none).  color_jitter: in place, BGR ->
 *      HSV (8U) -> V*bf, S*sf, H+hadd (fp32) -> clip, truncate -> BGR.  blur5: cv2.GaussianBlur
 *      5x5 sigma 1 (8U fixed point, BORDER_REFLECT_101), out of place.  finalize: cutout box
 *      [bx1, bx2) x [by1, by2) (rgb/x -> 0, label -> background; empty box: none) + ensure_size
 *      resize to oh x ow (linear / nearest) + (v/255 - mean)/std in fp64 -> float CHW; labels -> int64. */
int cmx_aug_resize_u8(const uint8_t* src, int h, int w, int C, uint8_t* dst, int oh, int ow, int nearest, int mirror, int clip_max, hipStream_t stream);
int cmx_aug_color_jitter_u8(uint8_t* img, int h, int w, float bf, float sf, float hadd, hipStream_t stream);
int cmx_aug_blur5_u8(const uint8_t* src, uint8_t* dst, int h, int w, int C, hipStream_t stream);
/* the four stages above over a whole minibatch, one launch per stage (TrainPre over the
 * DataLoader's batch, dataloader.py:85-112 + the default collate).  table: device array of
 * B records of 24 int64 words: [0] rgb, [1] x (h x w x 3 u8), [2] gt (h x w u8) sources;
 * [3] rs, [4] xs (sh x sw x 3), [5] gs (sh x sw) scaled images; [6] blur output (sh x sw x 3,
 * 0 = no blur); [7] rgb_out, [8] x_out (3 x oh x ow f32), [9] gt_out (oh x ow i64) batch slots;
 * [10] h, [11] w, [12] sh, [13] sw, [14] mirror, [15..18] cutout box bx1, by1, bx2, by2 (all
 * zero: none); [19] bf, [20] sf, [21] hue add (float bits in the low 32 bits); [22..23] 0.
 * max_sh / max_sw bound every record's sh / sw. */
int cmx_aug_batch(const int64_t* table, int B, int max_sh, int max_sw, int oh, int ow, int clip_max, int background, double m0, double m1, double m2, double s0, double s1, double s2, hipStream_t stream);
int cmx_aug_finalize(const uint8_t* rgb, const uint8_t* x, const uint8_t* gt, int h, int w, int oh, int ow, int bx1, int by1, int bx2, int by2, int background, double m0, double m1, double m2, double s0, double s1, double s2, float* rgb_out, float* x_out, int64_t* gt_out, hipStream_t stream);

/* ---- evaluation (engine/evaluator.py:306-396, utils/metric.py:8-15, eval.py:23-36).
 *      seg_window_accumulate: one sliding-window crop -- acc[k, sy+i, sx+j] += exp(s1[k, m0+i, m2+j]
 *      (+ s2[k, m0+i, cw-1-(m2+j)] when s2, the is_flip pass)), s1/s2 (K, ch, cw) fp32 logits of the crop,
 *      margins m0..m3 = top/bottom/left/right padding of the crop (pad_image_to_shape), acc (K, PH, PW) fp32.
 *      seg_argmax_confusion: pred = first argmax over K of score (K, HW) fp32; for labels in [0, n_cl):
 *      hist[n_cl*gt + pred] += 1, counts[0] (labeled) += 1, counts[1] (correct) += pred == gt.  hist (n_cl*n_cl)
 *      and counts (2) are int64 and ACCUMULATE; pred (int32, HW) may be NULL; label_dtype 0 = int64, 1 = uint8.
 *      score == NULL: pred is an INPUT class map (hist_info(n_cl, pred, gt)). */
int cmx_seg_window_accumulate(const float* s1, const float* s2, float* acc, int K, int ch, int cw, int m0, int m1, int m2, int m3, int PH, int PW, int sy, int sx, hipStream_t stream);
int cmx_seg_argmax_confusion(const float* score, int K, int64_t HW, const void* label, int label_dtype, int n_cl, int* pred, int64_t* hist, int64_t* counts, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
