// Evaluation kernels: the sliding-window evaluator's score accumulation and
// the mIoU confusion matrix, on the device, so a validation pass never copies a (K, H, W) score
// map to the host.
//
//  * cmx_seg_window_accumulate -- one crop of Evaluator.scale_process_rgbX
//    (engine/evaluator.py:345-368 with val_func_process_rgbX :374-396): the crop's logits
//    (and, with is_flip, the logits of the mirrored crop, mirrored back) are summed, exp'd and
//    added into the padded scale accumulator at (s_y, s_x), after dropping the crop's own
//    padding margin:  acc[k, s_y + i, s_x + j] += exp(s1[k, m0 + i, m2 + j]
//                                                     (+ s2[k, m0 + i, cw - 1 - (m2 + j)]))
//    The reference computes exp(score + flip(score_flip)) in fp32 and accumulates in fp32 on the
//    GPU, in the same order per element, so this is bit-exact against it.
//  * cmx_seg_argmax_confusion -- pred = argmax over classes of a (K, HW) score (numpy's
//    processed_pred.argmax(2): first maximum wins, evaluator.py:322) fused with hist_info
//    (utils/metric.py:8-15): for labels in [0, n_cl), hist[n_cl * gt + pred] += 1,
//    labeled += 1, correct += (pred == gt).  Integer counts: LDS-privatised per block
//    (32-bit LDS atomics), flushed with 64-bit global atomics -- order-independent, bit-exact.
//    With score == NULL the class map is READ from `pred` instead (hist_info(n_cl, pred, gt)).
//    Predictions outside [0, n_cl) count as labeled but land in no bin (numpy's bincount of
//    n_cl * gt + pred would shift them into a neighbouring bin or fail; the evaluator never
//    produces them).  The counts ACCUMULATE (the caller zeroes them once per validation pass), which is what
//    SegEvaluator.compute_metric does on the host (eval.py:69-78).
// Both kernels are HBM-bound: window accumulate reads K*ch*cw*(1 or 2) floats and
// read-modify-writes K*h*w; argmax+confusion reads K*HW floats + HW labels once.
#include "cmx_common.h"

namespace {

// one (class, crop row) per blockIdx.y row-chunk; lanes along the row (coalesced, no 64-bit
// index division per element)
__global__ void window_acc_kernel(const float* __restrict__ s1, const float* __restrict__ s2, float* __restrict__ acc,
                                  int K, int ch, int cw, int m0, int m2, int h, int w, int PH, int PW, int sy, int sx) {
  const int rows = K * h;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const int k = r / h, i = r - k * h;
    const float* a = s1 + ((long)k * ch + m0 + i) * cw;
    const float* b = s2 ? s2 + ((long)k * ch + m0 + i) * cw : nullptr;
    float* o = acc + ((long)k * PH + sy + i) * PW + sx;
    for (int j = threadIdx.x; j < w; j += blockDim.x) {
      float v = a[m2 + j];
      if (b) v += b[cw - 1 - (m2 + j)];
      o[j] += expf(v);
    }
  }
}

constexpr int CONF_THREADS = 256;

template <typename L>
__global__ __launch_bounds__(CONF_THREADS) void argmax_conf_kernel(const float* __restrict__ score, int K, long HW,
                                                                   const L* __restrict__ label, int n_cl,
                                                                   int* __restrict__ pred,
                                                                   unsigned long long* __restrict__ hist,
                                                                   unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned int sh[];            // n_cl * n_cl bins + labeled + correct
  const int nb = n_cl * n_cl;
  for (int b = threadIdx.x; b < nb + 2; b += blockDim.x) sh[b] = 0u;
  __syncthreads();
  unsigned int lab = 0, cor = 0;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += (long)gridDim.x * blockDim.x) {
    int bi;
    if (score) {
      // first maximum over classes (consecutive threads: consecutive pixels of one class row)
      // 8 class rows in flight per step (loads first, then the ordered comparisons)
      float best = score[p];
      bi = 0;
      bool bnan = best != best;
      for (int k0 = 1; k0 < K; k0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = k0 + u < K ? score[(long)(k0 + u) * HW + p] : -INFINITY;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (k0 + u < K && !bnan && (v[u] > best || v[u] != v[u])) {
            best = v[u];
            bi = k0 + u;
            bnan = v[u] != v[u];
          }
        }
      }
      if (pred) pred[p] = bi;
    } else {
      bi = pred[p];                               // hist_info on a given class map
    }
    const long long g = (long long)label[p];
    if (g >= 0 && g < n_cl) {
      ++lab;
      cor += (bi == (int)g);
      if (bi >= 0 && bi < n_cl) atomicAdd(&sh[(int)g * n_cl + bi], 1u);
    }
  }
  // per-thread labeled / correct -> LDS
  if (lab) atomicAdd(&sh[nb], lab);
  if (cor) atomicAdd(&sh[nb + 1], cor);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (sh[b]) atomicAdd(&hist[b], (unsigned long long)sh[b]);
  if (threadIdx.x == 0) {
    if (sh[nb]) atomicAdd(&counts[0], (unsigned long long)sh[nb]);
    if (sh[nb + 1]) atomicAdd(&counts[1], (unsigned long long)sh[nb + 1]);
  }
}

}  // namespace

extern "C" {

int cmx_seg_window_accumulate(const float* s1, const float* s2, float* acc, int K, int ch, int cw, int m0, int m1,
                              int m2, int m3, int PH, int PW, int sy, int sx, hipStream_t s) {
  const int h = ch - m0 - m1, w = cw - m2 - m3;
  CMX_REQUIRE(K > 0 && h > 0 && w > 0 && m0 >= 0 && m1 >= 0 && m2 >= 0 && m3 >= 0, CMX_ERR_SHAPE,
              "seg_window_accumulate: K=%d crop %dx%d margins %d %d %d %d", K, ch, cw, m0, m1, m2, m3);
  CMX_REQUIRE(sy >= 0 && sx >= 0 && sy + h <= PH && sx + w <= PW, CMX_ERR_SHAPE,
              "seg_window_accumulate: window (%d, %d) + %dx%d outside %dx%d", sy, sx, h, w, PH, PW);
  const long rows = (long)K * h;
  const unsigned blocks = (unsigned)(rows < 65536 ? rows : 65536);
  hipLaunchKernelGGL(window_acc_kernel, dim3(blocks), dim3(w >= 256 ? 256 : 64 * ((w + 63) / 64)), 0, s, s1, s2, acc,
                     K, ch, cw, m0, m2, h, w, PH, PW, sy, sx);
  return cmx_check_launch("seg_window_accumulate");
}

int cmx_seg_argmax_confusion(const float* score, int K, int64_t HW, const void* label, int label_dtype, int n_cl,
                             int* pred, int64_t* hist, int64_t* counts, hipStream_t s) {
  CMX_REQUIRE(score ? K > 0 : pred != nullptr, CMX_ERR_ARG, "seg_argmax_confusion: no score and no pred map");
  CMX_REQUIRE(HW > 0 && n_cl > 0 && n_cl <= 181, CMX_ERR_SHAPE,
              "seg_argmax_confusion: K=%d HW=%ld n_cl=%d (n_cl^2 bins must fit LDS)", K, (long)HW, n_cl);
  CMX_REQUIRE(label_dtype == 0 || label_dtype == 1, CMX_ERR_DTYPE,
              "seg_argmax_confusion: label dtype %d (0 = int64, 1 = uint8)", label_dtype);
  long blocks = (HW + CONF_THREADS - 1) / CONF_THREADS;
  if (blocks > 1024) blocks = 1024;
  const size_t sm = (size_t)(n_cl * n_cl + 2) * sizeof(unsigned int);
  auto* h = reinterpret_cast<unsigned long long*>(hist);
  auto* c = reinterpret_cast<unsigned long long*>(counts);
  if (label_dtype == 0)
    hipLaunchKernelGGL(argmax_conf_kernel<long long>, dim3((unsigned)blocks), dim3(CONF_THREADS), sm, s, score, K,
                       (long)HW, (const long long*)label, n_cl, pred, h, c);
  else
    hipLaunchKernelGGL(argmax_conf_kernel<unsigned char>, dim3((unsigned)blocks), dim3(CONF_THREADS), sm, s, score, K,
                       (long)HW, (const unsigned char*)label, n_cl, pred, h, c);
  return cmx_check_launch("seg_argmax_confusion");
}

}  // extern "C"
