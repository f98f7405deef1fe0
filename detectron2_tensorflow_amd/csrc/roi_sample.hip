// The ROI heads' label / take / mask-prep glue around the fused matcher and
// sampler, as two launches (lib/modeling/roi_heads/roi_heads.py:100-232
// label_and_sample_proposals, :35-62 select_foreground_proposals):
//   d2mi_roi_gt_classes   the per-proposal training class from the matcher's
//                         (matches, labels) -- torch's form is a gather and
//                         three selects;
//   d2mi_roi_sample_take  the sampled rows (boxes, class, matched GT row, GT
//                         box) in the sampler's order, and the mask branch's
//                         inputs over the first F slots per image in stable
//                         foreground-first order with the foreground count --
//                         torch's form is ~20 small launches (gathers, a
//                         strided-slice copy per tensor, a stable argsort, six
//                         index gathers, a sum), 4-28 us each.
// Pure data movement and comparisons: the outputs are the same values.
#include "common.h"

namespace d2mi {
namespace {

// one thread per (image, proposal)
__global__ __launch_bounds__(256) void roi_gt_classes_kernel(
    const int64_t* __restrict__ labels, const int64_t* __restrict__ matches,
    const void* __restrict__ gt_cls, int gt_cls_64, const uint8_t* __restrict__ pvalid, int N,
    int M, int G, int K, int64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * M) return;
  const int n = i / M;
  const int64_t lab = labels[i];
  int64_t v;
  if (lab == 1) {
    const int64_t g = matches[i];
    v = gt_cls_64 ? reinterpret_cast<const int64_t*>(gt_cls)[(size_t)n * G + g]
                  : (int64_t)reinterpret_cast<const int32_t*>(gt_cls)[(size_t)n * G + g];
  } else {
    v = lab == 0 ? (int64_t)K : lab;
  }
  out[i] = pvalid[i] ? v : (int64_t)-1;
}

constexpr int kTakeT = 1024;

// One workgroup: the take over every sampled slot, then the mask stage over
// the first F slots of each image (a workgroup scan for the stable order).
// The mask stage re-reads the sources (order -> proposal -> matched GT), not
// the take's outputs: nothing written here is read back.
__global__ __launch_bounds__(kTakeT) void roi_sample_take_kernel(
    const int64_t* __restrict__ order, const uint8_t* __restrict__ valid,
    const float4* __restrict__ boxes, const int64_t* __restrict__ gt_classes,
    const int64_t* __restrict__ matches, const float4* __restrict__ gt_boxes, int N, int M, int S,
    int G, int F, int K, float4* __restrict__ s_boxes, int64_t* __restrict__ s_cls,
    int64_t* __restrict__ s_gidx, float4* __restrict__ s_gtb, float4* __restrict__ m_boxes,
    int64_t* __restrict__ m_cls, uint8_t* __restrict__ m_fg, int32_t* __restrict__ m_img,
    int64_t* __restrict__ m_mind, float4* __restrict__ m_gtb, uint8_t* __restrict__ fg_all,
    int64_t* __restrict__ count) {
  __shared__ int s_wave[kTakeT / 64];
  __shared__ int s_run;  // foreground rows placed by earlier chunks
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = t; i < N * S; i += kTakeT) {
    const int n = i / S;
    const size_t p = (size_t)n * M + order[i];
    const int64_t g = matches[p];
    s_boxes[i] = boxes[p];
    s_cls[i] = gt_classes[p];
    s_gidx[i] = g;
    s_gtb[i] = gt_boxes[(size_t)n * G + g];
  }
  if (F == 0) return;
  const int R = N * F;
  // pass 1: the foreground count (every chunk's position needs it for the
  // background rows)
  int mine = 0;
  for (int i = t; i < R; i += kTakeT) {
    const int n = i / F, j = i - n * F;
    const int q = n * S + j;
    const size_t p = (size_t)n * M + order[q];
    mine += (valid[q] && gt_classes[p] < K) ? 1 : 0;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mine += __shfl_xor(mine, d);
  if (lane == 0) s_wave[w] = mine;
  if (t == 0) s_run = 0;
  __syncthreads();
  int total = 0;
#pragma unroll
  for (int k = 0; k < kTakeT / 64; ++k) total += s_wave[k];
  if (t == 0) count[0] = total;
  __syncthreads();  // (s_wave reused below)
  // pass 2: chunks of kTakeT rows in index order; a row's place is its rank
  // among its kind (foreground rows first, then the rest, index order each)
  for (int c0 = 0; c0 < R; c0 += kTakeT) {
    const int i = c0 + t;
    const bool live = i < R;
    const int n = live ? i / F : 0, j = live ? i - n * F : 0;
    const int q = n * S + j;
    size_t p = 0;
    bool fg = false;
    if (live) {
      p = (size_t)n * M + order[q];
      fg = valid[q] && gt_classes[p] < K;
    }
    const uint64_t bal = __ballot(fg);
    const int below = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[w] = __popcll(bal);
    __syncthreads();
    int before = s_run;  // foreground rows of earlier chunks
#pragma unroll
    for (int k = 0; k < kTakeT / 64; ++k) before += k < w ? s_wave[k] : 0;
    const int fg_rank = before + below;
    __syncthreads();
    if (t == kTakeT - 1) s_run = fg_rank + (fg ? 1 : 0);
    if (live) {
      const int pos = fg ? fg_rank : total + (i - fg_rank);
      const int64_t g = matches[p];
      fg_all[i] = fg ? 1 : 0;
      m_boxes[pos] = boxes[p];
      m_cls[pos] = gt_classes[p];
      m_fg[pos] = fg ? 1 : 0;
      m_img[pos] = n;
      m_mind[pos] = g + (int64_t)n * G;
      m_gtb[pos] = gt_boxes[(size_t)n * G + g];
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_roi_gt_classes(const int64_t* labels, const int64_t* matches,
                                   const void* gt_cls, int gt_cls_64, const uint8_t* pvalid, int N,
                                   int M, int G, int K, int64_t* out, void* stream) {
  D2MI_REQUIRE(N > 0 && M > 0 && G > 0 && (long long)N * M < (1LL << 31), "bad gt-classes shape");
  D2MI_REQUIRE(labels && matches && gt_cls && pvalid && out, "gt classes: null operand");
  const int n = N * M;
  hipLaunchKernelGGL(roi_gt_classes_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     as_stream(stream), labels, matches, gt_cls, gt_cls_64 ? 1 : 0, pvalid, N, M,
                     G, K, out);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_roi_sample_take(const int64_t* order, const uint8_t* valid,
                                    const float* boxes, const int64_t* gt_classes,
                                    const int64_t* matches, const float* gt_boxes, int N, int M,
                                    int S, int G, int F, int K, float* s_boxes, int64_t* s_cls,
                                    int64_t* s_gidx, float* s_gtb, float* m_boxes, int64_t* m_cls,
                                    uint8_t* m_fg, int32_t* m_img, int64_t* m_mind, float* m_gtb,
                                    uint8_t* fg_all, int64_t* count, void* stream) {
  D2MI_REQUIRE(N > 0 && M > 0 && S > 0 && G > 0 && F >= 0 && F <= S &&
                   (long long)N * S < (1LL << 30) && (long long)N * M < (1LL << 31),
               "bad sample-take shape");
  D2MI_REQUIRE(order && valid && boxes && gt_classes && matches && gt_boxes && s_boxes && s_cls &&
                   s_gidx && s_gtb,
               "sample take: null operand");
  D2MI_REQUIRE(F == 0 || (m_boxes && m_cls && m_fg && m_img && m_mind && m_gtb && fg_all && count),
               "sample take: null mask-stage operand");
  const void* v4[] = {boxes, gt_boxes, s_boxes, s_gtb, m_boxes, m_gtb};
  for (const void* p : v4)
    D2MI_REQUIRE(((uintptr_t)p & 15) == 0, "sample take: box arrays must be 16-byte aligned");
  hipLaunchKernelGGL(roi_sample_take_kernel, dim3(1), dim3(kTakeT), 0, as_stream(stream), order,
                     valid, reinterpret_cast<const float4*>(boxes), gt_classes, matches,
                     reinterpret_cast<const float4*>(gt_boxes), N, M, S, G, F, K,
                     reinterpret_cast<float4*>(s_boxes), s_cls, s_gidx,
                     reinterpret_cast<float4*>(s_gtb), reinterpret_cast<float4*>(m_boxes), m_cls,
                     m_fg, m_img, m_mind, reinterpret_cast<float4*>(m_gtb), fg_all, count);
  D2MI_LAUNCH_CHECK();
  return 0;
}
