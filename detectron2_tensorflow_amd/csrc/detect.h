// Detection helpers shared by the proposal / post-processing translation
// units (proposals.hip, topk.hip, retina_post.hip): per-level anchor geometry,
// box-delta configuration, and the sigmoid-key search of the dense top-k.
#pragma once
#include "internal.h"

namespace d2mi {

constexpr int kMaxA = 12;

// Per-level geometry of a pyramid's score / delta tensors and its anchors.
struct Levels {
  int64_t off_a[D2MI_MAX_LEVELS];  // element offset of level l's tensor from base_a
  int64_t off_b[D2MI_MAX_LEVELS];  // element offset of level l's tensor from base_b
  // image strides of level l's tensors (a: elements per K, b: float4s); by
  // default H * W * A (each level a dense [N, H, W, A(*K)] tensor)
  int64_t img_a[D2MI_MAX_LEVELS];
  int64_t img_b[D2MI_MAX_LEVELS];
  int H[D2MI_MAX_LEVELS], W[D2MI_MAX_LEVELS];
  int stride[D2MI_MAX_LEVELS];
  float cell[D2MI_MAX_LEVELS][kMaxA][4];
  int L, A;
};

// Anchor a at flat position hw of level l (anchor_generator.py:31-40, :92-109).
__device__ __forceinline__ float4 anchor_at(const Levels& lv, int l, int hw, int a) {
  const int h = hw / lv.W[l], w = hw - h * lv.W[l];
  // tf.range(0, H*stride, stride) cast to float32, then + cell anchor (float32)
  const float sy = (float)(h * lv.stride[l]);
  const float sx = (float)(w * lv.stride[l]);
  return make_float4(sy + lv.cell[l][a][0], sx + lv.cell[l][a][1], sy + lv.cell[l][a][2],
                     sx + lv.cell[l][a][3]);
}

struct DeltaCfg {
  float wy, wx, wh, ww, clamp;
};

// Host: fills lv from the per-level pointers / shapes (error code on bad input).
int make_levels(Levels& lv, const float* const* a_ptrs, const float* const* b_ptrs,
                const int32_t* level_hw, const float* strides, const float* cell, int L, int A);
DeltaCfg make_dc(const float* w4, float clamp);

// tf.nn.sigmoid as the oracle states it (1 / (1 + exp(-x)), float32).
__device__ __forceinline__ float sigmoidf_tf(float v) { return 1.f / (1.f + expf(-v)); }

constexpr uint32_t kKeyNegInf = 0x007fffffu;  // orderable(-inf)
constexpr uint32_t kKeyPosInf = 0xff800000u;  // orderable(+inf)
constexpr uint32_t kWindowMargin = 256;       // keys below a solved tie edge still tested

// sigmoid(from_orderable(u)) over a key range, as a function of the key:
// monotone non-decreasing (sigmoid is).  Smallest key in [lo, hi] whose
// sigmoid is >= s, or hi + 1.
__device__ inline uint32_t lower_bound_sig(uint32_t lo, uint32_t hi, float s) {
  uint32_t a = lo, b = hi + 1;  // search [a, b)
  while (a < b) {
    const uint32_t m = a + ((b - a) >> 1);
    if (sigmoidf_tf(from_orderable(m)) >= s) b = m;
    else a = m + 1;
  }
  return a;
}
// Largest key in [lo, hi] whose sigmoid is <= s (lo's sigmoid must be <= s).
__device__ inline uint32_t upper_bound_sig(uint32_t lo, uint32_t hi, float s) {
  uint32_t a = lo, b = hi;
  while (a < b) {
    const uint32_t m = a + ((b - a + 1) >> 1);
    if (sigmoidf_tf(from_orderable(m)) <= s) a = m;
    else b = m - 1;
  }
  return a;
}
// The same two searches by one whole wave (every lane calls with the same
// arguments and gets the same result): each round the 64 lanes test the last
// key of 64 equal chunks of the range, so 2^32 keys take 6 rounds of one
// sigmoid per lane instead of 32 dependent ones.  gt = false: smallest key in
// [lo, hi] whose sigmoid is >= s, or hi + 1 (lower_bound_sig); gt = true:
// smallest key whose sigmoid is > s, or hi + 1.
__device__ inline uint32_t wave_bound_sig(uint32_t lo, uint32_t hi, float s, bool gt) {
  const uint64_t lane = threadIdx.x & 63;
  uint64_t a = lo, b = (uint64_t)hi + 1;  // search [a, b)
  while (a < b) {
    const uint64_t step = (b - a + 63) >> 6;
    uint64_t m = a + (lane + 1) * step - 1;
    if (m > b - 1) m = b - 1;
    const float sm = sigmoidf_tf(from_orderable((uint32_t)m));
    const uint64_t bal = __ballot(gt ? sm > s : sm >= s);  // monotone in the lane
    if (bal == 0) return (uint32_t)b;  // (only when b = hi + 1: the range never shrinks from above otherwise)
    const uint64_t f = (uint64_t)(__ffsll((unsigned long long)bal) - 1);
    if (step == 1) return (uint32_t)(a + f);
    const uint64_t mf = a + (f + 1) * step - 1 < b - 1 ? a + (f + 1) * step - 1 : b - 1;
    a = a + f * step;  // the previous chunk's last key failed
    b = mf + 1;        // mf satisfies: the answer is <= mf
  }
  return (uint32_t)a;
}
__device__ inline uint32_t wave_lower_bound_sig(uint32_t lo, uint32_t hi, float s) {
  return wave_bound_sig(lo, hi, s, false);
}
// upper_bound_sig by one wave: the key before the first whose sigmoid is > s.
__device__ inline uint32_t wave_upper_bound_sig(uint32_t lo, uint32_t hi, float s) {
  return wave_bound_sig(lo, hi, s, true) - 1;
}

// RetinaNet inference in four launches (retina_post.hip).
bool retina_fused_eligible(int L, int k, int max_det);
size_t retina_fused_workspace_size(int N, int L, const int32_t* level_hw, int A, int K, int k);
int retinanet_fused(const float* const* cls, const float* const* box, const Levels& lv,
                    const int32_t* level_hw, int K, int N, int k, float score_thresh,
                    float nms_thresh, int max_det, DeltaCfg dc, float* out_boxes,
                    float* out_scores, int32_t* out_classes, uint8_t* out_valid, void* workspace,
                    size_t workspace_bytes, hipStream_t st, bool force_exact);

}  // namespace d2mi
