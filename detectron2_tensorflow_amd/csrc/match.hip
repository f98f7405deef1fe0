// IoU + Matcher fused: the pairwise IoU of ground truth against anchors /
// proposals (box_list_ops.pairwise_iou, :295-372) and Matcher.__call__
// (lib/modeling/matcher.py:8-173) without materialising the [N, G, P] IoU
// matrix or the dozen [N, P] passes of the tensor formulation.
//
//  best_gt_kernel (low-quality matches only): per valid GT, the max IoU over
//    all P boxes -- per-workgroup maxima combined with an atomic max on the
//    order-preserving integer image of the float (exact: max is order-free).
//  match_kernel: per box, the first GT of maximal IoU among valid GT, the
//    threshold labels, the low-quality hits (IoU == that GT's best), no-GT ->
//    background, then crowd (-1 where background and max crowd IoU > 1e-3)
//    and difficult (-1 where background and max difficult IoU > thr[1]).
//
// IoU float sequence: ih = min(y2a,y2b) - max(y1a,y1b) clamped at 0, iw the
// same, inter = ih * iw, union = (area_a + area_b) - inter, inter / union
// (0 when union == 0): the tensor code's order, so labels are identical.
#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kMaxGt = 256;
// boxes per thread of best_gt_kernel: each workgroup ends in one device-scope
// atomic max per GT, and those serialize per address across the XCDs, so
// fewer, fuller workgroups (r6: 16 per thread, 4,096 boxes per workgroup;
// 4 before: 263 atomics per GT per image at 1333x800)
constexpr int kBestPer = 16;

__device__ __forceinline__ float iou_of(const float4 a, const float4 b) {
  const float ih = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
  const float iw = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
  const float inter = ih * iw;
  const float area_a = (a.z - a.x) * (a.w - a.y);
  const float area_b = (b.z - b.x) * (b.w - b.y);
  const float uni = area_a + area_b - inter;
  return uni == 0.f ? 0.f : inter / uni;
}

__device__ __forceinline__ unsigned ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

struct MatchConf {
  float thr[5];  // interval bounds (thr[0] = -inf ... thr[n] = +inf)
  int lab[4];
  int n;
  int allow_low;
  float crowd_thr, diff_thr;
};

// flags: bit0 valid (matchable), bit1 crowd, bit2 difficult -- packed int32
// per GT, or (packed null) three byte masks (crowd / difficult nullable):
// d2mi_match_boxes_ex takes the bool tensors as they are, no packing passes,
// and matches against the valid GT that are neither crowd nor difficult (the
// reference's valid_gt_boxlist, rpn_outputs.py:255-264, roi_heads.py:160-180).
struct FlagSrc {
  const int* packed;
  const uint8_t* m;
  const uint8_t* c;
  const uint8_t* d;
};
__device__ __forceinline__ int flag_at(const FlagSrc& f, size_t i) {
  if (f.packed) return f.packed[i];
  const bool c = f.c && f.c[i], d = f.d && f.d[i];
  return (f.m[i] && !c && !d ? 1 : 0) | (c ? 2 : 0) | (d ? 4 : 0);
}

__global__ __launch_bounds__(256) void best_gt_kernel(const float4* __restrict__ gt,
                                                      const FlagSrc flags,
                                                      const float4* __restrict__ boxes,
                                                      long long box_stride, int G, int P,
                                                      unsigned* __restrict__ best) {
  __shared__ float4 g_s[kMaxGt];
  __shared__ int f_s[kMaxGt];
  __shared__ float red[4];
  const int n = blockIdx.y;
  for (int g = threadIdx.x; g < G; g += 256) {
    g_s[g] = gt[(size_t)n * G + g];
    f_s[g] = flag_at(flags, (size_t)n * G + g);
  }
  __syncthreads();
  constexpr int kPer = kBestPer;
  float4 b[kPer];
  bool ok[kPer];
  const int p0 = blockIdx.x * 256 * kPer + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int p = p0 + k * 256;
    ok[k] = p < P;
    b[k] = ok[k] ? boxes[n * box_stride + p] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int g = 0; g < G; ++g) {
    if (!(f_s[g] & 1)) continue;  // block-uniform
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (ok[k]) m = fmaxf(m, iou_of(g_s[g], b[k]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) red[wv] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      atomicMax(&best[(size_t)n * G + g], ord(bm));
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void match_kernel(const float4* __restrict__ gt,
                                                    const FlagSrc flags,
                                                    const float4* __restrict__ boxes,
                                                    long long box_stride, int G, int P,
                                                    MatchConf c, const unsigned* __restrict__ best,
                                                    long long* __restrict__ matches,
                                                    long long* __restrict__ labels) {
  __shared__ float4 g_s[kMaxGt];
  __shared__ int f_s[kMaxGt];
  __shared__ float b_s[kMaxGt];
  const int n = blockIdx.y;
  for (int g = threadIdx.x; g < G; g += 256) {
    g_s[g] = gt[(size_t)n * G + g];
    f_s[g] = flag_at(flags, (size_t)n * G + g);
    b_s[g] = (c.allow_low && (f_s[g] & 1)) ? unord(best[(size_t)n * G + g]) : 0.f;
  }
  __syncthreads();
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float4 b = boxes[n * box_stride + p];
  float v = -INFINITY, crowd = 0.f, diff = 0.f;
  int arg = 0;
  bool any = false, hit = false;
  for (int g = 0; g < G; ++g) {
    const int f = f_s[g];
    if (!(f & 7)) continue;
    const float q = iou_of(g_s[g], b);
    if (f & 1) {
      any = true;
      if (q > v) {
        v = q;
        arg = g;
      }
      if (c.allow_low && q == b_s[g]) hit = true;
    }
    if (f & 2) crowd = fmaxf(crowd, q);
    if (f & 4) diff = fmaxf(diff, q);
  }
  long long lab = 0;
  for (int i = 0; i < c.n; ++i)
    if (v >= c.thr[i] && v < c.thr[i + 1]) lab = c.lab[i];
  if (hit) lab = 1;
  if (!any) {
    lab = 0;
    arg = 0;
  }
  if (lab == 0 && crowd > c.crowd_thr) lab = -1;
  if (lab == 0 && diff > c.diff_thr) lab = -1;
  matches[(size_t)n * P + p] = arg;
  labels[(size_t)n * P + p] = lab;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_match_workspace_size(int N, int G) {
  return (size_t)(N > 0 ? N : 0) * (size_t)(G > 0 ? G : 0) * sizeof(unsigned);
}

static int match_core(const float* gt_boxes, FlagSrc gt_flags, const float* boxes,
                      int boxes_per_image, int N, int G, int P, const float* thresholds,
                      const int* labels_of, int n_intervals, int allow_low_quality,
                      float crowd_thr, float difficult_thr, long long* matches, long long* labels,
                      void* workspace, size_t workspace_bytes, void* stream);

extern "C" int d2mi_match_boxes(const float* gt_boxes, const int* gt_flags, const float* boxes,
                                int boxes_per_image, int N, int G, int P,
                                const float* thresholds, const int* labels_of, int n_intervals,
                                int allow_low_quality, float crowd_thr, float difficult_thr,
                                long long* matches, long long* labels, void* workspace,
                                size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(gt_flags != nullptr || G == 0, "match: null flags");
  return match_core(gt_boxes, FlagSrc{gt_flags, nullptr, nullptr, nullptr}, boxes,
                    boxes_per_image, N, G, P, thresholds, labels_of, n_intervals,
                    allow_low_quality, crowd_thr, difficult_thr, matches, labels, workspace,
                    workspace_bytes, stream);
}

extern "C" int d2mi_match_boxes_ex(const float* gt_boxes, const uint8_t* valid,
                                   const uint8_t* crowd, const uint8_t* difficult,
                                   const float* boxes, int boxes_per_image, int N, int G, int P,
                                   const float* thresholds, const int* labels_of, int n_intervals,
                                   int allow_low_quality, float crowd_thr, float difficult_thr,
                                   long long* matches, long long* labels, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(valid != nullptr || G == 0, "match: null valid mask");
  return match_core(gt_boxes, FlagSrc{nullptr, valid, crowd, difficult}, boxes,
                    boxes_per_image, N, G, P, thresholds, labels_of, n_intervals,
                    allow_low_quality, crowd_thr, difficult_thr, matches, labels, workspace,
                    workspace_bytes, stream);
}

static int match_core(const float* gt_boxes, FlagSrc gt_flags, const float* boxes,
                      int boxes_per_image, int N, int G, int P, const float* thresholds,
                      const int* labels_of, int n_intervals, int allow_low_quality,
                      float crowd_thr, float difficult_thr, long long* matches, long long* labels,
                      void* workspace, size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N > 0 && G >= 0 && P >= 0, "bad match shape");
  D2MI_REQUIRE(G <= kMaxGt, "match: at most %d ground-truth boxes per image (got %d)", kMaxGt, G);
  D2MI_REQUIRE(n_intervals >= 1 && n_intervals <= 4, "match: 1..4 threshold intervals");
  D2MI_REQUIRE(((uintptr_t)gt_boxes & 15) == 0 && ((uintptr_t)boxes & 15) == 0,
               "match: boxes must be 16-byte aligned");
  if (P == 0) return 0;
  MatchConf c;
  for (int i = 0; i <= n_intervals; ++i) c.thr[i] = thresholds[i];
  for (int i = 0; i < n_intervals; ++i) c.lab[i] = labels_of[i];
  c.n = n_intervals;
  c.allow_low = allow_low_quality && G > 0;
  c.crowd_thr = crowd_thr;
  c.diff_thr = difficult_thr;
  const long long bstride = boxes_per_image ? (long long)P : 0;
  hipStream_t st = as_stream(stream);
  unsigned* best = static_cast<unsigned*>(workspace);
  if (c.allow_low) {
    D2MI_REQUIRE(workspace && workspace_bytes >= d2mi_match_workspace_size(N, G),
                 "match workspace too small");
    D2MI_REQUIRE(fill_bytes(best, d2mi_match_workspace_size(N, G), 0, st) == 0, "fill failed");
    hipLaunchKernelGGL(best_gt_kernel, dim3((P + 256 * kBestPer - 1) / (256 * kBestPer), N), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(gt_boxes), gt_flags,
                       reinterpret_cast<const float4*>(boxes), bstride, G, P, best);
    D2MI_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(match_kernel, dim3((P + 255) / 256, N), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(gt_boxes), gt_flags,
                     reinterpret_cast<const float4*>(boxes), bstride, G, P, c, best, matches,
                     labels);
  D2MI_LAUNCH_CHECK();
  return 0;
}
