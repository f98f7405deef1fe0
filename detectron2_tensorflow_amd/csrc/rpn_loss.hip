// RPN losses in two passes (rpn_outputs.py:306-401, RPNOutputs.losses):
// the sigmoid cross-entropy of the objectness logits over the sampled
// anchors and the smooth-L1 of the box deltas over the positive anchors,
// with the regression targets (box_regression.py:38-74, get_deltas) formed
// on the fly from the anchor and its matched ground truth -- instead of the
// gather / encode / cat / where / loss / sum chain of ~30 tensor passes over
// [N, 268,569(, 4)].  Forward: per-workgroup partial sums (summed in a fixed
// order by the caller); backward: d logits = g_cls (sigmoid(x) - z) on the
// sampled anchors, d deltas = g_loc smooth-L1'(p - t) on the positives, with
// (g_cls, g_loc) read from the device (no host synchronisation).
// Element formulas follow ATen's binary_cross_entropy_with_logits and the
// smooth_l1_loss of layers/loss.py.
#include "common.h"

namespace d2mi {
namespace {

struct RpnLossArgs {
  const float* logits;        // [N, P]
  const float4* deltas;       // [N, P] float4
  const float4* anchors;      // [P]
  const float4* gt;           // [N, G]
  const long long* matches;   // [N, P]
  const unsigned char* pos;   // [N, P]
  const unsigned char* samp;  // [N, P]
  int N, P, G;
  float wy, wx, wh, ww, beta;
};

__device__ __forceinline__ float4 target_of(const RpnLossArgs& a, int n, int p) {
  const float4 s = a.anchors[p];
  const float4 t = a.gt[(size_t)n * a.G + (int)a.matches[(size_t)n * a.P + p]];
  const float sh = s.z - s.x, sw = s.w - s.y;
  const float scy = s.x + 0.5f * sh, scx = s.y + 0.5f * sw;
  const float th = t.z - t.x, tw = t.w - t.y;
  const float tcy = t.x + 0.5f * th, tcx = t.y + 0.5f * tw;
  return make_float4(a.wy * (tcy - scy) / sh, a.wx * (tcx - scx) / sw, a.wh * logf(th / sh),
                     a.ww * logf(tw / sw));
}

__device__ __forceinline__ float sl1(float t, float p, float beta) {
  const float d = fabsf(t - p);
  return beta < 1e-5f ? d : (d < beta ? 0.5f * (d * d) / beta : d - 0.5f * beta);
}

__device__ __forceinline__ float sl1_grad(float t, float p, float beta) {
  const float d = p - t;  // d|t - p| / dp = sign(p - t)
  const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  if (beta < 1e-5f) return sg;
  return fabsf(d) < beta ? d / beta : sg;
}

__global__ __launch_bounds__(256) void rpn_loss_fwd_kernel(RpnLossArgs a, float2* __restrict__ part) {
  __shared__ float2 red[4];
  const int n = blockIdx.y;
  float cls = 0.f, loc = 0.f;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < a.P; p += gridDim.x * 256) {
    const size_t i = (size_t)n * a.P + p;
    if (a.samp[i]) {
      const float x = a.logits[i], z = a.pos[i] ? 1.f : 0.f;
      const float m = fmaxf(-x, 0.f);
      cls += (1.f - z) * x + m + logf(expf(-m) + expf(-x - m));
    }
    if (a.pos[i]) {
      const float4 t = target_of(a, n, p), d = a.deltas[i];
      loc += ((sl1(t.x, d.x, a.beta) + sl1(t.y, d.y, a.beta)) + sl1(t.z, d.z, a.beta)) +
             sl1(t.w, d.w, a.beta);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cls += __shfl_down(cls, o, 64);
    loc += __shfl_down(loc, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = make_float2(cls, loc);
  __syncthreads();
  if (threadIdx.x == 0) {
    float2 s = red[0];
    for (int k = 1; k < 4; ++k) {
      s.x += red[k].x;
      s.y += red[k].y;
    }
    part[(size_t)n * gridDim.x + blockIdx.x] = s;
  }
}

// g_cls / g_loc: device scalars (null: a zero gradient), times `scale`
// (the loss normaliser folded in: g * f32(scale), the value autograd's
// multiply by that scale would give)
__global__ __launch_bounds__(256) void rpn_loss_bwd_kernel(RpnLossArgs a,
                                                           const float* __restrict__ g_cls_p,
                                                           const float* __restrict__ g_loc_p,
                                                           float scale,
                                                           float* __restrict__ d_logits,
                                                           float4* __restrict__ d_deltas) {
  const int n = blockIdx.y;
  const float g_cls = g_cls_p ? g_cls_p[0] * scale : 0.f;
  const float g_loc = g_loc_p ? g_loc_p[0] * scale : 0.f;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < a.P; p += gridDim.x * 256) {
    const size_t i = (size_t)n * a.P + p;
    float dl = 0.f;
    if (a.samp[i]) {
      const float x = a.logits[i], z = a.pos[i] ? 1.f : 0.f;
      dl = g_cls * (1.f / (1.f + expf(-x)) - z);
    }
    d_logits[i] = dl;
    float4 dd = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.pos[i]) {
      const float4 t = target_of(a, n, p), d = a.deltas[i];
      dd = make_float4(g_loc * sl1_grad(t.x, d.x, a.beta), g_loc * sl1_grad(t.y, d.y, a.beta),
                       g_loc * sl1_grad(t.z, d.z, a.beta), g_loc * sl1_grad(t.w, d.w, a.beta));
    }
    d_deltas[i] = dd;
  }
}

RpnLossArgs make_args(const float* logits, const float* deltas, const float* anchors,
                      const float* gt, const long long* matches, const unsigned char* pos,
                      const unsigned char* sampled, int N, int P, int G, const float* w,
                      float beta) {
  RpnLossArgs a;
  a.logits = logits;
  a.deltas = reinterpret_cast<const float4*>(deltas);
  a.anchors = reinterpret_cast<const float4*>(anchors);
  a.gt = reinterpret_cast<const float4*>(gt);
  a.matches = matches;
  a.pos = pos;
  a.samp = sampled;
  a.N = N;
  a.P = P;
  a.G = G;
  a.wy = w[0];
  a.wx = w[1];
  a.wh = w[2];
  a.ww = w[3];
  a.beta = beta;
  return a;
}

constexpr int kLossBlocks = 256;  // per image

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_rpn_loss_blocks(void) { return kLossBlocks; }

extern "C" int d2mi_rpn_loss_fwd(const float* logits, const float* deltas, const float* anchors,
                                 const float* gt_boxes, const long long* matches,
                                 const unsigned char* pos, const unsigned char* sampled, int N,
                                 int P, int G, const float* weights, float beta, float* partial,
                                 void* stream) {
  D2MI_REQUIRE(N > 0 && P > 0 && G > 0, "bad rpn-loss shape");
  D2MI_REQUIRE(((uintptr_t)deltas & 15) == 0 && ((uintptr_t)anchors & 15) == 0 &&
                   ((uintptr_t)gt_boxes & 15) == 0,
               "rpn loss: 16-byte aligned boxes / deltas");
  const RpnLossArgs a = make_args(logits, deltas, anchors, gt_boxes, matches, pos, sampled, N, P,
                                  G, weights, beta);
  hipLaunchKernelGGL(rpn_loss_fwd_kernel, dim3(kLossBlocks, N), dim3(256), 0, as_stream(stream),
                     a, reinterpret_cast<float2*>(partial));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_rpn_loss_bwd_ex(const float* logits, const float* deltas,
                                    const float* anchors, const float* gt_boxes,
                                    const long long* matches, const unsigned char* pos,
                                    const unsigned char* sampled, int N, int P, int G,
                                    const float* weights, float beta, const float* g_cls,
                                    const float* g_loc, float scale, float* d_logits,
                                    float* d_deltas, void* stream) {
  D2MI_REQUIRE(N > 0 && P > 0 && G > 0, "bad rpn-loss shape");
  D2MI_REQUIRE(((uintptr_t)d_deltas & 15) == 0, "rpn loss: 16-byte aligned d_deltas");
  const RpnLossArgs a = make_args(logits, deltas, anchors, gt_boxes, matches, pos, sampled, N, P,
                                  G, weights, beta);
  hipLaunchKernelGGL(rpn_loss_bwd_kernel, dim3((P + 255) / 256 < 2048 ? (P + 255) / 256 : 2048, N),
                     dim3(256), 0, as_stream(stream), a, g_cls, g_loc, scale, d_logits,
                     reinterpret_cast<float4*>(d_deltas));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_rpn_loss_bwd(const float* logits, const float* deltas, const float* anchors,
                                 const float* gt_boxes, const long long* matches,
                                 const unsigned char* pos, const unsigned char* sampled, int N,
                                 int P, int G, const float* weights, float beta,
                                 const float* grads, float* d_logits, float* d_deltas,
                                 void* stream) {
  D2MI_REQUIRE(grads != nullptr, "rpn loss: null grads");
  return d2mi_rpn_loss_bwd_ex(logits, deltas, anchors, gt_boxes, matches, pos, sampled, N, P, G,
                              weights, beta, grads, grads + 1, 1.0f, d_logits, d_deltas, stream);
}

// ------------------------------------------------ RPN head output layout
namespace d2mi {
namespace {
constexpr int kMaxHeadLevels = 8;
struct HeadLevels {
  const float* y[kMaxHeadLevels];
  float* gy[kMaxHeadLevels];
  int t0[kMaxHeadLevels + 1];  // first pixel of level l in the concatenation
  int L;
};

__device__ __forceinline__ int head_level(const HeadLevels& h, int t) {
  int l = 0;
#pragma unroll
  for (int i = 1; i < kMaxHeadLevels; ++i)
    if (i < h.L && t >= h.t0[i]) l = i;
  return l;
}

// One thread per (image, pixel): its A logits and 4A deltas.
__global__ __launch_bounds__(256) void rpn_head_gather_kernel(HeadLevels h, int N, int A, int C,
                                                              float* __restrict__ logits,
                                                              float* __restrict__ deltas) {
  const int T = h.t0[h.L];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * T) return;
  const int n = (int)(i / T), t = (int)(i - (long long)n * T);
  const int l = head_level(h, t);
  const int hw = t - h.t0[l], HW = h.t0[l + 1] - h.t0[l];
  const float* src = h.y[l] + ((size_t)n * HW + hw) * C;
  float* lo = logits + i * A;
  float* de = deltas + i * 4 * A;
  for (int a = 0; a < A; ++a) lo[a] = src[a];
  for (int j = 0; j < 4 * A; ++j) de[j] = src[A + j];
}

__global__ __launch_bounds__(256) void rpn_head_scatter_kernel(HeadLevels h, int N, int A, int C,
                                                               const float* __restrict__ gl,
                                                               const float* __restrict__ gd) {
  const int T = h.t0[h.L];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * T) return;
  const int n = (int)(i / T), t = (int)(i - (long long)n * T);
  const int l = head_level(h, t);
  const int hw = t - h.t0[l], HW = h.t0[l + 1] - h.t0[l];
  float* dst = h.gy[l] + ((size_t)n * HW + hw) * C;
  for (int c = 0; c < C; ++c) {
    float v = 0.f;
    if (c < A) v = gl ? gl[i * A + c] : 0.f;
    else if (c < 5 * A) v = gd ? gd[i * 4 * A + (c - A)] : 0.f;
    dst[c] = v;
  }
}

// float4 forms (the FPN RPN head: A = 3 anchors, C = 16 channels -- 15 used
// -- and 16-B aligned level outputs / gradients: r5): a lane moves its pixel's C channels as C / 4
// float4s, the 4A deltas as A float4s (4A floats at i * 4A: 16-B aligned)
// and the A logits as scalars; a wave's loads and stores cover whole cache
// lines in order (the scalar loops above read every 64-B pixel record one
// float at a time: 12 / 22 us per step for ~22 MB).
template <int A, int C>
__global__ __launch_bounds__(256) void rpn_head_gather4_kernel(HeadLevels h, int N,
                                                               float* __restrict__ logits,
                                                               float* __restrict__ deltas) {
  const int T = h.t0[h.L];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * T) return;
  const int n = (int)(i / T), t = (int)(i - (long long)n * T);
  const int l = head_level(h, t);
  const int hw = t - h.t0[l], HW = h.t0[l + 1] - h.t0[l];
  const float4* src = reinterpret_cast<const float4*>(h.y[l] + ((size_t)n * HW + hw) * C);
  float v[C];
#pragma unroll
  for (int q = 0; q < C / 4; ++q) {
    const float4 x = src[q];
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
  float* lo = logits + i * A;
#pragma unroll
  for (int a = 0; a < A; ++a) lo[a] = v[a];
  float4* de = reinterpret_cast<float4*>(deltas + i * 4 * A);
#pragma unroll
  for (int a = 0; a < A; ++a)
    de[a] = make_float4(v[A + 4 * a], v[A + 4 * a + 1], v[A + 4 * a + 2], v[A + 4 * a + 3]);
}

template <int A, int C>
__global__ __launch_bounds__(256) void rpn_head_scatter4_kernel(HeadLevels h, int N,
                                                                const float* __restrict__ gl,
                                                                const float* __restrict__ gd) {
  const int T = h.t0[h.L];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * T) return;
  const int n = (int)(i / T), t = (int)(i - (long long)n * T);
  const int l = head_level(h, t);
  const int hw = t - h.t0[l], HW = h.t0[l + 1] - h.t0[l];
  float v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = 0.f;
#pragma unroll
  for (int a = 0; a < A; ++a)
    if (gl) v[a] = gl[i * A + a];
  if (gd) {
    const float4* g4 = reinterpret_cast<const float4*>(gd + i * 4 * A);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float4 x = g4[a];
      v[A + 4 * a] = x.x; v[A + 4 * a + 1] = x.y; v[A + 4 * a + 2] = x.z; v[A + 4 * a + 3] = x.w;
    }
  }
  float4* dst = reinterpret_cast<float4*>(h.gy[l] + ((size_t)n * HW + hw) * C);
#pragma unroll
  for (int q = 0; q < C / 4; ++q) dst[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

int head_levels(HeadLevels& h, const int32_t* hw, int L) {
  D2MI_REQUIRE(L >= 1 && L <= kMaxHeadLevels, "RPN head: %d levels (1..%d)", L, kMaxHeadLevels);
  h.L = L;
  h.t0[0] = 0;
  for (int l = 0; l < L; ++l) {
    D2MI_REQUIRE(hw[l] > 0, "RPN head: empty level %d", l);
    h.t0[l + 1] = h.t0[l] + hw[l];
  }
  return 0;
}
}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_rpn_head_gather(const float* const* ys, const int32_t* level_hw_flat, int L,
                                    int N, int A, int C, float* logits, float* deltas,
                                    void* stream) {
  HeadLevels h = {};
  const int rc = head_levels(h, level_hw_flat, L);
  if (rc) return rc;
  D2MI_REQUIRE(N >= 1 && A >= 1 && C >= 5 * A && ys && logits && deltas, "bad RPN head gather");
  bool v4 = A == 3 && C == 16 && ((uintptr_t)deltas & 15) == 0;  // (the FPN RPN head)
  for (int l = 0; l < L; ++l) {
    h.y[l] = ys[l];
    v4 = v4 && ((uintptr_t)ys[l] & 15) == 0;
  }
  const long long n = (long long)N * h.t0[L];
  if (v4)
    hipLaunchKernelGGL((rpn_head_gather4_kernel<3, 16>), dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, as_stream(stream), h, N, logits, deltas);
  else
    hipLaunchKernelGGL(rpn_head_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), h, N, A, C, logits, deltas);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_rpn_head_scatter(const float* g_logits, const float* g_deltas,
                                     const int32_t* level_hw_flat, int L, int N, int A, int C,
                                     float* const* gys, void* stream) {
  HeadLevels h = {};
  const int rc = head_levels(h, level_hw_flat, L);
  if (rc) return rc;
  D2MI_REQUIRE(N >= 1 && A >= 1 && C >= 5 * A && gys, "bad RPN head scatter");
  bool v4 = A == 3 && C == 16 && (!g_deltas || ((uintptr_t)g_deltas & 15) == 0);
  for (int l = 0; l < L; ++l) {
    h.gy[l] = gys[l];
    v4 = v4 && ((uintptr_t)gys[l] & 15) == 0;
  }
  const long long n = (long long)N * h.t0[L];
  if (v4)
    hipLaunchKernelGGL((rpn_head_scatter4_kernel<3, 16>), dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, as_stream(stream), h, N, g_logits, g_deltas);
  else
    hipLaunchKernelGGL(rpn_head_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), h, N, A, C, g_logits, g_deltas);
  D2MI_LAUNCH_CHECK();
  return 0;
}
