// RetinaNet training losses in two passes (lib/modeling/single_stage_heads/
// retinanet.py:147-210, RetinaNet.losses; lib/layers/loss.py:9-58
// smooth_l1_loss, :59-104 sigmoid_focal_loss):
//   loss_cls = sum over valid anchors (label != ignore) and all K classes of
//              alpha_t * CE(x, t) * (1 - p_t)^gamma,  t = [class == k]
//   loss_box = sum over foreground anchors of smooth_l1(delta - target)
// straight from the head's per-level NHWC outputs [N, H, W, A*K] and
// [N, H, W, A*4] (the reference's reshape_to_N_HWA_K + concat order: levels,
// then (h, w, a)), the matcher's per-anchor labels / matches and the GT --
// no one-hot [N*R, K] target, no concatenated logits copy (2 x 16.1 M floats
// per image at 1333x800), no gathers.  The regression targets
// (box_regression.py:38-74 get_deltas) are formed on the fly from the
// anchor and its matched GT.  Forward: per-workgroup partial sums (the
// caller sums them in a fixed order); backward: the element gradients of
// the same expressions (TF's autodiff of them: d CE = sigmoid(x) - t, d p =
// p (1 - p), d pow = gamma (1 - p_t)^(gamma - 1)), times the upstream
// gradients read from the device.  Memory-bound: one read of the logits
// forward, one read + one write backward.
#include "common.h"

namespace d2mi {
namespace {

constexpr int kMaxRetinaLevels = 8;

struct RetinaLossArgs {
  const float* cls[kMaxRetinaLevels];    // [N, HW_l, A*K]
  const float* box[kMaxRetinaLevels];    // [N, HW_l, A*4]
  float* dcls[kMaxRetinaLevels];
  float* dbox[kMaxRetinaLevels];
  long long abase[kMaxRetinaLevels + 1];  // first anchor index of each level (per image)
  int L, N, K, A, G;
  long long R;                            // anchors per image
  const float4* anchors;                  // [R]
  const float4* gt;                       // [N, G]
  const long long* gt_classes;            // [N, G]
  const long long* matches;               // [N, R]
  const long long* labels;                // [N, R]: 1 fg, 0 bg, -1 ignore
  float alpha, gamma, beta;
  float wy, wx, wh, ww;
};

// target class of anchor r of image n: the matched GT's class (fg), K (bg),
// -1 (ignored)
__device__ __forceinline__ long long class_of(const RetinaLossArgs& a, int n, long long r) {
  const long long lb = a.labels[(size_t)n * a.R + r];
  if (lb < 0) return -1;
  if (lb == 0) return a.K;
  return a.gt_classes[(size_t)n * a.G + a.matches[(size_t)n * a.R + r]];
}

__device__ __forceinline__ void level_of(const RetinaLossArgs& a, long long r, int& l) {
  l = 0;
  while (l + 1 < a.L && r >= a.abase[l + 1]) ++l;
}

__device__ __forceinline__ float focal(float x, float t, float alpha, float gamma) {
  // sigmoid_focal_loss (loss.py:86-95): p = sigmoid(x); ce =
  // sigmoid_cross_entropy_with_logits (max(x, 0) - x t + log1p(exp(-|x|)));
  // p_t = p t + (1 - p)(1 - t); ce (1 - p_t)^gamma, times alpha_t
  const float p = 1.f / (1.f + expf(-x));
  const float ce = (fmaxf(x, 0.f) - x * t) + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  float loss = ce * powf(1.f - pt, gamma);
  if (alpha >= 0.f) loss = (alpha * t + (1.f - alpha) * (1.f - t)) * loss;
  return loss;
}

__device__ __forceinline__ float focal_grad(float x, float t, float alpha, float gamma) {
  const float p = 1.f / (1.f + expf(-x));
  const float ce = (fmaxf(x, 0.f) - x * t) + log1pf(expf(-fabsf(x)));
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float q = 1.f - pt;
  const float dp = p * (1.f - p);
  const float dpt = dp * t - dp * (1.f - t);
  // d(q^gamma)/dx = gamma q^(gamma - 1) * (-d p_t); 0 for gamma = 0 (plain
  // BCE: torch's pow backward for a zero exponent) -- q^(-1) is inf at q = 0
  const float dmod = gamma == 0.f ? 0.f : gamma * powf(q, gamma - 1.f) * -dpt;
  float g = (p - t) * (gamma == 0.f ? 1.f : powf(q, gamma)) + ce * dmod;
  if (alpha >= 0.f) g = (alpha * t + (1.f - alpha) * (1.f - t)) * g;
  return g;
}

__device__ __forceinline__ float4 target_of(const RetinaLossArgs& a, int n, long long r) {
  const float4 s = a.anchors[r];
  const float4 t = a.gt[(size_t)n * a.G + a.matches[(size_t)n * a.R + r]];
  const float sh = s.z - s.x, sw = s.w - s.y;
  const float scy = s.x + 0.5f * sh, scx = s.y + 0.5f * sw;
  const float th = t.z - t.x, tw = t.w - t.y;
  const float tcy = t.x + 0.5f * th, tcx = t.y + 0.5f * tw;
  return make_float4(a.wy * (tcy - scy) / sh, a.wx * (tcx - scx) / sw, a.wh * logf(th / sh),
                     a.ww * logf(tw / sw));
}

__device__ __forceinline__ float sl1(float t, float p, float beta) {
  const float d = fabsf(p - t);
  return beta < 1e-5f ? d : (d < beta ? 0.5f * (d * d) / beta : d - 0.5f * beta);
}

__device__ __forceinline__ float sl1_grad(float t, float p, float beta) {
  const float d = p - t;
  const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  if (beta < 1e-5f) return sg;
  return fabsf(d) < beta ? d / beta : sg;
}

// grid (blocks, N): the image's R*K/4 logit float4s (every level), then its
// R anchors' deltas; partial[n][block] = (cls, box)
__global__ __launch_bounds__(256) void retina_loss_fwd_kernel(RetinaLossArgs a,
                                                              float2* __restrict__ part) {
  __shared__ float2 red[4];
  const int n = blockIdx.y;
  const int K4 = a.K / 4;
  float cls = 0.f, box = 0.f;
  const unsigned total4 = (unsigned)(a.R * K4);  // < 2^31 (make_args)
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total4; i += gridDim.x * 256u) {
    const unsigned r = i / (unsigned)K4;
    const int k0 = (int)(i - r * K4) * 4;
    const long long c = class_of(a, n, r);
    if (c < 0) continue;
    int l;
    level_of(a, r, l);
    const long long lr = r - a.abase[l];
    const long long per = (a.abase[l + 1] - a.abase[l]) * a.K;  // level elements per image
    const float4 x = *reinterpret_cast<const float4*>(a.cls[l] + (size_t)n * per + lr * a.K + k0);
    cls += ((focal(x.x, c == k0 ? 1.f : 0.f, a.alpha, a.gamma) +
             focal(x.y, c == k0 + 1 ? 1.f : 0.f, a.alpha, a.gamma)) +
            focal(x.z, c == k0 + 2 ? 1.f : 0.f, a.alpha, a.gamma)) +
           focal(x.w, c == k0 + 3 ? 1.f : 0.f, a.alpha, a.gamma);
  }
  for (long long r = blockIdx.x * 256ll + threadIdx.x; r < a.R; r += gridDim.x * 256ll) {
    if (a.labels[(size_t)n * a.R + r] != 1) continue;
    int l;
    level_of(a, r, l);
    const long long lr = r - a.abase[l];
    const long long per = (a.abase[l + 1] - a.abase[l]) * 4;
    const float4 d = *reinterpret_cast<const float4*>(a.box[l] + (size_t)n * per + lr * 4);
    const float4 t = target_of(a, n, r);
    box += ((sl1(t.x, d.x, a.beta) + sl1(t.y, d.y, a.beta)) + sl1(t.z, d.z, a.beta)) +
           sl1(t.w, d.w, a.beta);
  }
  for (int o = 32; o > 0; o >>= 1) {
    cls += __shfl_down(cls, o, 64);
    box += __shfl_down(box, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = make_float2(cls, box);
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

// every element of every d_cls / d_box level written (0 where it does not count)
__global__ __launch_bounds__(256) void retina_loss_bwd_kernel(RetinaLossArgs a,
                                                              const float* __restrict__ g_cls_p,
                                                              const float* __restrict__ g_box_p) {
  const int n = blockIdx.y;
  const int K4 = a.K / 4;
  const float g_cls = g_cls_p ? g_cls_p[0] : 0.f;
  const float g_box = g_box_p ? g_box_p[0] : 0.f;
  const unsigned total4 = (unsigned)(a.R * K4);  // < 2^31 (make_args)
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total4; i += gridDim.x * 256u) {
    const unsigned r = i / (unsigned)K4;
    const int k0 = (int)(i - r * K4) * 4;
    const long long c = class_of(a, n, r);
    int l;
    level_of(a, r, l);
    const long long lr = r - a.abase[l];
    const size_t off = (size_t)n * (a.abase[l + 1] - a.abase[l]) * a.K + lr * a.K + k0;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c >= 0) {
      const float4 x = *reinterpret_cast<const float4*>(a.cls[l] + off);
      g = make_float4(g_cls * focal_grad(x.x, c == k0 ? 1.f : 0.f, a.alpha, a.gamma),
                      g_cls * focal_grad(x.y, c == k0 + 1 ? 1.f : 0.f, a.alpha, a.gamma),
                      g_cls * focal_grad(x.z, c == k0 + 2 ? 1.f : 0.f, a.alpha, a.gamma),
                      g_cls * focal_grad(x.w, c == k0 + 3 ? 1.f : 0.f, a.alpha, a.gamma));
    }
    *reinterpret_cast<float4*>(a.dcls[l] + off) = g;
  }
  for (long long r = blockIdx.x * 256ll + threadIdx.x; r < a.R; r += gridDim.x * 256ll) {
    int l;
    level_of(a, r, l);
    const long long lr = r - a.abase[l];
    const size_t off = (size_t)n * (a.abase[l + 1] - a.abase[l]) * 4 + lr * 4;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.labels[(size_t)n * a.R + r] == 1) {
      const float4 d = *reinterpret_cast<const float4*>(a.box[l] + off);
      const float4 t = target_of(a, n, r);
      g = make_float4(g_box * sl1_grad(t.x, d.x, a.beta), g_box * sl1_grad(t.y, d.y, a.beta),
                      g_box * sl1_grad(t.z, d.z, a.beta), g_box * sl1_grad(t.w, d.w, a.beta));
    }
    *reinterpret_cast<float4*>(a.dbox[l] + off) = g;
  }
}

constexpr int kRetinaLossBlocks = 512;  // per image

int make_args(RetinaLossArgs& a, const float* const* cls, const float* const* box,
              float* const* dcls, float* const* dbox, const long long* level_anchors, int L,
              int N, int K, int A, const float* anchors, const float* gt_boxes,
              const long long* gt_classes, int G, const long long* matches,
              const long long* labels, float alpha, float gamma, float beta,
              const float* weights) {
  D2MI_REQUIRE(L >= 1 && L <= kMaxRetinaLevels, "retina loss: 1..8 levels");
  D2MI_REQUIRE(N > 0 && K > 0 && K % 4 == 0 && A > 0 && G > 0, "retina loss: bad shape (K %% 4)");
  D2MI_REQUIRE(((uintptr_t)anchors & 15) == 0 && ((uintptr_t)gt_boxes & 15) == 0,
               "retina loss: 16-byte aligned anchors / GT boxes");
  a = RetinaLossArgs{};
  a.abase[0] = 0;
  for (int l = 0; l < L; ++l) {
    D2MI_REQUIRE(level_anchors[l] > 0, "retina loss: empty level");
    a.cls[l] = cls ? cls[l] : nullptr;
    a.box[l] = box ? box[l] : nullptr;
    a.dcls[l] = dcls ? dcls[l] : nullptr;
    a.dbox[l] = dbox ? dbox[l] : nullptr;
    for (const void* p : {(const void*)a.cls[l], (const void*)a.box[l], (const void*)a.dcls[l],
                          (const void*)a.dbox[l]})
      D2MI_REQUIRE(((uintptr_t)p & 15) == 0, "retina loss: 16-byte aligned level tensors");
    a.abase[l + 1] = a.abase[l] + level_anchors[l];
  }
  a.L = L;
  a.N = N;
  a.K = K;
  a.A = A;
  a.G = G;
  a.R = a.abase[L];
  D2MI_REQUIRE(a.R * (K / 4) < (1ll << 31), "retina loss: R * K / 4 must fit 31 bits");
  a.anchors = reinterpret_cast<const float4*>(anchors);
  a.gt = reinterpret_cast<const float4*>(gt_boxes);
  a.gt_classes = gt_classes;
  a.matches = matches;
  a.labels = labels;
  a.alpha = alpha;
  a.gamma = gamma;
  a.beta = beta;
  a.wy = weights[0];
  a.wx = weights[1];
  a.wh = weights[2];
  a.ww = weights[3];
  return 0;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_retina_loss_blocks(void) { return kRetinaLossBlocks; }

extern "C" int d2mi_retina_loss_fwd(const float* const* cls, const float* const* box,
                                    const long long* level_anchors, int L, int N, int K, int A,
                                    const float* anchors, const float* gt_boxes,
                                    const long long* gt_classes, int G, const long long* matches,
                                    const long long* labels, float alpha, float gamma,
                                    float beta, const float* weights, float* partial,
                                    void* stream) {
  D2MI_REQUIRE(cls && box && partial, "retina loss: null pointers");
  RetinaLossArgs a;
  int rc = make_args(a, cls, box, nullptr, nullptr, level_anchors, L, N, K, A, anchors, gt_boxes,
                     gt_classes, G, matches, labels, alpha, gamma, beta, weights);
  if (rc) return rc;
  hipLaunchKernelGGL(retina_loss_fwd_kernel, dim3(kRetinaLossBlocks, N), dim3(256), 0,
                     as_stream(stream), a, reinterpret_cast<float2*>(partial));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_retina_loss_bwd(const float* const* cls, const float* const* box,
                                    float* const* d_cls, float* const* d_box,
                                    const long long* level_anchors, int L, int N, int K, int A,
                                    const float* anchors, const float* gt_boxes,
                                    const long long* gt_classes, int G, const long long* matches,
                                    const long long* labels, float alpha, float gamma,
                                    float beta, const float* weights, const float* g_cls,
                                    const float* g_box, void* stream) {
  D2MI_REQUIRE(cls && box && d_cls && d_box, "retina loss: null pointers");
  RetinaLossArgs a;
  int rc = make_args(a, cls, box, d_cls, d_box, level_anchors, L, N, K, A, anchors, gt_boxes,
                     gt_classes, G, matches, labels, alpha, gamma, beta, weights);
  if (rc) return rc;
  hipLaunchKernelGGL(retina_loss_bwd_kernel, dim3(kRetinaLossBlocks * 2, N), dim3(256), 0,
                     as_stream(stream), a, g_cls, g_box);
  D2MI_LAUNCH_CHECK();
  return 0;
}
