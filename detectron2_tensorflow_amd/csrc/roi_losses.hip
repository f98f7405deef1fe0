// ROI-head training losses, fused (fast_rcnn.py:269-357 FastRCNNOutputs.losses,
// mask_head.py:17-68 mask_rcnn_loss), on the dense fixed-layout rows the
// sampler produces (valid / foreground masks instead of boolean_mask):
//
//   Fast R-CNN  loss_cls = sum over valid rows of softmax-CE(logits, gt class) / R
//               loss_box = sum over foreground rows of smooth-L1(
//                            deltas[gt class] - get_deltas(proposal, gt box)) / R
//               R = max(1, #valid rows)
//   mask        loss = sum over foreground rows and the Hm x Wm map of
//                      sigmoid-BCE(logits[.., gt class], target) / max(1, #fg * Hm * Wm)
//
// Instead of the ~80 elementwise / gather / reduction tensor passes of the
// autograd formulation, each loss is a per-row kernel (one wave per row; the
// row terms go to a small buffer), a one-workgroup fixed-order reduction
// (deterministic) and one backward kernel that writes the whole input
// gradient (zeros included) from the upstream gradients read on the device.
// Element formulas: the CE as log-softmax (x_c - max) - log(sum exp(x - max)),
// get_deltas as box_regression.py:38-74, smooth-L1 as layers/loss.py, the
// BCE as ATen's binary_cross_entropy_with_logits.
#include "common.h"

namespace d2mi {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float sl1(float t, float p, float beta) {
  const float d = fabsf(t - p);
  return beta < 1e-5f ? d : (d < beta ? 0.5f * (d * d) / beta : d - 0.5f * beta);
}

__device__ __forceinline__ float sl1_grad(float t, float p, float beta) {
  const float d = p - t;
  const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  if (beta < 1e-5f) return sg;
  return fabsf(d) < beta ? d / beta : sg;
}

struct FrcnArgs {
  const float* logits;          // [B, K1]
  const float* deltas;          // [B, nreg * 4]
  const float4* proposals;      // [B]
  const long long* gt_classes;  // [B]
  const float4* gt_boxes;       // [B]
  const unsigned char* valid;   // [B]
  int B, K1, nreg;
  float wy, wx, wh, ww, beta;
};

__device__ __forceinline__ float4 frcn_target(const FrcnArgs& a, int r) {
  const float4 s = a.proposals[r], t = a.gt_boxes[r];
  const float sh = s.z - s.x, sw = s.w - s.y;
  const float scy = s.x + 0.5f * sh, scx = s.y + 0.5f * sw;
  const float th = t.z - t.x, tw = t.w - t.y;
  const float tcy = t.x + 0.5f * th, tcx = t.y + 0.5f * tw;
  return make_float4(a.wy * (tcy - scy) / sh, a.wx * (tcx - scx) / sw, a.wh * logf(th / sh),
                     a.ww * logf(tw / sw));
}

// row class (where(valid, gt, 0)), foreground flag, regression column
__device__ __forceinline__ void frcn_row(const FrcnArgs& a, int r, bool& valid, int& cls, bool& fg,
                                         int& col) {
  valid = a.valid[r] != 0;
  const long long c = a.gt_classes[r];
  cls = valid ? (int)c : 0;
  fg = valid && c >= 0 && c < a.K1 - 1;
  col = (a.nreg == 1 || !fg) ? 0 : cls;
}

// max and sum(exp(x - max)) of a row's logits, over the wave
__device__ __forceinline__ void row_lse(const float* x, int K1, int lane, float& mx, float& se) {
  float m = -INFINITY;
  for (int j = lane; j < K1; j += 64) m = fmaxf(m, x[j]);
  mx = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < K1; j += 64) s += expf(x[j] - mx);
  se = wave_sum(s);
}

// one wave per row: terms[r] = (CE, smooth-L1 sum, valid)
__global__ __launch_bounds__(256) void frcn_loss_rows_kernel(FrcnArgs a, float* __restrict__ terms) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= a.B) return;
  bool valid, fg;
  int cls, col;
  frcn_row(a, r, valid, cls, fg, col);
  float ce = 0.f, l1 = 0.f;
  if (valid) {
    const float* x = a.logits + (size_t)r * a.K1;
    float mx, se;
    row_lse(x, a.K1, lane, mx, se);
    ce = -((x[cls] - mx) - logf(se));
  }
  if (fg) {
    const float4 t = frcn_target(a, r);
    const float* p = a.deltas + (size_t)r * a.nreg * 4 + col * 4;
    l1 = ((sl1(t.x, p[0], a.beta) + sl1(t.y, p[1], a.beta)) + sl1(t.z, p[2], a.beta)) +
         sl1(t.w, p[3], a.beta);
  }
  if (lane == 0) {
    terms[3 * r] = ce;
    terms[3 * r + 1] = l1;
    terms[3 * r + 2] = valid ? 1.f : 0.f;
  }
}

// One workgroup: out[k] = sum of terms[.][k] in a fixed order; with div:
// out[0..ndiv) /= max(1, out[cnt]) (the count column), out[nterms] = that
// normaliser.
__global__ __launch_bounds__(256) void rows_reduce_kernel(const float* __restrict__ terms, int rows,
                                                          int nterms, int cnt, float cnt_scale,
                                                          int ndiv, float* __restrict__ out) {
  __shared__ float red[4][256];
  const int t = threadIdx.x;
  for (int k = 0; k < nterms; ++k) {
    float s = 0.f;
    for (int r = t; r < rows; r += 256) s += terms[(size_t)r * nterms + k];
    red[k][t] = s;
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
      for (int k = 0; k < nterms; ++k) red[k][t] += red[k][t + w];
    __syncthreads();
  }
  if (t == 0) {
    const float n = fmaxf(red[cnt][0] * cnt_scale, 1.f);
    for (int k = 0; k < nterms; ++k) out[k] = k < ndiv ? red[k][0] / n : red[k][0];
    out[nterms] = n;
  }
}

// one wave per row: d logits (softmax - onehot) * g_cls / R on valid rows, d
// deltas smooth-L1' * g_box / R on the foreground row's class slot, 0 elsewhere
__global__ __launch_bounds__(256) void frcn_loss_bwd_kernel(FrcnArgs a, const float* __restrict__ stats,
                                                            const float* __restrict__ grads,
                                                            float* __restrict__ d_logits,
                                                            float* __restrict__ d_deltas) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= a.B) return;
  bool valid, fg;
  int cls, col;
  frcn_row(a, r, valid, cls, fg, col);
  const float R = stats[3];
  const float gc = grads[0] / R, gb = grads[1] / R;
  const float* x = a.logits + (size_t)r * a.K1;
  float* dx = d_logits + (size_t)r * a.K1;
  if (valid) {
    float mx, se;
    row_lse(x, a.K1, lane, mx, se);
    for (int j = lane; j < a.K1; j += 64)
      dx[j] = gc * (expf(x[j] - mx) / se - (j == cls ? 1.f : 0.f));
  } else {
    for (int j = lane; j < a.K1; j += 64) dx[j] = 0.f;
  }
  const int D = a.nreg * 4;
  float* dd = d_deltas + (size_t)r * D;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (fg) t = frcn_target(a, r);
  const float* p = a.deltas + (size_t)r * D + col * 4;
  for (int j = lane; j < D; j += 64) {
    float v = 0.f;
    if (fg && j >= col * 4 && j < col * 4 + 4) {
      const int k = j - col * 4;
      const float tk = k == 0 ? t.x : (k == 1 ? t.y : (k == 2 ? t.z : t.w));
      v = gb * sl1_grad(tk, p[k], a.beta);
    }
    dd[j] = v;
  }
}

struct MaskArgs {
  const float* logits;          // [B, P, C]  (P = Hm * Wm)
  const float* target;          // [B, P]
  const long long* classes;     // [B]
  const unsigned char* fg;      // [B]
  int B, P, C;
};

__device__ __forceinline__ int mask_channel(const MaskArgs& a, int r) {
  if (a.C == 1) return 0;
  const long long c = a.fg[r] ? a.classes[r] : 0;
  return (int)(c < 0 ? 0 : (c > a.C - 1 ? a.C - 1 : c));
}

__device__ __forceinline__ float bce(float x, float z) {
  const float m = fmaxf(-x, 0.f);
  return (1.f - z) * x + m + logf(expf(-m) + expf(-x - m));
}

// one wave per row: terms[r] = (BCE sum over the map, fg)
__global__ __launch_bounds__(256) void mask_loss_rows_kernel(MaskArgs a, float* __restrict__ terms) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= a.B) return;
  const bool fg = a.fg[r] != 0;
  float s = 0.f;
  if (fg) {
    const int c = mask_channel(a, r);
    const float* x = a.logits + (size_t)r * a.P * a.C + c;
    const float* z = a.target + (size_t)r * a.P;
    for (int p = lane; p < a.P; p += 64) s += bce(x[(size_t)p * a.C], z[p]);
    s = wave_sum(s);
  }
  if (lane == 0) {
    terms[2 * r] = s;
    terms[2 * r + 1] = fg ? 1.f : 0.f;
  }
}

// d logits over [B, P, C] as float4 (C % 4 == 0) or scalars
template <bool VEC4>
__global__ __launch_bounds__(256) void mask_loss_bwd_kernel(MaskArgs a, const float* __restrict__ stats,
                                                            const float* __restrict__ grads,
                                                            float* __restrict__ d_logits) {
  const int W = VEC4 ? 4 : 1;
  const int CW = a.C / W;
  const size_t total = (size_t)a.B * a.P * CW;
  const float g = grads[0] / stats[2];
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int cw = (int)(e % CW);
    const size_t rp = e / CW;
    const int r = (int)(rp / a.P);
    const int c0 = cw * W;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.fg[r]) {
      const int c = mask_channel(a, r);
      if (c >= c0 && c < c0 + W) {
        const float x = a.logits[rp * a.C + c], z = a.target[rp];
        v[c - c0] = g * (1.f / (1.f + expf(-x)) - z);
      }
    }
    if (VEC4)
      *reinterpret_cast<float4*>(d_logits + rp * a.C + c0) = make_float4(v[0], v[1], v[2], v[3]);
    else
      d_logits[rp * a.C + c0] = v[0];
  }
}

FrcnArgs frcn_args(const float* logits, const float* deltas, const float* proposals,
                   const long long* gt_classes, const float* gt_boxes, const unsigned char* valid,
                   int B, int K1, int nreg, const float* w, float beta) {
  FrcnArgs a;
  a.logits = logits;
  a.deltas = deltas;
  a.proposals = reinterpret_cast<const float4*>(proposals);
  a.gt_classes = gt_classes;
  a.gt_boxes = reinterpret_cast<const float4*>(gt_boxes);
  a.valid = valid;
  a.B = B;
  a.K1 = K1;
  a.nreg = nreg;
  a.wy = w[0];
  a.wx = w[1];
  a.wh = w[2];
  a.ww = w[3];
  a.beta = beta;
  return a;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_fast_rcnn_loss_workspace_size(int B) { return (size_t)B * 3 * sizeof(float); }

extern "C" int d2mi_fast_rcnn_loss_fwd(const float* logits, const float* deltas,
                                       const float* proposals, const long long* gt_classes,
                                       const float* gt_boxes, const unsigned char* valid, int B,
                                       int K1, int nreg, const float* weights, float beta,
                                       float* stats, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  D2MI_REQUIRE(B > 0 && K1 >= 2 && nreg >= 1, "bad Fast R-CNN loss shape");
  D2MI_REQUIRE(((uintptr_t)proposals & 15) == 0 && ((uintptr_t)gt_boxes & 15) == 0,
               "Fast R-CNN loss: 16-byte aligned boxes");
  D2MI_REQUIRE(workspace_bytes >= d2mi_fast_rcnn_loss_workspace_size(B),
               "Fast R-CNN loss workspace too small");
  const FrcnArgs a = frcn_args(logits, deltas, proposals, gt_classes, gt_boxes, valid, B, K1,
                               nreg, weights, beta);
  hipStream_t st = as_stream(stream);
  float* terms = (float*)workspace;
  hipLaunchKernelGGL(frcn_loss_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, st, a, terms);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(rows_reduce_kernel, dim3(1), dim3(256), 0, st, terms, B, 3, 2, 1.f, 2,
                     stats);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_fast_rcnn_loss_bwd(const float* logits, const float* deltas,
                                       const float* proposals, const long long* gt_classes,
                                       const float* gt_boxes, const unsigned char* valid, int B,
                                       int K1, int nreg, const float* weights, float beta,
                                       const float* stats, const float* grads, float* d_logits,
                                       float* d_deltas, void* stream) {
  D2MI_REQUIRE(B > 0 && K1 >= 2 && nreg >= 1, "bad Fast R-CNN loss shape");
  const FrcnArgs a = frcn_args(logits, deltas, proposals, gt_classes, gt_boxes, valid, B, K1,
                               nreg, weights, beta);
  hipLaunchKernelGGL(frcn_loss_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, as_stream(stream), a,
                     stats, grads, d_logits, d_deltas);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_mask_loss_workspace_size(int B) { return (size_t)B * 2 * sizeof(float); }

extern "C" int d2mi_mask_loss_fwd(const float* logits, const float* target,
                                  const long long* classes, const unsigned char* fg, int B, int P,
                                  int C, float* stats, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  D2MI_REQUIRE(B > 0 && P > 0 && C > 0, "bad mask loss shape");
  D2MI_REQUIRE(workspace_bytes >= d2mi_mask_loss_workspace_size(B), "mask loss workspace too small");
  MaskArgs a{logits, target, classes, fg, B, P, C};
  hipStream_t st = as_stream(stream);
  float* terms = (float*)workspace;
  hipLaunchKernelGGL(mask_loss_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, st, a, terms);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(rows_reduce_kernel, dim3(1), dim3(256), 0, st, terms, B, 2, 1, (float)P, 1,
                     stats);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_mask_loss_bwd(const float* logits, const float* target,
                                  const long long* classes, const unsigned char* fg, int B, int P,
                                  int C, const float* stats, const float* grads, float* d_logits,
                                  void* stream) {
  D2MI_REQUIRE(B > 0 && P > 0 && C > 0, "bad mask loss shape");
  MaskArgs a{logits, target, classes, fg, B, P, C};
  const bool v4 = C % 4 == 0 && ((uintptr_t)d_logits & 15) == 0;
  const size_t total = (size_t)B * P * (v4 ? C / 4 : C);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
  if (v4)
    hipLaunchKernelGGL(mask_loss_bwd_kernel<true>, dim3(grid), dim3(256), 0, as_stream(stream), a,
                       stats, grads, d_logits);
  else
    hipLaunchKernelGGL(mask_loss_bwd_kernel<false>, dim3(grid), dim3(256), 0, as_stream(stream),
                       a, stats, grads, d_logits);
  D2MI_LAUNCH_CHECK();
  return 0;
}
