// SOLOv2 Matrix-NMS (lib/layers/nms.py:29-83, called at solo_v2.py:541-545).
//   inter = M M^T          -> the MFMA implicit-GEMM conv kernel as a 1x1 conv
//                             (pixels = masks, Cin = H*W, Cout = masks)
//   iou[i][j] = inter / (s_i + s_j - inter) for i < j and class_i == class_j, else 0
//   comp[j]   = max_i iou[i][j]
//   decay[i][j] = exp(-sigma * (iou[i][j]^2 - comp[i]^2))   (gaussian)
//               = (1 - iou[i][j]) / (1 - comp[i])             (linear)
//   out[j] = scores[j] * min_i decay[i][j]
// For 0/1 masks the intersection counts are integers < 2^24, exact in f32 in
// any summation order.
#include "common.h"

extern "C" int d2mi_conv2d_nhwc(const float* x, const float* w_packed, const float* bias,
                                const float* topdown, const float* residual, float* y, int N,
                                int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad_beg, int pad_end, int act, void* stream);

namespace d2mi {
namespace {

__global__ __launch_bounds__(256) void row_sum_kernel(const float* __restrict__ m, int HW,
                                                      float* __restrict__ out) {
  const int i = blockIdx.x;
  float acc = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) acc += m[(size_t)i * HW + p];
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[i] = red[0];
}

__device__ __forceinline__ float iou_at(const float* inter, const float* s, const int64_t* cls,
                                        int M, int i, int j) {
  if (i >= j || cls[i] != cls[j]) return 0.f;
  const float it = inter[(size_t)i * M + j];
  const float uni = (s[j] + s[i]) - it;  // sum_matrix + sum_matrix^T - inter
  return it / uni;
}

// comp[j] = max over i of iou[i][j]: one 256-thread workgroup per column,
// threads over the rows, tree max (exact in any order).
__global__ __launch_bounds__(256) void comp_kernel(const float* inter, const float* s,
                                                   const int64_t* cls, int M, float* comp) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  float mx = 0.f;  // every column has the zero entries of the lower triangle
  for (int i = threadIdx.x; i < j; i += blockDim.x) mx = fmaxf(mx, iou_at(inter, s, cls, M, i, j));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) comp[j] = red[0];
}

// one workgroup per column: min over the rows of the decay, tree min
__global__ __launch_bounds__(256) void decay_kernel(const float* inter, const float* s,
                                                    const int64_t* cls, const float* comp,
                                                    const float* scores, int M, int kernel,
                                                    float sigma, float* out) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  float mn = INFINITY;
  const float ns = -1.f * sigma;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const float v = iou_at(inter, s, cls, M, i, j);
    const float c = comp[i];
    float d;
    if (kernel == 0) d = expf(ns * (v * v - c * c));
    else d = (1.f - v) / (1.f - c);
    mn = fminf(mn, d);
  }
  red[threadIdx.x] = mn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fminf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = scores[j] * red[0];
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_matrix_nms_workspace_size(int M) {
  WorkspaceSizer z;
  z.take<float>((size_t)M * M);
  z.take<float>(M);
  z.take<float>(M);
  return z.off;
}

extern "C" int d2mi_matrix_nms(const float* masks, const int64_t* classes, const float* scores,
                               const float* sum_masks, int M, int HW, int kernel, float sigma,
                               float* out_scores, void* workspace, size_t workspace_bytes,
                               void* stream) {
  D2MI_REQUIRE(M >= 0 && HW > 0, "bad matrix_nms sizes");
  D2MI_REQUIRE(kernel == 0 || kernel == 1, "NMS kernel must be gaussian (0) or linear (1)");
  D2MI_REQUIRE(HW % 4 == 0, "H*W must be a multiple of 4 (got %d)", HW);
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  float* inter = w.take<float>((size_t)M * M);
  float* sums = w.take<float>(M);
  float* comp = w.take<float>(M);
  D2MI_REQUIRE(w.ok(), "matrix_nms workspace too small (%zu < %zu)", workspace_bytes, w.off);
  // inter = masks . masks^T : a 1x1 conv over M "pixels" with Cin = HW, Cout = M,
  // whose packed [Cout][Cin] weight is the mask matrix itself.
  int rc = d2mi_conv2d_nhwc(masks, masks, nullptr, nullptr, nullptr, inter, 1, 1, M, HW, M, 1, 1,
                            1, 0, 0, 0, stream);
  if (rc) return rc;
  const float* s = sum_masks;
  if (!s) {
    hipLaunchKernelGGL(row_sum_kernel, dim3(M), dim3(256), 0, st, masks, HW, sums);
    D2MI_LAUNCH_CHECK();
    s = sums;
  }
  hipLaunchKernelGGL(comp_kernel, dim3(M), dim3(256), 0, st, inter, s, classes, M, comp);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(decay_kernel, dim3(M), dim3(256), 0, st, inter, s, classes, comp, scores, M,
                     kernel, sigma, out_scores);
  D2MI_LAUNCH_CHECK();
  return 0;
}
