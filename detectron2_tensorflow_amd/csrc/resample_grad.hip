// Gradients of the two resampling steps around the hot-path convs, each as
// one pass that writes every output element exactly once:
//
//  * d2mi_upsample2x_grad: adjoint of the FPN top-down nearest 2x upsample
//    (lib/modeling/backbone/fpn.py:138-149, fused into the lateral conv's
//    epilogue forward): gtd[n,i,j,c] = sum of gy over the (up to) 2x2 output
//    pixels (2i+di, 2j+dj) that copy it, added in the fixed order
//    (0,0), (0,1), (1,0), (1,1).  Replaces a zero pad of odd maps + a strided
//    reduce.
//  * d2mi_stride_scatter: the input gradient of a 1x1 stride-s conv from the
//    GEMM on its strided grid: out[n,h,w,c] = (h%s == 0 && w%s == 0 ?
//    g[n,h/s,w/s,c] : 0) (+ add[n,h,w,c]).  Replaces zeros + a strided copy
//    (+ autograd's add of the other consumer's gradient).
//    d2mi_stride_scatter_ex adds a second operand and a ReLU gate: the last
//    of three consumers of a ReLU output forms its whole gradient in one pass.
//
// NHWC f32, C % 4 == 0: one float4 of channels per thread, grid-stride.
#include "common.h"

namespace d2mi {
namespace {

// I: the element index type -- uint32_t when the tensor has < 2^31 float4s
// (r6: the int64 divisions and remainders were most of these HBM passes'
// instructions), int64_t otherwise
template <typename I>
__global__ void upsample2x_grad_kernel(const float4* __restrict__ gy, int N, int OH, int OW,
                                       int C4, int TH, int TW, float4* __restrict__ gtd) {
  const I total = (I)N * TH * TW * C4;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int c = (int)(i % (I)C4);
    I p = i / (I)C4;
    const int tw = (int)(p % (I)TW);
    p /= (I)TW;
    const int th = (int)(p % (I)TH);
    const int n = (int)(p / (I)TH);
    const int h0 = 2 * th, w0 = 2 * tw;
    const float4* row = gy + (((int64_t)n * OH + h0) * OW + w0) * C4 + c;
    float4 s = row[0];
    const bool wr = w0 + 1 < OW, hr = h0 + 1 < OH;
    if (wr) {
      const float4 v = row[C4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (hr) {
      const float4 v = row[(int64_t)OW * C4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      if (wr) {
        const float4 u = row[(int64_t)OW * C4 + C4];
        s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
      }
    }
    gtd[i] = s;
  }
}

template <typename I>
__global__ void stride_scatter_kernel(const float4* __restrict__ g, const float4* __restrict__ add,
                                      const float4* __restrict__ add2,
                                      const float4* __restrict__ gate, int N, int H, int W, int C4,
                                      int stride, int GH, int GW, float4* __restrict__ out) {
  const I total = (I)N * H * W * C4;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int c = (int)(i % (I)C4);
    I p = i / (I)C4;
    const int w = (int)(p % (I)W);
    p /= (I)W;
    const int h = (int)(p % (I)H);
    const int n = (int)(p / (I)H);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h % stride == 0 && w % stride == 0)
      v = g[(((int64_t)n * GH + h / stride) * GW + w / stride) * C4 + c];
    if (add) {
      const float4 a = add[i];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (add2) {  // (scatter + add) + add2: autograd's order for a third consumer
      const float4 a = add2[i];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (gate) {  // threshold_backward(v, gate, 0): kept where gate > 0
      const float4 q = gate[i];
      v.x = q.x > 0.f ? v.x : 0.f;
      v.y = q.y > 0.f ? v.y : 0.f;
      v.z = q.z > 0.f ? v.z : 0.f;
      v.w = q.w > 0.f ? v.w : 0.f;
    }
    out[i] = v;
  }
}

int grid_for(int64_t total) { return (int)std::min<int64_t>((total + 255) / 256, 16384); }
// 32-bit element indices suffice: the index never passes 2^31 (total + one
// grid stride)
bool narrow_index(int64_t total) { return total + 256ll * grid_for(total) < (1ll << 31); }

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_upsample2x_grad(const float* gy, int N, int OH, int OW, int C, float* gtd,
                                    void* stream) {
  D2MI_REQUIRE(N > 0 && OH > 0 && OW > 0 && C > 0 && C % 4 == 0, "bad upsample-grad shape");
  D2MI_REQUIRE(gy && gtd && ((uintptr_t)gy & 15) == 0 && ((uintptr_t)gtd & 15) == 0,
               "gy / gtd must be 16-byte aligned");
  const int TH = (OH + 1) / 2, TW = (OW + 1) / 2;
  const int64_t total = (int64_t)N * TH * TW * (C / 4);
  if (narrow_index(total))
    hipLaunchKernelGGL(upsample2x_grad_kernel<uint32_t>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(gy), N, OH, OW, C / 4, TH,
                       TW, reinterpret_cast<float4*>(gtd));
  else
    hipLaunchKernelGGL(upsample2x_grad_kernel<int64_t>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(gy), N, OH, OW, C / 4, TH,
                       TW, reinterpret_cast<float4*>(gtd));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_stride_scatter_ex(const float* g, const float* add, const float* add2,
                                      const float* gate, int N, int H, int W, int C, int stride,
                                      float* out, void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && stride > 0,
               "bad stride-scatter shape");
  D2MI_REQUIRE(g && out && ((uintptr_t)g & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                   ((uintptr_t)add & 15) == 0 && ((uintptr_t)add2 & 15) == 0 &&
                   ((uintptr_t)gate & 15) == 0,
               "g / add / add2 / gate / out must be 16-byte aligned");
  const int GH = (H - 1) / stride + 1, GW = (W - 1) / stride + 1;
  const int64_t total = (int64_t)N * H * W * (C / 4);
  if (narrow_index(total))
    hipLaunchKernelGGL(stride_scatter_kernel<uint32_t>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(g),
                       reinterpret_cast<const float4*>(add), reinterpret_cast<const float4*>(add2),
                       reinterpret_cast<const float4*>(gate), N, H, W, C / 4, stride, GH, GW,
                       reinterpret_cast<float4*>(out));
  else
    hipLaunchKernelGGL(stride_scatter_kernel<int64_t>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), reinterpret_cast<const float4*>(g),
                       reinterpret_cast<const float4*>(add), reinterpret_cast<const float4*>(add2),
                       reinterpret_cast<const float4*>(gate), N, H, W, C / 4, stride, GH, GW,
                       reinterpret_cast<float4*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_stride_scatter(const float* g, const float* add, int N, int H, int W, int C,
                                   int stride, float* out, void* stream) {
  return d2mi_stride_scatter_ex(g, add, nullptr, nullptr, N, H, W, C, stride, out, stream);
}
