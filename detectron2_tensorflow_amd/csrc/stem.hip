// The ResNet stem's tail in one pass (lib/modeling/backbone/resnet.py:73-82,
// BasicStem): relu(conv1 + shift) of the frozen, BN-folded 7x7 conv, the
// tf.pad of one zero pixel on each side and the 3x3 / stride-2 VALID max
// pool -- one read of the conv output, one write of the pooled map (instead
// of a bias-add pass, a ReLU pass, a padded copy and the pool).
// Max over the window with 0 as the start value is exact: every ReLU output
// is >= 0 and the padded pixels are 0.
#include "common.h"

namespace d2mi {
namespace {

__global__ void stem_pool_kernel(const float4* __restrict__ y, const float4* __restrict__ shift,
                                 int N, int H, int W, int C4, int OH, int OW,
                                 float4* __restrict__ out) {
  const int64_t total = (int64_t)N * OH * OW * C4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    int64_t p = i / C4;
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    const float4 b = shift ? shift[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int h = 2 * oh - 1 + dy;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int w = 2 * ow - 1 + dx;
        if (w < 0 || w >= W) continue;
        const float4 v = y[(((int64_t)n * H + h) * W + w) * C4 + c];
        m.x = fmaxf(m.x, fmaxf(v.x + b.x, 0.f));
        m.y = fmaxf(m.y, fmaxf(v.y + b.y, 0.f));
        m.z = fmaxf(m.z, fmaxf(v.z + b.z, 0.f));
        m.w = fmaxf(m.w, fmaxf(v.w + b.w, 0.f));
      }
    }
    out[i] = m;
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_stem_pool(const float* y, const float* shift, int N, int H, int W, int C,
                              float* out, void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0, "bad stem-pool shape");
  D2MI_REQUIRE(y && out && ((uintptr_t)y & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                   ((uintptr_t)shift & 15) == 0,
               "stem pool: 16-byte aligned operands");
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int64_t total = (int64_t)N * OH * OW * (C / 4);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(stem_pool_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(y), reinterpret_cast<const float4*>(shift), N,
                     H, W, C / 4, OH, OW, reinterpret_cast<float4*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}
