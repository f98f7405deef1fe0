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

// The stem's 7x7 / stride-2 conv itself (Cin = 3, Cout = 64; fix_padding's
// symmetric pad of 3 then VALID, lib/layers/convolutional.py:12-24) on the
// bf16 MFMA with the exact 3-term split of both operands and the six
// products of the conv kernels (f32-class arithmetic, csrc/conv_mfma.hip).
// GEMM view: M = output pixels, N = 64, K = 7 * 7 * 3 = 147 (HWIO order,
// padded to 160: ten 16-deep MFMA steps).  A workgroup takes 128 consecutive
// output pixels of one output row (4 waves x 32 pixels, both 32-channel
// halves per wave); its input footprint -- 7 input rows x (2 * 128 + 5)
// columns x 3 channels, zero outside the image -- is staged in LDS once
// (each row one contiguous NHWC run), and each lane gathers its A fragment
// (8 K values of its pixel) from LDS and splits it in registers.  B arrives
// pre-split: [3][64][160] bf16 planes of the transposed, K-padded weights.
// Output: the raw conv sums (stem_pool_kernel adds the shift, applies the
// ReLU, pads and pools).
typedef float stem_floatx16 __attribute__((ext_vector_type(16)));
typedef short stem_bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kStemTile = 128, kStemK = 160, kStemCols = 2 * kStemTile + 5;
constexpr int kStemPatch = 7 * kStemCols * 3;

// LDS offset of K index k (HWIO: k = (kh * 7 + kw) * 3 + c) for pixel 0; pixel
// p adds 6 * p (two input columns of 3 channels).  -1: K padding.
__host__ __device__ constexpr int stem_koff(int k) {
  return k >= 147 ? -1 : ((k / 21) * kStemCols + (k / 3) % 7) * 3 + k % 3;
}

__device__ __forceinline__ void split8(const float (&v)[8], stem_bf16x8& h, stem_bf16x8& m,
                                       stem_bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t hb = __float_as_uint(v[j]) & 0xffff0000u;
    const float r = v[j] - __uint_as_float(hb);
    const uint32_t mb = __float_as_uint(r) & 0xffff0000u;
    const uint32_t lb = __float_as_uint(r - __uint_as_float(mb));
    h[j] = (short)(hb >> 16);
    m[j] = (short)(mb >> 16);
    l[j] = (short)(lb >> 16);
  }
}

__global__ __launch_bounds__(256) void stem_conv_kernel(const float* __restrict__ x,
                                                        const uint16_t* __restrict__ w3, int H,
                                                        int W, int OH, int OW,
                                                        float* __restrict__ y) {
  __shared__ float patch[kStemPatch];
  const int tiles_per_row = (OW + kStemTile - 1) / kStemTile;
  int b = blockIdx.x;
  const int tw = b % tiles_per_row;
  b /= tiles_per_row;
  const int oh = b % OH, n = b / OH;
  const int ow0 = tw * kStemTile;
  const int ih0 = 2 * oh - 3, iw0 = 2 * ow0 - 3;
  for (int i = threadIdx.x; i < kStemPatch; i += 256) {
    const int r = i / (kStemCols * 3), e = i - r * (kStemCols * 3);
    const int ih = ih0 + r, iw = iw0 + e / 3;
    float v = 0.f;
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = x[(((size_t)n * H + ih) * W) * 3 + (ptrdiff_t)iw0 * 3 + e];
    patch[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int pbase = 6 * (wave * 32 + li);
  stem_floatx16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
  for (int s = 0; s < kStemK / 16; ++s) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o0 = stem_koff(16 * s + j), o1 = stem_koff(16 * s + 8 + j);
      const int o = lh ? o1 : o0;
      a[j] = o >= 0 ? patch[o + pbase] : 0.f;
    }
    stem_bf16x8 fa[3], fb[3][2];
    split8(a, fa[0], fa[1], fa[2]);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        fb[pl][t] = *reinterpret_cast<const stem_bf16x8*>(
            w3 + ((size_t)pl * 64 + t * 32 + li) * kStemK + 16 * s + 8 * lh);
    // the conv kernels' product order: m*m, l*h, h*l, h*m, m*h, h*h
    constexpr int PA[6] = {1, 2, 0, 0, 1, 0};
    constexpr int PB[6] = {1, 0, 2, 1, 0, 0};
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PA[q]], fb[PB[q]][t], acc[t], 0, 0, 0);
  }
  // C/D map: channel = li, pixel row = (r & 3) + 8 * (r >> 2) + 4 * lh
  float* yrow = y + ((size_t)n * OH + oh) * OW * 64;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ow = ow0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    if (ow < OW) {
#pragma unroll
      for (int t = 0; t < 2; ++t) yrow[(size_t)ow * 64 + t * 32 + li] = acc[t][r];
    }
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_stem_conv(const float* x, const uint16_t* w3, int N, int H, int W, float* y,
                              void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0, "bad stem conv shape");
  D2MI_REQUIRE(x && w3 && y && ((uintptr_t)w3 & 15) == 0, "stem conv: null or unaligned operand");
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long blocks = (long long)N * OH * ((OW + kStemTile - 1) / kStemTile);
  D2MI_REQUIRE(blocks < (1LL << 31) && (long long)N * H * W * 3 < (1LL << 40), "stem conv too large");
  hipLaunchKernelGGL(stem_conv_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), x,
                     w3, H, W, OH, OW, y);
  D2MI_LAUNCH_CHECK();
  return 0;
}

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
