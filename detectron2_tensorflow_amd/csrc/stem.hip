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

// grid (row chunks, N * OH): one pooled row per blockIdx.y, threads over its
// (column, channel quad) pairs -- 32-bit index math (r5: a flat index split
// by 64-bit divisions, three per element).
__global__ __launch_bounds__(256) void stem_pool_kernel(const float4* __restrict__ y,
                                                        const float4* __restrict__ shift, int N,
                                                        int H, int W, int C4, int OH, int OW,
                                                        float4* __restrict__ out) {
  const int row = blockIdx.y;  // n * OH + oh
  const int n = row / OH, oh = row - n * OH;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= OW * C4) return;
  const int ow = i / C4, c = i - ow * C4;
  const float4 b = shift ? shift[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int h = 2 * oh - 1 + dy;
    if (h < 0 || h >= H) continue;
    const float4* yr = y + ((size_t)n * H + h) * W * C4 + c;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int w = 2 * ow - 1 + dx;
      if (w < 0 || w >= W) continue;
      const float4 v = yr[(size_t)w * C4];
      m.x = fmaxf(m.x, fmaxf(v.x + b.x, 0.f));
      m.y = fmaxf(m.y, fmaxf(v.y + b.y, 0.f));
      m.z = fmaxf(m.z, fmaxf(v.z + b.z, 0.f));
      m.w = fmaxf(m.w, fmaxf(v.w + b.w, 0.f));
    }
  }
  out[(size_t)row * OW * C4 + i] = m;
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

// r5: a wave computes TWO 32-pixel tiles (64 pixels, 4 accumulators) and a
// workgroup is 2 waves over the same 128-pixel patch, so each weight fragment
// (loaded from L2) feeds twice the MFMAs and half as many waves wait on it:
// the kernel was bound by the waits around its MFMAs (ablation: 1/6 of the
// MFMAs 130 -> 51 us, no input loads -> 97, no stores -> 118), not by VALU.
// The patch is staged row by row with 32-bit offsets and split ONCE into its
// bf16 planes as it enters LDS (hi | mid packed in a word, lo in a half-word;
// every element feeds ~12 output pixels' fragments, each of which split it
// again before).  The planes are split3's, each accumulator's products and
// their order are the conv kernels' (m*m, l*h, h*l, h*m, m*h, h*h per step):
// the sums are the same as before, bit for bit.
constexpr int kStemWaves = 2, kStemThreads = 64 * kStemWaves;
__global__ __launch_bounds__(kStemThreads) void stem_conv_kernel(const float* __restrict__ x,
                                                                 const uint16_t* __restrict__ w3,
                                                                 int H, int W, int OH, int OW,
                                                                 float* __restrict__ y) {
  __shared__ uint32_t phm[kStemPatch];  // (hi << 16) | mid
  __shared__ uint16_t plo[kStemPatch];
  const int tiles_per_row = (OW + kStemTile - 1) / kStemTile;
  int b = blockIdx.x;
  const int tw = b % tiles_per_row;
  b /= tiles_per_row;
  const int oh = b % OH, n = b / OH;
  const int ow0 = tw * kStemTile;
  const int ih0 = 2 * oh - 3, iw0 = 2 * ow0 - 3;
  // 7 rows x 783 contiguous floats; a thread takes elements t, t + 128, ...
  // of a row, the row's loads in flight before its splits and LDS stores
  constexpr int kRowE = kStemCols * 3, kPerRow = (kRowE + kStemThreads - 1) / kStemThreads;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int ih = ih0 + r;
    const bool row_ok = (unsigned)ih < (unsigned)H;
    const float* xr = x + ((size_t)n * H + (row_ok ? ih : 0)) * W * 3;
    float pv[kPerRow];
#pragma unroll
    for (int u = 0; u < kPerRow; ++u) {
      const int e = (int)threadIdx.x + u * kStemThreads;
      const int iw = iw0 + e / 3;
      const bool ok = row_ok && e < kRowE && (unsigned)iw < (unsigned)W;
      pv[u] = ok ? xr[iw0 * 3 + e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kPerRow; ++u) {
      const int e = (int)threadIdx.x + u * kStemThreads;
      if (e < kRowE) {
        const float v = pv[u];
        const uint32_t hb = __float_as_uint(v) & 0xffff0000u;
        const float rr = v - __uint_as_float(hb);
        const uint32_t mb = __float_as_uint(rr) & 0xffff0000u;
        const uint32_t lb = __float_as_uint(rr - __uint_as_float(mb));
        phm[r * kRowE + e] = hb | (mb >> 16);
        plo[r * kRowE + e] = (uint16_t)(lb >> 16);
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  int pbase[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) pbase[m] = 6 * (wave * 64 + m * 32 + li);
  stem_floatx16 acc[2][2];  // [tile][32-channel half]
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][t][r] = 0.f;
  constexpr int kSteps = kStemK / 16;
  stem_bf16x8 fb[2][3][2];  // [step % 2][plane][32-channel half]
  auto load_b = [&](int st, stem_bf16x8 (&f)[3][2]) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        f[pl][t] = *reinterpret_cast<const stem_bf16x8*>(
            w3 + ((size_t)pl * 64 + t * 32 + li) * kStemK + 16 * st + 8 * lh);
  };
  load_b(0, fb[0]);
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    if (s + 1 < kSteps) load_b(s + 1, fb[(s + 1) % 2]);
    stem_bf16x8 fa[2][3];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      uint32_t hm[8];
      uint32_t lo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int o0 = stem_koff(16 * s + j), o1 = stem_koff(16 * s + 8 + j);
        const int o = lh ? o1 : o0;
        hm[j] = o >= 0 ? phm[o + pbase[m]] : 0u;
        lo[j] = o >= 0 ? (uint32_t)plo[o + pbase[m]] : 0u;
      }
      uint4 h, md, l;
      h.x = (hm[0] >> 16) | (hm[1] & 0xffff0000u);
      h.y = (hm[2] >> 16) | (hm[3] & 0xffff0000u);
      h.z = (hm[4] >> 16) | (hm[5] & 0xffff0000u);
      h.w = (hm[6] >> 16) | (hm[7] & 0xffff0000u);
      md.x = (hm[0] & 0xffffu) | (hm[1] << 16);
      md.y = (hm[2] & 0xffffu) | (hm[3] << 16);
      md.z = (hm[4] & 0xffffu) | (hm[5] << 16);
      md.w = (hm[6] & 0xffffu) | (hm[7] << 16);
      l.x = lo[0] | (lo[1] << 16);
      l.y = lo[2] | (lo[3] << 16);
      l.z = lo[4] | (lo[5] << 16);
      l.w = lo[6] | (lo[7] << 16);
      fa[m][0] = __builtin_bit_cast(stem_bf16x8, h);
      fa[m][1] = __builtin_bit_cast(stem_bf16x8, md);
      fa[m][2] = __builtin_bit_cast(stem_bf16x8, l);
    }
    // the conv kernels' product order per accumulator: m*m, l*h, h*l, h*m, m*h, h*h
    constexpr int PA[6] = {1, 2, 0, 0, 1, 0};
    constexpr int PB[6] = {1, 0, 2, 1, 0, 0};
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][PA[q]], fb[s % 2][PB[q]][t],
                                                              acc[m][t], 0, 0, 0);
  }
  // C/D map: channel = li, pixel row = (r & 3) + 8 * (r >> 2) + 4 * lh
  float* yrow = y + ((size_t)n * OH + oh) * OW * 64;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ow = ow0 + wave * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (ow < OW) {
#pragma unroll
        for (int t = 0; t < 2; ++t) yrow[(size_t)ow * 64 + t * 32 + li] = acc[m][t][r];
      }
    }
}

// The input pipeline ahead of the stem in one pass (lib/modeling/meta_arch/
// rcnn.py:146-157 preprocess_image, structures/image_list.py:89-100):
// (image - mean) / std per channel, the channel flip to BGR, and the zero
// pad to the size divisibility -- one read of the image, one write of the
// padded map (torch's form: a subtract, a divide, a flip gather, a fill and a
// copy, five launches of ~12 us each over the whole image per step).  The
// same two IEEE operations per value, so the result is the same bits.
// grid (row chunks, N * OHp): one padded output row per blockIdx.y, FOUR
// consecutive output floats per thread (a float4 store when the row is a
// whole number of float4s); the input row (W * 3 floats) is read by scalars.
template <bool VEC>
__global__ __launch_bounds__(256) void preprocess_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ stdv, int H,
                                                         int W, int OHp, int OWp, int flip,
                                                         float* __restrict__ out) {
  const int row = blockIdx.y;  // n * OHp + y
  const int n = row / OHp, y = row - n * OHp;
  const int f0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  const int rowf = OWp * 3;
  if (f0 >= rowf) return;
  const float m[3] = {mean[0], mean[1], mean[2]};
  const float s[3] = {stdv[0], stdv[1], stdv[2]};
  const float* xr = x + ((size_t)n * H + y) * W * 3;
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = f0 + k;
    const int px = f / 3, c = f - 3 * px;
    const int cs = flip ? 2 - c : c;
    // (the register arrays by a selected constant: no dynamic index into scratch)
    const float mc = cs == 0 ? m[0] : (cs == 1 ? m[1] : m[2]);
    const float sc = cs == 0 ? s[0] : (cs == 1 ? s[1] : s[2]);
    v[k] = (y < H && px < W && f < rowf) ? (xr[(size_t)px * 3 + cs] - mc) / sc : 0.f;
  }
  float* orow = out + (size_t)row * rowf;
  if (VEC) {
    *reinterpret_cast<float4*>(orow + f0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (f0 + k < rowf) orow[f0 + k] = v[k];
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_preprocess_images(const float* x, const float* mean, const float* stdv, int N,
                                      int H, int W, int OHp, int OWp, int flip, float* out,
                                      void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && OHp >= H && OWp >= W, "bad preprocess shape");
  D2MI_REQUIRE(x && mean && stdv && out && x != out, "preprocess: null or aliased operand");
  D2MI_REQUIRE((long long)N * OHp < 65536 && (long long)OWp * 3 < (1LL << 30),
               "preprocess: too many rows or a row too long");
  const int rowf = OWp * 3;
  const dim3 grid((unsigned)((rowf / 4 + 1 + 255) / 256), (unsigned)(N * OHp));
  const bool vec = rowf % 4 == 0 && ((uintptr_t)out & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(preprocess_kernel<true>, grid, dim3(256), 0, as_stream(stream), x, mean,
                       stdv, H, W, OHp, OWp, flip ? 1 : 0, out);
  else
    hipLaunchKernelGGL(preprocess_kernel<false>, grid, dim3(256), 0, as_stream(stream), x, mean,
                       stdv, H, W, OHp, OWp, flip ? 1 : 0, out);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_stem_conv(const float* x, const uint16_t* w3, int N, int H, int W, float* y,
                              void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0, "bad stem conv shape");
  D2MI_REQUIRE(x && w3 && y && ((uintptr_t)w3 & 15) == 0, "stem conv: null or unaligned operand");
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long blocks = (long long)N * OH * ((OW + kStemTile - 1) / kStemTile);
  D2MI_REQUIRE(blocks < (1LL << 31) && (long long)N * H * W * 3 < (1LL << 40), "stem conv too large");
  hipLaunchKernelGGL(stem_conv_kernel, dim3((unsigned)blocks), dim3(kStemThreads), 0,
                     as_stream(stream), x, w3, H, W, OH, OW, y);
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
  D2MI_REQUIRE((int64_t)OW * (C / 4) < (1 << 30) && (int64_t)N * OH < 65536,
               "stem pool: row too long or too many rows");
  const dim3 grid((unsigned)((OW * (C / 4) + 255) / 256), (unsigned)(N * OH));
  hipLaunchKernelGGL(stem_pool_kernel, grid, dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(y), reinterpret_cast<const float4*>(shift), N,
                     H, W, C / 4, OH, OW, reinterpret_cast<float4*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}
