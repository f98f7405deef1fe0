// NHWC implicit-GEMM convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the tf.layers.Conv2D / tf.nn.conv2d calls of
//   lib/layers/convolutional.py:12-23   fix_padding (explicit symmetric pad, then VALID)
//   lib/layers/convolutional.py:198-263 Conv2D.call (+ bias, + activation)
// for the FPN lateral 1x1 / output 3x3 convs (lib/modeling/necks/fpn.py:121-159),
// the RPN head (rpn.py:83-96) and the mask head convs (mask_head.py:165-170),
// with the FPN top-down merge  prev = lateral(x) + up2_nearest(prev)  fused
// into the lateral conv's epilogue (fpn.py:138-149, functional.py:58-90).
//
// GEMM view: M = N*OH*OW pixels, N = Cout, K = KH*KW*Cin (tap-major, channel-minor).
// Tile 128 pixels x 128 couts x 32 k per 256-thread workgroup (4 waves in 2x2, each
// wave 64x64 = 2x2 MFMA 32x32 tiles, 64 f32 accumulators per lane).  Both
// operands are staged through LDS as [row][32 k] images padded to 36 floats
// (conflict-free ds_read_b128 for the 4x16-lane groups), which requires the
// weights packed as [KH][KW][Cout][Cin] (d2mi_conv_pack_weights, done once per
// weight version by the host layer).  Within a 32-deep k tile, MFMA step s
// feeds lane half h with k = 16h + s, so every lane fetches the operands of four
// consecutive MFMA steps with one ds_read_b128.  The next k tile is prefetched
// into registers while the current one feeds the MFMAs.  fp32 in / fp32
// accumulate: exact-f32 products, so results differ from a CPU conv only by
// summation order (the parity tests bound it).
#include "common.h"

namespace d2mi {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32, LDSP = 36;

struct ConvArgs {
  const float* x;
  const float* w;  // [KH][KW][Cout][Cin]
  const float* bias;
  const float* topdown;
  const float* residual;
  float* y;
  int N, H, W, Cin, Cout, KH, KW, stride, pad, OH, OW, act;
  int M, nM, nN, ntiles;
  int tdH, tdW;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float As[BM * LDSP];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LDSP];

  // XCD-aware tile order: consecutive tiles (the Cout tiles of one pixel tile
  // and neighbouring pixel tiles, which share input halo rows) land on one XCD.
  const int orig = blockIdx.x;
  const int q = a.ntiles / 8, r8 = a.ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int mt = tile / a.nN, nt = tile - mt * a.nN;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  // staging assignment: 4 rows per thread, one float4 (4 k) each
  const int srow = tid >> 3, schunk = (tid & 7) * 4;
  int pn[4], ph[4], pw[4];
  bool pv[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int m = m0 + srow + 32 * p;
    pv[p] = m < a.M;
    const int mm = pv[p] ? m : 0;
    pn[p] = mm / (a.OH * a.OW);
    const int rem = mm - pn[p] * a.OH * a.OW;
    ph[p] = rem / a.OW;
    pw[p] = rem - ph[p] * a.OW;
  }
  const int cchunks = (a.Cin + BK - 1) / BK;
  const int nk = a.KH * a.KW * cchunks;

  float4 ra[4], rb[4];
  auto load_tile = [&](int kt) {
    const int tap = kt / cchunks;
    const int c0 = (kt - tap * cchunks) * BK + schunk;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int ih = ph[p] * a.stride - a.pad + kh;
      const int iw = pw[p] * a.stride - a.pad + kw;
      const bool ok = pv[p] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W && c0 < a.Cin;
      ra[p] = ok ? ld4(a.x + (((size_t)pn[p] * a.H + ih) * a.W + iw) * a.Cin + c0)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      const int co = n0 + srow + 32 * p;
      const bool okb = co < a.Cout && c0 < a.Cin;
      rb[p] = okb ? ld4(a.w + (((size_t)tap * a.Cout + co) * a.Cin + c0))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      *reinterpret_cast<float4*>(&As[(srow + 32 * p) * LDSP + schunk]) = ra[p];
      *reinterpret_cast<float4*>(&Bs[(srow + 32 * p) * LDSP + schunk]) = rb[p];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_tile(0);
  store_tile();
  __syncthreads();

  const int li = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
    for (int s0 = 0; s0 < 16; s0 += 4) {
      float4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const float4*>(
            &As[(wr * 64 + i * 32 + li) * LDSP + lh * 16 + s0]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *reinterpret_cast<const float4*>(
            &Bs[(wc * 64 + j * 32 + li) * LDSP + lh * 16 + s0]);
#pragma unroll
      for (int ss = 0; ss < 4; ++ss) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][ss], fb[j][ss], acc[i][j], 0,
                                                              0, 0);
      }
    }
    __syncthreads();
    if (kt + 1 < nk) {
      store_tile();
      __syncthreads();
    }
  }

  // epilogue: C/D map for 32x32: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int co = n0 + wc * 64 + j * 32 + li;
    if (co >= a.Cout) continue;
    const float bv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bv;
        if (a.act == 1) v = fmaxf(v, 0.f);
        if (a.topdown) {
          const int n = m / (a.OH * a.OW);
          const int rem = m - n * a.OH * a.OW;
          const int oh = rem / a.OW, ow = rem - oh * a.OW;
          v = v + a.topdown[(((size_t)n * a.tdH + (oh >> 1)) * a.tdW + (ow >> 1)) * a.Cout + co];
        }
        if (a.residual) v = v + a.residual[(size_t)m * a.Cout + co];
        a.y[(size_t)m * a.Cout + co] = v;
      }
    }
  }
}

__global__ void pack_weights_kernel(const float* __restrict__ w, int taps, int Cin, int Cout,
                                    float* __restrict__ out) {
  const int64_t total = (int64_t)taps * Cin * Cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    // i indexes the output [tap][co][ci]
    const int64_t ci = i % Cin;
    const int64_t t2 = i / Cin;
    const int64_t co = t2 % Cout;
    const int64_t tap = t2 / Cout;
    out[i] = w[(tap * Cin + ci) * Cout + co];
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_conv_pack_weights(const float* w_hwio, int KH, int KW, int Cin, int Cout,
                                      float* w_packed, void* stream) {
  D2MI_REQUIRE(KH > 0 && KW > 0 && Cin > 0 && Cout > 0, "bad conv weight shape");
  const int64_t total = (int64_t)KH * KW * Cin * Cout;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(grid), dim3(256), 0, as_stream(stream), w_hwio,
                     KH * KW, Cin, Cout, w_packed);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_conv2d_nhwc(const float* x, const float* w_packed, const float* bias,
                                const float* topdown, const float* residual, float* y, int N,
                                int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad_beg, int pad_end, int act, void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0,
               "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0, "Cin must be a multiple of 4 (got %d)", Cin);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_packed & 15) == 0,
               "x and w must be 16-byte aligned");
  D2MI_REQUIRE(act == 0 || act == 1, "act must be 0 (none) or 1 (relu)");
  ConvArgs a;
  a.x = x;
  a.w = w_packed;
  a.bias = bias;
  a.topdown = topdown;
  a.residual = residual;
  a.y = y;
  a.N = N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.Cout = Cout;
  a.KH = KH;
  a.KW = KW;
  a.stride = stride;
  a.pad = pad_beg;
  a.OH = (H + pad_beg + pad_end - KH) / stride + 1;
  a.OW = (W + pad_beg + pad_end - KW) / stride + 1;
  D2MI_REQUIRE(a.OH > 0 && a.OW > 0, "conv output is empty");
  a.act = act;
  a.M = N * a.OH * a.OW;
  a.nM = (a.M + BM - 1) / BM;
  a.nN = (Cout + BN - 1) / BN;
  a.ntiles = a.nM * a.nN;
  a.tdH = (a.OH + 1) / 2;
  a.tdW = (a.OW + 1) / 2;
  hipLaunchKernelGGL(conv_mfma_kernel, dim3(a.ntiles), dim3(256), 0, as_stream(stream), a);
  D2MI_LAUNCH_CHECK();
  return 0;
}
