// Weight gradient of the NHWC convolution on gfx950 fp32 MFMA
// (v_mfma_f32_32x32x2_f32) — the backward of the FPN output / RPN share /
// mask-head 3x3 convs (lib/layers/convolutional.py:198-263 under tf.gradients).
//
//   dW[kh][kw][ci][co] = sum over pixels p=(n,oy,ox) of
//                        X[n, oy*s - pad + kh, ox*s - pad + kw, ci] * dY[p][co]
//
// GEMM view per tap (kh, kw): C[ci][co] = A^T B with A = X shifted [P][Cin] and
// B = dY [P][Cout] — both stored pixel-major with the OUTPUT dims contiguous
// ("TN" GEMM).  That is the natural operand order of the f32 32x32x2 MFMA,
// where lane l supplies A[l%32][k = l/32]: the LDS image keeps global rows as
// they are (k = pixel rows, channels contiguous) and every operand fetch is one
// conflict-free ds_read_b32 (the row pitch puts the two lane halves on
// disjoint bank halves).  A 256-thread workgroup (2x2 waves, TMxTN 32x32 MFMA
// tiles per wave) owns a (BM channels) x (BN out-channels) tile of one tap and
// walks a contiguous range of 32-pixel chunks; the pixel range is split over
// gridDim.y workgroups whose partial tiles are summed by a second kernel in a
// FIXED split order (deterministic).  Global loads of the next chunk are issued
// before the current chunk's MFMAs (register double buffering).
#include "common.h"

namespace d2mi {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KP = 32;  // pixels per k-step

struct WgradArgs {
  const float* x;   // [N,H,W,Cin]
  const float* dy;  // [N,OH,OW,Cout]
  float* dw;        // [KH,KW,Cin,Cout]
  float* partial;   // [splits][KH*KW*Cin*Cout] when splits > 1
  float* dbias;     // [Cout] bias gradient sum_p dy[p][co] (nullable)
  float* pbias;     // [splits][Cout] partial bias sums when splits > 1
  int N, H, W, Cin, Cout, KH, KW, stride, pad, OH, OW;
  int P;                      // N*OH*OW
  int nCi, nCo, ntiles;       // channel tiles per tap, co tiles, total tiles
  int splits, chunks_per_split, nchunks;
};

template <int TM, int TN>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int BM = 2 * TM * 32, BN = 2 * TN * 32;
  constexpr int PA = BM + 32, PB = BN + 32;  // row pitch: lane halves on disjoint banks
  constexpr int CA = BM / 4, CB = BN / 4;    // float4 columns per row
  constexpr int RA = KP * CA / 256, RB = KP * CB / 256;  // float4 loads per thread
  __shared__ __attribute__((aligned(16))) float As[KP * PA];
  __shared__ __attribute__((aligned(16))) float Bs[KP * PB];

  const int tile = blockIdx.x;
  const int per_tap = a.nCi * a.nCo;
  const int tap = tile / per_tap;
  const int rem = tile - tap * per_tap;
  const int cit = rem / a.nCo, cot = rem - cit * a.nCo;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const int ci0 = cit * BM, co0 = cot * BN;
  const int split = blockIdx.y;
  const int c_begin = split * a.chunks_per_split;
  const int c_end = min(a.nchunks, c_begin + a.chunks_per_split);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  float4 ra[RA], rb[RB];
  auto load_chunk = [&](int ch) {
    const int pbase = ch * KP;
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / CA, c4 = idx - row * CA;
      const int p = pbase + row;
      const int ci = ci0 + c4 * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < a.P && ci < a.Cin) {
        const int n = p / (a.OH * a.OW);
        const int r2 = p - n * a.OH * a.OW;
        const int oy = r2 / a.OW, ox = r2 - oy * a.OW;
        const int iy = oy * a.stride - a.pad + kh, ix = ox * a.stride - a.pad + kw;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          v = *reinterpret_cast<const float4*>(a.x + (((size_t)n * a.H + iy) * a.W + ix) * a.Cin +
                                               ci);
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / CB, c4 = idx - row * CB;
      const int p = pbase + row;
      const int co = co0 + c4 * 4;
      rb[q] = (p < a.P && co < a.Cout)
                  ? *reinterpret_cast<const float4*>(a.dy + (size_t)p * a.Cout + co)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / CA, c4 = idx - row * CA;
      *reinterpret_cast<float4*>(&As[row * PA + c4 * 4]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / CB, c4 = idx - row * CB;
      *reinterpret_cast<float4*>(&Bs[row * PB + c4 * 4]) = rb[q];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // the tap-0 / first-channel-tile blocks also sum dy's columns (bias gradient)
  const bool do_bias = a.dbias != nullptr && tap == 0 && cit == 0;
  float bsum = 0.f;

  if (c_begin < c_end) {
    load_chunk(c_begin);
    for (int ch = c_begin; ch < c_end; ++ch) {
      store_chunk();
      __syncthreads();
      if (ch + 1 < c_end) load_chunk(ch + 1);
      if (do_bias && tid < BN) {
#pragma unroll 8
        for (int k = 0; k < KP; ++k) bsum += Bs[k * PB + tid];
      }
#pragma unroll 4
      for (int k = 0; k < KP; k += 2) {
        const float* Ar = &As[(k + lh) * PA + wr * TM * 32 + li];
        const float* Br = &Bs[(k + lh) * PB + wc * TN * 32 + li];
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = Ar[i * 32];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = Br[j * 32];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
    }
  }

  if (do_bias && tid < BN && co0 + tid < a.Cout) {
    if (a.splits > 1) a.pbias[(size_t)split * a.Cout + co0 + tid] = bsum;
    else a.dbias[co0 + tid] = bsum;
  }

  // C/D map for 32x32: col (co) = lane & 31, row (ci) = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const size_t wsz = (size_t)a.KH * a.KW * a.Cin * a.Cout;
  float* out = a.splits > 1 ? a.partial + (size_t)split * wsz : a.dw;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = co0 + (wc * TN + j) * 32 + li;
    if (co >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cb = ci0 + (wr * TM + i) * 32 + 4 * lh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = cb + (r & 3) + 8 * (r >> 2);
        if (ci < a.Cin) out[((size_t)tap * a.Cin + ci) * a.Cout + co] = acc[i][j][r];
      }
    }
  }
}

// Fixed split order (deterministic); the last Cout entries are the bias
// gradient when pbias follows the weight partials.
__global__ void wgrad_reduce_kernel(const float* __restrict__ partial, int splits, size_t total,
                                    float* __restrict__ dw, const float* __restrict__ pbias,
                                    int Cout, float* __restrict__ dbias) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total + Cout;
       i += (size_t)gridDim.x * blockDim.x) {
    if (i < total) {
      float s = 0.f;
      for (int k = 0; k < splits; ++k) s += partial[(size_t)k * total + i];
      dw[i] = s;
    } else if (dbias) {
      const size_t c = i - total;
      float s = 0.f;
      for (int k = 0; k < splits; ++k) s += pbias[(size_t)k * Cout + c];
      dbias[c] = s;
    }
  }
}

struct WPlan {
  int TM, TN, BM, BN, ntiles, splits, chunks_per_split, nchunks;
};

WPlan wplan(int N, int OH, int OW, int Cin, int Cout, int KH, int KW) {
  WPlan p;
  // 128 x 128 tiles for 256-wide channels; 64-wide when a dimension is small
  p.TM = Cin > 64 ? 2 : 1;
  p.TN = Cout > 64 ? 2 : 1;
  p.BM = 64 * p.TM;
  p.BN = 64 * p.TN;
  p.ntiles = KH * KW * ((Cin + p.BM - 1) / p.BM) * ((Cout + p.BN - 1) / p.BN);
  const long long P = (long long)N * OH * OW;
  p.nchunks = (int)((P + KP - 1) / KP);
  // about 2 workgroups per CU in total, each walking >= 16 chunks
  int splits = std::max(1, 512 / p.ntiles);
  splits = std::min(splits, std::max(1, p.nchunks / 16));
  splits = std::min(splits, 64);
  p.chunks_per_split = (p.nchunks + splits - 1) / splits;
  p.splits = (p.nchunks + p.chunks_per_split - 1) / p.chunks_per_split;
  return p;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_conv2d_wgrad_workspace_size(int N, int H, int W, int Cin, int Cout, int KH,
                                                   int KW, int stride, int pad_beg, int pad_end) {
  if (N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0)
    return 0;
  const int OH = (H + pad_beg + pad_end - KH) / stride + 1;
  const int OW = (W + pad_beg + pad_end - KW) / stride + 1;
  if (OH <= 0 || OW <= 0) return 0;
  const WPlan p = wplan(N, OH, OW, Cin, Cout, KH, KW);
  return p.splits > 1 ? (size_t)p.splits * ((size_t)KH * KW * Cin * Cout + Cout) * sizeof(float)
                      : 0;
}

extern "C" int d2mi_conv2d_wgrad(const float* x, const float* dy, float* dw_hwio, float* dbias,
                                 int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                 int stride, int pad_beg, int pad_end, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0,
               "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0 && Cout % 4 == 0, "Cin and Cout must be multiples of 4 (%d, %d)",
               Cin, Cout);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0,
               "x and dy must be 16-byte aligned");
  WgradArgs a;
  a.x = x;
  a.dy = dy;
  a.dw = dw_hwio;
  a.dbias = dbias;
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
  D2MI_REQUIRE((long long)N * a.OH * a.OW < (1LL << 31), "too many pixels");
  a.P = N * a.OH * a.OW;
  WPlan p = wplan(N, a.OH, a.OW, Cin, Cout, KH, KW);
  const size_t need = d2mi_conv2d_wgrad_workspace_size(N, H, W, Cin, Cout, KH, KW, stride,
                                                       pad_beg, pad_end);
  if (need > workspace_bytes || workspace == nullptr) {  // no workspace: one split
    p.splits = 1;
    p.chunks_per_split = p.nchunks;
  }
  a.nCi = (Cin + p.BM - 1) / p.BM;
  a.nCo = (Cout + p.BN - 1) / p.BN;
  a.ntiles = p.ntiles;
  a.splits = p.splits;
  a.chunks_per_split = p.chunks_per_split;
  a.nchunks = p.nchunks;
  a.partial = p.splits > 1 ? (float*)workspace : nullptr;
  a.pbias = p.splits > 1 ? (float*)workspace + (size_t)p.splits * KH * KW * Cin * Cout : nullptr;
  hipStream_t st = as_stream(stream);
  dim3 grid(a.ntiles, a.splits);
  if (p.TM == 2 && p.TN == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 2>), grid, dim3(256), 0, st, a);
  else if (p.TM == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 1>), grid, dim3(256), 0, st, a);
  else if (p.TN == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<1, 2>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<1, 1>), grid, dim3(256), 0, st, a);
  D2MI_LAUNCH_CHECK();
  if (a.splits > 1) {
    const size_t total = (size_t)KH * KW * Cin * Cout;
    const int g = (int)std::min<size_t>((total + Cout + 255) / 256, 4096);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(g), dim3(256), 0, st, a.partial, a.splits, total,
                       dw_hwio, a.pbias, Cout, dbias);
    D2MI_LAUNCH_CHECK();
  }
  return 0;
}
