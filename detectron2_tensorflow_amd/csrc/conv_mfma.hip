// NHWC implicit-GEMM convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the tf.layers.Conv2D / tf.nn.conv2d calls of
//   lib/layers/convolutional.py:12-23   fix_padding (explicit symmetric pad, then VALID)
//   lib/layers/convolutional.py:198-263 Conv2D.call (+ bias, + activation)
// for the FPN lateral 1x1 / output 3x3 convs (lib/modeling/necks/fpn.py:121-159),
// the RPN head (rpn.py:83-96), the mask head (mask_head.py:165-170) and the
// ResNet 1x1 convs, with the FPN top-down merge  prev = lateral(x) + up2(prev)
// (fpn.py:138-149) or a residual add + ReLU (blocks.py:143-186) fused into the
// epilogue.
//
// GEMM view: M = N*OH*OW pixels, N = Cout, K = KH*KW*Cin (tap-major, channel-minor).
// A 256-thread workgroup (4 waves) owns a BM x BN output tile; each wave owns
// TM x TN MFMA tiles of 32 x 32 (f32 accumulators: 16 per lane per tile).
// Configurations: 128x128 (2x2 waves of 2x2 tiles, the FPN / RPN / mask-head
// shapes), 128x64 and 128x32 (narrow Cout: RPN 1x1, mask predictor).  K is
// staged 32 deep per step through a DOUBLE-BUFFERED LDS image [row][36]
// (rows padded to 36 floats: the 16-lane groups of ds_read_b128 hit 16
// distinct 4-bank slots), one barrier per k-step: while the MFMAs consume
// buffer b, the next k-step's global loads (issued before the MFMAs) land in
// registers and are written to buffer b^1.  Inside a 32-deep step, MFMA step
// s feeds lane half h with k = 16h + s, so one ds_read_b128 per operand covers
// four MFMA steps.  Weights are packed [KH][KW][Cout][Cin] (d2mi_conv_pack_weights)
// so both operands stage identically.  Small-M shapes (FPN p5/p6, 1x1 laterals
// on res5) split K over up to 16 workgroups per tile; partial sums go to a
// caller-provided workspace and a second kernel adds them in a FIXED order
// (deterministic) and applies the epilogue.
// fp32 in / fp32 accumulate: exact-f32 products; results differ from a CPU
// conv only by summation order (the parity tests bound it).
#include "common.h"

namespace d2mi {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32, LDSP = 36;

enum EpiFlags { kRelu = 1, kReluAfterResidual = 2 };

struct ConvArgs {
  const float* x;
  const float* w;  // [KH][KW][Cout][Cin]
  const float* bias;
  const float* topdown;
  const float* residual;
  float* y;
  float* partial;  // split-K workspace [splits][M][Cout] (nullable)
  int N, H, W, Cin, Cout, KH, KW, stride, pad, OH, OW, flags;
  int M, nM, nN, ntiles, splits, kt_per_split, nk, cchunks;
  int tdH, tdW;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float epilogue(const ConvArgs& a, float acc, int m, int co) {
  float v = acc + (a.bias ? a.bias[co] : 0.f);
  if ((a.flags & kRelu) && !(a.flags & kReluAfterResidual)) v = fmaxf(v, 0.f);
  if (a.topdown) {
    const int n = m / (a.OH * a.OW);
    const int rem = m - n * a.OH * a.OW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    v = v + a.topdown[(((size_t)n * a.tdH + (oh >> 1)) * a.tdW + (ow >> 1)) * a.Cout + co];
  }
  if (a.residual) v = v + a.residual[(size_t)m * a.Cout + co];
  if ((a.flags & kRelu) && (a.flags & kReluAfterResidual)) v = fmaxf(v, 0.f);
  return v;
}

// DB: double-buffered LDS (one barrier per k-step, 2 workgroups/CU for the
// 128x128 tile) vs single-buffered (two barriers per k-step, 36 KiB LDS, up to
// 3 workgroups/CU).  Large-M shapes prefer the higher occupancy.
template <int WM, int WN, int TM, int TN, bool DB>
__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(ConvArgs a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int RA = BM / 32, RB = BN / 32;  // staged rows per thread (8 threads per row)
  constexpr int NB = DB ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float As[NB][BM * LDSP];
  __shared__ __attribute__((aligned(16))) float Bs[NB][BN * LDSP];

  // XCD-aware tile order: consecutive tiles (the Cout tiles of one pixel tile
  // and neighbouring pixel tiles, which share input halo rows) land on one XCD.
  const int orig = blockIdx.x;
  const int q = a.ntiles / 8, r8 = a.ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int mt = tile / a.nN, nt = tile - mt * a.nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int split = blockIdx.y;
  const int kt0 = split * a.kt_per_split;
  const int kt1 = min(a.nk, kt0 + a.kt_per_split);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;

  const int srow = tid >> 3, schunk = (tid & 7) * 4;
  int pn[RA], ph[RA], pw[RA];
  bool pv[RA];
#pragma unroll
  for (int p = 0; p < RA; ++p) {
    const int m = m0 + srow + 32 * p;
    pv[p] = m < a.M;
    const int mm = pv[p] ? m : 0;
    pn[p] = mm / (a.OH * a.OW);
    const int rem = mm - pn[p] * a.OH * a.OW;
    ph[p] = rem / a.OW;
    pw[p] = rem - ph[p] * a.OW;
  }

  float4 ra[RA], rb[RB];
  auto load_tile = [&](int kt) {
    const int tap = kt / a.cchunks;
    const int c0 = (kt - tap * a.cchunks) * BK + schunk;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const bool cok = c0 < a.Cin;
#pragma unroll
    for (int p = 0; p < RA; ++p) {
      const int ih = ph[p] * a.stride - a.pad + kh;
      const int iw = pw[p] * a.stride - a.pad + kw;
      const bool ok = cok && pv[p] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      ra[p] = ok ? ld4(a.x + (((size_t)pn[p] * a.H + ih) * a.W + iw) * a.Cin + c0)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int co = n0 + srow + 32 * p;
      rb[p] = (cok && co < a.Cout) ? ld4(a.w + (((size_t)tap * a.Cout + co) * a.Cin + c0))
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int p = 0; p < RA; ++p)
      *reinterpret_cast<float4*>(&As[buf][(srow + 32 * p) * LDSP + schunk]) = ra[p];
#pragma unroll
    for (int p = 0; p < RB; ++p)
      *reinterpret_cast<float4*>(&Bs[buf][(srow + 32 * p) * LDSP + schunk]) = rb[p];
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      const float* A = As[buf];
      const float* B = Bs[buf];
#pragma unroll
      for (int s0 = 0; s0 < 16; s0 += 4) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[i] = *reinterpret_cast<const float4*>(
              &A[((wr * TM + i) * 32 + li) * LDSP + lh * 16 + s0]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const float4*>(
              &B[((wc * TN + j) * 32 + li) * LDSP + lh * 16 + s0]);
#pragma unroll
        for (int ss = 0; ss < 4; ++ss)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][ss], fb[j][ss], acc[i][j],
                                                                0, 0, 0);
      }
      if (DB) {
        if (more) store_tile(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      } else {
        __syncthreads();
        if (more) {
          store_tile(0);
          __syncthreads();
        }
      }
    }
  }

  // C/D map for 32x32: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool simple = a.splits == 1 && !a.topdown && !a.residual;
  const bool relu = (a.flags & kRelu) != 0;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + (wc * TN + j) * 32 + li;
    if (co >= a.Cout) continue;
    const float bv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + (wr * TM + i) * 32 + 4 * lh;
      if (simple) {  // bias (+ relu) only: the common case, no per-element branches
        float* yp = a.y + (size_t)mb * a.Cout + co;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          if (mb + dm < a.M) {
            float v = acc[i][j][r] + bv;
            yp[(size_t)dm * a.Cout] = relu ? fmaxf(v, 0.f) : v;
          }
        }
        continue;
      }
      if (a.splits > 1) {
        float* pp = a.partial + ((size_t)split * a.M + mb) * a.Cout + co;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          if (mb + dm < a.M) pp[(size_t)dm * a.Cout] = acc[i][j][r];
        }
        continue;
      }
      // residual / top-down operands: all 16 loads issued before any store
      // (y may not alias them; without this the loads serialise behind the stores)
      float add[16];
      // pixel coordinates of row mb, then stepped (dm < 32): no per-element division
      int tn = 0, toh = 0, tow = 0, last = 0;
      if (a.topdown) {
        const int mm = min(mb, a.M - 1);
        tn = mm / (a.OH * a.OW);
        const int rem = mm - tn * a.OH * a.OW;
        toh = rem / a.OW;
        tow = rem - toh * a.OW;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const int m = mb + dm;
        float v = 0.f;
        if (a.topdown) {  // advance (n, oh, ow) from row mb + last to mb + dm
          tow += dm - last;
          last = dm;
          while (tow >= a.OW) {
            tow -= a.OW;
            if (++toh == a.OH) { toh = 0; ++tn; }
          }
        }
        if (m < a.M) {
          if (a.residual) v = a.residual[(size_t)m * a.Cout + co];
          if (a.topdown)
            v = v + a.topdown[(((size_t)tn * a.tdH + (toh >> 1)) * a.tdW + (tow >> 1)) * a.Cout +
                              co];
        }
        add[r] = v;
      }
      const bool relu_after = (a.flags & kReluAfterResidual) != 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bv;
        if (relu && !relu_after) v = fmaxf(v, 0.f);
        // epilogue() order: conv + bias, (+ top-down) (+ residual)
        if (a.topdown && a.residual) {
          v = epilogue(a, acc[i][j][r], m, co);
        } else {
          v = v + add[r];
          if (relu && relu_after) v = fmaxf(v, 0.f);
        }
        a.y[(size_t)m * a.Cout + co] = v;
      }
    }
  }
}

// Fixed-order split-K reduction + epilogue (deterministic).
__global__ void splitk_reduce_kernel(ConvArgs a) {
  const int64_t total = (int64_t)a.M * a.Cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < a.splits; ++s) acc += a.partial[(size_t)s * total + i];
    const int m = (int)(i / a.Cout), co = (int)(i - (int64_t)m * a.Cout);
    a.y[i] = epilogue(a, acc, m, co);
  }
}

__global__ void pack_weights_kernel(const float* __restrict__ w, int taps, int Cin, int Cout,
                                    float* __restrict__ out) {
  const int64_t total = (int64_t)taps * Cin * Cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ci = i % Cin;  // i indexes the output [tap][co][ci]
    const int64_t t2 = i / Cin;
    const int64_t co = t2 % Cout;
    const int64_t tap = t2 / Cout;
    out[i] = w[(tap * Cin + ci) * Cout + co];
  }
}

struct Plan {
  int cfg;  // 0: 128x128, 1: 128x64, 2: 128x32
  int BM, BN, splits, kt_per_split, nk, ntiles;
};

Plan make_plan(int M, int Cout, int KH, int KW, int Cin) {
  Plan p;
  p.cfg = Cout <= 32 ? 2 : (Cout <= 64 ? 1 : 0);
  p.BM = 128;
  p.BN = p.cfg == 0 ? 128 : (p.cfg == 1 ? 64 : 32);
  const int nM = (M + p.BM - 1) / p.BM, nN = (Cout + p.BN - 1) / p.BN;
  p.ntiles = nM * nN;
  p.nk = KH * KW * ((Cin + BK - 1) / BK);
  p.splits = 1;
  // Fewer tiles than 2 workgroups per CU (512) and a long K: split K.
  if (p.ntiles < 384 && p.nk >= 16) {
    p.splits = std::min(std::max(1, 512 / p.ntiles), std::min(p.nk / 8, 16));
  }
  p.kt_per_split = (p.nk + p.splits - 1) / p.splits;
  p.splits = (p.nk + p.kt_per_split - 1) / p.kt_per_split;
  return p;
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

static int conv_dims(int H, int W, int KH, int KW, int stride, int pb, int pe, int& OH, int& OW) {
  OH = (H + pb + pe - KH) / stride + 1;
  OW = (W + pb + pe - KW) / stride + 1;
  return (OH > 0 && OW > 0) ? 0 : -1;
}

extern "C" size_t d2mi_conv2d_workspace_size(int N, int H, int W, int Cin, int Cout, int KH,
                                             int KW, int stride, int pad_beg, int pad_end) {
  int OH, OW;
  if (conv_dims(H, W, KH, KW, stride, pad_beg, pad_end, OH, OW)) return 0;
  const Plan p = make_plan(N * OH * OW, Cout, KH, KW, Cin);
  return p.splits > 1 ? (size_t)p.splits * N * OH * OW * Cout * sizeof(float) : 0;
}

extern "C" int d2mi_conv2d_nhwc_ex(const float* x, const float* w_packed, const float* bias,
                                   const float* topdown, const float* residual, float* y, int N,
                                   int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                   int pad_beg, int pad_end, int flags, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0,
               "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0, "Cin must be a multiple of 4 (got %d)", Cin);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_packed & 15) == 0,
               "x and w must be 16-byte aligned");
  D2MI_REQUIRE((flags & ~3) == 0, "flags: bit0 relu, bit1 relu after the residual/top-down add");
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
  D2MI_REQUIRE(conv_dims(H, W, KH, KW, stride, pad_beg, pad_end, a.OH, a.OW) == 0,
               "conv output is empty");
  a.flags = flags;
  a.M = N * a.OH * a.OW;
  Plan p = make_plan(a.M, Cout, KH, KW, Cin);
  const size_t need = p.splits > 1 ? (size_t)p.splits * a.M * Cout * sizeof(float) : 0;
  if (need > workspace_bytes || workspace == nullptr) {  // no workspace: no split-K
    p.splits = 1;
    p.kt_per_split = p.nk;
  }
  a.nM = (a.M + p.BM - 1) / p.BM;
  a.nN = (Cout + p.BN - 1) / p.BN;
  a.ntiles = p.ntiles;
  a.splits = p.splits;
  a.kt_per_split = p.kt_per_split;
  a.nk = p.nk;
  a.cchunks = (Cin + BK - 1) / BK;
  a.partial = p.splits > 1 ? (float*)workspace : nullptr;
  a.tdH = (a.OH + 1) / 2;
  a.tdW = (a.OW + 1) / 2;
  hipStream_t st = as_stream(stream);
  dim3 grid(a.ntiles, a.splits);
  // workgroups per launch well above 2 per CU: single-buffered (occupancy);
  // otherwise double-buffered.  D2MI_CONV_DB=0/1 forces one (tuning).
  static const char* force = getenv("D2MI_CONV_DB");
  bool db = (size_t)a.ntiles * a.splits < 1024;
  if (force && (force[0] == '0' || force[0] == '1')) db = force[0] == '1';
  if (p.cfg == 0) {
    if (db) hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, false>), grid, dim3(256), 0, st, a);
  } else if (p.cfg == 1) {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 2, true>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 1, true>), grid, dim3(256), 0, st, a);
  }
  D2MI_LAUNCH_CHECK();
  if (a.splits > 1) {
    const int64_t total = (int64_t)a.M * Cout;
    const int g = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, st, a);
    D2MI_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int d2mi_conv2d_nhwc(const float* x, const float* w_packed, const float* bias,
                                const float* topdown, const float* residual, float* y, int N,
                                int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad_beg, int pad_end, int act, void* stream) {
  D2MI_REQUIRE(act == 0 || act == 1, "act must be 0 (none) or 1 (relu)");
  return d2mi_conv2d_nhwc_ex(x, w_packed, bias, topdown, residual, y, N, H, W, Cin, Cout, KH, KW,
                             stride, pad_beg, pad_end, act ? kRelu : 0, nullptr, 0, stream);
}
