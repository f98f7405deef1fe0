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
#include "internal.h"

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
  // the partial slabs are written (splits > 1, or an accumulating call:
  // the reduce then adds the sum into dw / dbias)
  int part;
  int x_bytes, dy_bytes;  // buffer ranges (split kernel; < 2 GiB)
  // D2MI_WGRAD_PRIO (default 1, 0 off): wave priority 1 while issuing the
  // chunk's MFMAs, as conv_mfma.hip.  Measured (tools/ab_prio.sh): the wgrad
  // set 1.9 % faster in total (FPN p2 3x3 1025 -> 1008 us, res5 3x3 97 -> 92),
  // the training bench +1.4 % (89.6 -> 90.9 img/s, two alternating pairs).
  int prio;
  // tuning "wgrad_xcd" (default 1): the (tile, split) grid walked in an
  // XCD-contiguous order -- the tiles of one pixel range (its taps and channel
  // blocks, which read the same x rows and dY chunk) land on one XCD, so the
  // re-reads meet in that XCD's L2 instead of eight.  Bit-identical (each
  // workgroup's (tile, split) work is unchanged, only its placement).
  int xcd;
};

// (tile, split) of this workgroup: blockIdx as launched, or its XCD-contiguous
// remap (hardware dispatch puts linear workgroup L on XCD L % 8; logical index
// l = the L-th of XCD L % 8's contiguous block, tile fastest).
__device__ __forceinline__ void wgrad_tile_split(const WgradArgs& a, int& tile, int& split) {
  if (!a.xcd) {
    tile = blockIdx.x;
    split = blockIdx.y;
    return;
  }
  const int nwg = gridDim.x * gridDim.y;
  const int L = blockIdx.x + blockIdx.y * gridDim.x;
  const int q = nwg / 8, r8 = nwg % 8, x8 = L % 8;
  const int l = (x8 < r8 ? x8 * (q + 1) : r8 * (q + 1) + (x8 - r8) * q) + L / 8;
  split = l / gridDim.x;
  tile = l - split * gridDim.x;
}

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
    if (a.part) a.pbias[(size_t)split * a.Cout + co0 + tid] = bsum;
    else a.dbias[co0 + tid] = bsum;
  }

  // C/D map for 32x32: col (co) = lane & 31, row (ci) = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const size_t wsz = (size_t)a.KH * a.KW * a.Cin * a.Cout;
  float* out = a.part ? a.partial + (size_t)split * wsz : a.dw;
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
// float4 form (total % 4 == 0, 16-B aligned): the same per-element split
// order, four elements and their split loads in flight per thread.
// accum: dw / dbias += the sum (a level accumulator: the old value plus this
// call's gradient, autograd's order for a weight shared by several calls).
__global__ void wgrad_reduce4_kernel(const float4* __restrict__ partial, int splits, size_t total4,
                                     float4* __restrict__ dw, const float* __restrict__ pbias,
                                     int Cout, float* __restrict__ dbias, int accum) {
  const size_t n = total4 + (dbias ? (size_t)Cout : 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    if (i < total4) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
      for (int k = 0; k < splits; ++k) {
        const float4 v = partial[(size_t)k * total4 + i];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
      if (accum) {
        const float4 o = dw[i];
        s.x = o.x + s.x;
        s.y = o.y + s.y;
        s.z = o.z + s.z;
        s.w = o.w + s.w;
      }
      dw[i] = s;
    } else {
      const size_t c = i - total4;
      float s = 0.f;
#pragma unroll 8  // (loads in flight; the sum stays in split order)
      for (int k = 0; k < splits; ++k) s += pbias[(size_t)k * Cout + c];
      dbias[c] = accum ? dbias[c] + s : s;
    }
  }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ partial, int splits, size_t total,
                                    float* __restrict__ dw, const float* __restrict__ pbias,
                                    int Cout, float* __restrict__ dbias, int accum) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total + Cout;
       i += (size_t)gridDim.x * blockDim.x) {
    if (i < total) {
      float s = 0.f;
#pragma unroll 4
      for (int k = 0; k < splits; ++k) s += partial[(size_t)k * total + i];
      dw[i] = accum ? dw[i] + s : s;
    } else if (dbias) {
      const size_t c = i - total;
      float s = 0.f;
#pragma unroll 8  // (loads in flight; the sum stays in split order)
      for (int k = 0; k < splits; ++k) s += pbias[(size_t)k * Cout + c];
      dbias[c] = accum ? dbias[c] + s : s;
    }
  }
}

// ---------------------------------------------------------------------------
// Split-product variant (d2mi_conv2d_wgrad_ex flags bit 2): the same GEMM on
// the bf16 MFMA with each f32 operand split exactly into three bf16 terms
// (h + m + l == x, truncation) and six products per k-step, as
// conv_mfma.hip's SPLIT path.  The MFMA operand wants 8 consecutive PIXELS of
// one channel, so each thread loads 4 pixels x 4 channels (four float4),
// transposes them in registers, splits, and writes 4 pixels (8 B) per plane
// per channel into [plane][channel][32 pixels] LDS images with XOR-swizzled
// 16-B chunks.  The bias gradient is summed from the f32 dY values before
// the split and reduced over the pixel groups in a fixed order.

typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int LDW = 32;  // bf16 per LDS row (one 32-pixel chunk)

__device__ __forceinline__ int wswz(int row, int elem) {
  return row * LDW + ((((elem >> 3) ^ (row >> 2)) & 3) << 3) + (elem & 7);
}

__device__ __forceinline__ void split3w(const float4 v, uint2& h, uint2& m, uint2& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t hb[4], mb[4], lb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hb[e] = __float_as_uint(x[e]) & 0xffff0000u;
    const float r = x[e] - __uint_as_float(hb[e]);
    mb[e] = __float_as_uint(r) & 0xffff0000u;
    lb[e] = __float_as_uint(r - __uint_as_float(mb[e]));
  }
  // each pair packed by one byte permute (the high halves of two words)
  h.x = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
  h.y = __builtin_amdgcn_perm(hb[3], hb[2], 0x07060302u);
  m.x = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
  m.y = __builtin_amdgcn_perm(mb[3], mb[2], 0x07060302u);
  l.x = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
  l.y = __builtin_amdgcn_perm(lb[3], lb[2], 0x07060302u);
}

// n / d for 0 <= n < 2^31 by multiply-high (Granlund-Montgomery).
struct FastDiv {
  uint32_t d, m, l;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.l;
}

template <int TM, int TN, int OCC = 2>
__global__ __launch_bounds__(256, OCC) void conv_wgrad_split_kernel(WgradArgs a, FastDiv fd_hw,
                                                                    FastDiv fd_w) {
  constexpr int BM = 2 * TM * 32, BN = 2 * TN * 32;
  constexpr int GA = BM / 4, GB = BN / 4;  // 4-channel groups
  __shared__ __attribute__((aligned(16))) uint16_t As[3 * BM * LDW];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[3 * BN * LDW];
  __shared__ float bred[8][BN];

  int tile, split;
  wgrad_tile_split(a, tile, split);
  const int per_tap = a.nCi * a.nCo;
  const int tap = tile / per_tap;
  const int rem = tile - tap * per_tap;
  const int cit = rem / a.nCo, cot = rem - cit * a.nCo;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const int ci0 = cit * BM, co0 = cot * BN;
  const int c_begin = split * a.chunks_per_split;
  const int c_end = min(a.nchunks, c_begin + a.chunks_per_split);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  // A items: (cg, pg) = (tid % GA, tid / GA) for tid < 8 * GA; B likewise
  const bool a_on = tid < 8 * GA, b_on = tid < 8 * GB;
  const int cga = tid % GA, pga = tid / GA;
  const int cgb = tid % GB, pgb = tid / GB;
  const int ci = ci0 + 4 * cga, co = co0 + 4 * cgb;
  const bool ci_ok = a_on && ci < a.Cin, co_ok = b_on && co < a.Cout;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x), 0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.dy), 0, a.dy_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;

  float4 ra[4], rb[4];
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = ch * KP + 4 * pga + q;
      const uint32_t n = fdiv((uint32_t)p, fd_hw);
      const int r2 = p - (int)n * (a.OH * a.OW);
      const int oy = (int)fdiv((uint32_t)r2, fd_w), ox = r2 - oy * a.OW;
      const int iy = oy * a.stride - a.pad + kh, ix = ox * a.stride - a.pad + kw;
      const bool ok = ci_ok & (p < a.P) & ((unsigned)iy < (unsigned)a.H) &
                      ((unsigned)ix < (unsigned)a.W);
      const uint32_t off = ok ? (uint32_t)(((((int)n * a.H + iy) * a.W + ix) * a.Cin + ci) * 4) : kOOB;
      ra[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      const int pb = ch * KP + 4 * pgb + q;
      const uint32_t offb = (co_ok & (pb < a.P)) ? (uint32_t)((pb * a.Cout + co) * 4) : kOOB;
      rb[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(yr, offb, 0, 0));
    }
  };
  const bool do_bias = a.dbias != nullptr && tap == 0 && cit == 0;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  auto store_chunk = [&]() {
    if (a_on) {
      const float* f = reinterpret_cast<const float*>(ra);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 h, m, l;
        split3w(make_float4(f[j], f[4 + j], f[8 + j], f[12 + j]), h, m, l);
        const int o = wswz(4 * cga + j, 4 * pga);
        *reinterpret_cast<uint2*>(&As[o]) = h;
        *reinterpret_cast<uint2*>(&As[BM * LDW + o]) = m;
        *reinterpret_cast<uint2*>(&As[2 * BM * LDW + o]) = l;
      }
    }
    if (b_on) {
      const float* f = reinterpret_cast<const float*>(rb);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = make_float4(f[j], f[4 + j], f[8 + j], f[12 + j]);
        if (do_bias) bsum[j] += ((v.x + v.y) + v.z) + v.w;
        uint2 h, m, l;
        split3w(v, h, m, l);
        const int o = wswz(4 * cgb + j, 4 * pgb);
        *reinterpret_cast<uint2*>(&Bs[o]) = h;
        *reinterpret_cast<uint2*>(&Bs[BN * LDW + o]) = m;
        *reinterpret_cast<uint2*>(&Bs[2 * BN * LDW + o]) = l;
      }
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (c_begin < c_end) {
    load_chunk(c_begin);
    for (int ch = c_begin; ch < c_end; ++ch) {
      store_chunk();
      __syncthreads();
      if (ch + 1 < c_end) load_chunk(ch + 1);
      if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fa[3][TM], fb[3][TN];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[pl][i] = *reinterpret_cast<const bf16x8*>(
                &As[pl * BM * LDW + wswz((wr * TM + i) * 32 + li, ks * 16 + lh * 8)]);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[pl][j] = *reinterpret_cast<const bf16x8*>(
                &Bs[pl * BN * LDW + wswz((wc * TN + j) * 32 + li, ks * 16 + lh * 8)]);
        }
        constexpr int PAi[6] = {1, 2, 0, 0, 1, 0};
        constexpr int PBi[6] = {1, 0, 2, 1, 0, 0};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PAi[t]][i], fb[PBi[t]][j],
                                                                   acc[i][j], 0, 0, 0);
      }
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      __syncthreads();
    }
  }

  if (do_bias) {  // fixed-order reduction over the 8 pixel groups
    if (b_on) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bred[pgb][4 * cgb + j] = bsum[j];
    }
    __syncthreads();
    if (tid < BN && co0 + tid < a.Cout) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) s += bred[g][tid];
      if (a.part) a.pbias[(size_t)split * a.Cout + co0 + tid] = s;
      else a.dbias[co0 + tid] = s;
    }
  }

  const size_t wsz = (size_t)a.KH * a.KW * a.Cin * a.Cout;
  float* out = a.part ? a.partial + (size_t)split * wsz : a.dw;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int oc = co0 + (wc * TN + j) * 32 + li;
    if (oc >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cb = ci0 + (wr * TM + i) * 32 + 4 * lh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = cb + (r & 3) + 8 * (r >> 2);
        if (c < a.Cin) out[((size_t)tap * a.Cin + c) * a.Cout + oc] = acc[i][j][r];
      }
    }
  }
}


// Warp-specialised split wgrad (the conv_ws_kernel structure of
// conv_mfma.hip for the weight gradient): a 256 (ci) x 128 (co) tile of one
// tap, 16 waves, one workgroup per CU.  Waves 0-7 compute (4 x 2 blocks of
// 64 x 64, ds_read + MFMA only); waves 8-15 stage: the 32-pixel chunks of X
// (shifted by the tap) and dY into registers two chunks ahead, transposed to
// [channel][pixel], split exactly into bf16 planes and written to one of two
// LDS stages; one barrier per chunk.  Stager threads 0-511 each own one
// (4-channel, 4-pixel) item of X; threads 256-511 also one item of dY (and
// its bias-gradient partial sums, reduced in the fixed order of the 128 x 128
// kernel).  Same pixel order, product order and accumulation sequence as
// conv_wgrad_split_kernel: bit-identical for equal pixel splits.
template <int LD, bool INC = false>
__global__ __launch_bounds__(1024, 1) void conv_wgrad_ws_kernel(WgradArgs a, FastDiv fd_hw,
                                                                FastDiv fd_w) {
  constexpr int TM = 2, TN = 2, BM = 256, BN = 128, S = 2;
  constexpr int GA = BM / 4, GB = BN / 4;  // 4-channel groups
  constexpr int A_H = 3 * BM * LDW, B_H = 3 * BN * LDW;  // halfwords per stage
  constexpr int STAGE = A_H + B_H;                      // 36864 halfwords = 72 KiB
  __shared__ __attribute__((aligned(16))) uint16_t smem[S * STAGE];
  __shared__ float bred[8][BN];

  int tile, split;
  wgrad_tile_split(a, tile, split);
  const int per_tap = a.nCi * a.nCo;
  const int tap = tile / per_tap;
  const int rem = tile - tap * per_tap;
  const int cit = rem / a.nCo, cot = rem - cit * a.nCo;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const int ci0 = cit * BM, co0 = cot * BN;
  const int c_begin = split * a.chunks_per_split;
  const int c_end = min(a.nchunks, c_begin + a.chunks_per_split);
  const int nks = max(c_end - c_begin, 0);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;  // compute waves 0-7: 4 x 2
  const int li = lane & 31, lh = lane >> 5;
  const bool do_bias = a.dbias != nullptr && tap == 0 && cit == 0;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (wave >= 8) {
    // ------------------------------------------------------------ stagers
    const int st = tid - 512;
    const int cga = st % GA, pga = st / GA;             // X item (all 512)
    const bool b_on = st >= 256;                        // dY item (threads 256-511)
    const int sb = st - 256;
    const int cgb = (b_on ? sb : 0) % GB, pgb = (b_on ? sb : 0) / GB;
    const int ci = ci0 + 4 * cga, co = co0 + 4 * cgb;
    const bool ci_ok = ci < a.Cin, co_ok = b_on && co < a.Cout;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x), 0, a.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.dy), 0, a.dy_bytes, 0x00020000);
    constexpr uint32_t kOOB = 0x80000000u;
    float4 ra[LD][4], rb[LD][4];
    // The loads walk the split's chunks in order (then the last one again).
    // INC (same-size stride-1 convs: the 3x3 / 1x1 this kernel takes, see
    // the launch): input pixel = output pixel + a uniform tap shift, so a
    // per-thread (oy, ox) cursor of its first pixel, advanced by 32 pixels
    // per chunk, gives the range test, and 24-bit multiplies the offsets --
    // two fast divisions and four 32-bit multiplies per pixel fewer.  Else
    // per-pixel division.  dY offsets advance by one uniform stride.  Same
    // addresses either way.
    const int clast = c_begin + max(nks, 1) - 1;
    int c_ch = c_begin;
    int p0 = c_begin * KP + 4 * pga;   // first of this thread's 4 X pixels
    int pb0 = c_begin * KP + 4 * pgb;  // (dY)
    int oy0 = 0, ox0 = 0;
    if (INC) {
      const int r2 = p0 - (int)fdiv((uint32_t)p0, fd_hw) * (a.OH * a.OW);
      oy0 = (int)fdiv((uint32_t)r2, fd_w);
      ox0 = r2 - oy0 * a.OW;
    }
    const int dy32 = KP / a.OW, dx32 = KP - (KP / a.OW) * a.OW;  // (uniform)
    const int ybase = kh - a.pad, xbase = kw - a.pad;
    const int tsh = ybase * a.W + xbase;  // INC: input pixel - output pixel
    const uint32_t bstride = (uint32_t)KP * (uint32_t)a.Cout * 4u;
    uint32_t boff = (uint32_t)(pb0 * a.Cout + co) * 4u;
    auto load = [&](float4 (&la)[4], float4 (&lb)[4]) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = p0 + q;
        uint32_t off;
        if (INC) {
          int ox = ox0 + q, oy = oy0;
          const bool wrap = ox >= a.OW;
          ox = wrap ? ox - a.OW : ox;
          oy = wrap ? oy + 1 : oy;
          oy = oy >= a.OH ? oy - a.OH : oy;
          const bool ok = ci_ok & (p < a.P) & ((unsigned)(oy + ybase) < (unsigned)a.H) &
                          ((unsigned)(ox + xbase) < (unsigned)a.W);
          off = ok ? (__umul24((uint32_t)(p + tsh), (uint32_t)a.Cin) + (uint32_t)ci) * 4u : kOOB;
        } else {
          const int n = (int)fdiv((uint32_t)p, fd_hw);
          const int r2 = p - n * (a.OH * a.OW);
          const int oy = (int)fdiv((uint32_t)r2, fd_w), ox = r2 - oy * a.OW;
          const int iy = oy * a.stride - a.pad + kh, ix = ox * a.stride - a.pad + kw;
          const bool ok = ci_ok & (p < a.P) & ((unsigned)iy < (unsigned)a.H) &
                          ((unsigned)ix < (unsigned)a.W);
          off = ok ? (uint32_t)(((((int)n * a.H + iy) * a.W + ix) * a.Cin + ci) * 4) : kOOB;
        }
        la[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        const uint32_t offb = (co_ok & (pb0 + q < a.P)) ? boff + (uint32_t)(q * a.Cout * 4) : kOOB;
        lb[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(yr, offb, 0, 0));
      }
      if (c_ch < clast) {  // advance to the next chunk (uniform condition)
        ++c_ch;
        p0 += KP;
        pb0 += KP;
        boff += bstride;
        if (INC) {
          ox0 += dx32;
          oy0 += dy32;
          const bool wrap = ox0 >= a.OW;
          ox0 = wrap ? ox0 - a.OW : ox0;
          oy0 = wrap ? oy0 + 1 : oy0;
          oy0 = oy0 >= a.OH ? oy0 - a.OH : oy0;
        }
      }
    };
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    auto write = [&](int buf, const float4 (&la)[4], const float4 (&lb)[4]) {
      uint16_t* As = smem + buf * STAGE;
      uint16_t* Bs = As + A_H;
      const float* f = reinterpret_cast<const float*>(la);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint2 h, m, l;
        split3w(make_float4(f[j], f[4 + j], f[8 + j], f[12 + j]), h, m, l);
        const int o = wswz(4 * cga + j, 4 * pga);
        *reinterpret_cast<uint2*>(&As[o]) = h;
        *reinterpret_cast<uint2*>(&As[BM * LDW + o]) = m;
        *reinterpret_cast<uint2*>(&As[2 * BM * LDW + o]) = l;
      }
      if (b_on) {
        const float* g = reinterpret_cast<const float*>(lb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 v = make_float4(g[j], g[4 + j], g[8 + j], g[12 + j]);
          if (do_bias) bsum[j] += ((v.x + v.y) + v.z) + v.w;
          uint2 h, m, l;
          split3w(v, h, m, l);
          const int o = wswz(4 * cgb + j, 4 * pgb);
          *reinterpret_cast<uint2*>(&Bs[o]) = h;
          *reinterpret_cast<uint2*>(&Bs[BN * LDW + o]) = m;
          *reinterpret_cast<uint2*>(&Bs[2 * BN * LDW + o]) = l;
        }
      }
    };
    // unconditional loads (chunks past the end re-load the last one): hipcc
    // then counts the loads in flight instead of draining them
#pragma unroll
    for (int j = 0; j < LD; ++j) load(ra[j], rb[j]);
    if (nks > 0) write(0, ra[0], rb[0]);
    load(ra[0], rb[0]);
    __syncthreads();  // B_{-1}
    int u0 = 0;
    for (; u0 + LD <= nks; u0 += LD) {
#pragma unroll
      for (int j = 0; j < LD; ++j) {
        const int v = u0 + j + 1;
        const int set = (j + 1) % LD;
        if (v < nks) write(v & 1, ra[set], rb[set]);
        load(ra[set], rb[set]);  // chunk v + LD (clamped)
        __syncthreads();  // B_u
      }
    }
#pragma unroll
    for (int j = 0; j < LD - 1; ++j) {
      if (u0 + j < nks) {
        const int v = u0 + j + 1;
        const int set = (j + 1) % LD;
        if (v < nks) write(v & 1, ra[set], rb[set]);
        __syncthreads();
      }
    }
    if (do_bias && b_on) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bred[pgb][4 * cgb + j] = bsum[j];
    }
  } else {
    // ------------------------------------------------------------ compute
    bf16x8 fa[3][TM], fb[3][TN];
    auto ld1 = [&](const uint16_t* As, const uint16_t* Bs, int pa, int pb, int ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[pa][i] = *reinterpret_cast<const bf16x8*>(
            &As[pa * BM * LDW + wswz((wr * TM + i) * 32 + li, ks * 16 + lh * 8)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[pb][j] = *reinterpret_cast<const bf16x8*>(
            &Bs[pb * BN * LDW + wswz((wc * TN + j) * 32 + li, ks * 16 + lh * 8)]);
    };
    auto mm1 = [&](int pa, int pb) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[pa][i], fb[pb][j], acc[i][j], 0, 0, 0);
    };
    // products in the split kernel's order {mm, lh, hl, hm, mh, hh}, reads in
    // three plane batches one MFMA group ahead of their first use
    auto step16 = [&](const uint16_t* As, const uint16_t* Bs, int ks) {
      ld1(As, Bs, 1, 1, ks);
      __builtin_amdgcn_sched_barrier(0);
      ld1(As, Bs, 2, 0, ks);
      mm1(1, 1);
      __builtin_amdgcn_sched_barrier(0);
      ld1(As, Bs, 0, 2, ks);
      mm1(2, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm1(0, 2);
      mm1(0, 1);
      mm1(1, 0);
      mm1(0, 0);
    };
    __syncthreads();  // B_{-1}
    for (int u = 0; u < nks; ++u) {
      const uint16_t* As = smem + (u & 1) * STAGE;
      const uint16_t* Bs = As + A_H;
      if (a.prio) __builtin_amdgcn_s_setprio(1);
      step16(As, Bs, 0);
      step16(As, Bs, 1);
      if (a.prio) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();  // B_u
    }
  }
  if (do_bias) {  // fixed-order reduction over the 8 pixel groups
    __syncthreads();
    if (tid < BN && co0 + tid < a.Cout) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) s += bred[g][tid];
      if (a.part) a.pbias[(size_t)split * a.Cout + co0 + tid] = s;
      else a.dbias[co0 + tid] = s;
    }
  }
  if (wave >= 8) return;
  const size_t wsz = (size_t)a.KH * a.KW * a.Cin * a.Cout;
  float* out = a.part ? a.partial + (size_t)split * wsz : a.dw;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int oc = co0 + (wc * TN + j) * 32 + li;
    if (oc >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cb = ci0 + (wr * TM + i) * 32 + 4 * lh;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = cb + (r & 3) + 8 * (r >> 2);
        if (c < a.Cin) out[((size_t)tap * a.Cin + c) * a.Cout + oc] = acc[i][j][r];
      }
    }
  }
}

FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.l = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}

struct WPlan {
  int TM, TN, BM, BN, ntiles, splits, chunks_per_split, nchunks;
  bool occ3;
  bool ws;  // conv_wgrad_ws_kernel (256 x 128 tiles, one workgroup per CU)
};

// The 128x128 split wgrad can run three workgroups per CU (168 VGPRs, 52 KiB
// LDS).  Measured (tools/conv_ab.py --set wgrad): 3% faster on the FPN p2 3x3
// (134,400 pixels), slower on everything smaller (the extra pixel splits cost
// more partial traffic than the occupancy gains), so only pixel counts of
// 64k and up take it.  D2MI_WGRAD_OCC=2 disables it (A/B).
static bool wgrad_occ3() {
  static const int on = [] {
    const char* e = getenv("D2MI_WGRAD_OCC");
    return !(e && e[0] == '2');
  }();
  return on;
}

// split3: the split-product math (the warp-specialised kernel exists only in
// that form).  It takes the KxK convs with Cin % 256 == 0, Cout % 128 == 0
// (tuning "wgrad_ws"; tools/ws_ab.py --key wgrad_ws: 3x3 shapes 10-20 %
// faster, the 1x1s 9 % slower -- their 8 chunks of 32 pixels per split are
// too short for its prologue).
WPlan wplan(int N, int OH, int OW, int Cin, int Cout, int KH, int KW, bool split3 = true) {
  WPlan p;
  // 128 x 128 tiles for 256-wide channels; 64-wide when a dimension is small
  p.TM = Cin > 64 ? 2 : 1;
  p.TN = Cout > 64 ? 2 : 1;
  // 1x1s (tuning "wgrad_ws1"): only from ~6 GFLOP up -- the smaller ones have
  // too few 256x128 tiles x 16-chunk splits to fill the chip (tools/wgrad_ws1_ab.sh:
  // the FPN p2 lateral 165 -> 140 us, the strided shortcuts 8-13 % faster,
  // the 4.4 GFLOP res4 1x1s 7 % slower)
  // (tuning value = the GFLOP threshold; 0 = off)
  const bool ws1 = KH * KW == 1 && tuning(kTuneWgradWS1) > 0 &&
                   2.0 * N * OH * OW * (double)Cin * Cout >= tuning(kTuneWgradWS1) * 1e9;
  p.ws = split3 && tuning(kTuneWgradWS) > 0 && (KH * KW > 1 || ws1) && Cin % 256 == 0 &&
         Cout % 128 == 0;
  p.BM = p.ws ? 256 : 64 * p.TM;
  p.BN = 64 * p.TN;
  p.ntiles = KH * KW * ((Cin + p.BM - 1) / p.BM) * ((Cout + p.BN - 1) / p.BN);
  const long long P = (long long)N * OH * OW;
  p.nchunks = (int)((P + KP - 1) / KP);
  // about one round of resident workgroups (2 or 3 per CU), each walking
  // >= 16 chunks
  // D2MI_WGRAD_OCC3_MIN_P: the pixel count from which the 3-per-CU kernel runs (A/B)
  static const long long occ3_min_p = [] {
    const char* e = getenv("D2MI_WGRAD_OCC3_MIN_P");
    return e ? atoll(e) : 65536LL;
  }();
  p.occ3 = !p.ws && p.TM == 2 && p.TN == 2 && P >= occ3_min_p && wgrad_occ3();
  // D2MI_WGRAD_SLOTS / D2MI_WGRAD_MINCH: the split target and the minimum
  // chunks per split (A/B knobs)
  static const int slots_env = [] {
    const char* e = getenv("D2MI_WGRAD_SLOTS");
    return e ? atoi(e) : 0;
  }();
  static const int minch = [] {
    const char* e = getenv("D2MI_WGRAD_MINCH");
    return e && atoi(e) > 0 ? atoi(e) : 16;
  }();
  const int G = slots_env > 0 ? slots_env : (p.ws ? 256 : (p.occ3 ? 768 : 512));
  int splits = std::max(1, G / p.ntiles);
  splits = std::min(splits, std::max(1, p.nchunks / minch));
  // D2MI_WGRAD_MAXSPLIT: the cap on splits (A/B knob)
  static const int maxsplit = [] {
    const char* e = getenv("D2MI_WGRAD_MAXSPLIT");
    return e && atoi(e) > 0 ? atoi(e) : 128;
  }();
  splits = std::min(splits, maxsplit);
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
  // the larger of the split-product and the f32 plans (either math mode fits)
  const int s = std::max(wplan(N, OH, OW, Cin, Cout, KH, KW, true).splits,
                         wplan(N, OH, OW, Cin, Cout, KH, KW, false).splits);
  return s > 1 ? (size_t)s * ((size_t)KH * KW * Cin * Cout + Cout) * sizeof(float) : 0;
}

extern "C" int d2mi_conv2d_wgrad_ex(const float* x, const float* dy, float* dw_hwio,
                                    float* dbias, int N, int H, int W, int Cin, int Cout, int KH,
                                    int KW, int stride, int pad_beg, int pad_end, int flags,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE((flags & ~12) == 0,
               "wgrad flags: bit2 = split-bf16 products, bit3 = accumulate into dw / dbias");
  const bool accum = (flags & 8) != 0;
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0,
               "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0 && Cout % 4 == 0, "Cin and Cout must be multiples of 4 (%d, %d)",
               Cin, Cout);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0,
               "x and dy must be 16-byte aligned");
  WgradArgs a = {};
  {
    static const char* e = getenv("D2MI_WGRAD_PRIO");
    a.prio = e ? atoi(e) : 1;
  }
  a.xcd = tuning(kTuneWgradXCD) > 0 ? 1 : 0;
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
  const bool split3 = (flags & 4) != 0;
  WPlan p = wplan(N, a.OH, a.OW, Cin, Cout, KH, KW, split3);
  const size_t need =
      p.splits > 1 ? (size_t)p.splits * ((size_t)KH * KW * Cin * Cout + Cout) * sizeof(float) : 0;
  if (need > workspace_bytes || workspace == nullptr) {  // no workspace: one split
    p.splits = 1;
    p.chunks_per_split = p.nchunks;
  }
  if (accum)  // the sum goes through the reduce, which adds it: one slab at least
    D2MI_REQUIRE(workspace != nullptr &&
                     workspace_bytes >= (size_t)p.splits *
                                            ((size_t)KH * KW * Cin * Cout + Cout) * sizeof(float),
                 "accumulating wgrad: workspace must hold %d slab(s)", p.splits);
  a.nCi = (Cin + p.BM - 1) / p.BM;
  a.nCo = (Cout + p.BN - 1) / p.BN;
  a.ntiles = p.ntiles;
  a.splits = p.splits;
  a.chunks_per_split = p.chunks_per_split;
  a.nchunks = p.nchunks;
  a.part = p.splits > 1 || accum;
  a.partial = a.part ? (float*)workspace : nullptr;
  a.pbias = a.part ? (float*)workspace + (size_t)p.splits * KH * KW * Cin * Cout : nullptr;
  hipStream_t st = as_stream(stream);
  dim3 grid(a.ntiles, a.splits);
  if (split3) {
    D2MI_REQUIRE((int64_t)N * H * W * Cin * 4 < (1ll << 31) &&
                     (int64_t)a.P * Cout * 4 < (1ll << 31),
                 "split wgrad: x and dy must each be < 2 GiB");
    a.x_bytes = (int)((int64_t)N * H * W * Cin * 4);
    a.dy_bytes = (int)((int64_t)a.P * Cout * 4);
    const FastDiv fhw = make_fastdiv((uint32_t)(a.OH * a.OW)), fw = make_fastdiv((uint32_t)a.OW);
    // tuning wgrad_ws: 1 = loads one chunk ahead (no spills), 2 = two chunks
    // ahead (10 VGPRs of the stagers' ring spill at the 128-VGPR budget)
    // the incremental pixel cursor (conv_wgrad_ws_kernel INC): same-size
    // stride-1 convs whose per-thread runs of 4 pixels and 32-pixel chunk
    // steps wrap at most one row and one image, pixel indices < 2^24
    const bool inc = a.stride == 1 && a.OH == H && a.OW == W && a.OW >= 4 &&
                     KP / a.OW + 1 <= a.OH && (int64_t)a.P + KP < (1 << 24) &&
                     tuning(kTuneWgradInc) > 0;
    if (p.ws && tuning(kTuneWgradWS) >= 2)
      hipLaunchKernelGGL((conv_wgrad_ws_kernel<2>), grid, dim3(1024), 0, st, a, fhw, fw);
    else if (p.ws && inc)
      hipLaunchKernelGGL((conv_wgrad_ws_kernel<1, true>), grid, dim3(1024), 0, st, a, fhw, fw);
    else if (p.ws)
      hipLaunchKernelGGL((conv_wgrad_ws_kernel<1>), grid, dim3(1024), 0, st, a, fhw, fw);
    else if (p.occ3)
      hipLaunchKernelGGL((conv_wgrad_split_kernel<2, 2, 3>), grid, dim3(256), 0, st, a, fhw, fw);
    else if (p.TM == 2 && p.TN == 2)
      hipLaunchKernelGGL((conv_wgrad_split_kernel<2, 2>), grid, dim3(256), 0, st, a, fhw, fw);
    else if (p.TM == 2)
      hipLaunchKernelGGL((conv_wgrad_split_kernel<2, 1>), grid, dim3(256), 0, st, a, fhw, fw);
    else if (p.TN == 2)
      hipLaunchKernelGGL((conv_wgrad_split_kernel<1, 2>), grid, dim3(256), 0, st, a, fhw, fw);
    else
      hipLaunchKernelGGL((conv_wgrad_split_kernel<1, 1>), grid, dim3(256), 0, st, a, fhw, fw);
  } else if (p.TM == 2 && p.TN == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 2>), grid, dim3(256), 0, st, a);
  else if (p.TM == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 1>), grid, dim3(256), 0, st, a);
  else if (p.TN == 2)
    hipLaunchKernelGGL((conv_wgrad_kernel<1, 2>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<1, 1>), grid, dim3(256), 0, st, a);
  D2MI_LAUNCH_CHECK();
  if (a.part) {
    const size_t total = (size_t)KH * KW * Cin * Cout;
    if (total % 4 == 0 && ((uintptr_t)a.partial & 15) == 0 && ((uintptr_t)dw_hwio & 15) == 0) {
      const size_t total4 = total / 4;
      const int g4 = (int)std::min<size_t>((total4 + Cout + 255) / 256, 8192);
      hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3(g4), dim3(256), 0, st,
                         reinterpret_cast<const float4*>(a.partial), a.splits, total4,
                         reinterpret_cast<float4*>(dw_hwio), a.pbias, Cout, dbias, (int)accum);
    } else {
      const int g = (int)std::min<size_t>((total + Cout + 255) / 256, 4096);
      hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(g), dim3(256), 0, st, a.partial, a.splits,
                         total, dw_hwio, a.pbias, Cout, dbias, (int)accum);
    }
    D2MI_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int d2mi_conv2d_wgrad(const float* x, const float* dy, float* dw_hwio, float* dbias,
                                 int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                 int stride, int pad_beg, int pad_end, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  return d2mi_conv2d_wgrad_ex(x, dy, dw_hwio, dbias, N, H, W, Cin, Cout, KH, KW, stride,
                              pad_beg, pad_end, 0, workspace, workspace_bytes, stream);
}
