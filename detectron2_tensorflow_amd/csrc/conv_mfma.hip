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
//
// SPLIT variant (flags bit 2, kSplit3): the same f32 operands, multiplied on
// the bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate per clock).
// Each f32 x is split EXACTLY into three bf16 terms by truncation,
//   h = x & 0xffff0000,  m = (x - h) & 0xffff0000,  l = x - h - m,
// (8 + 8 + 8 significant bits = f32's 24: h + m + l == x bit for bit), and
// a*b is formed from the six products whose order is <= 2^-16 relative,
//   ah*bh + ah*bm + am*bh + ah*bl + am*bm + al*bh,
// dropping am*bl + al*bm + al*bl (<= 2^-23 * |a*b| together, below f32's own
// rounding of the product, 2^-24 relative per accumulation step on top).
// The 3 bf16 planes of each staged A/B tile live in LDS as [plane][row][32]
// with XOR-swizzled 16-B chunks (swz(): conflict-free reads and writes).  Six bf16 MFMAs per 32x32x16 step = 2.67x the f32-MFMA rate at
// f32-class error (tests: error vs float64 within a small factor of the
// native f32 path's).
#include "common.h"
#include "internal.h"

#include <mutex>
#include <vector>

namespace d2mi {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32, LDSP = 36, LDSB = 32;
constexpr int kMaxConvLevels = 6;

// bf16 LDS images: 64-B rows (32 bf16 = one BK step) whose four 16-B chunks
// are XOR-swizzled by (row >> 2) & 3.  ds_read_b128 phases (lanes
// {0-3,12-15,20-27}, ... reading one chunk of 16 rows) and ds_write_b128 /
// b64 phases (2 whole rows) then touch every bank once: conflict-free.
__device__ __forceinline__ int swz(int row, int elem) {
  return row * LDSB + ((((elem >> 3) ^ (row >> 2)) & 3) << 3) + (elem & 7);
}

typedef short bf16x8 __attribute__((ext_vector_type(8)));

// kFlipTaps: read weight tap (KH*KW - 1 - tap) -- the spatially flipped kernel
// of a stride-1 dgrad, without materialising the flipped copy.
// kMaskByResidual: the residual operand is a ReLU output whose mask gates the
// result, out = residual > 0 ? conv + bias : 0 (a dgrad with the producer's
// ReLU backward fused; no add).  The host turns it into ConvArgs::gate; the
// gated entry point (d2mi_conv2d_nhwc_gated) passes a gate AND a residual:
// out = gate > 0 ? conv + bias + residual : 0 (a dgrad that also takes the
// other consumer's gradient of the same ReLU output).
enum EpiFlags {
  kRelu = 1, kReluAfterResidual = 2, kSplit3 = 4, kFlipTaps = 8, kMaskByResidual = 16
};

// Compile-time ablation bits of the split conv kernels, for timing
// experiments only: an ablation build of the library (tools/, D2MI_LIB)
// passes -DD2MI_CONV_ABLATE=<bits>; the production build has 0 and every
// ablation branch is compiled out.  1 = no global loads, 2 = no split / LDS
// writes (loaded values kept live), 4 = no MFMAs (fragments kept live),
// 8 = no epilogue.
#ifndef D2MI_CONV_ABLATE
#define D2MI_CONV_ABLATE 0
#endif
constexpr int kAblate = D2MI_CONV_ABLATE;

// Wave priority 1 while a wave issues its k-step's MFMAs (s_setprio): the
// SIMD's arbiter then prefers the MFMA stream over the staging VALU / LDS
// writes of the other resident workgroups (or the stager waves).  Measured
// (r2, tools/ab_prio.sh, 16 Mask R-CNN shapes): 1.3 % faster in total, 2-5 %
// on the res3-res5 3x3s and 1x1s; on the double-buffered narrow-Cout kernels
// 2-4 %; priority during the load-issue phase instead gained 0.2 %.  Fixed
// since r4 (was the runtime D2MI_CONV_PRIO).
constexpr bool kPrioMfma = true;

// Exact 3-term bf16 split of four floats (truncation; see the header).
// Each output packs 4 bf16 (element order = float4 order).
__device__ __forceinline__ void split3(const float4 v, uint2& h, uint2& m, uint2& l) {
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

struct ConvArgs {
  const float* x;
  const float* w;  // [KH][KW][Cout][Cin]
  const float* bias;
  const float* topdown;
  const float* residual;
  const float* gate;  // nullable: out = gate > 0 ? out : 0 (applied last)
  float* y;
  float* partial;  // split-K workspace [splits][M][Cout] (nullable)
  int N, H, W, Cin, Cout, KH, KW, stride, pad, OH, OW, flags;
  int M, nM, nN, ntiles, splits, kt_per_split, nk, cchunks;
  // this launch covers tiles [tile_base, tile_base + ntiles); split-K
  // partials cover output rows [m_base, m_end) (a main launch and a tail launch
  // last round would run mostly empty, see conv_core)
  int tile_base, m_base, m_end;
  int lds_epi;  // store_outputs_lds usable (Cout % 4 == 0, 16-B aligned operands)
  int nt_store;  // final outputs of the LDS epilogue / split-K reduce stored non-temporally
  int x_bytes, w_bytes;  // buffer-descriptor ranges (< 2 GiB)
  int tdH, tdW;
  int reg_partials;  // split-K partials stored from the accumulators (tuning conv_epi)
  int xcd2;  // xcd_tile(): the 2-D XCD-contiguous remap (tuning conv_xcd, default 1)
  // Multi-level launch (d2mi_conv2d_nhwc_levels): nlev > 0 levels share the
  // weights; level l owns tiles [lv_tile0[l], lv_tile0[l + 1]) and its own
  // input / output / gate maps.  The kernel swaps them into the fields above
  // at start, so everything after that is the single-level code.
  int nlev;
  const float* lv_x[kMaxConvLevels];
  float* lv_y[kMaxConvLevels];
  const float* lv_gate[kMaxConvLevels];
  int lv_H[kMaxConvLevels], lv_W[kMaxConvLevels], lv_OH[kMaxConvLevels], lv_OW[kMaxConvLevels];
  int lv_N[kMaxConvLevels], lv_xbytes[kMaxConvLevels], lv_tile0[kMaxConvLevels + 1];
  int lv_moff[kMaxConvLevels + 1];  // first row of each level in the split-K slab; [6] = total
};

// The per-level part of a launch's arguments: a single-level launch takes
// it from ConvArgs; a multi-level one (nlev > 0) from the tile's level, whose
// tile index it makes level-local.  A small struct of scalars (the kernels
// keep it in SGPRs; swapping fields of the whole ConvArgs put it in scratch).
struct Geo {
  const float* x;
  float* y;
  const float* gate;
  int N, H, W, OH, OW, M, m_end, x_bytes;
  // split-K partial rows: slab stride (rows per split) and the row that maps
  // to slab row 0 (single level: m_base; multi-level: minus the level's row
  // offset in the concatenated slab)
  int pstride, prow0;
};

__device__ __forceinline__ Geo geo_of(const ConvArgs& a) {
  return Geo{a.x, a.y, a.gate, a.N, a.H, a.W, a.OH, a.OW, a.M, a.m_end, a.x_bytes,
             a.m_end - a.m_base, a.m_base};
}

__device__ __forceinline__ Geo select_level(const ConvArgs& a, int& tile) {
  Geo r = geo_of(a);
  if (a.nlev == 0) return r;
  // unrolled over the level slots (constant indices: a runtime index into the
  // by-value kernel argument would copy it to scratch)
  int base = 0;
#pragma unroll
  for (int l = 0; l < kMaxConvLevels; ++l) {
    if (l < a.nlev && tile >= a.lv_tile0[l]) {
      base = a.lv_tile0[l];
      r.x = a.lv_x[l];
      r.y = a.lv_y[l];
      r.gate = a.lv_gate[l];
      r.N = a.lv_N[l];
      r.H = a.lv_H[l];
      r.W = a.lv_W[l];
      r.OH = a.lv_OH[l];
      r.OW = a.lv_OW[l];
      r.x_bytes = a.lv_xbytes[l];
      r.prow0 = -a.lv_moff[l];
    }
  }
  tile -= base;
  r.M = r.N * r.OH * r.OW;
  r.m_end = r.M;
  r.pstride = a.lv_moff[a.nlev > 0 ? kMaxConvLevels : 0];  // total rows (slot kMaxConvLevels)
  return r;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
typedef float ntv4 __attribute__((ext_vector_type(4)));
// streaming (non-temporal) float4 load / store: data touched once
__device__ __forceinline__ float4 ld4_nt(const float* p) {
  const ntv4 v = __builtin_nontemporal_load(reinterpret_cast<const ntv4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4_nt(float* p, float4 v) {
  ntv4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<ntv4*>(p));
}

__device__ __forceinline__ float epilogue(const ConvArgs& a, const Geo& g, float acc, int m,
                                          int co) {
  float v = acc + (a.bias ? a.bias[co] : 0.f);
  if ((a.flags & kRelu) && !(a.flags & kReluAfterResidual)) v = fmaxf(v, 0.f);
  if (a.topdown) {
    const int n = m / (g.OH * g.OW);
    const int rem = m - n * g.OH * g.OW;
    const int oh = rem / g.OW, ow = rem - oh * g.OW;
    v = v + a.topdown[(((size_t)n * a.tdH + (oh >> 1)) * a.tdW + (ow >> 1)) * a.Cout + co];
  }
  if (a.residual) v = v + a.residual[(size_t)m * a.Cout + co];
  if ((a.flags & kRelu) && (a.flags & kReluAfterResidual)) v = fmaxf(v, 0.f);
  if (g.gate && !(g.gate[(size_t)m * a.Cout + co] > 0.f)) v = 0.f;
  return v;
}

// Epilogue shared by the conv kernels: bias, ReLU, top-down / residual adds
// (or the split-K partial slab), written straight from the MFMA accumulators.
template <int WN, int TM, int TN>
__device__ __forceinline__ void store_outputs(const ConvArgs& a, const Geo& g,
                                              floatx16 (&acc)[TM][TN], int m0,
                                              int n0, int wr, int wc, int lane, int split,
                                              bool part) {
  const int li = lane & 31, lh = lane >> 5;
  // C/D map for 32x32: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool simple = !part && !a.topdown && !a.residual && !g.gate;
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
        float* yp = g.y + (size_t)mb * a.Cout + co;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          if (mb + dm < g.M) {
            float v = acc[i][j][r] + bv;
            yp[(size_t)dm * a.Cout] = relu ? fmaxf(v, 0.f) : v;
          }
        }
        continue;
      }
      if (part) {
        float* pp =
            a.partial + ((size_t)split * g.pstride + (mb - g.prow0)) * a.Cout + co;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dm = (r & 3) + 8 * (r >> 2);
          if (mb + dm < g.M) pp[(size_t)dm * a.Cout] = acc[i][j][r];
        }
        continue;
      }
      // residual / top-down operands: all 16 loads issued before any store
      // (y may not alias them; without this the loads serialise behind the stores)
      float add[16];
      // pixel coordinates of row mb, then stepped (dm < 32): no per-element division
      int tn = 0, toh = 0, tow = 0, last = 0;
      if (a.topdown) {
        const int mm = min(mb, g.M - 1);
        tn = mm / (g.OH * g.OW);
        const int rem = mm - tn * g.OH * g.OW;
        toh = rem / g.OW;
        tow = rem - toh * g.OW;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        const int m = mb + dm;
        float v = 0.f;
        if (a.topdown) {  // advance (n, oh, ow) from row mb + last to mb + dm
          tow += dm - last;
          last = dm;
          while (tow >= g.OW) {
            tow -= g.OW;
            if (++toh == g.OH) { toh = 0; ++tn; }
          }
        }
        if (m < g.M) {
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
        if (m >= g.M) continue;
        float v = acc[i][j][r] + bv;
        if (relu && !relu_after) v = fmaxf(v, 0.f);
        // epilogue() order: conv + bias, (+ top-down) (+ residual), gate last
        // (the gate comes with Cout % 4 == 0 dgrads: normally the LDS epilogue)
        if ((a.topdown && a.residual) || g.gate) {
          v = epilogue(a, g, acc[i][j][r], m, co);
        } else {
          v = v + add[r];
          if (relu && relu_after) v = fmaxf(v, 0.f);
        }
        g.y[(size_t)m * a.Cout + co] = v;
      }
    }
  }
}

// Split-K / stream-K partial slab straight from the accumulators (raw sums:
// the reduce applies the epilogue).  Slab `split`, rows mapped as store_outputs.
template <int WN, int TM, int TN>
__device__ __forceinline__ void store_partial(const ConvArgs& a, const Geo& g,
                                              floatx16 (&acc)[TM][TN], int m0, int n0, int wr,
                                              int wc, int lane, int split) {
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int co = n0 + (wc * TN + j) * 32 + li;
    if (co >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + (wr * TM + i) * 32 + 4 * lh;
      float* pp = a.partial + ((size_t)split * g.pstride + (mb - g.prow0)) * a.Cout + co;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int dm = (r & 3) + 8 * (r >> 2);
        if (mb + dm < g.M) pp[(size_t)dm * a.Cout] = acc[i][j][r];
      }
    }
  }
}

// LDS-staged epilogue (ConvArgs::lds_epi): the accumulators leave through
// LDS one 32-row slab at a time as row-major float4s, so every store
// instruction writes whole rows of the tile (BN * 4 bytes) instead of 32-float
// column pieces, and the slab's residual / gate / top-down operands are
// loaded as float4s BEFORE its LDS barrier (their latency overlaps the
// transpose).  Same arithmetic order as epilogue(); split-K partials are
// written raw.  smem: >= 32 * (BN + 4) floats of the kernel's LDS.
template <int WM, int WN, int TM, int TN, int NT = 256>
__device__ __forceinline__ void store_outputs_lds(const ConvArgs& a, const Geo& g,
                                                  floatx16 (&acc)[TM][TN],
                                                  int m0, int n0, int wr, int wc, int lane,
                                                  int split, bool part, float* smem) {
  constexpr int BN = WN * TN * 32;
  constexpr int LS = BN + 4;        // slab row stride (floats)
  constexpr int F4 = BN / 4;        // float4 per tile row
  constexpr int Q = 32 * F4 / NT;   // float4 per thread per slab
  const int tid = threadIdx.x;
  const int li = lane & 31, lh = lane >> 5;
  float* const dst = part ? a.partial + (size_t)split * g.pstride * a.Cout : g.y;
  const int mrow0 = part ? g.prow0 : 0;
  const bool relu = (a.flags & kRelu) != 0, relu_after = (a.flags & kReluAfterResidual) != 0;
  __syncthreads();  // the main loop's last LDS reads are complete
#pragma unroll
  for (int s = 0; s < WM * TM; ++s) {
    float4 res[Q], gt[Q], td[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int idx = tid + NT * q;
      const int row = idx / F4, c4 = idx - row * F4;
      const int m = m0 + s * 32 + row, co = n0 + c4 * 4;
      res[q] = gt[q] = td[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!part && m < g.M && co < a.Cout) {
        const size_t o = (size_t)m * a.Cout + co;
        if (a.residual) res[q] = ld4(a.residual + o);
        if (g.gate) gt[q] = ld4(g.gate + o);
        if (a.topdown) {
          const int n = m / (g.OH * g.OW);
          const int rem = m - n * g.OH * g.OW;
          const int oh = rem / g.OW, ow = rem - oh * g.OW;
          td[q] = ld4(a.topdown + (((size_t)n * a.tdH + (oh >> 1)) * a.tdW + (ow >> 1)) * a.Cout +
                      co);
        }
      }
    }
    if (wr == s / TM) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          smem[((r & 3) + 8 * (r >> 2) + 4 * lh) * LS + (wc * TN + j) * 32 + li] = acc[s % TM][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int idx = tid + NT * q;
      const int row = idx / F4, c4 = idx - row * F4;
      const int m = m0 + s * 32 + row, co = n0 + c4 * 4;
      if (m >= g.M || co >= a.Cout) continue;
      float4 v = *reinterpret_cast<const float4*>(&smem[row * LS + c4 * 4]);
      if (!part) {
        float* vv = reinterpret_cast<float*>(&v);
        const float* rr = reinterpret_cast<const float*>(&res[q]);
        const float* gg = reinterpret_cast<const float*>(&gt[q]);
        const float* tt = reinterpret_cast<const float*>(&td[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = vv[e] + (a.bias ? a.bias[co + e] : 0.f);
          if (relu && !relu_after) x = fmaxf(x, 0.f);
          if (a.topdown) x = x + tt[e];
          if (a.residual) x = x + rr[e];
          if (relu && relu_after) x = fmaxf(x, 0.f);
          if (g.gate && !(gg[e] > 0.f)) x = 0.f;
          vv[e] = x;
        }
      }
      if (!part && a.nt_store) st4_nt(dst + (size_t)(m - mrow0) * a.Cout + co, v);
      else *reinterpret_cast<float4*>(dst + (size_t)(m - mrow0) * a.Cout + co) = v;
    }
    __syncthreads();
  }
}

// DB: double-buffered LDS (one barrier per k-step, 2 workgroups/CU for the
// 128x128 tile) vs single-buffered (two barriers per k-step, 36 KiB LDS, up to
// 3 workgroups/CU).  Large-M shapes prefer the higher occupancy.
// Position of a k-step in the channel-chunk-major, tap-minor K order.  The
// staging loads walk k-steps in order: kseek() advances by one step with a
// few scalar adds and only re-derives the position by division on a jump.
struct KCursor {
  int kt, chunk, tap, kh, kw;
};
__device__ __forceinline__ void kseek(KCursor& c, int kt, int taps, int KW) {
  if (kt == c.kt) return;
  if (kt == c.kt + 1) {
    c.kt = kt;
    ++c.tap;
    if (++c.kw == KW) {
      c.kw = 0;
      ++c.kh;
    }
    if (c.tap == taps) {
      c.tap = c.kh = c.kw = 0;
      ++c.chunk;
    }
    return;
  }
  c.kt = kt;
  c.chunk = kt / taps;
  c.tap = kt - c.chunk * taps;
  c.kh = c.tap / KW;
  c.kw = c.tap - c.kh * KW;
}
__device__ __forceinline__ KCursor kcursor(int kt, int taps, int KW) {
  KCursor c;
  c.kt = kt;
  c.chunk = kt / taps;
  c.tap = kt - c.chunk * taps;
  c.kh = c.tap / KW;
  c.kw = c.tap - c.kh * KW;
  return c;
}

// XCD-contiguous remap of a (tiles x splits) grid: hardware dispatch puts
// linear workgroup L = x + y * gridDim.x on XCD L % 8; logical index l = the
// (L / 8)-th of XCD L % 8's contiguous block, tile fastest, so consecutive
// tiles of one split (which share input rows and the split's weight rows)
// meet in one XCD's L2.  xcd2 = 0 (tuning conv_xcd = 0, A/B): the 1-D remap of
// blockIdx.x alone with the split from blockIdx.y (exact XCD placement only
// when gridDim.x % 8 == 0).  Placement only: outputs are bit-identical.
__device__ __forceinline__ int xcd_tile(int xcd2, int& split) {
  const int nx = gridDim.x;
  const int nwg = xcd2 ? nx * gridDim.y : nx;
  const int L = xcd2 ? blockIdx.x + blockIdx.y * nx : blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, x8 = L % 8;
  const int l = (x8 < r8 ? x8 * (q + 1) : r8 * (q + 1) + (x8 - r8) * q) + L / 8;
  split = xcd2 ? l / nx : blockIdx.y;
  return xcd2 ? l - split * nx : l;
}

template <int WM, int WN, int TM, int TN, bool DB, bool SPLIT, int OCC = 2, bool ML = false>
__global__ __launch_bounds__(256, OCC) void conv_mfma_kernel(ConvArgs a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int RA = BM / 32, RB = BN / 32;  // staged rows per thread (8 threads per row)
  constexpr int NB = DB ? 2 : 1;
  // f32: [row][36] floats; SPLIT: [3 planes][row][40] bf16 (as uint16)
  constexpr int A_WORDS = SPLIT ? 3 * BM * LDSB / 2 : BM * LDSP;
  constexpr int B_WORDS = SPLIT ? 3 * BN * LDSB / 2 : BN * LDSP;
  __shared__ __attribute__((aligned(16))) float As[NB][A_WORDS];
  __shared__ __attribute__((aligned(16))) float Bs[NB][B_WORDS];
  static_assert(NB * A_WORDS >= 32 * (BN + 4), "LDS epilogue slab does not fit in As");

  // XCD-aware tile order: consecutive tiles (the Cout tiles of one pixel tile
  // and neighbouring pixel tiles, which share input halo rows) land on one XCD.
  int split;
  int tile = a.tile_base + xcd_tile(a.xcd2, split);
  const Geo g = ML ? select_level(a, tile) : geo_of(a);  // ML: a multi-level launch
  const int mt = tile / a.nN, nt = tile - mt * a.nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = split * a.kt_per_split;
  const int kt1 = min(a.nk, kt0 + a.kt_per_split);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;

  const int srow = tid >> 3, schunk = (tid & 7) * 4;
  // Per staged row: top-left input pixel of its receptive field (ih0, iw0)
  // and that pixel's element offset; invalid rows get ih0 = INT_MIN/2 so
  // every tap fails the range test.  Loads are raw buffer loads: an invalid
  // (row, tap) gets an out-of-range offset and the hardware range check
  // returns zeros (no branches around the loads, 32-bit offsets; the host
  // keeps x and w below 2 GiB per launch).
  int ih0[RA], iw0[RA], base[RA];
#pragma unroll
  for (int p = 0; p < RA; ++p) {
    const int m = m0 + srow + 32 * p;
    const int mm = m < g.M ? m : 0;
    const int n = mm / (g.OH * g.OW);
    const int rem = mm - n * g.OH * g.OW;
    const int oh = rem / g.OW, ow = rem - oh * g.OW;
    const int ihv = oh * a.stride - a.pad;
    ih0[p] = m < g.M ? ihv : -(1 << 29);
    iw0[p] = ow * a.stride - a.pad;
    base[p] = ((n * g.H + ihv) * g.W + iw0[p]) * a.Cin + schunk;
  }
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.x), 0, g.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.w), 0, a.w_bytes, 0x00020000);
  constexpr uint32_t kOOB = 0x80000000u;

  // Staging registers.  Single-buffered LDS runs a 2-deep prefetch of the
  // activation tile (k-step kt+2 loads while kt computes and kt+1 waits in
  // the other set) and a 1-deep prefetch of the weight tile (small and
  // L2-resident): an activation gather has two compute phases to return, one
  // phase (~0.6 us at 2 workgroups/CU) being below its loaded latency.
  // OCC 3 (three workgroups per CU): a 1-deep activation prefetch (fewer VGPRs)
  float4 ra[OCC >= 3 ? 1 : 2][RA], rb[RB];
  // channel-chunk-major, tap-minor K order: consecutive k-steps read the
  // same 32 channels at neighbouring pixels (the 3x3 taps), which are still
  // in L2 (tap-major order re-fetched them Cin/32 steps later)
  const int taps = a.KH * a.KW;
  KCursor ca = kcursor(kt0, taps, a.KW), cb = ca;  // (A and B loads run in k-step order)
  auto load_a = [&](int kt, float4 (&la)[RA]) {
    kseek(ca, kt, taps, a.KW);
    const int cc = ca.chunk * BK;
    const int kh = ca.kh, kw = ca.kw;
    const bool cok = cc + schunk < a.Cin;
    const int toff = (kh * g.W + kw) * a.Cin + cc;
#pragma unroll
    for (int p = 0; p < RA; ++p) {
      // bitwise &: no short-circuit branches around the loads
      const bool ok = cok & ((unsigned)(ih0[p] + kh) < (unsigned)g.H) &
                      ((unsigned)(iw0[p] + kw) < (unsigned)g.W);
      const uint32_t off = ok ? (uint32_t)(base[p] + toff) * 4u : kOOB;
      la[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrsrc, off, 0, 0));
    }
  };
  auto load_b = [&](int kt) {
    kseek(cb, kt, taps, a.KW);
    const int tap = (a.flags & kFlipTaps) ? taps - 1 - cb.tap : cb.tap;
    const int cc = cb.chunk * BK;
    const bool cok = cc + schunk < a.Cin;
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int co = n0 + srow + 32 * p;
      const uint32_t off = (cok & (co < a.Cout))
                               ? (uint32_t)((tap * a.Cout + co) * a.Cin + cc + schunk) * 4u
                               : kOOB;
      rb[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, off, 0, 0));
    }
  };
  auto store_tile = [&](int buf, const float4 (&la)[RA], const float4 (&lb)[RB]) {
    if constexpr (SPLIT) {
      uint16_t* A16 = reinterpret_cast<uint16_t*>(As[buf]);
      uint16_t* B16 = reinterpret_cast<uint16_t*>(Bs[buf]);
#pragma unroll
      for (int p = 0; p < RA; ++p) {
        uint2 h, m, l;
        split3(la[p], h, m, l);
        const int o = swz(srow + 32 * p, schunk);
        *reinterpret_cast<uint2*>(&A16[o]) = h;
        *reinterpret_cast<uint2*>(&A16[BM * LDSB + o]) = m;
        *reinterpret_cast<uint2*>(&A16[2 * BM * LDSB + o]) = l;
      }
#pragma unroll
      for (int p = 0; p < RB; ++p) {
        uint2 h, m, l;
        split3(lb[p], h, m, l);
        const int o = swz(srow + 32 * p, schunk);
        *reinterpret_cast<uint2*>(&B16[o]) = h;
        *reinterpret_cast<uint2*>(&B16[BN * LDSB + o]) = m;
        *reinterpret_cast<uint2*>(&B16[2 * BN * LDSB + o]) = l;
      }
    } else {
#pragma unroll
      for (int p = 0; p < RA; ++p)
        *reinterpret_cast<float4*>(&As[buf][(srow + 32 * p) * LDSP + schunk]) = la[p];
#pragma unroll
      for (int p = 0; p < RB; ++p)
        *reinterpret_cast<float4*>(&Bs[buf][(srow + 32 * p) * LDSP + schunk]) = lb[p];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    if constexpr (SPLIT) {
      const uint16_t* A16 = reinterpret_cast<const uint16_t*>(As[buf]);
      const uint16_t* B16 = reinterpret_cast<const uint16_t*>(Bs[buf]);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {  // two 16-deep bf16 MFMA steps per 32-deep stage
        bf16x8 fa[3][TM], fb[3][TN];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[pl][i] = *reinterpret_cast<const bf16x8*>(
                &A16[pl * BM * LDSB + swz((wr * TM + i) * 32 + li, ks * 16 + lh * 8)]);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[pl][j] = *reinterpret_cast<const bf16x8*>(
                &B16[pl * BN * LDSB + swz((wc * TN + j) * 32 + li, ks * 16 + lh * 8)]);
        }
        // small terms first, then the dominant h*h
        constexpr int PA[6] = {1, 2, 0, 0, 1, 0};
        constexpr int PB[6] = {1, 0, 2, 1, 0, 0};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[PA[t]][i], fb[PB[t]][j],
                                                                   acc[i][j], 0, 0, 0);
      }
    } else {
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
    }
  };

  if (kt0 < kt1) {
    if constexpr (DB) {
      load_a(kt0, ra[0]);
      load_b(kt0);
      store_tile(0, ra[0], rb);
      __syncthreads();
      int buf = 0;
      for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more) {
          load_a(kt + 1, ra[0]);
          load_b(kt + 1);
        }
        if (kPrioMfma) __builtin_amdgcn_s_setprio(1);
        compute(buf);
        if (kPrioMfma) __builtin_amdgcn_s_setprio(0);
        if (more) store_tile(buf ^ 1, ra[0], rb);
        __syncthreads();
        buf ^= 1;
      }
    } else if constexpr (OCC >= 3) {
      load_a(kt0, ra[0]);
      load_b(kt0);
      store_tile(0, ra[0], rb);
      __syncthreads();
      for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more && !(kAblate & 1)) {
          load_b(kt + 1);
          load_a(kt + 1, ra[0]);
        }
        if (kPrioMfma) __builtin_amdgcn_s_setprio(1);
        if (!(kAblate & 4)) compute(0);
        if (kPrioMfma) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        if (more) {
          if (!(kAblate & 2)) store_tile(0, ra[0], rb);
          __syncthreads();
        }
      }
    } else {
      // step(kt): activation set F is free (its k-step is in LDS), set X
      // holds kt + 1.  B(kt+1) is issued before A(kt+2), so the store of
      // k-step kt+1 leaves only A(kt+2) in flight.
      auto step = [&](int kt, float4 (&F)[RA], const float4 (&X)[RA]) {  // (OCC 2 only)
        if (kt + 1 < kt1) load_b(kt + 1);
        if (kt + 2 < kt1) load_a(kt + 2, F);
        compute(0);
        __syncthreads();
        if (kt + 1 < kt1) {
          store_tile(0, X, rb);
          __syncthreads();
        }
      };
      load_a(kt0, ra[0]);
      load_b(kt0);
      if (kt0 + 1 < kt1) load_a(kt0 + 1, ra[1]);
      store_tile(0, ra[0], rb);
      __syncthreads();
      for (int kt = kt0; kt < kt1; kt += 2) {
        step(kt, ra[0], ra[1]);
        if (kt + 1 < kt1) step(kt + 1, ra[1], ra[0]);
      }
    }
  }

  if constexpr ((kAblate & 8) != 0) return;
  // split-K partial slabs leave straight from the accumulators (each store
  // instruction writes two whole 128-B row segments; no LDS round trip and
  // none of its barriers) unless tuning conv_epi = 0
  if (a.splits > 1 && a.reg_partials) {
    store_outputs<WN, TM, TN>(a, g, acc, m0, n0, wr, wc, lane, split, true);
  } else if (WN * TN * 32 == 128 || a.lds_epi)  // 128-wide tiles: planned only with lds_epi
    store_outputs_lds<WM, WN, TM, TN>(a, g, acc, m0, n0, wr, wc, lane, split, a.splits > 1,
                                      &As[0][0]);
  else
    store_outputs<WN, TM, TN>(a, g, acc, m0, n0, wr, wc, lane, split, a.splits > 1);
}

// Streaming short-K 1x1 conv (r5, plan cfg 4; tuning "conv_stream").  The
// memory-bound launches of the step are the stride-1 1x1 convs with a short
// K (Cin 64-256: the bottleneck expand + residual, the conv1 dgrads with the
// ReLU gate and the shortcut's gradient): 2-8 k-steps per 128x128 tile, so
// the tiled kernel spends its time in prologue / epilogue latency and splits
// every activation row once per Cout tile (verdict r4 weak #4: 0.24 of HBM).
// Here a workgroup owns one BN-wide Cout slice for the whole launch: its
// weight slice (K x BN) is split into the three bf16 planes ONCE, resident in
// LDS, and its waves stream 32-row pixel strips -- each lane loads its MFMA A
// fragments straight from global memory (row = lane & 31, the 8 channels of
// each 16-deep step at 8 * (lane >> 5)), splits them in registers and
// multiplies with the pixels as the MFMA B operand (so a lane's accumulators
// are channel quads of one pixel); the epilogue operands (residual / gate)
// are loaded as row-contiguous float4s before the MFMAs, and the results
// leave through a per-wave LDS slab (64 channels at a time) as whole-row
// float4 stores.  No workgroup barrier after the prologue.
// Same K order (16-deep steps ascending), product order and accumulation
// sequence as conv_mfma_kernel<..., SPLIT = true>: bit-identical outputs.
// Grid: nslices x groups; slice = (blockIdx / 8) % nslices with the XCD
// (blockIdx % 8) fixed, so the slices of one strip run on one XCD and share
// its A rows in L2.
// RES / GATE: the epilogue operands present (their prefetch registers exist
// only then: 16 x TN floats per lane each).  LDS: the weight slice (K x BN x
// 6 B) + 8 KiB per wave (<= 160 KiB: K 128 at BN 128, K 256 at BN 64).
template <int TN, int KMAX, int WAVES, bool RES, bool GATE>
__global__ __launch_bounds__(64 * WAVES, 1) void conv1x1_stream_kernel(ConvArgs a, int nslices,
                                                                      int ntmode) {
  constexpr int BN = 32 * TN;
  static_assert(KMAX % 32 == 0, "K: whole 32-deep chunks");
  static_assert(TN == 2 || TN == 4, "64-column epilogue halves");
  constexpr int K = KMAX;  // host: Cin == KMAX (a compile-time K: A lives in registers)
  constexpr int NH = TN / 2;  // 64-column halves of the strip
  __shared__ __attribute__((aligned(16))) uint16_t Bs[KMAX / 32 * 3 * BN * LDSB];
  // per-wave epilogue slab: 32 pixel rows x 64 channels, float4 chunks XOR-
  // swizzled by row (conflict-free column writes, row-contiguous reads)
  __shared__ __attribute__((aligned(16))) float Slab[WAVES][32 * 64];
  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;
  const int slice = j8 % nslices;
  const int grp = (j8 / nslices) * 8 + xcd;
  const int ngrp = (gridDim.x / 8 / nslices) * 8;
  const int n0 = slice * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;

  // the weight slice, split once: chunk c, plane p, column n at
  // ((c * 3 + p) * BN) * 32 + swz(n, e) -- conv_mfma_kernel's per-step image
  {
    constexpr int k4n = K / 4;
    for (int f = tid; f < BN * k4n; f += 64 * WAVES) {
      const int n = f / k4n, k = (f - n * k4n) * 4;
      const int co = n0 + n;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (co < a.Cout) v = *reinterpret_cast<const float4*>(a.w + (size_t)co * K + k);
      uint2 h, m, l;
      split3(v, h, m, l);
      const int c = k >> 5, e = k & 31;
      uint16_t* base = Bs + (size_t)c * 3 * BN * LDSB;
      const int o = swz(n, e);
      *reinterpret_cast<uint2*>(&base[o]) = h;
      *reinterpret_cast<uint2*>(&base[BN * LDSB + o]) = m;
      *reinterpret_cast<uint2*>(&base[2 * BN * LDSB + o]) = l;
    }
  }
  __syncthreads();

  const bool relu = (a.flags & kRelu) != 0, relu_after = (a.flags & kReluAfterResidual) != 0;
  const int nstrips = (a.M + 31) / 32;
  constexpr int PA[6] = {1, 2, 0, 0, 1, 0};
  constexpr int PB[6] = {1, 0, 2, 1, 0, 0};
  float* slab = Slab[wave];
  // row-contiguous epilogue positions of this lane: q-th float4 at pixel row
  // (lane >> 4) + 4 q, channel chunk lane & 15 of the half
  const int erow = lane >> 4, ec4 = lane & 15;
  // Software-pipelined over the wave's strips: the next strip's A fragments
  // are issued as soon as this strip's MFMAs have consumed theirs (under this
  // strip's epilogue), and its epilogue operands as soon as this strip's
  // epilogue has used its own (under the next strip's MFMAs) -- the same
  // registers, one strip ahead.
  const int sstep = ngrp * WAVES;
  float4 ra[K / 16][2];
  float4 res[RES ? NH : 1][8], gt[GATE ? NH : 1][8];
  auto load_a = [&](int strip) {
    const int arow = min(strip * 32 + li, a.M - 1);
    const float* xr = a.x + (size_t)arow * K + lh * 8;
#pragma unroll
    for (int j = 0; j < K / 16; ++j) {
      ra[j][0] = *reinterpret_cast<const float4*>(xr + j * 16);
      ra[j][1] = *reinterpret_cast<const float4*>(xr + j * 16 + 4);
    }
  };
  auto load_e = [&](int strip) {  // the epilogue operands, row-contiguous float4s
    if constexpr (RES || GATE) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int m = strip * 32 + erow + 4 * q, co = n0 + h * 64 + ec4 * 4;
          const bool ok = m < a.M && co < a.Cout;
          const size_t o = (size_t)m * a.Cout + co;
          const bool nt = ntmode & 1;  // (uniform)
          if constexpr (RES)
            res[h][q] = ok ? (nt ? ld4_nt(a.residual + o) : ld4(a.residual + o))
                           : make_float4(0.f, 0.f, 0.f, 0.f);
          if constexpr (GATE)
            gt[h][q] = ok ? (nt ? ld4_nt(a.gate + o) : ld4(a.gate + o))
                          : make_float4(1.f, 1.f, 1.f, 1.f);
        }
    }
  };
  int s = grp * WAVES + wave;
  if (s < nstrips) {
    load_a(s);
    load_e(s);
  }
  for (; s < nstrips; s += sstep) {
    const int m0 = s * 32;
    const bool more = s + sstep < nstrips;
    // The MFMAs take the weights as the A operand and the pixels as B
    // (C^T = W X^T): lane li holds pixel m0 + li and, per 32-channel tile t,
    // the channels 32 t + 8 g + 4 lh + {0..3} in acc[t][4 g .. 4 g + 3]
    floatx16 acc[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    if (kPrioMfma) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < K / 16; ++j) {
      bf16x8 fa[3];
      {
        uint2 h0, m0_, l0, h1, m1, l1;
        split3(ra[j][0], h0, m0_, l0);
        split3(ra[j][1], h1, m1, l1);
        fa[0] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
        fa[1] = __builtin_bit_cast(bf16x8, make_uint4(m0_.x, m0_.y, m1.x, m1.y));
        fa[2] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
      }
      const uint16_t* base = Bs + (size_t)(j >> 1) * 3 * BN * LDSB;
      const int e = (j & 1) * 16 + lh * 8;
      // tile by tile (each accumulator's product sequence is the tiled
      // kernel's: activation plane PA[q] times weight plane PB[q])
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        bf16x8 fb[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          fb[p] = *reinterpret_cast<const bf16x8*>(&base[p * BN * LDSB + swz(t * 32 + li, e)]);
#pragma unroll
        for (int q = 0; q < 6; ++q)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[PB[q]], fa[PA[q]], acc[t], 0, 0, 0);
      }
      // keep the scheduler from hoisting every later step's LDS fragments
      // (and splits) above this step's MFMAs: their registers spill
      __builtin_amdgcn_sched_barrier(0);
    }
    if (kPrioMfma) __builtin_amdgcn_s_setprio(0);
    if (more) load_a(s + sstep);  // ra is free: the next strip's A under this epilogue
    // epilogue, one 64-channel half at a time through the wave's slab;
    // epilogue() order: conv + bias, ReLU (before), + residual, ReLU (after), gate
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int c4 = tt * 8 + gq * 2 + lh;  // chunk of channels 32 tt + 8 gq + 4 lh
          const floatx16& A = acc[2 * h + tt];
          *reinterpret_cast<float4*>(&slab[li * 64 + ((c4 ^ (li & 15)) << 2)]) =
              make_float4(A[4 * gq], A[4 * gq + 1], A[4 * gq + 2], A[4 * gq + 3]);
        }
      __builtin_amdgcn_wave_barrier();
      const int co = n0 + h * 64 + ec4 * 4;
      if (co >= a.Cout) continue;
      const float4 bv = a.bias ? ld4(a.bias + co) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int row = erow + 4 * q, m = m0 + row;
        const float4 c = *reinterpret_cast<const float4*>(&slab[row * 64 + ((ec4 ^ (row & 15)) << 2)]);
        float v[4] = {c.x + bv.x, c.y + bv.y, c.z + bv.z, c.w + bv.w};
        const float* rr = RES ? reinterpret_cast<const float*>(&res[RES ? h : 0][q]) : nullptr;
        const float* gg = GATE ? reinterpret_cast<const float*>(&gt[GATE ? h : 0][q]) : nullptr;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          if (relu && !relu_after) v[e4] = fmaxf(v[e4], 0.f);
          if constexpr (RES) v[e4] = v[e4] + rr[e4];
          if (relu && relu_after) v[e4] = fmaxf(v[e4], 0.f);
          if constexpr (GATE) {
            if (!(gg[e4] > 0.f)) v[e4] = 0.f;
          }
        }
        if (m < a.M) {
          const float4 o4 = make_float4(v[0], v[1], v[2], v[3]);
          if (ntmode & 2) st4_nt(a.y + (size_t)m * a.Cout + co, o4);
          else *reinterpret_cast<float4*>(a.y + (size_t)m * a.Cout + co) = o4;
        }
      }
    }
    if (more) load_e(s + sstep);  // res / gt are free: the next strip's, under its MFMAs
  }
}

// Warp-specialised split-product conv: a 256x128 tile, 16 waves (1024
// threads), one workgroup per CU.  Waves 0-7 only compute: each owns a
// 64x64 block (2x2 tiles of 32x32) and issues ds_read + MFMA.  Waves 8-15
// only stage: global loads LD k-steps ahead into registers, the exact bf16x3
// split, the LDS writes.  Two LDS stages of the split planes (72 KiB each):
// at iteration u the stagers write k-step u + 1 while the compute waves
// multiply k-step u -- one barrier per 32-deep k-step, and no compute wave
// waits for a global load.  Waves w, w + 4, w + 8, w + 12 share a SIMD
// (dispatch order 0 2 1 3): two MFMA streams (which hide each other's LDS
// latency) beside two staging streams on every SIMD.  The 256-row tile reads
// 48 KiB from L2 per k-step for twice the 128x128 tile's products (32 KiB).
// Same K order, product order and accumulation sequence as
// conv_mfma_kernel<..., SPLIT = true>: bit-identical outputs for equal splits.
template <int LD>
__global__ __launch_bounds__(1024, 1) void conv_ws_kernel(ConvArgs a) {
  constexpr int WM = 4, WN = 2, TM = 2, TN = 2;
  constexpr int BM = 256, BN = 128, RA = 4, RB = 2, S = 2;
  constexpr int A_WORDS = 3 * BM * LDSB / 2, B_WORDS = 3 * BN * LDSB / 2;
  constexpr int STAGE = A_WORDS + B_WORDS;  // 18432 words = 72 KiB
  __shared__ __attribute__((aligned(16))) float smem[S * STAGE];
  static_assert(S * STAGE >= 32 * (BN + 4), "LDS epilogue slab does not fit");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WN, wc = wave % WN;  // (stagers: wr >= 4, never an acc slab)

  // XCD-contiguous order of the workgroup index: consecutive tiles, which
  // share input halo rows and weight tiles, land on one XCD's L2.
  int split;
  const int tile = a.tile_base + xcd_tile(a.xcd2, split);
  const int kt0 = split * a.kt_per_split;
  const int kt1 = min(a.nk, kt0 + a.kt_per_split);
  const int nks = max(kt1 - kt0, 0);
  const Geo g = geo_of(a);
  const int mt = tile / a.nN, nt = tile - mt * a.nN;
  const int m0 = mt * BM, n0 = nt * BN;

  floatx16 acc[TM][TN];
  if (wave >= 8) {
    // ------------------------------------------------------------ stagers
    const int st = tid - 512;
    const int srow = st >> 3, schunk = (st & 7) * 4;  // rows srow + 64 p
    int ih0[RA], iw0[RA], base[RA];
#pragma unroll
    for (int p = 0; p < RA; ++p) {
      const int m = m0 + srow + 64 * p;
      const int mm = m < g.M ? m : 0;
      const int n = mm / (g.OH * g.OW);
      const int rem = mm - n * g.OH * g.OW;
      const int oh = rem / g.OW, ow = rem - oh * g.OW;
      const int ihv = oh * a.stride - a.pad;
      ih0[p] = m < g.M ? ihv : -(1 << 29);
      iw0[p] = ow * a.stride - a.pad;
      base[p] = ((n * g.H + ihv) * g.W + iw0[p]) * a.Cin + schunk;
    }
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g.x), 0, g.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), 0, a.w_bytes, 0x00020000);
    constexpr uint32_t kOOB = 0x80000000u;
    const int taps = a.KH * a.KW;
    // Per staged row, which taps land inside the image (bit t: tap t; the
    // plan gives this kernel <= 32 taps), so a k-step's range test is one bit
    // extract.
    // Closed form: the valid kw form one run of bits, [max(0, -iw0),
    // min(KW, W - iw0)), replicated at the KW-bit offsets of the valid kh.
    uint32_t tv[RA];
#pragma unroll
    for (int p = 0; p < RA; ++p) {
      const int kw0 = max(0, -iw0[p]), kw1 = min(a.KW, g.W - iw0[p]);
      const uint32_t cols = kw1 > kw0 ? (uint32_t)((1ull << kw1) - (1ull << kw0)) : 0u;
      uint32_t b = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        b |= ((unsigned)(ih0[p] + kh) < (unsigned)g.H ? cols : 0u) << (kh * a.KW);
      tv[p] = b;
    }
    // weight rows: element offset of (co, schunk) inside a tap's [Cout][Cin]
    int boff[RB];
    bool bco[RB];
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int co = n0 + srow + 64 * p;
      bco[p] = co < a.Cout;
      boff[p] = co * a.Cin + schunk;
    }
    // The loads run in k-step order (kt0, kt0 + 1, ..., then the last one
    // again): a uniform cursor (chunk, tap, kh, kw) advanced by one step
    // replaces two integer divisions per k-step.
    const int klast = kt0 + max(nks, 1) - 1;
    int c_kt = kt0, c_chunk = kt0 / taps, c_tap = kt0 - (kt0 / taps) * taps;
    int c_kh = c_tap / a.KW, c_kw = c_tap - (c_tap / a.KW) * a.KW;
    auto load = [&](float4 (&la)[RA], float4 (&lb)[RB]) {
      if constexpr ((kAblate & 1) != 0) return;
      const int cc = c_chunk * BK;
      const bool cok = cc + schunk < a.Cin;
      const int toff = (c_kh * g.W + c_kw) * a.Cin + cc;
      const int wtap = (a.flags & kFlipTaps) ? taps - 1 - c_tap : c_tap;
      const int wsc = wtap * a.Cout * a.Cin + cc;
#pragma unroll
      for (int p = 0; p < RB; ++p) {
        const uint32_t off = (cok & bco[p]) ? (uint32_t)(boff[p] + wsc) * 4u : kOOB;
        lb[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, off, 0, 0));
      }
#pragma unroll
      for (int p = 0; p < RA; ++p) {
        const bool inb = ((tv[p] >> c_tap) & 1u) != 0;
        const uint32_t off = (cok & inb) ? (uint32_t)(base[p] + toff) * 4u : kOOB;
        la[p] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xrsrc, off, 0, 0));
      }
      if (c_kt < klast) {  // advance the cursor (uniform)
        ++c_kt;
        ++c_tap;
        if (++c_kw == a.KW) {
          c_kw = 0;
          ++c_kh;
        }
        if (c_tap == taps) {
          c_tap = c_kh = c_kw = 0;
          ++c_chunk;
        }
      }
    };
    auto write = [&](int buf, const float4 (&la)[RA], const float4 (&lb)[RB]) {
      if constexpr ((kAblate & 2) != 0) {
#pragma unroll
        for (int p = 0; p < RA; ++p) asm volatile("" ::"v"(la[p].x));
#pragma unroll
        for (int p = 0; p < RB; ++p) asm volatile("" ::"v"(lb[p].x));
        return;
      }
      uint16_t* A16 = reinterpret_cast<uint16_t*>(smem + buf * STAGE);
      uint16_t* B16 = A16 + 3 * BM * LDSB;
#pragma unroll
      for (int p = 0; p < RA; ++p) {
        uint2 h, m, l;
        split3(la[p], h, m, l);
        const int o = swz(srow + 64 * p, schunk);
        *reinterpret_cast<uint2*>(&A16[o]) = h;
        *reinterpret_cast<uint2*>(&A16[BM * LDSB + o]) = m;
        *reinterpret_cast<uint2*>(&A16[2 * BM * LDSB + o]) = l;
      }
#pragma unroll
      for (int p = 0; p < RB; ++p) {
        uint2 h, m, l;
        split3(lb[p], h, m, l);
        const int o = swz(srow + 64 * p, schunk);
        *reinterpret_cast<uint2*>(&B16[o]) = h;
        *reinterpret_cast<uint2*>(&B16[BN * LDSB + o]) = m;
        *reinterpret_cast<uint2*>(&B16[2 * BN * LDSB + o]) = l;
      }
    };
    // Register ring of LD k-steps (static indices: the loops are unrolled by
    // LD).  Every load is UNCONDITIONAL (k-steps past the end re-load the last
    // one): with a data-dependent load count hipcc cannot count the loads in
    // flight and drains them all (vmcnt(0)) before each write.
    float4 ra[LD][RA], rb[LD][RB];
    if constexpr ((kAblate & 1) != 0) {
#pragma unroll
      for (int j = 0; j < LD; ++j) {
#pragma unroll
        for (int p = 0; p < RA; ++p) ra[j][p] = make_float4(1.f, 2.f, 3.f, 4.f);
#pragma unroll
        for (int p = 0; p < RB; ++p) rb[j][p] = make_float4(1.f, 2.f, 3.f, 4.f);
      }
    }
#pragma unroll
    for (int j = 0; j < LD; ++j) load(ra[j], rb[j]);
    if (nks > 0) write(0, ra[0], rb[0]);  // prologue: k-step 0 into buffer 0
    load(ra[0], rb[0]);
    __syncthreads();  // B_{-1}
    // iteration u: k-step v = u + 1 -> buffer v % 2 from register set v % LD,
    // that set re-filled with k-step v + LD; then B_u
    int u0 = 0;
    for (; u0 + LD <= nks; u0 += LD) {
#pragma unroll
      for (int j = 0; j < LD; ++j) {
        const int v = u0 + j + 1;
        const int set = (j + 1) % LD;  // (unrolled: a constant index)
        if (v < nks) write(v & 1, ra[set], rb[set]);
        load(ra[set], rb[set]);  // k-step v + LD (clamped)
        __syncthreads();  // B_u
      }
    }
#pragma unroll
    for (int j = 0; j < LD - 1; ++j) {  // the remaining nks % LD iterations
      if (u0 + j < nks) {
        const int v = u0 + j + 1;
        const int set = (j + 1) % LD;
        if (v < nks) write(v & 1, ra[set], rb[set]);
        __syncthreads();
      }
    }
  } else {
    // ------------------------------------------------------------ compute
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int li = lane & 31, lh = lane >> 5;
    bf16x8 fa[3][TM], fb[3][TN];
    // One 16-deep step with its LDS reads in three plane batches, each
    // issued one MFMA group ahead of its first use (products in the PA / PB
    // order of conv_mfma_kernel: small terms first, h*h last): after a
    // barrier all eight compute waves read at once, and 4 reads per wave
    // before the first MFMA (not 12) shorten that burst.
    auto ld1 = [&](const uint16_t* A16, const uint16_t* B16, int pa, int pb, int ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[pa][i] = *reinterpret_cast<const bf16x8*>(
            &A16[pa * BM * LDSB + swz((wr * TM + i) * 32 + li, ks * 16 + lh * 8)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[pb][j] = *reinterpret_cast<const bf16x8*>(
            &B16[pb * BN * LDSB + swz((wc * TN + j) * 32 + li, ks * 16 + lh * 8)]);
    };
    auto mm1 = [&](int pa, int pb) {
      if constexpr ((kAblate & 4) != 0) {  // ablation: no MFMAs (the fragments kept live)
        asm volatile("" ::"v"(fa[pa][0]), "v"(fa[pa][1]), "v"(fb[pb][0]), "v"(fb[pb][1]));
        return;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[pa][i], fb[pb][j], acc[i][j], 0, 0, 0);
    };
    auto step16 = [&](int buf, int ks) {
      const uint16_t* A16 = reinterpret_cast<const uint16_t*>(smem + buf * STAGE);
      const uint16_t* B16 = A16 + 3 * BM * LDSB;
      ld1(A16, B16, 1, 1, ks);
      __builtin_amdgcn_sched_barrier(0);
      ld1(A16, B16, 2, 0, ks);
      mm1(1, 1);  // m*m
      __builtin_amdgcn_sched_barrier(0);
      ld1(A16, B16, 0, 2, ks);
      mm1(2, 0);  // l*h
      __builtin_amdgcn_sched_barrier(0);
      mm1(0, 2);  // h*l
      mm1(0, 1);  // h*m
      mm1(1, 0);  // m*h
      mm1(0, 0);  // h*h
    };
    __syncthreads();  // B_{-1}
    for (int u = 0; u < nks; ++u) {
      const int buf = u & 1;
      if (kPrioMfma) __builtin_amdgcn_s_setprio(1);
      step16(buf, 0);
      step16(buf, 1);
      if (kPrioMfma) __builtin_amdgcn_s_setprio(0);
      // keep the MFMAs ahead of the barrier: moved past it, they would wait
      // for the stagers instead of overlapping them
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();  // B_u
    }
  }
  if constexpr ((kAblate & 8) != 0) return;  // (ablation: no epilogue)
  if (a.splits > 1 && a.reg_partials) {  // partial slabs straight from the accumulators
    if (wave < 8) store_partial<WN, TM, TN>(a, g, acc, m0, n0, wr, wc, lane, split);
    return;
  }
  store_outputs_lds<WM, WN, TM, TN, 1024>(a, g, acc, m0, n0, wr, wc, lane, split, a.splits > 1,
                                          smem);
}

// x [n] f32 -> [3][n] bf16 planes (h, m, l of the exact truncation split).
__global__ void split3_kernel(const float4* __restrict__ x, int64_t n4, uint2* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint2 h, m, l;
    split3(x[i], h, m, l);
    out[i] = h;
    out[n4 + i] = m;
    out[2 * n4 + i] = l;
  }
}

// Fixed-order split-K reduction + epilogue (deterministic).
__global__ void splitk_reduce_kernel(ConvArgs a) {
  const Geo g = geo_of(a);
  const int64_t total = (int64_t)(a.m_end - a.m_base) * a.Cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
#pragma unroll 4
    for (int s = 0; s < a.splits; ++s) acc += a.partial[(size_t)s * total + i];
    const int ml = (int)(i / a.Cout), co = (int)(i - (int64_t)ml * a.Cout);
    const int m = a.m_base + ml;
    a.y[(size_t)m * a.Cout + co] = epilogue(a, g, acc, m, co);
  }
}

// float4 form (Cout % 4 == 0, 16-B aligned partial / y): same split order.
// epilogue() on four consecutive channels of one row (Cout % 4 == 0, co % 4
// == 0): the same operations in the same order per channel, with the bias,
// top-down, residual and gate operands read as one float4 each (r6: the
// per-channel form issued four scalar loads of each)
__device__ __forceinline__ float4 epilogue4(const ConvArgs& a, const Geo& g, float4 acc, int m,
                                            int co) {
  float4 v = acc;
  if (a.bias) {
    const float4 b = *reinterpret_cast<const float4*>(a.bias + co);
    v = make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
  } else {
    v = make_float4(v.x + 0.f, v.y + 0.f, v.z + 0.f, v.w + 0.f);
  }
  const bool relu = (a.flags & kRelu) != 0, after = (a.flags & kReluAfterResidual) != 0;
  if (relu && !after) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
  if (a.topdown) {
    const int n = m / (g.OH * g.OW);
    const int rem = m - n * g.OH * g.OW;
    const int oh = rem / g.OW, ow = rem - oh * g.OW;
    const float4 t = *reinterpret_cast<const float4*>(
        a.topdown + (((size_t)n * a.tdH + (oh >> 1)) * a.tdW + (ow >> 1)) * a.Cout + co);
    v = make_float4(v.x + t.x, v.y + t.y, v.z + t.z, v.w + t.w);
  }
  if (a.residual) {
    const float4 r = *reinterpret_cast<const float4*>(a.residual + (size_t)m * a.Cout + co);
    v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
  }
  if (relu && after) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
  if (g.gate) {
    const float4 q = *reinterpret_cast<const float4*>(g.gate + (size_t)m * a.Cout + co);
    if (!(q.x > 0.f)) v.x = 0.f;
    if (!(q.y > 0.f)) v.y = 0.f;
    if (!(q.z > 0.f)) v.z = 0.f;
    if (!(q.w > 0.f)) v.w = 0.f;
  }
  return v;
}

// The split-K sum in split order + the epilogue, one float4 of channels per
// thread and step.  32-bit row / channel arithmetic when the slab has < 2^31
// float4s (every training shape; the 64-bit division cost more VALU than the
// loads it indexed), the float4 epilogue operands, and the split loads eight
// at a time.
__global__ void splitk_reduce4_kernel(ConvArgs a) {
  const Geo g = geo_of(a);
  const int64_t total = (int64_t)(a.m_end - a.m_base) * a.Cout;
  const int64_t total4 = total / 4;
  const float4* p4 = reinterpret_cast<const float4*>(a.partial);
  if (total4 < (1ll << 31) - (int64_t)gridDim.x * blockDim.x) {
    const int t4 = (int)total4, C4 = a.Cout >> 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < t4; i += gridDim.x * blockDim.x) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
      for (int s = 0; s < a.splits; ++s) {
        const float4 v = p4[(size_t)s * t4 + i];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      const int ml = i / C4, co = 4 * (i - ml * C4);
      const int m = a.m_base + ml;
      const float4 o = epilogue4(a, g, acc, m, co);
      if (a.nt_store) st4_nt(a.y + (size_t)m * a.Cout + co, o);
      else *reinterpret_cast<float4*>(a.y + (size_t)m * a.Cout + co) = o;
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int s = 0; s < a.splits; ++s) {
      const float4 v = p4[(size_t)s * total4 + i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    const int64_t e = 4 * i;
    const int ml = (int)(e / a.Cout), co = (int)(e - (int64_t)ml * a.Cout);
    const int m = a.m_base + ml;
    float4 o;
    o.x = epilogue(a, g, acc.x, m, co);
    o.y = epilogue(a, g, acc.y, m, co + 1);
    o.z = epilogue(a, g, acc.z, m, co + 2);
    o.w = epilogue(a, g, acc.w, m, co + 3);
    if (a.nt_store) st4_nt(a.y + (size_t)m * a.Cout + co, o);
    else *reinterpret_cast<float4*>(a.y + (size_t)m * a.Cout + co) = o;
  }
}

// Multi-level split-K: rows of the concatenated slab -> (level, row), fixed
// split order, + bias (+ ReLU); float4 over channels (Cout % 4 == 0).
__global__ void splitk_reduce_levels_kernel(ConvArgs a) {
  const int C4 = a.Cout / 4;
  const int rows = a.lv_moff[kMaxConvLevels];
  const int64_t total = (int64_t)rows * C4;
  const bool relu = (a.flags & kRelu) != 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / C4), c = (int)(e - (int64_t)r * C4) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int sp = 0; sp < a.splits; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(a.partial + ((size_t)sp * rows + r) * a.Cout + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (a.bias) {
      acc.x += a.bias[c]; acc.y += a.bias[c + 1]; acc.z += a.bias[c + 2]; acc.w += a.bias[c + 3];
    }
    if (relu) {
      acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f);
      acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
    }
    float* y = a.lv_y[0];
    int m = r;
#pragma unroll
    for (int l = 1; l < kMaxConvLevels; ++l)
      if (l < a.nlev && r >= a.lv_moff[l]) {
        y = a.lv_y[l];
        m = r - a.lv_moff[l];
      }
    *reinterpret_cast<float4*>(y + (size_t)m * a.Cout + c) = acc;
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

// Tiled HWIO -> [tap][co][ci] (Cin % 64 == 0): 64 x 64 tiles through LDS, reads
// along co and writes along ci both coalesced.
__global__ __launch_bounds__(256) void pack_weights_tiled_kernel(const float* __restrict__ w,
                                                                 int Cin, int Cout,
                                                                 float* __restrict__ out) {
  __shared__ float tile[64][65];
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64, tap = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = wv; i < 64; i += 4)
    tile[i][lane] = co0 + lane < Cout ? w[((size_t)tap * Cin + ci0 + i) * Cout + co0 + lane] : 0.f;
  __syncthreads();
  for (int j = wv; j < 64; j += 4)
    if (co0 + j < Cout) out[((size_t)tap * Cout + co0 + j) * Cin + ci0 + lane] = tile[lane][j];
}

// Many weight tensors packed by ONE launch (d2mi_conv_pack_weights_many): the
// tiled transpose above over a table of up to kMaxPack tensors with
// Cin % 64 == 0, a workgroup's tensor found from the per-tensor first-block
// table (block-uniform, so the table reads are scalar).
constexpr int kMaxPack = 32;
struct PackMany {
  const float* w[kMaxPack];
  float* out[kMaxPack];
  int Cin[kMaxPack], Cout[kMaxPack];
  int block0[kMaxPack + 1];
  int n;
};

__global__ __launch_bounds__(256) void pack_weights_many_kernel(PackMany p) {
  __shared__ float tile[64][65];
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < p.n && b >= p.block0[e + 1]) ++e;
  const int Cin = p.Cin[e], Cout = p.Cout[e];
  const int nco = (Cout + 63) / 64, nci = Cin / 64;
  const int local = b - p.block0[e];
  const int tap = local / (nco * nci);
  const int rem = local - tap * nco * nci;
  const int ci0 = (rem / nco) * 64, co0 = (rem % nco) * 64;
  const float* __restrict__ w = p.w[e];
  float* __restrict__ out = p.out[e];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = wv; i < 64; i += 4)
    tile[i][lane] = co0 + lane < Cout ? w[((size_t)tap * Cin + ci0 + i) * Cout + co0 + lane] : 0.f;
  __syncthreads();
  for (int j = wv; j < 64; j += 4)
    if (co0 + j < Cout) out[((size_t)tap * Cout + co0 + j) * Cin + ci0 + lane] = tile[lane][j];
}

struct Plan {
  int cfg;  // 0: 128x128, 1: 128x64, 2: 128x32
  int BM, BN, splits, kt_per_split, nk, ntiles;
  // tail split: the first full_tiles run as whole tiles, the remaining
  // tail_tiles (whole pixel-row blocks) split K tail_splits ways
  int full_tiles, tail_tiles, tail_splits, tail_kt_per_split;
  int main_m_end;  // output rows of the main launch (its split-K partial rows)
  size_t ws_bytes;
};

// Resident workgroups of the 128-wide conv tiles: 2 per CU.
// Resident workgroups per CU of a plan's kernel: the 128x128 split kernel
// runs three (168 VGPRs, 48 KiB LDS: conv_mfma_kernel<..., OCC = 3>), the
// others two.  D2MI_CONV_OCC=2 keeps the 128x128 split kernel at two (A/B).
static bool occ3_enabled() {
  static const int on = [] {
    const char* e = getenv("D2MI_CONV_OCC");
    return !(e && e[0] == '2');
  }();
  return on;
}

static int wg_slots(int cfg) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        c <= 0)
      c = 256;  // MI355X
    cus = c;
  }
  if (cfg == 3) return cus;  // the warp-specialised kernel: one per CU
  return (cfg == 0 && occ3_enabled() ? 3 : 2) * cus;
}

// wide_ok: the 128x128 tile may be used -- its kernels only carry the LDS
// epilogue (Cout % 4 == 0 and 16-B aligned operands); otherwise 128x64.
// split: the split-product math (kSplit3); cfg 3 (the warp-specialised
// 256x128 kernel, tuning "conv_ws") exists only in that form, and takes the
// long-K convs (>= 16 k-steps: every 3x3 with Cin >= 64, the 1x1s with
// Cin >= 512), where its deeper staging pipeline pays; the short-K 1x1s
// (2-8 k-steps) stay on the 3-per-CU kernel, whose prologue / epilogue
// overlap across workgroups (tools/ws_ab.py, 16 Mask R-CNN shapes).
// The stride-1 1x1 shapes with K = 256 that the streaming kernel takes
// (stream1x1_variant: 1.17x into 64 channels, 1.12x into 512 at >= 32 k
// pixels, profiles/r5_stream_ab_force_tn_rule.log); the tiled plan of these
// shapes never splits its tail tiles' K, so both kernels round alike.
static bool stream256_shape(int M, int Cout, int KH, int KW, int Cin) {
  return KH == 1 && KW == 1 && Cin == 256 && M >= 32768 && (Cout <= 64 || Cout == 512) &&
         Cout % 4 == 0;
}

Plan make_plan(int M, int Cout, int KH, int KW, int Cin, bool wide_ok, bool split = true) {
  Plan p;
  p.cfg = Cout <= 32 ? 2 : (Cout <= 64 || !wide_ok ? 1 : 0);
  // tuning "conv_ws_mink": the fewest k-steps that go to the WS kernel (A/B)
  if (p.cfg == 0 && split && tuning(kTuneConvWS) > 0 &&
      KH * KW * ((Cin + BK - 1) / BK) >= tuning(kTuneConvWSMinK) &&
      KH * KW <= 32 &&  // (the WS stagers keep a 32-bit tap mask per row)
      // (tuning "conv_ws_mintiles": the fewest 256x128 tiles that go to the WS kernel, A/B)
      ((M + 255) / 256) * ((Cout + 127) / 128) >= tuning(kTuneConvWSMinTiles))
    p.cfg = 3;
  p.BM = p.cfg == 3 ? 256 : 128;
  p.BN = (p.cfg == 0 || p.cfg == 3) ? 128 : (p.cfg == 1 ? 64 : 32);
  const int nM = (M + p.BM - 1) / p.BM, nN = (Cout + p.BN - 1) / p.BN;
  p.ntiles = nM * nN;
  p.nk = KH * KW * ((Cin + BK - 1) / BK);
  p.splits = 1;
  const int G = wg_slots(p.cfg);
  // Fewer tiles than resident workgroups and a long K: split K (to about
  // GS workgroups: every split writes and the reduce reads one more partial
  // slab of the output).
  static const int GS = [] {
    const char* e = getenv("D2MI_CONV_SPLIT_SLOTS");
    return e ? atoi(e) : 0;
  }();
  // target: two workgroups per CU even for the 3-per-CU kernel (A/B over
  // 384..1024 slots on the training step: 512 fastest, +2.5 % over 768 -- fewer
  // splits, less partial-slab traffic for the reduce)
  const int gs = GS > 0 ? GS : (p.cfg == 3 ? wg_slots(3) : wg_slots(1));
  if (4 * p.ntiles < 3 * gs && p.nk >= 16) {
    p.splits = std::min(std::max(1, gs / p.ntiles), std::min(p.nk / 8, 16));
  }
  p.kt_per_split = (p.nk + p.splits - 1) / p.splits;
  p.splits = (p.nk + p.kt_per_split - 1) / p.kt_per_split;
  p.ws_bytes = p.splits > 1 ? (size_t)p.splits * M * Cout * sizeof(float) : 0;
  // Tail split: with more tiles than resident workgroups, a last round that
  // is mostly empty (1050 tiles = 2 rounds of 512 + 26 on the FPN p2 3x3,
  // 525 = 512 + 13 on p3) costs about a whole round for a few tiles.  Those
  // tiles (whole pixel-row blocks) are split along K over the idle slots
  // instead and reduced in a fixed order.
  p.full_tiles = p.ntiles;
  p.tail_tiles = 0;
  p.tail_splits = 1;
  p.tail_kt_per_split = p.nk;
  p.main_m_end = M;
  static const char* tail_env = getenv("D2MI_CONV_TAIL");  // "0": no tail split (A/B)
  // (tuning "conv_tail_mink": the fewest k-steps whose tail tiles are split, A/B)
  if (p.splits == 1 && p.ntiles > G && p.nk >= std::max(2, tuning(kTuneConvTailMinK)) &&
      !(tail_env && tail_env[0] == '0') &&
      !stream256_shape(M, Cout, KH, KW, Cin)) {
    const int full = (p.ntiles / G) * G / nN * nN;
    const int tail = p.ntiles - full;
    if (tail > 0 && 2 * tail <= G) {
      int S = std::min(std::min(G / tail, p.nk / 4), 32);
      if (S >= 2) {
        const int kps = (p.nk + S - 1) / S;
        S = (p.nk + kps - 1) / kps;
        p.full_tiles = full;
        p.tail_tiles = tail;
        p.tail_splits = S;
        p.tail_kt_per_split = kps;
        const int m_base = full / nN * p.BM;
        p.ws_bytes = (size_t)S * (M - m_base) * Cout * sizeof(float);
      }
    }
  }
  return p;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_conv_pack_weights_many(int n, const float* const* w_hwio, const int32_t* dims,
                                           float* const* w_packed, void* stream) {
  D2MI_REQUIRE(n >= 0 && (n == 0 || (w_hwio && dims && w_packed)), "bad pack table");
  PackMany p = {};
  auto flush = [&]() -> int {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(pack_weights_many_kernel, dim3(p.block0[p.n]), dim3(256), 0,
                       as_stream(stream), p);
    D2MI_LAUNCH_CHECK();
    p = PackMany{};
    return 0;
  };
  for (int i = 0; i < n; ++i) {
    const int KH = dims[4 * i], KW = dims[4 * i + 1], Cin = dims[4 * i + 2], Cout = dims[4 * i + 3];
    D2MI_REQUIRE(KH > 0 && KW > 0 && Cin > 0 && Cout > 0, "bad conv weight shape (entry %d)", i);
    if (Cin % 64 != 0) {  // the generic kernel, alone
      const int rc = d2mi_conv_pack_weights(w_hwio[i], KH, KW, Cin, Cout, w_packed[i], stream);
      if (rc) return rc;
      continue;
    }
    const long long blocks = (long long)KH * KW * ((Cout + 63) / 64) * (Cin / 64);
    if (p.n == kMaxPack || (long long)p.block0[p.n] + blocks > (1LL << 30)) {
      const int rc = flush();
      if (rc) return rc;
    }
    p.w[p.n] = w_hwio[i];
    p.out[p.n] = w_packed[i];
    p.Cin[p.n] = Cin;
    p.Cout[p.n] = Cout;
    p.block0[p.n + 1] = p.block0[p.n] + (int)blocks;
    ++p.n;
  }
  return flush();
}

extern "C" int d2mi_conv_pack_weights(const float* w_hwio, int KH, int KW, int Cin, int Cout,
                                      float* w_packed, void* stream) {
  D2MI_REQUIRE(KH > 0 && KW > 0 && Cin > 0 && Cout > 0, "bad conv weight shape");
  if (Cin % 64 == 0) {
    hipLaunchKernelGGL(pack_weights_tiled_kernel, dim3((Cout + 63) / 64, Cin / 64, KH * KW),
                       dim3(256), 0, as_stream(stream), w_hwio, Cin, Cout, w_packed);
    D2MI_LAUNCH_CHECK();
    return 0;
  }
  const int64_t total = (int64_t)KH * KW * Cin * Cout;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(pack_weights_kernel, dim3(grid), dim3(256), 0, as_stream(stream), w_hwio,
                     KH * KW, Cin, Cout, w_packed);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// D2MI_CONV_WS / d2mi_set_tuning("conv_ws", d): the warp-specialised
// 256x128 split kernel (conv_ws_kernel, plan cfg 3): 0 off, > 0 on.  r3: a
// 16-deep, 3/4-stage read-ahead variant measured bit-identical but slower;
// r4 removed the other measured-slower A/B forms (stream-K, the in-launch
// split-K fix-up, the multi-level WS launch, the pre-split-plane kernel) --
// DESIGN section 5 keeps their numbers.

template <bool SPLIT>
static void launch_conv(int cfg, bool db, dim3 grid, hipStream_t st, const ConvArgs& a) {
  if (cfg == 3) {  // the warp-specialised 256x128 split kernel (plan cfg 3)
    // (LD = 3 does not fit the 128-VGPR budget of 4 waves per SIMD: it spills)
    if constexpr (SPLIT) hipLaunchKernelGGL((conv_ws_kernel<2>), grid, dim3(1024), 0, st, a);
    return;
  }
  if (cfg == 0 && !db && occ3_enabled()) {
    hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, false, SPLIT, 3>), grid, dim3(256), 0, st, a);
    return;
  }
  if (cfg == 0) {
    if (db)
      hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, true, SPLIT>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, false, SPLIT>), grid, dim3(256), 0, st, a);
  } else if (cfg == 1) {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 2, true, SPLIT>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 1, true, SPLIT>), grid, dim3(256), 0, st, a);
  }
}

// Multi-level launches (ConvArgs::nlev > 0): no split-K, single-buffered.
template <bool SPLIT>
static void launch_conv_levels(int cfg, dim3 grid, hipStream_t st, const ConvArgs& a) {
  if (cfg == 0) {
    if (occ3_enabled())
      hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, false, SPLIT, 3, true>), grid, dim3(256), 0,
                         st, a);
    else
      hipLaunchKernelGGL((conv_mfma_kernel<2, 2, 2, 2, false, SPLIT, 2, true>), grid, dim3(256), 0,
                         st, a);
  } else if (cfg == 1) {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 2, true, SPLIT, 2, true>), grid, dim3(256), 0, st,
                       a);
  } else {
    hipLaunchKernelGGL((conv_mfma_kernel<4, 1, 1, 1, true, SPLIT, 2, true>), grid, dim3(256), 0, st,
                       a);
  }
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
  const Plan p = make_plan(N * OH * OW, Cout, KH, KW, Cin, Cout % 4 == 0);
  return p.ws_bytes;
}

// conv1x1_stream_kernel's variant for a launch (0: not eligible): stride-1
// unpadded 1x1, split products, no top-down, Cin 64 / 128 / 256, Cout % 4
// == 0, 16-B aligned operands, and enough pixel strips to fill the chip
// (tuning "conv_stream": 0 off; else the fewest output pixels).
static int stream1x1_variant(const ConvArgs& a, const Plan& p, int flags) {
  const int tv = tuning(kTuneConvStream);
  const bool force = tv < 0;  // (A/B: every eligible shape of >= -tv pixels)
  const int minM = force ? -tv : tv;
  if (tv == 0 || !(flags & kSplit3) || a.KH != 1 || a.KW != 1 || a.stride != 1 || a.pad != 0 ||
      a.topdown || !(a.Cin == 64 || a.Cin == 128 || a.Cin == 256) || a.M < minM)
    return 0;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (a.Cout % 4 != 0 || !al16(a.x) || !al16(a.w) || !al16(a.y) || !al16(a.residual) ||
      !al16(a.gate) || !al16(a.bias))
    return 0;
  if (a.Cin == 256 && a.residual && a.gate) return 0;  // (its registers spill)
  // where it measured faster than the tiled kernel (tools/stream_ab.py,
  // profiles/r5_stream_ab_force_tn_rule.log, with TN 2 when 128-wide slices
  // leave too few strip tasks): every K = 64 and K = 128 launch.  K = 256
  // (1.12-1.17x into <= 64 or 512 channels) only under force: the tiled
  // kernel splits the K of its tail tiles there (>= 8 k-steps), so the two
  // kernels' results differ in the last bit, and a launch whose operands
  // are not 16-B aligned (a gradient bucket view) would then round
  // differently from an aligned one (tests/test_gpu_dp.py's one-rank RCCL
  // equality).  For K <= 128 both kernels sum in the same order: bit-identical.
  if (a.Cin == 64 || a.Cin == 128) return a.Cin == 64 ? 1 : 2;
  // r5b: K = 256 into <= 64 or 512 channels (where it wins) -- make_plan
  // keeps those shapes' tiles whole (no tail split, stream256_shape), so the
  // tiled fallback sums K in the stream kernel's order: bit-identical again
  if (force || stream256_shape(a.M, a.Cout, a.KH, a.KW, a.Cin)) return 3;
  return 0;
}

template <int TN, int KMAX>
static void launch_stream1x1_t(dim3 grid, hipStream_t st, const ConvArgs& a, int nslices) {
  // tuning "conv_stream_nt": bit 0 streaming loads of the epilogue operands, bit 1
  // streaming (non-temporal) stores of the output -- default 2: the stores
  // alone (tools/stream_ab.py --nt, profiles/r5_stream_nt_*.log: 64 -> 256 +
  // residual at 134 k pixels 82.2 -> 66.6 us, 0.58 of HBM; the loads alone
  // lose on 128 -> 512; in-step -0.20 %, profiles/r5_ab_stream_nt.log)
  const int nt = tuning(kTuneConvStreamNt);
  constexpr int W = 8;
  const bool r = a.residual != nullptr, g = a.gate != nullptr;
  if (r && g) {
    if constexpr (TN == 2)  // (both operands' registers: BN 64, launch_stream1x1)
      hipLaunchKernelGGL((conv1x1_stream_kernel<TN, KMAX, W, true, true>), grid, dim3(64 * W), 0,
                         st, a, nslices, nt);
  } else if (r) {
    hipLaunchKernelGGL((conv1x1_stream_kernel<TN, KMAX, W, true, false>), grid, dim3(64 * W), 0,
                       st, a, nslices, nt);
  } else if (g) {
    hipLaunchKernelGGL((conv1x1_stream_kernel<TN, KMAX, W, false, true>), grid, dim3(64 * W), 0,
                       st, a, nslices, nt);
  } else {
    hipLaunchKernelGGL((conv1x1_stream_kernel<TN, KMAX, W, false, false>), grid, dim3(64 * W), 0,
                       st, a, nslices, nt);
  }
}

// variant: 1 K = 64, 2 K = 128, 3 K = 256.  BN 128 (TN 4) for K <= 128 with
// at most one epilogue operand, else BN 64 (TN 2): the registers of a
// residual AND a gate, and K = 256's A fragments, leave no room for TN 4.
static int launch_stream1x1(int variant, const ConvArgs& a, void* stream) {
  constexpr int WAVES = 8;
  const bool both = a.residual && a.gate;
  // TN 2 also when 128-wide slices leave fewer strip tasks than the chip has
  // waves (one 8-wave workgroup per CU)
  const int strips = (a.M + 31) / 32;
  const bool few = (long long)strips * ((a.Cout + 127) / 128) < 8LL * wg_slots(3);
  const int TN = (variant == 3 || both || few) ? 2 : 4;
  const int BN = 32 * TN;
  const int nslices = (a.Cout + BN - 1) / BN;
  const int nstrips = (a.M + 31) / 32;
  // one resident workgroup per CU (LDS: the weight slice + the slabs) over
  // all slices, whole XCD rounds, and no group without a strip for each of
  // its waves
  int groups = std::max(1, wg_slots(3) / nslices / 8);
  groups = std::min(groups, std::max(1, nstrips / WAVES / 8));
  const dim3 grid(8 * groups * nslices);
  hipStream_t st = as_stream(stream);
  if (variant == 1 && TN == 4)
    launch_stream1x1_t<4, 64>(grid, st, a, nslices);
  else if (variant == 1)
    launch_stream1x1_t<2, 64>(grid, st, a, nslices);
  else if (variant == 2 && TN == 4)
    launch_stream1x1_t<4, 128>(grid, st, a, nslices);
  else if (variant == 2)
    launch_stream1x1_t<2, 128>(grid, st, a, nslices);
  else
    launch_stream1x1_t<2, 256>(grid, st, a, nslices);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// Shared launcher of the f32-operand convs (the split or native-f32 MFMA
// products, flags bit 2).
static int conv_core(const float* x, const float* w_packed, const float* bias,
                     const float* topdown, const float* residual, const float* gate, float* y,
                     int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                     int pad_beg, int pad_end, int flags, void* workspace,
                     size_t workspace_bytes, void* stream) {
  ConvArgs a = {};
  a.x = x;
  const int64_t xe = (int64_t)N * H * W * Cin, we = (int64_t)KH * KW * Cin * Cout;
  a.x_bytes = (int)(xe * 4);
  a.w_bytes = (int)(we * 4);
  a.w = w_packed;
  a.bias = bias;
  a.topdown = topdown;
  a.residual = residual;
  a.gate = gate;
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
  {
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    a.lds_epi = Cout % 4 == 0 && al16(y) && al16(residual) && al16(gate) && al16(topdown) &&
                al16(workspace);
  }
  a.reg_partials = tuning(kTuneConvEpi) != 0;
  a.xcd2 = tuning(kTuneConvXCD) != 0;
  a.nt_store = tuning(kTuneConvNt) != 0;  // (tuning "conv_nt", A/B)
  Plan p = make_plan(a.M, Cout, KH, KW, Cin, a.lds_epi != 0, (flags & kSplit3) != 0);
  if (p.ws_bytes > workspace_bytes || workspace == nullptr) {  // no workspace: no split-K
    p.splits = 1;
    p.kt_per_split = p.nk;
    p.full_tiles = p.ntiles;
    p.tail_tiles = 0;
    p.main_m_end = a.M;
  }
  a.nM = (a.M + p.BM - 1) / p.BM;
  a.nN = (Cout + p.BN - 1) / p.BN;
  a.ntiles = p.full_tiles;
  a.tile_base = 0;
  a.m_base = 0;
  a.m_end = p.main_m_end;
  a.splits = p.splits;
  a.kt_per_split = p.kt_per_split;
  a.nk = p.nk;
  a.cchunks = (Cin + BK - 1) / BK;
  a.partial = p.splits > 1 ? (float*)workspace : nullptr;
  a.tdH = (a.OH + 1) / 2;
  a.tdW = (a.OW + 1) / 2;
  hipStream_t st = as_stream(stream);
  ConvArgs t = a;  // the tail launch (when planned)
  if (p.tail_tiles > 0) {
    t.tile_base = p.full_tiles;
    t.ntiles = p.tail_tiles;
    t.m_base = p.full_tiles / a.nN * p.BM;
    t.m_end = a.M;
    t.splits = p.tail_splits;
    t.kt_per_split = p.tail_kt_per_split;
    t.partial = (float*)workspace +
                (p.splits > 1 ? (size_t)p.splits * p.main_m_end * Cout : (size_t)0);
  }
  // 128x128 tiles: single-buffered LDS (two barriers per k-step, 3 workgroups
  // per CU) measured faster than double-buffered on every Mask R-CNN shape,
  // f32 and split, large grids and small.
  const bool db = false;
  // r5: the streaming short-K 1x1 kernel (conv1x1_stream_kernel) for the
  // memory-bound stride-1 1x1s, when the plan has no split-K
  {
    const int sk = stream1x1_variant(a, p, flags);
    if (sk > 0) return launch_stream1x1(sk, a, stream);
  }
  // Split-K partials go to the workspace and a second launch sums them in a
  // fixed order + applies the epilogue (deterministic).  r3 measured the
  // in-launch alternative (the last-arriving workgroup of each tile sums its
  // tile, agent-scope release / acquire): bit-identical but 6 % slower in the
  // step -- one workgroup reads its tile's 64-128 KiB slabs at ~100 GB/s --
  // and r4 removed it.
  auto launch = [&](const ConvArgs& c) {
    const dim3 g(c.ntiles, c.splits);
    if (flags & kSplit3)
      launch_conv<true>(p.cfg, db, g, st, c);
    else
      launch_conv<false>(p.cfg, db, g, st, c);
    D2MI_LAUNCH_CHECK();
    if (c.splits > 1) {
      const int64_t total = (int64_t)(c.m_end - c.m_base) * Cout;
      // (the float4 epilogue reads bias / top-down / residual / gate as float4s)
      const uintptr_t ops4 = (uintptr_t)c.bias | (uintptr_t)c.topdown | (uintptr_t)c.residual |
                             (uintptr_t)c.gate;
      if (Cout % 4 == 0 && ((uintptr_t)c.partial & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
          (ops4 & 15) == 0) {
        const int gr = (int)std::min<int64_t>((total / 4 + 255) / 256, 8192);
        hipLaunchKernelGGL(splitk_reduce4_kernel, dim3(gr), dim3(256), 0, st, c);
      } else {
        const int gr = (int)std::min<int64_t>((total + 255) / 256, 4096);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gr), dim3(256), 0, st, c);
      }
      D2MI_LAUNCH_CHECK();
    }
    return 0;
  };
  if (a.ntiles > 0) {
    const int rc = launch(a);
    if (rc) return rc;
  }
  if (p.tail_tiles > 0) return launch(t);
  return 0;
}


// f32-operand conv with the >= 2 GiB-batch image chunking (32-bit buffer offsets).
static int conv_f32(const float* x, const float* w_packed, const float* bias,
                    const float* topdown, const float* residual, const float* gate, float* y,
                    int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                    int pad_beg, int pad_end, int flags, void* workspace, size_t workspace_bytes,
                    void* stream) {
  D2MI_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0,
               "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0, "Cin must be a multiple of 4 (got %d)", Cin);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_packed & 15) == 0,
               "x and w must be 16-byte aligned");
  const int64_t img_bytes = (int64_t)H * W * Cin * sizeof(float);
  D2MI_REQUIRE(img_bytes < (1ll << 31), "one conv input image must be < 2 GiB");
  D2MI_REQUIRE((int64_t)KH * KW * Cin * Cout * sizeof(float) < (1ll << 31),
               "conv weights must be < 2 GiB");
  if ((int64_t)N * img_bytes >= (1ll << 31)) {
    int OH0, OW0;
    D2MI_REQUIRE(conv_dims(H, W, KH, KW, stride, pad_beg, pad_end, OH0, OW0) == 0,
                 "conv output is empty");
    const int chunk = (int)(((1ll << 31) - 1) / img_bytes);
    const size_t xs = (size_t)H * W * Cin, ys = (size_t)OH0 * OW0 * Cout;
    const size_t ts = (size_t)((OH0 + 1) / 2) * ((OW0 + 1) / 2) * Cout;
    for (int n0 = 0; n0 < N; n0 += chunk) {
      const int nn = std::min(chunk, N - n0);
      const int rc = conv_f32(
          x + n0 * xs, w_packed, bias, topdown ? topdown + n0 * ts : nullptr,
          residual ? residual + n0 * ys : nullptr, gate ? gate + n0 * ys : nullptr, y + n0 * ys,
          nn, H, W, Cin, Cout, KH, KW, stride, pad_beg, pad_end, flags, workspace,
          workspace_bytes, stream);
      if (rc) return rc;
    }
    return 0;
  }
  return conv_core(x, w_packed, bias, topdown, residual, gate, y, N, H, W, Cin, Cout, KH, KW,
                   stride, pad_beg, pad_end, flags, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_conv2d_nhwc_ex(const float* x, const float* w_packed, const float* bias,
                                   const float* topdown, const float* residual, float* y, int N,
                                   int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                   int pad_beg, int pad_end, int flags, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE((flags & ~31) == 0,
               "flags: bit0 relu, bit1 relu after the residual/top-down add, bit2 split-bf16 "
               "MFMA products, bit3 flipped weight taps, bit4 residual is a ReLU gate");
  D2MI_REQUIRE(!(flags & kMaskByResidual) || (residual && !topdown && !(flags & 3)),
               "the ReLU gate (bit4) needs the residual operand and no relu / top-down");
  if (flags & kMaskByResidual)
    return conv_f32(x, w_packed, bias, nullptr, nullptr, residual, y, N, H, W, Cin, Cout, KH, KW,
                    stride, pad_beg, pad_end, flags & ~kMaskByResidual, workspace,
                    workspace_bytes, stream);
  return conv_f32(x, w_packed, bias, topdown, residual, nullptr, y, N, H, W, Cin, Cout, KH, KW,
                  stride, pad_beg, pad_end, flags, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_conv2d_nhwc_gated(const float* x, const float* w_packed, const float* bias,
                                      const float* residual, const float* gate, float* y, int N,
                                      int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                      int pad_beg, int pad_end, int flags, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE((flags & ~(kSplit3 | kFlipTaps)) == 0,
               "gated conv flags: bit2 split-bf16 MFMA products, bit3 flipped weight taps");
  D2MI_REQUIRE(gate != nullptr, "gated conv needs its gate");
  return conv_f32(x, w_packed, bias, nullptr, residual, gate, y, N, H, W, Cin, Cout, KH, KW,
                  stride, pad_beg, pad_end, flags, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_conv2d_nhwc(const float* x, const float* w_packed, const float* bias,
                                const float* topdown, const float* residual, float* y, int N,
                                int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad_beg, int pad_end, int act, void* stream) {
  D2MI_REQUIRE(act == 0 || act == 1, "act must be 0 (none) or 1 (relu)");
  return d2mi_conv2d_nhwc_ex(x, w_packed, bias, topdown, residual, y, N, H, W, Cin, Cout, KH, KW,
                             stride, pad_beg, pad_end, act ? kRelu : 0, nullptr, 0, stream);
}

// Split-K plan of a multi-level launch: the single-level rule on the total
// tile count (Cout % 4 == 0 for the level-aware reduce).
static int levels_splits(const int32_t* dims, int nlev, int Cin, int Cout, int KH, int KW,
                         int stride, int pad_beg, int pad_end, int64_t* rows, int* ntiles) {
  const Plan p0 = make_plan(1, Cout, KH, KW, Cin, Cout % 4 == 0, false);  // (no cfg 3)
  const int nN = (Cout + p0.BN - 1) / p0.BN;
  int64_t r = 0;
  int t = 0;
  for (int l = 0; l < nlev; ++l) {
    int OH = 0, OW = 0;
    conv_dims(dims[3 * l + 1], dims[3 * l + 2], KH, KW, stride, pad_beg, pad_end, OH, OW);
    const int64_t M = (int64_t)dims[3 * l] * OH * OW;
    r += M;
    t += (int)((M + p0.BM - 1) / p0.BM) * nN;
  }
  *rows = r;
  *ntiles = t;
  const int G = wg_slots(p0.cfg);
  const int nk = KH * KW * ((Cin + BK - 1) / BK);
  if (Cout % 4 || !(4 * t < 3 * G && nk >= 16)) return 1;
  const int S = std::min(std::max(1, G / std::max(t, 1)), std::min(nk / 8, 16));
  const int kps = (nk + S - 1) / S;
  return (nk + kps - 1) / kps;
}

extern "C" size_t d2mi_conv2d_levels_workspace_size(const int32_t* dims, int nlev, int Cin,
                                                    int Cout, int KH, int KW, int stride,
                                                    int pad_beg, int pad_end) {
  if (nlev < 1 || nlev > kMaxConvLevels) return 0;
  int64_t rows;
  int t;
  const int S = levels_splits(dims, nlev, Cin, Cout, KH, KW, stride, pad_beg, pad_end, &rows, &t);
  return S > 1 ? (size_t)S * rows * Cout * sizeof(float) : 0;
}

extern "C" int d2mi_conv2d_nhwc_levels(const float* const* xs, const int32_t* dims, int nlev,
                                       const float* w_packed, const float* bias, float* const* ys,
                                       int Cin, int Cout, int KH, int KW, int stride, int pad_beg,
                                       int pad_end, int flags, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(nlev >= 1 && nlev <= kMaxConvLevels, "nlev=%d out of [1,%d]", nlev, kMaxConvLevels);
  D2MI_REQUIRE(Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0, "bad conv shape");
  D2MI_REQUIRE(Cin % 4 == 0, "Cin must be a multiple of 4 (got %d)", Cin);
  D2MI_REQUIRE((flags & ~(kRelu | kSplit3)) == 0,
               "multi-level conv flags: bit0 relu, bit2 split-bf16 MFMA products");
  D2MI_REQUIRE(((uintptr_t)w_packed & 15) == 0, "w must be 16-byte aligned");
  D2MI_REQUIRE((int64_t)KH * KW * Cin * Cout * sizeof(float) < (1ll << 31),
               "conv weights must be < 2 GiB");
  ConvArgs a = {};
  a.w = w_packed;
  a.w_bytes = (int)((int64_t)KH * KW * Cin * Cout * 4);
  a.bias = bias;
  a.Cin = Cin;
  a.Cout = Cout;
  a.KH = KH;
  a.KW = KW;
  a.stride = stride;
  a.pad = pad_beg;
  a.flags = flags;
  a.nlev = nlev;
  bool al = (Cout % 4) == 0;
  int64_t Mtot = 0;
  for (int l = 0; l < nlev; ++l) {
    const int N = dims[3 * l], H = dims[3 * l + 1], W = dims[3 * l + 2];
    int OH, OW;
    D2MI_REQUIRE(N > 0 && H > 0 && W > 0 &&
                     conv_dims(H, W, KH, KW, stride, pad_beg, pad_end, OH, OW) == 0,
                 "level %d: bad or empty conv geometry", l);
    D2MI_REQUIRE((int64_t)N * H * W * Cin * 4 < (1ll << 31), "level %d input must be < 2 GiB", l);
    D2MI_REQUIRE(((uintptr_t)xs[l] & 15) == 0, "level %d input must be 16-byte aligned", l);
    al = al && ((uintptr_t)ys[l] & 15) == 0;
    a.lv_x[l] = xs[l];
    a.lv_y[l] = ys[l];
    a.lv_gate[l] = nullptr;
    a.lv_N[l] = N;
    a.lv_H[l] = H;
    a.lv_W[l] = W;
    a.lv_OH[l] = OH;
    a.lv_OW[l] = OW;
    a.lv_xbytes[l] = (int)((int64_t)N * H * W * Cin * 4);
    Mtot += (int64_t)N * OH * OW;
  }
  a.lds_epi = al;
  // multi-level launches keep the 128-row kernels (no cfg 3: r3 measured the
  // multi-level warp-specialised form neutral for Mask R-CNN and 2-8 %
  // slower for the RetinaNet / SOLOv2 towers; removed in r4)
  a.reg_partials = 0;
  const Plan p = make_plan((int)std::min<int64_t>(Mtot, 1 << 30), Cout, KH, KW, Cin, al, false);
  a.nN = (Cout + p.BN - 1) / p.BN;
  int t = 0;
  for (int l = 0; l < nlev; ++l) {
    a.lv_tile0[l] = t;
    t += (a.lv_N[l] * a.lv_OH[l] * a.lv_OW[l] + p.BM - 1) / p.BM * a.nN;
  }
  a.lv_tile0[nlev] = t;
  a.ntiles = t;
  a.tile_base = 0;
  a.nk = KH * KW * ((Cin + BK - 1) / BK);
  {
    int64_t rows;
    int tt;
    int S = levels_splits(dims, nlev, Cin, Cout, KH, KW, stride, pad_beg, pad_end, &rows, &tt);
    if (S > 1 && (workspace == nullptr || workspace_bytes < (size_t)S * rows * Cout * 4 ||
                  ((uintptr_t)workspace & 15) != 0 || !al))
      S = 1;  // no (usable) workspace: one pass per tile
    a.splits = S;
    a.kt_per_split = (a.nk + S - 1) / S;
    a.partial = S > 1 ? (float*)workspace : nullptr;
    int64_t off = 0;
    for (int l = 0; l <= kMaxConvLevels; ++l) {
      a.lv_moff[l] = (int)off;
      if (l < nlev) off += (int64_t)a.lv_N[l] * a.lv_OH[l] * a.lv_OW[l];
    }
    for (int l = nlev; l <= kMaxConvLevels; ++l) a.lv_moff[l] = (int)rows;
  }
  a.cchunks = (Cin + BK - 1) / BK;
  // level 0's geometry in the single-level fields (unused by the kernel)
  a.x = xs[0];
  a.y = ys[0];
  a.N = a.lv_N[0];
  a.H = a.lv_H[0];
  a.W = a.lv_W[0];
  a.OH = a.lv_OH[0];
  a.OW = a.lv_OW[0];
  a.M = a.N * a.OH * a.OW;
  a.m_end = a.M;
  a.x_bytes = a.lv_xbytes[0];
  a.tdH = a.tdW = 1;
  const dim3 grid(a.ntiles, a.splits);
  if (flags & kSplit3)
    launch_conv_levels<true>(p.cfg, grid, as_stream(stream), a);
  else
    launch_conv_levels<false>(p.cfg, grid, as_stream(stream), a);
  D2MI_LAUNCH_CHECK();
  if (a.splits > 1) {
    const int64_t total = (int64_t)a.lv_moff[kMaxConvLevels] * (Cout / 4);
    const int gr = (int)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(splitk_reduce_levels_kernel, dim3(gr), dim3(256), 0, as_stream(stream), a);
    D2MI_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int d2mi_split_bf16x3(const float* x, int64_t n, uint16_t* out, void* stream) {
  D2MI_REQUIRE(n >= 0 && n % 4 == 0, "split: n must be a multiple of 4 (got %lld)", (long long)n);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 7) == 0, "split: misaligned buffers");
  if (n == 0) return 0;
  const int64_t n4 = n / 4;
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 16384);
  hipLaunchKernelGGL(split3_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(x), n4, reinterpret_cast<uint2*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}
