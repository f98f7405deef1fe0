// FrozenBN folded into the preceding convolution, forward and backward, as two
// fused kernels instead of the ~14 elementwise launches per conv autograd makes
// of  scale = gamma * rsqrt(var + eps),  w_eff = w * scale,  b_eff = beta - mean*scale
// (+ bias * scale).
//
// Reference: lib/layers/normalization.py:15-119 (BatchNorm with training=False:
// moving statistics, gamma / beta trainable above FREEZE_AT — the
// resnet_arg_scope of lib/modeling/backbone/resnet.py:22-46) applied after
// Conv2D (lib/layers/convolutional.py:198-263).  conv(x, w) * scale + shift ==
// conv(x, w * scale) + shift, so the frozen affine folds into the weights.
//
// Layout: w HWIO [rows = KH*KW*Cin][Cout] (Cout contiguous).  Forward writes
// w_eff (HWIO) and/or the MFMA-packed copy [KH][KW][Cout][Cin] in the same
// pass.  Backward: gw = gw_eff * scale (elementwise, same pass) and the
// per-channel reductions  sum_rows gw_eff * w  split over row chunks into a
// workspace and summed in a FIXED chunk order by a second kernel, which also
// forms d gamma, d beta and d bias.
#include "common.h"

namespace d2mi {
namespace {

constexpr int kRowChunks = 32;

__device__ __forceinline__ float bn_inv(const float* var, float eps, int c) {
  return 1.f / sqrtf(var[c] + eps);
}

__global__ void fold_bn_kernel(const float* __restrict__ w, const float* __restrict__ bias,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ mean, const float* __restrict__ var,
                               float eps, int rows, int Cout, int taps, int Cin,
                               float* __restrict__ w_eff, float* __restrict__ w_packed,
                               float* __restrict__ b_eff) {
  const int co = blockIdx.x * 64 + (threadIdx.x & 63);
  if (co >= Cout) return;
  const float inv = bn_inv(var, eps, co);
  const float scale = gamma ? inv * gamma[co] : inv;
  if (blockIdx.y == 0 && threadIdx.x < 64) {
    float shift = -mean[co] * scale;
    if (beta) shift = shift + beta[co];
    b_eff[co] = bias ? bias[co] * scale + shift : shift;
  }
  const int rstep = gridDim.y * (blockDim.x >> 6);
  for (int r = blockIdx.y * (blockDim.x >> 6) + (threadIdx.x >> 6); r < rows; r += rstep) {
    const float v = w[(size_t)r * Cout + co] * scale;
    if (w_eff) w_eff[(size_t)r * Cout + co] = v;
    if (w_packed) {  // [tap][co][ci]
      const int tap = r / Cin, ci = r - tap * Cin;
      w_packed[((size_t)tap * Cout + co) * Cin + ci] = v;
    }
  }
}

// Tiled variant (Cin % 64 == 0, i.e. every ResNet conv): a 64 (ci) x 64 (co)
// tile of one tap per workgroup; w / w_eff rows are read and written along
// co, the packed [tap][co][ci] copy is written along ci from an LDS transpose
// -- both coalesced (the per-element version above writes the packed copy
// with a stride of Cin between lanes).
__global__ __launch_bounds__(256) void fold_bn_tiled_kernel(
    const float* __restrict__ w, const float* __restrict__ bias, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ var,
    float eps, int Cout, int Cin, float* __restrict__ w_eff, float* __restrict__ w_packed,
    float* __restrict__ b_eff) {
  __shared__ float tile[64][65];
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64, tap = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int co = co0 + lane;
  const bool live = co < Cout;
  float scale = 0.f;
  if (live) {
    const float inv = bn_inv(var, eps, co);
    scale = gamma ? inv * gamma[co] : inv;
    if (blockIdx.y == 0 && tap == 0 && wv == 0) {
      float shift = -mean[co] * scale;
      if (beta) shift = shift + beta[co];
      b_eff[co] = bias ? bias[co] * scale + shift : shift;
    }
  }
  for (int i = wv; i < 64; i += 4) {  // rows ci0 + i of this tap, lanes over co
    const size_t r = (size_t)tap * Cin + ci0 + i;
    const float v = live ? w[r * Cout + co] * scale : 0.f;
    if (w_eff && live) w_eff[r * Cout + co] = v;
    tile[i][lane] = v;
  }
  if (!w_packed) return;
  __syncthreads();
  for (int j = wv; j < 64; j += 4) {  // packed rows co0 + j, lanes over ci
    if (co0 + j < Cout)
      w_packed[((size_t)tap * Cout + co0 + j) * Cin + ci0 + lane] = tile[lane][j];
  }
}

// partial[chunk][0][co] = sum gw_eff * w over the chunk's rows; gw = gw_eff * scale.
__global__ void fold_bn_bwd_kernel(const float* __restrict__ gw_eff, const float* __restrict__ w,
                                   const float* __restrict__ gamma, const float* __restrict__ var,
                                   float eps, int rows, int Cout, float* __restrict__ gw,
                                   float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int co = blockIdx.x * 64 + lane;
  const bool live = co < Cout;
  const int chunk = blockIdx.y;
  const int per = (rows + kRowChunks - 1) / kRowChunks;
  const int r0 = chunk * per, r1 = min(rows, r0 + per);
  float scale = 0.f;
  if (live) {
    const float inv = bn_inv(var, eps, co);
    scale = gamma ? inv * gamma[co] : inv;
  }
  float s = 0.f;
  if (live) {
    for (int r = r0 + wv; r < r1; r += 4) {
      const float g = gw_eff[(size_t)r * Cout + co];
      s += g * w[(size_t)r * Cout + co];
      if (gw) gw[(size_t)r * Cout + co] = g * scale;
    }
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && live)
    partial[(size_t)chunk * Cout + co] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ void fold_bn_bwd_finish_kernel(const float* __restrict__ partial,
                                          const float* __restrict__ gb_eff,
                                          const float* __restrict__ bias,
                                          const float* __restrict__ gamma,
                                          const float* __restrict__ mean,
                                          const float* __restrict__ var, float eps, int Cout,
                                          float* __restrict__ gbias, float* __restrict__ ggamma,
                                          float* __restrict__ gbeta) {
  const int co = blockIdx.x * blockDim.x + threadIdx.x;
  if (co >= Cout) return;
  float gs = 0.f;
  for (int k = 0; k < kRowChunks; ++k) gs += partial[(size_t)k * Cout + co];
  const float inv = bn_inv(var, eps, co);
  const float scale = gamma ? inv * gamma[co] : inv;
  const float gb = gb_eff ? gb_eff[co] : 0.f;
  // b_eff = bias * scale + beta - mean * scale
  gs = gs + gb * ((bias ? bias[co] : 0.f) - mean[co]);
  if (ggamma) ggamma[co] = gs * inv;
  if (gbeta) gbeta[co] = gb;
  if (gbias) gbias[co] = gb * scale;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_fold_frozen_bn(const float* w_hwio, const float* bias, const float* gamma,
                                   const float* beta, const float* mean, const float* var,
                                   float eps, int KH, int KW, int Cin, int Cout, float* w_eff,
                                   float* w_packed, float* b_eff, void* stream) {
  D2MI_REQUIRE(KH > 0 && KW > 0 && Cin > 0 && Cout > 0, "bad weight shape");
  D2MI_REQUIRE(w_hwio && mean && var && b_eff, "w, mean, var and b_eff are required");
  const int rows = KH * KW * Cin;
  if (Cin % 64 == 0) {
    dim3 grid((Cout + 63) / 64, Cin / 64, KH * KW);
    hipLaunchKernelGGL(fold_bn_tiled_kernel, grid, dim3(256), 0, as_stream(stream), w_hwio, bias,
                       gamma, beta, mean, var, eps, Cout, Cin, w_eff, w_packed, b_eff);
    D2MI_LAUNCH_CHECK();
    return 0;
  }
  const int gy = std::min(64, std::max(1, rows / 64));
  dim3 grid((Cout + 63) / 64, gy);
  hipLaunchKernelGGL(fold_bn_kernel, grid, dim3(256), 0, as_stream(stream), w_hwio, bias, gamma,
                     beta, mean, var, eps, rows, Cout, KH * KW, Cin, w_eff, w_packed, b_eff);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_fold_frozen_bn_bwd_workspace_size(int Cout) {
  return (size_t)kRowChunks * (size_t)(Cout > 0 ? Cout : 0) * sizeof(float);
}

extern "C" int d2mi_fold_frozen_bn_bwd(const float* gw_eff, const float* gb_eff,
                                       const float* w_hwio, const float* bias, const float* gamma,
                                       const float* mean, const float* var, float eps, int KH,
                                       int KW, int Cin, int Cout, float* gw, float* gbias,
                                       float* ggamma, float* gbeta, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(KH > 0 && KW > 0 && Cin > 0 && Cout > 0, "bad weight shape");
  D2MI_REQUIRE(gw_eff && w_hwio && mean && var, "gw_eff, w, mean and var are required");
  D2MI_REQUIRE(workspace_bytes >= d2mi_fold_frozen_bn_bwd_workspace_size(Cout) && workspace,
               "fold_frozen_bn_bwd workspace too small");
  const int rows = KH * KW * Cin;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(fold_bn_bwd_kernel, dim3((Cout + 63) / 64, kRowChunks), dim3(256), 0, st,
                     gw_eff, w_hwio, gamma, var, eps, rows, Cout, gw, (float*)workspace);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(fold_bn_bwd_finish_kernel, dim3((Cout + 255) / 256), dim3(256), 0, st,
                     (const float*)workspace, gb_eff, bias, gamma, mean, var, eps, Cout, gbias,
                     ggamma, gbeta);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------ batched fold
// Every BN-conv of the backbone folded by ONE forward launch and ONE backward
// pair, driven by a table of d2mi_fold_entry (include/d2mi.h) instead of ~50
// launches of each kernel above per step.  Each workgroup finds its entry by
// binary search over the entries' first-block indices (the table is small and
// sits in L2 after the first wave), then does the same work as
// fold_bn_tiled_kernel / fold_bn_bwd_kernel / fold_bn_bwd_finish_kernel with
// ci / co tails guarded, so any Cin works.  Sums keep the fixed row-chunk order
// of the per-conv kernels: results are bit-identical to them.
namespace d2mi {
namespace {

__device__ __forceinline__ int find_entry(const d2mi_fold_entry* __restrict__ t, int n, int b,
                                          int which) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last entry whose begin <= b
    const int mid = (lo + hi + 1) >> 1;
    const int beg = which == 0 ? t[mid].fwd_begin : which == 1 ? t[mid].bwd_begin : t[mid].co_begin;
    if (beg <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void fold_bn_many_kernel(const d2mi_fold_entry* __restrict__ tab,
                                                           int n) {
  __shared__ float tile[64][65];
  const d2mi_fold_entry& e = tab[find_entry(tab, n, blockIdx.x, 0)];
  const int Cout = e.Cout, Cin = e.Cin;
  const int nco = (Cout + 63) / 64, nci = (Cin + 63) / 64;
  int local = blockIdx.x - e.fwd_begin;
  const int cot = local % nco; local /= nco;
  const int cit = local % nci;
  const int tap = local / nci;
  const int co0 = cot * 64, ci0 = cit * 64;
  // float4 form (Cin, Cout multiples of 4, 16-B aligned tensors: every ResNet
  // conv): 16 threads per 64-channel row, 16-B loads and stores, the same
  // per-element product (bit-identical)
  const bool al = ((reinterpret_cast<uintptr_t>(e.w) | reinterpret_cast<uintptr_t>(e.w_eff) |
                    reinterpret_cast<uintptr_t>(e.w_packed)) & 15) == 0;
  if (Cout % 4 == 0 && Cin % 4 == 0 && al) {
    const int t = threadIdx.x;
    const int cq = t & 15, ri = t >> 4;  // channel quad, row phase
    const int c4 = co0 + 4 * cq;
    const bool live4 = c4 < Cout;        // (Cout % 4 == 0: the quad is whole)
    float sc[4] = {0.f, 0.f, 0.f, 0.f};
    if (live4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float inv = bn_inv(e.var, e.eps, c4 + q);
        sc[q] = e.gamma ? inv * e.gamma[c4 + q] : inv;
      }
      if (cit == 0 && tap == 0 && ri == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float shift = -e.mean[c4 + q] * sc[q];
          if (e.beta) shift = shift + e.beta[c4 + q];
          e.b_eff[c4 + q] = e.bias ? e.bias[c4 + q] * sc[q] + shift : shift;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = ri + 16 * k;
      const bool row = ci0 + i < Cin;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (live4 && row) {
        const size_t o = ((size_t)tap * Cin + ci0 + i) * Cout + c4;
        const float4 w4 = *reinterpret_cast<const float4*>(e.w + o);
        v = make_float4(w4.x * sc[0], w4.y * sc[1], w4.z * sc[2], w4.w * sc[3]);
        if (e.w_eff) *reinterpret_cast<float4*>(e.w_eff + o) = v;
      }
      tile[i][4 * cq] = v.x;
      tile[i][4 * cq + 1] = v.y;
      tile[i][4 * cq + 2] = v.z;
      tile[i][4 * cq + 3] = v.w;
    }
    if (!e.w_packed) return;
    __syncthreads();
    const int ciq = t & 15, cj = t >> 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = cj + 16 * k;
      const int ci = ci0 + 4 * ciq;
      if (co0 + j < Cout && ci < Cin)
        *reinterpret_cast<float4*>(e.w_packed + ((size_t)tap * Cout + co0 + j) * Cin + ci) =
            make_float4(tile[4 * ciq][j], tile[4 * ciq + 1][j], tile[4 * ciq + 2][j],
                        tile[4 * ciq + 3][j]);
    }
    return;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int co = co0 + lane;
  const bool live = co < Cout;
  float scale = 0.f;
  if (live) {
    const float inv = bn_inv(e.var, e.eps, co);
    scale = e.gamma ? inv * e.gamma[co] : inv;
    if (cit == 0 && tap == 0 && wv == 0) {
      float shift = -e.mean[co] * scale;
      if (e.beta) shift = shift + e.beta[co];
      e.b_eff[co] = e.bias ? e.bias[co] * scale + shift : shift;
    }
  }
  for (int i = wv; i < 64; i += 4) {
    const bool row = ci0 + i < Cin;
    const size_t r = (size_t)tap * Cin + ci0 + i;
    const float v = live && row ? e.w[r * Cout + co] * scale : 0.f;
    if (e.w_eff && live && row) e.w_eff[r * Cout + co] = v;
    tile[i][lane] = v;
  }
  if (!e.w_packed) return;
  __syncthreads();
  for (int j = wv; j < 64; j += 4) {
    if (co0 + j < Cout && ci0 + lane < Cin)
      e.w_packed[((size_t)tap * Cout + co0 + j) * Cin + ci0 + lane] = tile[lane][j];
  }
}

__global__ __launch_bounds__(256) void fold_bn_bwd_many_kernel(
    const d2mi_fold_entry* __restrict__ tab, int n, float* __restrict__ ws) {
  __shared__ float red[4][64];
  const d2mi_fold_entry& e = tab[find_entry(tab, n, blockIdx.x, 1)];
  const int Cout = e.Cout, rows = e.taps * e.Cin;
  const int nco = (Cout + 63) / 64;
  const int local = blockIdx.x - e.bwd_begin;
  const int cot = local % nco, chunk = local / nco;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int co = cot * 64 + lane;
  const bool live = co < Cout;
  const int per = (rows + kRowChunks - 1) / kRowChunks;
  const int r0 = chunk * per, r1 = min(rows, r0 + per);
  if (!e.ggamma) {
    // no gamma gradient (FrozenBN: gamma is a constant): only gw = gw_eff *
    // scale -- the sum of gw_eff * w (and so the read of w) is not needed;
    // float4 rows where aligned, 16 threads per 64-channel row
    if (!e.gw) return;
    const bool al = ((reinterpret_cast<uintptr_t>(e.gw_eff) | reinterpret_cast<uintptr_t>(e.gw)) &
                     15) == 0;
    if (Cout % 4 == 0 && al) {
      const int t = threadIdx.x, cq = t & 15, ri = t >> 4;
      const int c4 = cot * 64 + 4 * cq;
      if (c4 >= Cout) return;
      float sc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float inv = bn_inv(e.var, e.eps, c4 + q);
        sc[q] = e.gamma ? inv * e.gamma[c4 + q] : inv;
      }
#pragma unroll 4
      for (int r = r0 + ri; r < r1; r += 16) {
        const size_t o = (size_t)r * Cout + c4;
        const float4 g = e.gw_eff ? *reinterpret_cast<const float4*>(e.gw_eff + o)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(e.gw + o) =
            make_float4(g.x * sc[0], g.y * sc[1], g.z * sc[2], g.w * sc[3]);
      }
      return;
    }
    if (!live) return;
    const float inv = bn_inv(e.var, e.eps, co);
    const float scale = e.gamma ? inv * e.gamma[co] : inv;
#pragma unroll 8
    for (int r = r0 + wv; r < r1; r += 4) {
      const float g = e.gw_eff ? e.gw_eff[(size_t)r * Cout + co] : 0.f;
      e.gw[(size_t)r * Cout + co] = g * scale;
    }
    return;
  }
  float scale = 0.f;
  if (live) {
    const float inv = bn_inv(e.var, e.eps, co);
    scale = e.gamma ? inv * e.gamma[co] : inv;
  }
  float s = 0.f;
  if (live) {
    // unrolled: eight rows' loads in flight per lane (the sum keeps its order)
#pragma unroll 8
    for (int r = r0 + wv; r < r1; r += 4) {
      const float g = e.gw_eff ? e.gw_eff[(size_t)r * Cout + co] : 0.f;
      s += g * e.w[(size_t)r * Cout + co];
      if (e.gw) e.gw[(size_t)r * Cout + co] = g * scale;
    }
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && live)
    ws[e.partial_offset + (size_t)chunk * Cout + co] =
        ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ void fold_bn_bwd_many_finish_kernel(const d2mi_fold_entry* __restrict__ tab, int n,
                                               int total_cout, const float* __restrict__ ws) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total_cout) return;
  const d2mi_fold_entry& e = tab[find_entry(tab, n, g, 2)];
  const int Cout = e.Cout, co = g - e.co_begin;
  const float* partial = ws + e.partial_offset;
  float gs = 0.f;
  if (e.ggamma)  // (the partials exist only then: fold_bn_bwd_many_kernel)
    for (int k = 0; k < kRowChunks; ++k) gs += partial[(size_t)k * Cout + co];
  const float inv = bn_inv(e.var, e.eps, co);
  const float scale = e.gamma ? inv * e.gamma[co] : inv;
  const float gb = e.gb_eff ? e.gb_eff[co] : 0.f;
  gs = gs + gb * ((e.bias ? e.bias[co] : 0.f) - e.mean[co]);
  if (e.ggamma) e.ggamma[co] = gs * inv;
  if (e.gbeta) e.gbeta[co] = gb;
  if (e.gbias) e.gbias[co] = gb * scale;
}

}  // namespace
}  // namespace d2mi

extern "C" int d2mi_fold_many_sizes(int* entry_bytes, int* row_chunks) {
  if (entry_bytes) *entry_bytes = (int)sizeof(d2mi_fold_entry);
  if (row_chunks) *row_chunks = kRowChunks;
  return 0;
}

extern "C" int d2mi_fold_frozen_bn_many(const d2mi_fold_entry* table, int num_entries,
                                        int fwd_blocks, void* stream) {
  D2MI_REQUIRE(table && num_entries > 0 && fwd_blocks > 0, "empty fold table");
  hipLaunchKernelGGL(fold_bn_many_kernel, dim3(fwd_blocks), dim3(256), 0, as_stream(stream), table,
                     num_entries);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_fold_frozen_bn_bwd_many(const d2mi_fold_entry* table, int num_entries,
                                            int bwd_blocks, int total_cout, float* workspace,
                                            void* stream) {
  D2MI_REQUIRE(table && num_entries > 0 && bwd_blocks > 0 && total_cout > 0, "empty fold table");
  D2MI_REQUIRE(workspace, "fold_frozen_bn_bwd_many needs its workspace");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(fold_bn_bwd_many_kernel, dim3(bwd_blocks), dim3(256), 0, st, table,
                     num_entries, workspace);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(fold_bn_bwd_many_finish_kernel, dim3((total_cout + 255) / 256), dim3(256), 0,
                     st, table, num_entries, total_cout, (const float*)workspace);
  D2MI_LAUNCH_CHECK();
  return 0;
}
