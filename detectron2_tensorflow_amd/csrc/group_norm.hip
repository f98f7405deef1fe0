// GroupNorm on NHWC (lib/layers/normalization.py:174-260: tf.nn.moments over
// (H, W, channels of the group), then tf.nn.batch_normalization:
// inv = rsqrt(var + eps) * gamma, y = x * inv + (beta - mean * inv)), with
// the ops that follow it in the SOLOv2 heads fused into the apply pass:
// ReLU (the conv's activation, solo_v2.py:173-183 / :659-669), the nearest
// x2 upsample of MaskFeatureBranch (wrappers.py:104-116 — the reference's
// Upsample ignores its method) and the running sum of the scale heads
// (solo_v2.py:705-721: res = res + head(feature)).
//
// Five launches, deterministic (fixed-order reductions, no atomics):
//   gn_sum_kernel        per (image, pixel chunk) per-group partial sums
//   gn_reduce_kernel     -> mean
//   gn_sum_kernel        per-group partial sums of (x - mean)^2 (the
//                        two-pass variance of tf.nn.moments)
//   gn_reduce_kernel     -> var
//   gn_apply_kernel      per-channel inv / shift, apply (+ ReLU, up2, sum)
// Each pass reads x once (float4 over channels, coalesced whole pixels).
#include <algorithm>

#include "common.h"

namespace d2mi {
namespace {

constexpr int kGnThreads = 256;
constexpr int kGnMaxGroups = 64;

// partial[(n * chunks + chunk) * G + g]
__global__ __launch_bounds__(kGnThreads) void gn_sum_kernel(const float* __restrict__ x, int HW,
                                                           int C, int G, int chunk_px,
                                                           const float* __restrict__ mean,
                                                           float* __restrict__ partial) {
  __shared__ float red[kGnThreads];
  const int chunk = blockIdx.x, n = blockIdx.y, chunks = gridDim.x;
  const int C4 = C / 4;
  const int tc = threadIdx.x % C4;             // this thread's channel quad
  const int tp = threadIdx.x / C4;             // pixel slot
  const int ppi = kGnThreads / C4;             // pixels per iteration
  const int cpg = C / G;                       // channels per group
  const int g = tc * 4 / cpg;                  // the group of the quad (cpg % 4 == 0)
  const float mu = mean ? mean[n * G + g] : 0.f;
  const int p0 = chunk * chunk_px, p1 = min(HW, p0 + chunk_px);
  const float* xb = x + (size_t)n * HW * C;
  float acc = 0.f;
  if (threadIdx.x < ppi * C4) {
    for (int p = p0 + tp; p < p1; p += ppi) {
      const float4 v = *reinterpret_cast<const float4*>(xb + (size_t)p * C + tc * 4);
      if (mean) {
        const float a = v.x - mu, b = v.y - mu, c = v.z - mu, d = v.w - mu;
        acc += (a * a + b * b) + (c * c + d * d);
      } else {
        acc += (v.x + v.y) + (v.z + v.w);
      }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  // per group: the quads of the group over every pixel slot, fixed order
  for (int gg = threadIdx.x; gg < G; gg += kGnThreads) {
    float s = 0.f;
    const int q0 = gg * cpg / 4, q1 = (gg + 1) * cpg / 4;
    for (int t = 0; t < ppi; ++t)
      for (int q = q0; q < q1; ++q) s += red[t * C4 + q];
    partial[((size_t)n * chunks + chunk) * G + gg] = s;
  }
}

// mean[n * G + g] (or var) = sum over chunks / count
__global__ void gn_reduce_kernel(const float* __restrict__ partial, int chunks, int G, float inv_count,
                                 float* __restrict__ out) {
  const int n = blockIdx.x;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < chunks; ++c) s += partial[((size_t)n * chunks + c) * G + g];
    out[n * G + g] = s * inv_count;
  }
}

// y = x * inv + shift (+ ReLU); up2: each pixel to its 2x2 block of the
// output [N, 2H, 2W, C]; accumulate: y += instead of y =.
template <bool UP2, bool ACC>
__global__ __launch_bounds__(kGnThreads) void gn_apply_kernel(
    const float* __restrict__ x, int H, int W, int C, int G, const float* __restrict__ mean,
    const float* __restrict__ var, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int relu, float* __restrict__ y, int N) {
  const int C4 = C / 4, cpg = C / G;
  const size_t total = (size_t)N * H * W * C4;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int q = (int)(e % C4);
    const size_t px = e / C4;
    const int n = (int)(px / ((size_t)H * W));
    const int c = q * 4;
    const int g = c / cpg;
    const float mu = mean[n * G + g];
    const float r = rsqrtf(var[n * G + g] + eps);
    const float4 v = *reinterpret_cast<const float4*>(x + px * C + c);
    const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
    const float4 bt = *reinterpret_cast<const float4*>(beta + c);
    float4 o;
    {
      const float i0 = r * gm.x, i1 = r * gm.y, i2 = r * gm.z, i3 = r * gm.w;
      o.x = v.x * i0 + (bt.x - mu * i0);
      o.y = v.y * i1 + (bt.y - mu * i1);
      o.z = v.z * i2 + (bt.z - mu * i2);
      o.w = v.w * i3 + (bt.w - mu * i3);
    }
    if (relu) {
      o.x = fmaxf(o.x, 0.f);
      o.y = fmaxf(o.y, 0.f);
      o.z = fmaxf(o.z, 0.f);
      o.w = fmaxf(o.w, 0.f);
    }
    if (!UP2) {
      float4* d = reinterpret_cast<float4*>(y + px * C + c);
      if (ACC) {
        const float4 t = *d;
        o.x = t.x + o.x;
        o.y = t.y + o.y;
        o.z = t.z + o.z;
        o.w = t.w + o.w;
      }
      *d = o;
    } else {
      const int rem = (int)(px - (size_t)n * H * W);
      const int h = rem / W, w = rem - h * W;
      const int OW = 2 * W;
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          float4* d = reinterpret_cast<float4*>(
              y + (((size_t)n * 2 * H + 2 * h + dy) * OW + 2 * w + dx) * C + c);
          float4 oo = o;
          if (ACC) {
            const float4 t = *d;
            oo.x = t.x + o.x;
            oo.y = t.y + o.y;
            oo.z = t.z + o.z;
            oo.w = t.w + o.w;
          }
          *d = oo;
        }
    }
  }
}

static int gn_chunks(int HW, int& chunk_px) {
  // ~32 pixel-chunks per image (enough workgroups for N >= 2 at every SOLO
  // level), at least 16 pixels each
  int chunks = std::max(1, std::min(64, HW / 16));
  chunk_px = (HW + chunks - 1) / chunks;
  chunks = (HW + chunk_px - 1) / chunk_px;
  return chunks;
}

// ---------------------------------------------------------------- levels
// Multi-level GroupNorm (d2mi_group_norm_nhwc_levels): the same layer over
// up to six feature levels (the SOLOv2 tower GroupNorms after a multi-level
// conv launch) in five launches total instead of five per level.  Level l's
// sum workgroups are [wg0[l], wg0[l + 1]) (one per (image, chunk): the
// partial row of that index), its statistics rows [st0[l], st0[l + 1]) (one
// per image), its apply elements [e0[l], e0[l + 1]) (float4 quads).  Per
// level the arithmetic is gn_sum / gn_reduce / gn_apply's, in the same order.
constexpr int kGnMaxLevels = 6;
struct GnLevels {
  const float* x[kGnMaxLevels];
  float* y[kGnMaxLevels];
  int HW[kGnMaxLevels], chunks[kGnMaxLevels], chunk_px[kGnMaxLevels];
  float inv_count[kGnMaxLevels];
  int wg0[kGnMaxLevels + 1], st0[kGnMaxLevels + 1];
  long long e0[kGnMaxLevels + 1];
  int L;
};

__device__ __forceinline__ int gn_level_of(const int* first, int L, int i) {
  int l = 0;
  while (l + 1 < L && i >= first[l + 1]) ++l;
  return l;
}

__global__ __launch_bounds__(kGnThreads) void gn_sum_levels_kernel(GnLevels lv, int C, int G,
                                                                  const float* __restrict__ mean,
                                                                  float* __restrict__ partial) {
  __shared__ float red[kGnThreads];
  const int l = gn_level_of(lv.wg0, lv.L, blockIdx.x);
  const int local = blockIdx.x - lv.wg0[l];
  const int chunks = lv.chunks[l];
  const int n = local / chunks, chunk = local - n * chunks;
  const int HW = lv.HW[l];
  const int C4 = C / 4;
  const int tc = threadIdx.x % C4;
  const int tp = threadIdx.x / C4;
  const int ppi = kGnThreads / C4;
  const int cpg = C / G;
  const int g = tc * 4 / cpg;
  const int srow = lv.st0[l] + n;
  const float mu = mean ? mean[srow * G + g] : 0.f;
  const int p0 = chunk * lv.chunk_px[l], p1 = min(HW, p0 + lv.chunk_px[l]);
  const float* xb = lv.x[l] + (size_t)n * HW * C;
  float acc = 0.f;
  if (threadIdx.x < ppi * C4) {
    for (int p = p0 + tp; p < p1; p += ppi) {
      const float4 v = *reinterpret_cast<const float4*>(xb + (size_t)p * C + tc * 4);
      if (mean) {
        const float a = v.x - mu, b = v.y - mu, c = v.z - mu, d = v.w - mu;
        acc += (a * a + b * b) + (c * c + d * d);
      } else {
        acc += (v.x + v.y) + (v.z + v.w);
      }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int gg = threadIdx.x; gg < G; gg += kGnThreads) {
    float sum = 0.f;
    const int q0 = gg * cpg / 4, q1 = (gg + 1) * cpg / 4;
    for (int t = 0; t < ppi; ++t)
      for (int q = q0; q < q1; ++q) sum += red[t * C4 + q];
    partial[(size_t)blockIdx.x * G + gg] = sum;
  }
}

// one workgroup per (level, image): out[row * G + g] = sum over its chunks / count
__global__ void gn_reduce_levels_kernel(GnLevels lv, const float* __restrict__ partial, int G,
                                        float* __restrict__ out) {
  const int row = blockIdx.x;
  const int l = gn_level_of(lv.st0, lv.L, row);
  const int n = row - lv.st0[l];
  const int chunks = lv.chunks[l];
  const size_t base = (size_t)lv.wg0[l] + (size_t)n * chunks;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    float sum = 0.f;
    for (int c = 0; c < chunks; ++c) sum += partial[(base + c) * G + g];
    out[row * G + g] = sum * lv.inv_count[l];
  }
}

__global__ __launch_bounds__(kGnThreads) void gn_apply_levels_kernel(
    GnLevels lv, int C, int G, const float* __restrict__ mean, const float* __restrict__ var,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int relu) {
  const int C4 = C / 4, cpg = C / G;
  const long long total = lv.e0[lv.L];
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < lv.L && e >= lv.e0[l + 1]) ++l;
    const long long le = e - lv.e0[l];
    const int q = (int)(le % C4);
    const long long px = le / C4;
    const int n = (int)(px / lv.HW[l]);
    const int c = q * 4;
    const int g = c / cpg;
    const int srow = lv.st0[l] + n;
    const float mu = mean[srow * G + g];
    const float r = rsqrtf(var[srow * G + g] + eps);
    const float4 v = *reinterpret_cast<const float4*>(lv.x[l] + px * C + c);
    const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
    const float4 bt = *reinterpret_cast<const float4*>(beta + c);
    float4 o;
    const float i0 = r * gm.x, i1 = r * gm.y, i2 = r * gm.z, i3 = r * gm.w;
    o.x = v.x * i0 + (bt.x - mu * i0);
    o.y = v.y * i1 + (bt.y - mu * i1);
    o.z = v.z * i2 + (bt.z - mu * i2);
    o.w = v.w * i3 + (bt.w - mu * i3);
    if (relu) {
      o.x = fmaxf(o.x, 0.f);
      o.y = fmaxf(o.y, 0.f);
      o.z = fmaxf(o.z, 0.f);
      o.w = fmaxf(o.w, 0.f);
    }
    *reinterpret_cast<float4*>(lv.y[l] + px * C + c) = o;
  }
}

// level table + workspace layout of a multi-level call
static int gn_levels_plan(const int32_t* dims, int nlev, int C, int G, GnLevels& lv,
                          size_t& n_partial, size_t& n_stats) {
  lv = GnLevels{};
  lv.L = nlev;
  int wg = 0, st = 0;
  long long e = 0;
  for (int l = 0; l < nlev; ++l) {
    const int N = dims[3 * l], H = dims[3 * l + 1], W = dims[3 * l + 2];
    if (N < 0 || H <= 0 || W <= 0) return -1;
    lv.HW[l] = H * W;
    lv.chunks[l] = gn_chunks(H * W, lv.chunk_px[l]);
    lv.inv_count[l] = 1.f / (float)((size_t)H * W * (C / G));
    lv.wg0[l] = wg;
    lv.st0[l] = st;
    lv.e0[l] = e;
    wg += N * lv.chunks[l];
    st += N;
    e += (long long)N * H * W * (C / 4);
  }
  lv.wg0[nlev] = wg;
  lv.st0[nlev] = st;
  lv.e0[nlev] = e;
  n_partial = (size_t)wg * G;
  n_stats = (size_t)st * G;
  return 0;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_group_norm_workspace_size(int N, int H, int W, int C, int G) {
  int cp;
  const int chunks = gn_chunks(H * W, cp);
  WorkspaceSizer z;
  z.take<float>((size_t)N * chunks * G);
  z.take<float>((size_t)N * G);
  z.take<float>((size_t)N * G);
  return z.off;
}

extern "C" int d2mi_group_norm_nhwc(const float* x, int N, int H, int W, int C, int G,
                                    const float* gamma, const float* beta, float eps, int relu,
                                    int up2, int accumulate, float* y, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N >= 0 && H > 0 && W > 0 && C > 0 && G > 0 && G <= kGnMaxGroups,
               "bad GroupNorm sizes (groups <= %d)", kGnMaxGroups);
  D2MI_REQUIRE(C % G == 0 && (C / G) % 4 == 0, "GroupNorm: C / G must be a multiple of 4");
  D2MI_REQUIRE(C / 4 <= kGnThreads, "GroupNorm: C <= %d", 4 * kGnThreads);
  D2MI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                   ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0,
               "GroupNorm operands must be 16-B aligned");
  if (N == 0) return 0;
  hipStream_t st = as_stream(stream);
  int chunk_px;
  const int HW = H * W;
  const int chunks = gn_chunks(HW, chunk_px);
  Workspace w(workspace, workspace_bytes);
  float* partial = w.take<float>((size_t)N * chunks * G);
  float* mean = w.take<float>((size_t)N * G);
  float* var = w.take<float>((size_t)N * G);
  D2MI_REQUIRE(w.ok(), "GroupNorm workspace too small (%zu < %zu)", workspace_bytes, w.off);
  const float inv_count = 1.f / (float)((size_t)HW * (C / G));
  hipLaunchKernelGGL(gn_sum_kernel, dim3(chunks, N), dim3(kGnThreads), 0, st, x, HW, C, G,
                     chunk_px, nullptr, partial);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_reduce_kernel, dim3(N), dim3(64), 0, st, partial, chunks, G, inv_count,
                     mean);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_sum_kernel, dim3(chunks, N), dim3(kGnThreads), 0, st, x, HW, C, G,
                     chunk_px, mean, partial);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_reduce_kernel, dim3(N), dim3(64), 0, st, partial, chunks, G, inv_count,
                     var);
  D2MI_LAUNCH_CHECK();
  const size_t total = (size_t)N * HW * (C / 4);
  const int grid = (int)std::min<size_t>((total + kGnThreads - 1) / kGnThreads, 16384);
#define GN_APPLY(U, A)                                                                          \
  hipLaunchKernelGGL((gn_apply_kernel<U, A>), dim3(grid), dim3(kGnThreads), 0, st, x, H, W, C, \
                     G, mean, var, gamma, beta, eps, relu, y, N)
  if (up2 && accumulate) GN_APPLY(true, true);
  else if (up2) GN_APPLY(true, false);
  else if (accumulate) GN_APPLY(false, true);
  else GN_APPLY(false, false);
#undef GN_APPLY
  D2MI_LAUNCH_CHECK();
  return 0;
}

// Reference: the per-level GroupNorm calls of the SOLOv2 towers
// (solo_v2.py:173-183) — d2mi_group_norm_nhwc per level, as ONE set of launches.
extern "C" size_t d2mi_group_norm_levels_workspace_size(const int32_t* dims, int nlev, int C,
                                                        int G) {
  if (nlev < 1 || nlev > kGnMaxLevels || G <= 0) return 0;
  GnLevels lv;
  size_t np = 0, ns = 0;
  if (gn_levels_plan(dims, nlev, C, G, lv, np, ns)) return 0;
  WorkspaceSizer z;
  z.take<float>(np);
  z.take<float>(ns);
  z.take<float>(ns);
  return z.off;
}

extern "C" int d2mi_group_norm_nhwc_levels(const float* const* xs, const int32_t* dims, int nlev,
                                           int C, int G, const float* gamma, const float* beta,
                                           float eps, int relu, float* const* ys, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(nlev >= 1 && nlev <= kGnMaxLevels, "GroupNorm levels: 1..%d levels", kGnMaxLevels);
  D2MI_REQUIRE(C > 0 && G > 0 && G <= kGnMaxGroups, "bad GroupNorm sizes (groups <= %d)",
               kGnMaxGroups);
  D2MI_REQUIRE(C % G == 0 && (C / G) % 4 == 0, "GroupNorm: C / G must be a multiple of 4");
  D2MI_REQUIRE(C / 4 <= kGnThreads, "GroupNorm: C <= %d", 4 * kGnThreads);
  D2MI_REQUIRE(((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0,
               "GroupNorm operands must be 16-B aligned");
  GnLevels lv;
  size_t np = 0, ns = 0;
  D2MI_REQUIRE(gn_levels_plan(dims, nlev, C, G, lv, np, ns) == 0, "bad GroupNorm level dims");
  for (int l = 0; l < nlev; ++l) {
    D2MI_REQUIRE(((uintptr_t)xs[l] & 15) == 0 && ((uintptr_t)ys[l] & 15) == 0,
                 "GroupNorm level %d operands must be 16-B aligned", l);
    lv.x[l] = xs[l];
    lv.y[l] = ys[l];
  }
  if (lv.wg0[nlev] == 0) return 0;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  float* partial = w.take<float>(np);
  float* mean = w.take<float>(ns);
  float* var = w.take<float>(ns);
  D2MI_REQUIRE(w.ok(), "GroupNorm workspace too small (%zu < %zu)", workspace_bytes, w.off);
  hipLaunchKernelGGL(gn_sum_levels_kernel, dim3(lv.wg0[nlev]), dim3(kGnThreads), 0, st, lv, C, G,
                     nullptr, partial);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_reduce_levels_kernel, dim3(lv.st0[nlev]), dim3(64), 0, st, lv, partial, G,
                     mean);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_sum_levels_kernel, dim3(lv.wg0[nlev]), dim3(kGnThreads), 0, st, lv, C, G,
                     mean, partial);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_reduce_levels_kernel, dim3(lv.st0[nlev]), dim3(64), 0, st, lv, partial, G,
                     var);
  D2MI_LAUNCH_CHECK();
  const long long total = lv.e0[nlev];
  const int grid = (int)std::min<long long>((total + kGnThreads - 1) / kGnThreads, 16384);
  hipLaunchKernelGGL(gn_apply_levels_kernel, dim3(grid), dim3(kGnThreads), 0, st, lv, C, G, mean,
                     var, gamma, beta, eps, relu);
  D2MI_LAUNCH_CHECK();
  return 0;
}
