// Weight + bias gradient of a 1x1 conv with few output channels (the RPN
// head's fused objectness + anchor-delta 1x1, rpn.py:31-96: Cout = A + 4A =
// 15 -> 16 with a zero pad column) over every pixel of a pyramid level:
//   gw[ci][co] = sum_p x[p][ci] * g[p][co],   gb[co] = sum_p g[p][co]
// i.e. X^T G with a short output (Cin x Cout <= 256 x 16) and a reduction
// over up to ~135k pixels.  A GEMM tiling leaves 5/6 of every MFMA tile
// empty here (hipBLASLt took 0.5 ms for Cout = 3 on p2); this is an HBM-bound
// streaming pass instead: each 256-thread workgroup takes a chunk of kChunk
// pixels, one input channel per thread (one coalesced 1 KiB row read per
// pixel for Cin = 256), the chunk's G rows staged in LDS and broadcast, 16
// f32 accumulators per thread; per-chunk partials then reduced in chunk
// order by a second kernel (deterministic, no atomics).
#include <algorithm>

#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kChunk = 128;    // pixels per workgroup
constexpr int kMaxCout = 16;

__global__ __launch_bounds__(256) void wgrad_skinny_partial_kernel(
    const float* __restrict__ x, const float* __restrict__ g, int P, int Cin, int Cout,
    float* __restrict__ partial /* [chunks][Cin + 1][Cout] */) {
  __shared__ float gs[kChunk * kMaxCout];
  const int chunk = blockIdx.x;
  const int p0 = chunk * kChunk;
  const int np = min(kChunk, P - p0);
  // LDS rows padded to kMaxCout (zeros): compile-time strides, so the
  // broadcast reads below are 16-B LDS loads
  for (int i = threadIdx.x; i < kChunk * kMaxCout; i += blockDim.x) {
    const int p = i / kMaxCout, j = i - p * kMaxCout;
    gs[i] = (p < np && j < Cout) ? g[(size_t)(p0 + p) * Cout + j] : 0.f;
  }
  __syncthreads();
  float* out = partial + (size_t)chunk * (Cin + 1) * Cout;
  for (int c = threadIdx.x; c < Cin; c += blockDim.x) {
    float acc[kMaxCout];
#pragma unroll
    for (int j = 0; j < kMaxCout; ++j) acc[j] = 0.f;
    const float* xp = x + (size_t)p0 * Cin + c;
    int p = 0;
    for (; p + 4 <= np; p += 4) {  // 4 row loads in flight
      float xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) xv[u] = xp[(size_t)(p + u) * Cin];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < kMaxCout; ++j) acc[j] = fmaf(xv[u], gs[(p + u) * kMaxCout + j], acc[j]);
    }
    for (; p < np; ++p) {
      const float xv = xp[(size_t)p * Cin];
#pragma unroll
      for (int j = 0; j < kMaxCout; ++j) acc[j] = fmaf(xv, gs[p * kMaxCout + j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < kMaxCout; ++j)
      if (j < Cout) out[(size_t)c * Cout + j] = acc[j];
  }
  if (threadIdx.x < Cout) {  // bias row: column sums of the chunk's G
    float s = 0.f;
    for (int p = 0; p < np; ++p) s += gs[p * kMaxCout + threadIdx.x];
    out[(size_t)Cin * Cout + threadIdx.x] = s;
  }
}

// float4 form (Cin % 4 == 0, 16-B aligned x): a lane owns 4 input channels,
// the four waves take every 4th pixel of the chunk (each row read is one
// 1 KiB float4 wave load for Cin = 256, four rows in flight per wave: 4x the
// bytes per load of the scalar form, which left this pass latency-bound),
// and the waves' sums are combined in wave order through LDS before the
// chunk partial is written.  kChunk4 pixels per workgroup.
constexpr int kChunk4 = 128;

__device__ __forceinline__ void skinny_partial4(const float* __restrict__ x,
                                                const float* __restrict__ g, int P, int Cin,
                                                int Cout, int chunk,
                                                float* __restrict__ partial, float4* lds) {
  float* gs = reinterpret_cast<float*>(lds);
  const int p0 = chunk * kChunk4;
  const int np = min(kChunk4, P - p0);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* out = partial + (size_t)chunk * (Cin + 1) * Cout;
  for (int cb = 0; cb < Cin; cb += 256) {  // 256 input channels per pass
    __syncthreads();
    for (int i = threadIdx.x; i < kChunk4 * kMaxCout; i += blockDim.x) {
      const int p = i / kMaxCout, j = i - p * kMaxCout;
      gs[i] = (p < np && j < Cout) ? g[(size_t)(p0 + p) * Cout + j] : 0.f;
    }
    __syncthreads();
    const int c = cb + 4 * lane;
    const bool live = c < Cin;
    float4 acc[kMaxCout];
#pragma unroll
    for (int j = 0; j < kMaxCout; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
      const float* xp = x + (size_t)p0 * Cin + c;
      int p = wv;
      for (; p + 12 < np; p += 16) {  // 4 rows in flight per wave
        float4 xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) xv[u] = *reinterpret_cast<const float4*>(xp + (size_t)(p + 4 * u) * Cin);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* gr = gs + (p + 4 * u) * kMaxCout;
#pragma unroll
          for (int j = 0; j < kMaxCout; ++j) {
            const float gv = gr[j];
            acc[j].x = fmaf(xv[u].x, gv, acc[j].x);
            acc[j].y = fmaf(xv[u].y, gv, acc[j].y);
            acc[j].z = fmaf(xv[u].z, gv, acc[j].z);
            acc[j].w = fmaf(xv[u].w, gv, acc[j].w);
          }
        }
      }
      for (; p < np; p += 4) {
        const float4 xv = *reinterpret_cast<const float4*>(xp + (size_t)p * Cin);
        const float* gr = gs + p * kMaxCout;
#pragma unroll
        for (int j = 0; j < kMaxCout; ++j) {
          const float gv = gr[j];
          acc[j].x = fmaf(xv.x, gv, acc[j].x);
          acc[j].y = fmaf(xv.y, gv, acc[j].y);
          acc[j].z = fmaf(xv.z, gv, acc[j].z);
          acc[j].w = fmaf(xv.w, gv, acc[j].w);
        }
      }
    }
    // bias row of this chunk (once): column sums of G in pixel order
    float bsum = 0.f;
    if (cb == 0 && threadIdx.x < Cout)
      for (int q = 0; q < np; ++q) bsum += gs[q * kMaxCout + threadIdx.x];
    __syncthreads();  // gs no longer read: the region takes the wave sums
    if (wv > 0) {
#pragma unroll
      for (int j = 0; j < kMaxCout; ++j) lds[((wv - 1) * 64 + lane) * kMaxCout + j] = acc[j];
    }
    __syncthreads();
    if (wv == 0 && live) {
      // ((w0 + w1) + w2) + w3 per output, one output column at a time
#pragma unroll
      for (int j = 0; j < kMaxCout; ++j) {
        float4 t = acc[j];
        for (int w = 0; w < 3; ++w) {
          const float4 v = lds[(w * 64 + lane) * kMaxCout + j];
          t.x += v.x;
          t.y += v.y;
          t.z += v.z;
          t.w += v.w;
        }
        if (j < Cout) {
          out[(size_t)c * Cout + j] = t.x;
          out[(size_t)(c + 1) * Cout + j] = t.y;
          out[(size_t)(c + 2) * Cout + j] = t.z;
          out[(size_t)(c + 3) * Cout + j] = t.w;
        }
      }
    }
    if (cb == 0 && threadIdx.x < Cout) out[(size_t)Cin * Cout + threadIdx.x] = bsum;
  }
}

__global__ __launch_bounds__(256, 2) void wgrad_skinny_partial4_kernel(
    const float* __restrict__ x, const float* __restrict__ g, int P, int Cin, int Cout,
    float* __restrict__ partial /* [chunks][Cin + 1][Cout] */) {
  // the chunk's G rows (16 KiB); reused for the wave combine (3 x 64 lanes x
  // 64 floats = 48 KiB)
  __shared__ float4 lds[3 * 64 * 16];
  skinny_partial4(x, g, P, Cin, Cout, blockIdx.x, partial, lds);
}

// Several calls' (levels') passes in one launch: the levels' chunks one
// after another, level l's partials at chunk offset cb[l] (each level's
// chunk partials exactly the single-level kernel's).
constexpr int kSkinnyMaxLevels = 8;
struct SkinnyLevels {
  const float* x[kSkinnyMaxLevels];
  const float* g[kSkinnyMaxLevels];
  int P[kSkinnyMaxLevels];
  int cb[kSkinnyMaxLevels + 1];
  int L;
};

__global__ __launch_bounds__(256, 2) void wgrad_skinny_partial4_levels_kernel(
    SkinnyLevels lv, int Cin, int Cout, float* __restrict__ partial) {
  __shared__ float4 lds[3 * 64 * 16];
  int l = 0;
  while (l + 1 < lv.L && (int)blockIdx.x >= lv.cb[l + 1]) ++l;
  skinny_partial4(lv.x[l], lv.g[l], lv.P[l], Cin, Cout, blockIdx.x - lv.cb[l],
                  partial + (size_t)lv.cb[l] * (Cin + 1) * Cout, lds);
}

// Sum the chunk partials (gw rows, then the gb row) in a fixed order: 16
// outputs per workgroup, 16 chunk segments per output summed in chunk order
// by 16 threads, then the 16 segment sums in segment order (one thread per
// chunk range left the p2 reduction latency-bound at ~0.3 ms).
constexpr int kRedOut = 16, kRedSeg = 16;

__global__ __launch_bounds__(256) void wgrad_skinny_reduce_kernel(
    const float* __restrict__ partial, int chunks, int Cin, int Cout, float* __restrict__ gw,
    float* __restrict__ gb, int accumulate) {
  __shared__ float red[kRedSeg][kRedOut];
  const int n = (Cin + 1) * Cout;
  const int ol = threadIdx.x % kRedOut, sg = threadIdx.x / kRedOut;
  const int o = blockIdx.x * kRedOut + ol;
  const int per = (chunks + kRedSeg - 1) / kRedSeg;
  const int k0 = sg * per, k1 = min(chunks, k0 + per);
  float s = 0.f;
  if (o < n)
#pragma unroll 8  // (loads in flight; the sum stays in chunk order)
    for (int k = k0; k < k1; ++k) s += partial[(size_t)k * n + o];
  red[sg][ol] = s;
  __syncthreads();
  if (sg == 0 && o < n) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < kRedSeg; ++j) t += red[j][ol];
    // accumulate: old + new, the rounding of autograd's sum of two gradients
    if (o < Cin * Cout) gw[o] = accumulate ? gw[o] + t : t;
    else if (gb) gb[o - Cin * Cout] = accumulate ? gb[o - Cin * Cout] + t : t;
  }
}

// The levels' reduces in one launch: per output, each level's chunk partials
// summed exactly as wgrad_skinny_reduce_kernel sums one call's (16 ordered
// segments, then the segments in order), and the levels added in launch
// order -- the rounding of one call per level with accumulate (old + new).
__global__ __launch_bounds__(256) void wgrad_skinny_reduce_levels_kernel(
    const float* __restrict__ partial, SkinnyLevels lv, int Cin, int Cout,
    float* __restrict__ gw, float* __restrict__ gb, int accumulate) {
  __shared__ float red[kRedSeg][kRedOut];
  const int n = (Cin + 1) * Cout;
  const int ol = threadIdx.x % kRedOut, sg = threadIdx.x / kRedOut;
  const int o = blockIdx.x * kRedOut + ol;
  // accumulate: start from the old value (old + t0, then + t1 ...)
  float acc = 0.f;
  if (accumulate && sg == 0 && o < n) acc = o < Cin * Cout ? gw[o] : (gb ? gb[o - Cin * Cout] : 0.f);
  for (int l = 0; l < lv.L; ++l) {
    const int chunks = lv.cb[l + 1] - lv.cb[l];
    const float* part = partial + (size_t)lv.cb[l] * n;
    const int per = (chunks + kRedSeg - 1) / kRedSeg;
    const int k0 = sg * per, k1 = min(chunks, k0 + per);
    float s = 0.f;
    if (o < n)
#pragma unroll 8  // (loads in flight; the sum stays in chunk order)
      for (int k = k0; k < k1; ++k) s += part[(size_t)k * n + o];
    __syncthreads();  // (the previous level's red reads are done)
    red[sg][ol] = s;
    __syncthreads();
    if (sg == 0) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < kRedSeg; ++j) t += red[j][ol];
      acc = (l == 0 && !accumulate) ? t : acc + t;
    }
  }
  if (sg == 0 && o < n) {
    if (o < Cin * Cout) gw[o] = acc;
    else if (gb) gb[o - Cin * Cout] = acc;
  }
}

// Column sums of a row-major [rows, cols] matrix (the bias gradient of a conv
// whose weight gradient ran as a library GEMM): workgroup (col chunk of 256,
// row chunk of kColRows) sums its rows in order -> partial[row chunk][col];
// then the row chunks are summed in order (wgrad_skinny_reduce_kernel's
// two-level scheme with Cin = 0).
constexpr int kColRows = 32;

__global__ __launch_bounds__(256) void column_sum_partial_kernel(const float* __restrict__ x,
                                                                 long long rows, int cols,
                                                                 float* __restrict__ partial) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const long long r0 = (long long)blockIdx.y * kColRows;
  const long long r1 = r0 + kColRows < rows ? r0 + kColRows : rows;
  if (c >= cols) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 independent chains, fixed order
  long long r = r0;
  for (; r + 4 <= r1; r += 4) {
    s0 += x[(size_t)r * cols + c];
    s1 += x[(size_t)(r + 1) * cols + c];
    s2 += x[(size_t)(r + 2) * cols + c];
    s3 += x[(size_t)(r + 3) * cols + c];
  }
  for (; r < r1; ++r) s0 += x[(size_t)r * cols + c];
  partial[(size_t)blockIdx.y * cols + c] = (s0 + s1) + (s2 + s3);
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_column_sum_workspace_size(long long rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (size_t)((rows + kColRows - 1) / kColRows) * cols * sizeof(float);
}

extern "C" int d2mi_column_sum(const float* x, long long rows, int cols, float* out,
                               void* workspace, size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(rows > 0 && cols > 0, "column_sum: rows=%lld cols=%d", rows, cols);
  const size_t need = d2mi_column_sum_workspace_size(rows, cols);
  D2MI_REQUIRE(workspace && workspace_bytes >= need, "column_sum workspace too small");
  const long long chunks = (rows + kColRows - 1) / kColRows;
  D2MI_REQUIRE(chunks < 65536, "column_sum: too many rows");
  hipStream_t st = as_stream(stream);
  float* partial = static_cast<float*>(workspace);
  hipLaunchKernelGGL(column_sum_partial_kernel, dim3((cols + 255) / 256, (unsigned)chunks),
                     dim3(256), 0, st, x, rows, cols, partial);
  D2MI_LAUNCH_CHECK();
  // reduce: rows of the partial = chunks, "Cin" = 0, Cout = cols -> gb = out
  hipLaunchKernelGGL(wgrad_skinny_reduce_kernel, dim3((cols + kRedOut - 1) / kRedOut), dim3(256),
                     0, st, partial, (int)chunks, 0, cols, nullptr, out, 0);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_wgrad_skinny_workspace_size(int P, int Cin, int Cout) {
  if (P <= 0 || Cin <= 0 || Cout <= 0) return 0;
  const size_t chunks = ((size_t)P + kChunk - 1) / kChunk;  // >= the float4 form's
  return chunks * (size_t)(Cin + 1) * Cout * sizeof(float);
}

extern "C" int d2mi_wgrad_skinny(const float* x, const float* g, int P, int Cin, int Cout,
                                 float* gw, float* gb, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  return d2mi_wgrad_skinny_ex(x, g, P, Cin, Cout, gw, gb, 0, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_wgrad_skinny_ex(const float* x, const float* g, int P, int Cin, int Cout,
                                    float* gw, float* gb, int accumulate, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(P > 0 && Cin > 0 && Cout > 0 && Cout <= kMaxCout,
               "wgrad_skinny: P=%d Cin=%d Cout=%d (Cout must be 1..%d)", P, Cin, Cout, kMaxCout);
  const size_t need = d2mi_wgrad_skinny_workspace_size(P, Cin, Cout);
  D2MI_REQUIRE(workspace && workspace_bytes >= need, "wgrad_skinny workspace too small: %zu < %zu",
               workspace_bytes, need);
  const bool v4 = Cin % 4 == 0 && ((uintptr_t)x & 15) == 0;
  const int chunks = v4 ? (P + kChunk4 - 1) / kChunk4 : (P + kChunk - 1) / kChunk;
  hipStream_t st = as_stream(stream);
  float* partial = static_cast<float*>(workspace);
  if (v4)
    hipLaunchKernelGGL(wgrad_skinny_partial4_kernel, dim3(chunks), dim3(256), 0, st, x, g, P, Cin,
                       Cout, partial);
  else
    hipLaunchKernelGGL(wgrad_skinny_partial_kernel, dim3(chunks), dim3(256), 0, st, x, g, P, Cin,
                       Cout, partial);
  D2MI_LAUNCH_CHECK();
  const int n = (Cin + 1) * Cout;
  hipLaunchKernelGGL(wgrad_skinny_reduce_kernel, dim3((n + kRedOut - 1) / kRedOut), dim3(256), 0,
                     st, partial, chunks, Cin, Cout, gw, gb, accumulate);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_wgrad_skinny_levels_workspace_size(const int* P, int L, int Cin, int Cout) {
  if (!P || L <= 0 || L > kSkinnyMaxLevels || Cin <= 0 || Cout <= 0) return 0;
  size_t chunks = 0;
  for (int l = 0; l < L; ++l) chunks += ((size_t)std::max(P[l], 0) + kChunk4 - 1) / kChunk4;
  return chunks * (size_t)(Cin + 1) * Cout * sizeof(float);
}

extern "C" int d2mi_wgrad_skinny_levels(const float* const* x, const float* const* g, const int* P,
                                        int L, int Cin, int Cout, float* gw, float* gb,
                                        int accumulate, void* workspace, size_t workspace_bytes,
                                        void* stream) {
  D2MI_REQUIRE(x && g && P && L > 0 && L <= kSkinnyMaxLevels,
               "wgrad_skinny_levels: 1..%d levels", kSkinnyMaxLevels);
  D2MI_REQUIRE(Cin > 0 && Cin % 4 == 0 && Cout > 0 && Cout <= kMaxCout,
               "wgrad_skinny_levels: Cin=%d (a multiple of 4) Cout=%d (1..%d)", Cin, Cout,
               kMaxCout);
  SkinnyLevels lv = {};
  lv.L = L;
  lv.cb[0] = 0;
  for (int l = 0; l < L; ++l) {
    D2MI_REQUIRE(P[l] > 0 && x[l] && g[l] && ((uintptr_t)x[l] & 15) == 0,
                 "wgrad_skinny_levels: level %d (P=%d) needs 16-B aligned x", l, P[l]);
    lv.x[l] = x[l];
    lv.g[l] = g[l];
    lv.P[l] = P[l];
    lv.cb[l + 1] = lv.cb[l] + (P[l] + kChunk4 - 1) / kChunk4;
  }
  const size_t need = d2mi_wgrad_skinny_levels_workspace_size(P, L, Cin, Cout);
  D2MI_REQUIRE(workspace && workspace_bytes >= need,
               "wgrad_skinny_levels workspace too small: %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  float* partial = static_cast<float*>(workspace);
  hipLaunchKernelGGL(wgrad_skinny_partial4_levels_kernel, dim3(lv.cb[L]), dim3(256), 0, st, lv,
                     Cin, Cout, partial);
  D2MI_LAUNCH_CHECK();
  const int n = (Cin + 1) * Cout;
  hipLaunchKernelGGL(wgrad_skinny_reduce_levels_kernel, dim3((n + kRedOut - 1) / kRedOut),
                     dim3(256), 0, st, partial, lv, Cin, Cout, gw, gb, accumulate);
  D2MI_LAUNCH_CHECK();
  return 0;
}
