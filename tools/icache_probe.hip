// Instruction-fetch cost of straight-line code in a one-shot workgroup
// (tools/icache_probe.py): a kernel whose body is N copies of a short
// dependent VALU sequence, fully unrolled (code size ~ N * 16 B), run by ONE
// workgroup, timed by its own wall-clock stamps (100 MHz) -- cold (after a
// kernel that streams 1 GiB through the caches) and warm (launched again
// right after).  Against the same work as a rolled loop (a few cache lines).
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int N>
__global__ __launch_bounds__(256) void straight_kernel(float* out, uint64_t* t, float a) {
  const uint64_t t0 = wall_clock64();
  float x = a + threadIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    x = __builtin_fmaf(x, 1.0001f, (float)i * 0.5f);
    x = __builtin_fmaf(x, 0.9999f, -(float)i * 0.25f);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    t[0] = t0;
    t[1] = wall_clock64();
  }
}

__global__ __launch_bounds__(256) void rolled_kernel(float* out, uint64_t* t, float a, int n) {
  const uint64_t t0 = wall_clock64();
  float x = a + threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < n; ++i) {
    x = __builtin_fmaf(x, 1.0001f, (float)i * 0.5f);
    x = __builtin_fmaf(x, 0.9999f, -(float)i * 0.25f);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    t[0] = t0;
    t[1] = wall_clock64();
  }
}

__global__ void stream_kernel(const float4* __restrict__ in, float* out, size_t n4) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

extern "C" int probe_straight(int which, float* out, uint64_t* t, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (which) {
    case 0: hipLaunchKernelGGL(straight_kernel<256>, dim3(1), dim3(256), 0, st, out, t, 1.f); break;
    case 1: hipLaunchKernelGGL(straight_kernel<1024>, dim3(1), dim3(256), 0, st, out, t, 1.f); break;
    case 2: hipLaunchKernelGGL(straight_kernel<4096>, dim3(1), dim3(256), 0, st, out, t, 1.f); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int probe_rolled(int n, float* out, uint64_t* t, void* stream) {
  hipLaunchKernelGGL(rolled_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, out, t, 1.f, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int probe_stream(const float* in, float* out, size_t n, void* stream) {
  hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(in), out, n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
