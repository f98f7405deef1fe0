// Fused Momentum-SGD step over every trainable tensor: the L2 regulariser
// gradient, per-tensor clip_by_norm and tf.train.MomentumOptimizer in two
// launches (instead of one elementwise kernel per tensor per operation).
//
// Restates lib/engine/trainer.py:116-139 (+ lib/solver/regularizer.py:6-24):
//   g' = g + wd * w                       slim.l2_regularizer(wd) gradient
//   g'' = g' * clip / max(|g'|_2, clip)   clip_by_norm of EACH gradient tensor
//                                         (slim.learning.clip_gradient_norms)
//   accum = accum * momentum + g''        ApplyMomentum
//   w -= lr * accum
// Tensors are split into chunks of at most kChunk elements (a host-built
// table).  Pass 1 writes each chunk's sum of g'^2; pass 2 sums a tensor's
// chunk partials in chunk order (every chunk of the tensor recomputes the same
// fixed-order sum: deterministic, no atomics) and updates its chunk.
#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kChunk = 65536;

struct SgdTensor {
  float* w;
  const float* g;      // null: zero gradient
  float* accum;
  long long numel;
  float wd;
  int first_chunk, num_chunks;
  int pad;
};

struct SgdChunk {
  int tensor;
  int pad;
  long long begin, end;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;  // valid in thread 0
}

__global__ __launch_bounds__(256) void sgd_sumsq_kernel(const SgdTensor* __restrict__ tensors,
                                                        const SgdChunk* __restrict__ chunks,
                                                        float* __restrict__ partial) {
  __shared__ float red[4];
  const SgdChunk c = chunks[blockIdx.x];
  const SgdTensor t = tensors[c.tensor];
  float s = 0.f;
  if (t.g && t.wd == 0.f) {
    for (long long i = c.begin + threadIdx.x; i < c.end; i += blockDim.x) s += t.g[i] * t.g[i];
  } else if (t.g) {
    for (long long i = c.begin + threadIdx.x; i < c.end; i += blockDim.x) {
      const float g = t.g[i] + t.wd * t.w[i];
      s += g * g;
    }
  } else if (t.wd != 0.f) {
    for (long long i = c.begin + threadIdx.x; i < c.end; i += blockDim.x) {
      const float g = t.wd * t.w[i];
      s += g * g;
    }
  }
  const float tot = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void sgd_update_kernel(const SgdTensor* __restrict__ tensors,
                                                         const SgdChunk* __restrict__ chunks,
                                                         const float* __restrict__ partial,
                                                         float clip, float momentum, float lr) {
  __shared__ float scale_s;
  const SgdChunk c = chunks[blockIdx.x];
  const SgdTensor t = tensors[c.tensor];
  if (threadIdx.x == 0) {
    float ss = 0.f;
    if (clip > 0.f)
      for (int k = 0; k < t.num_chunks; ++k) ss += partial[t.first_chunk + k];
    // tf.clip_by_norm: l2norm = sqrt(sum) (0 when sum == 0); t * clip / max(l2norm, clip)
    const float nrm = ss > 0.f ? sqrtf(ss) : 0.f;
    scale_s = clip > 0.f ? fmaxf(nrm, clip) : 0.f;  // divisor; 0 = no clipping
  }
  __syncthreads();
  const float div = scale_s;
  for (long long i = c.begin + threadIdx.x; i < c.end; i += blockDim.x) {
    const float w = t.w[i];
    float g = (t.g ? t.g[i] : 0.f) + t.wd * w;
    if (div > 0.f) g = g * clip / div;
    const float a = t.accum[i] * momentum + g;
    t.accum[i] = a;
    t.w[i] = w - lr * a;
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

// Host helper: the table layout the caller uploads (see include/d2mi.h).
extern "C" int d2mi_sgd_table_sizes(int* tensor_bytes, int* chunk_bytes, int* chunk_elems) {
  *tensor_bytes = (int)sizeof(SgdTensor);
  *chunk_bytes = (int)sizeof(SgdChunk);
  *chunk_elems = kChunk;
  return 0;
}

extern "C" int d2mi_momentum_sgd(const void* tensor_table, const void* chunk_table, int num_chunks,
                                 float* partial, float clip_norm, float momentum, float lr,
                                 void* stream) {
  D2MI_REQUIRE(num_chunks >= 0, "num_chunks < 0");
  if (num_chunks == 0) return 0;
  hipStream_t st = as_stream(stream);
  const SgdTensor* t = static_cast<const SgdTensor*>(tensor_table);
  const SgdChunk* c = static_cast<const SgdChunk*>(chunk_table);
  if (clip_norm > 0.f) {
    hipLaunchKernelGGL(sgd_sumsq_kernel, dim3(num_chunks), dim3(256), 0, st, t, c, partial);
    D2MI_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(sgd_update_kernel, dim3(num_chunks), dim3(256), 0, st, t, c, partial,
                     clip_norm, momentum, lr);
  D2MI_LAUNCH_CHECK();
  return 0;
}
