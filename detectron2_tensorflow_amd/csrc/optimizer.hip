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

// float4 body when every pointer of the tensor is 16-B aligned (chunk
// boundaries are multiples of kChunk), scalar tail; 4 vectors in flight per
// thread.  Per-thread sums are in a fixed order, so results stay deterministic.
__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

__device__ __forceinline__ float sq_term(const SgdTensor& t, long long i) {
  const float g = (t.g ? t.g[i] : 0.f) + t.wd * t.w[i];
  return g * g;
}

__global__ __launch_bounds__(256) void sgd_sumsq_kernel(const SgdTensor* __restrict__ tensors,
                                                        const SgdChunk* __restrict__ chunks,
                                                        float* __restrict__ partial) {
  __shared__ float red[4];
  const SgdChunk c = chunks[blockIdx.x];
  const SgdTensor t = tensors[c.tensor];
  float s = 0.f;
  if (t.g || t.wd != 0.f) {
    long long i0 = c.begin;
    if (al16(t.w) && (!t.g || al16(t.g))) {
      const long long n4 = (c.end - c.begin) / 4;
      const float4* g4 = t.g ? reinterpret_cast<const float4*>(t.g + c.begin) : nullptr;
      const float4* w4 = reinterpret_cast<const float4*>(t.w + c.begin);
#pragma unroll 4
      for (long long k = threadIdx.x; k < n4; k += blockDim.x) {
        float4 g = g4 ? g4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (t.wd != 0.f) {
          const float4 w = w4[k];
          g.x = g.x + t.wd * w.x;
          g.y = g.y + t.wd * w.y;
          g.z = g.z + t.wd * w.z;
          g.w = g.w + t.wd * w.w;
        }
        s += g.x * g.x;
        s += g.y * g.y;
        s += g.z * g.z;
        s += g.w * g.w;
      }
      i0 = c.begin + 4 * n4;
    } else {
      // operands not 16-B aligned (a gradient that is a view into an
      // all-reduce bucket, engine/reducer.py): scalar loads, but the float4
      // body's summation order -- thread k adds elements 4k .. 4k+3 in turn --
      // so the norm, and the clip factor, do not depend on the alignment
      const long long n4 = (c.end - c.begin) / 4;
      for (long long k = threadIdx.x; k < n4; k += blockDim.x) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long long i = c.begin + 4 * k + u;
          float g = t.g ? t.g[i] : 0.f;
          if (t.wd != 0.f) g = g + t.wd * t.w[i];
          s += g * g;
        }
      }
      i0 = c.begin + 4 * n4;
    }
    for (long long i = i0 + threadIdx.x; i < c.end; i += blockDim.x) s += sq_term(t, i);
  }
  const float tot = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void sgd_update_kernel(const SgdTensor* __restrict__ tensors,
                                                         const SgdChunk* __restrict__ chunks,
                                                         const float* __restrict__ partial,
                                                         float clip, float momentum, float lr,
                                                         const float* __restrict__ lr_dev,
                                                         int rev) {
  __shared__ float scale_s;
  if (lr_dev) lr = *lr_dev;  // (a captured graph's step: the LR lives on the device)
  // rev: chunks in reverse order, so that the operands the sum-of-squares pass
  // read last come first (tuning "sgd_rev", off: no MALL reuse measured,
  // 151-157 us per step either way, profiles/r5_sgd_rev_ab.log); each chunk's
  // arithmetic is the same either way
  const SgdChunk c = chunks[rev ? gridDim.x - 1 - blockIdx.x : blockIdx.x];
  const SgdTensor t = tensors[c.tensor];
  if (threadIdx.x == 0) {
    float ss = 0.f;
    if (clip > 0.f) {
#pragma unroll 8  // (loads in flight; the sum stays in chunk order)
      for (int k = 0; k < t.num_chunks; ++k) ss += partial[t.first_chunk + k];
    }
    // tf.clip_by_norm: l2norm = sqrt(sum) (0 when sum == 0); t * clip / max(l2norm, clip)
    const float nrm = ss > 0.f ? sqrtf(ss) : 0.f;
    scale_s = clip > 0.f ? fmaxf(nrm, clip) : 0.f;  // divisor; 0 = no clipping
  }
  __syncthreads();
  const float div = scale_s;
  auto upd = [&](float w, float g, float a, float& wo, float& ao) {
    g = g + t.wd * w;
    if (div > 0.f) g = g * clip / div;
    ao = a * momentum + g;
    wo = w - lr * ao;
  };
  long long i0 = c.begin;
  if (al16(t.w) && al16(t.accum) && (!t.g || al16(t.g))) {
    const long long n4 = (c.end - c.begin) / 4;
    float4* w4 = reinterpret_cast<float4*>(t.w + c.begin);
    float4* a4 = reinterpret_cast<float4*>(t.accum + c.begin);
    const float4* g4 = t.g ? reinterpret_cast<const float4*>(t.g + c.begin) : nullptr;
#pragma unroll 4
    for (long long k = threadIdx.x; k < n4; k += blockDim.x) {
      const float4 w = w4[k], a = a4[k];
      const float4 g = g4 ? g4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 wo, ao;
      upd(w.x, g.x, a.x, wo.x, ao.x);
      upd(w.y, g.y, a.y, wo.y, ao.y);
      upd(w.z, g.z, a.z, wo.z, ao.z);
      upd(w.w, g.w, a.w, wo.w, ao.w);
      a4[k] = ao;
      w4[k] = wo;
    }
    i0 = c.begin + 4 * n4;
  }
  for (long long i = i0 + threadIdx.x; i < c.end; i += blockDim.x) {
    float wo, ao;
    upd(t.w[i], t.g ? t.g[i] : 0.f, t.accum[i], wo, ao);
    t.accum[i] = ao;
    t.w[i] = wo;
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

// lr_dev: when non-null the learning rate is read from this device float at
// run time (a step captured in a hipGraph replays with each step's LR, which
// the host writes there); lr is then ignored.
extern "C" int d2mi_momentum_sgd_ex(const void* tensor_table, const void* chunk_table,
                                    int num_chunks, float* partial, float clip_norm,
                                    float momentum, float lr, const float* lr_dev, void* stream) {
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
                     clip_norm, momentum, lr, lr_dev,
                     clip_norm > 0.f && tuning(kTuneSgdRev) != 0 ? 1 : 0);  // (tuning "sgd_rev")
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_momentum_sgd(const void* tensor_table, const void* chunk_table, int num_chunks,
                                 float* partial, float clip_norm, float momentum, float lr,
                                 void* stream) {
  return d2mi_momentum_sgd_ex(tensor_table, chunk_table, num_chunks, partial, clip_norm, momentum,
                              lr, nullptr, stream);
}
