// Segmented sort of 64-bit (score, index) keys.
// Small segments (<= 8192 keys: RPN levels, RetinaNet candidates, NMS inputs)
// are sorted by a stable counting rank spread over len/64 workgroups per
// segment (keys staged in LDS, 64 KiB at most); larger capacities fall back
// to rocPRIM's segmented radix sort.
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "internal.h"

namespace d2mi {
namespace {

// Stable counting-rank sort: rank(i) = #{j : key_j < key_i} + #{j < i : key_j
// == key_i}, a permutation of [0, len).  A workgroup ranks 64 keys of its
// segment against all of them (each of its 4 waves a quarter of the segment,
// keys broadcast from LDS; 16 waves = 1,024 threads: each wave a sixteenth
// of the segment), so a segment spreads over len/64 workgroups
// instead of one workgroup running a bitonic network (13*14/2 LDS passes).
constexpr int kRankI = 64, kRankT = 1024, kRankW = kRankT / 64;
__global__ __launch_bounds__(kRankT) void rank_sort_kernel(const uint64_t* __restrict__ in,
                                                        uint64_t* __restrict__ out,
                                                        const int32_t* __restrict__ lens,
                                                        int cap) {
  extern __shared__ uint64_t s[];
  __shared__ uint32_t part[kRankT];
  const int seg = blockIdx.y;
  const int len = min(lens[seg], cap);
  const int i0 = blockIdx.x * kRankI;
  if (i0 >= len) return;
  const uint64_t* src = in + (size_t)seg * cap;
  // 8 global loads in flight per thread, 8 LDS broadcast reads in flight per
  // comparison step (one dependent load per key made both loops latency-bound:
  // 84 us for the RetinaNet NMS inputs, 2 x 5,000 keys)
  for (int j0 = 0; j0 < len; j0 += 8 * kRankT) {
    uint64_t e[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * kRankT + threadIdx.x;
      e[u] = j < len ? src[j] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * kRankT + threadIdx.x;
      if (j < len) s[j] = e[u];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = i0 + lane;
  const uint64_t mine = i < len ? s[i] : ~0ull;
  const int q = (len + kRankW - 1) / kRankW;
  const int j0 = w * q, j1 = min(len, j0 + q);
  uint32_t r = 0;
  int j = j0;
  for (; j + 8 <= j1; j += 8) {
    uint64_t o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = s[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) r += (o[u] < mine || (o[u] == mine && j + u < i)) ? 1u : 0u;
  }
  for (; j < j1; ++j) {
    const uint64_t o = s[j];
    r += (o < mine || (o == mine && j < i)) ? 1u : 0u;
  }
  part[threadIdx.x] = r;
  __syncthreads();
  if (w == 0 && i < len) {
    uint32_t rank = 0;
#pragma unroll
    for (int v = 0; v < kRankW; ++v) rank += part[v * 64 + lane];
    out[(size_t)seg * cap + rank] = mine;
  }
}

__global__ void seg_bounds_kernel(const int32_t* lens, int S, int cap, int* begin, int* end) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < S) {
    begin[s] = s * cap;
    end[s] = s * cap + min(lens[s], cap);
  }
}

size_t rocprim_tmp_bytes(int S, int cap) {
  size_t bytes = 0;
  rocprim::segmented_radix_sort_keys((void*)nullptr, bytes, (const uint64_t*)nullptr,
                                     (uint64_t*)nullptr, (unsigned int)((size_t)S * cap),
                                     (unsigned int)S, (const int*)nullptr, (const int*)nullptr,
                                     0u, 64u, (hipStream_t)0, false);
  return bytes;
}

}  // namespace

size_t sort_workspace_size(int S, int cap) {
  if (cap <= kLdsSortCap) return 0;
  WorkspaceSizer z;
  z.take<int>(S);
  z.take<int>(S);
  z.take<char>(rocprim_tmp_bytes(S, cap));
  return z.off;
}

int sort_keys_segmented(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* lens, int S,
                        int cap, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (S == 0 || cap == 0) return 0;
  if (cap <= kLdsSortCap) {
    hipLaunchKernelGGL(rank_sort_kernel, dim3((cap + kRankI - 1) / kRankI, S), dim3(kRankT),
                       cap * sizeof(uint64_t), stream, keys_in, keys_out, lens, cap);
    D2MI_LAUNCH_CHECK();
    return 0;
  }
  Workspace w(ws, ws_bytes);
  int* begin = w.take<int>(S);
  int* end = w.take<int>(S);
  size_t tmp_bytes = rocprim_tmp_bytes(S, cap);
  void* tmp = w.take<char>(tmp_bytes);
  D2MI_REQUIRE(w.ok(), "sort workspace too small (%zu < %zu)", ws_bytes, w.off);
  hipLaunchKernelGGL(seg_bounds_kernel, dim3((S + 255) / 256), dim3(256), 0, stream, lens, S, cap,
                     begin, end);
  D2MI_LAUNCH_CHECK();
  D2MI_HIP(rocprim::segmented_radix_sort_keys(tmp, tmp_bytes, keys_in, keys_out,
                                              (unsigned int)((size_t)S * cap), (unsigned int)S,
                                              (const int*)begin, (const int*)end, 0u, 64u, stream,
                                              false));
  return 0;
}

}  // namespace d2mi
