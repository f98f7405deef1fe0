// Segmented sort of 64-bit (score, index) keys.
// Small segments (<= 8192 keys: RPN levels, RetinaNet candidates, NMS inputs)
// are sorted by a stable counting rank spread over len/64 workgroups per
// segment (keys staged in LDS, 64 KiB at most).  Larger capacities (the
// class-offset NMS of fast_rcnn_inference over up to 80k boxes,
// fast_rcnn.py:145): the same rank sort on 8192-key tiles, then merge passes
// that double the sorted run width -- each key finds its place in the merged
// run by a binary search of the partner run (merge-path by rank), one launch
// per pass, ping-ponging through a workspace copy.  Hand-written (r4: no
// vendor sort on the hot path); deterministic and a permutation for any keys.
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

// Rank sort of fixed-size tiles: tile t of segment seg = blockIdx.y / nt
// holds keys [t * tile, min((t + 1) * tile, len)) -- rank_sort_kernel on a
// virtual segment of at most `tile` keys.
__global__ __launch_bounds__(kRankT) void rank_sort_tiles_kernel(const uint64_t* __restrict__ in,
                                                              uint64_t* __restrict__ out,
                                                              const int32_t* __restrict__ lens,
                                                              int cap, int tile, int nt) {
  extern __shared__ uint64_t s[];
  __shared__ uint32_t part[kRankT];
  const int seg = blockIdx.y / nt, t = blockIdx.y - seg * nt;
  const int len = min(max(min(lens[seg], cap) - t * tile, 0), tile);
  const int i0 = blockIdx.x * kRankI;
  if (i0 >= len) return;
  const size_t base = (size_t)seg * cap + (size_t)t * tile;
  const uint64_t* src = in + base;
  for (int j = threadIdx.x; j < len; j += kRankT) s[j] = src[j];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = i0 + lane;
  const uint64_t mine = i < len ? s[i] : ~0ull;
  const int q = (len + kRankW - 1) / kRankW;
  const int j0 = w * q, j1 = min(len, j0 + q);
  uint32_t r = 0;
  for (int j = j0; j < j1; ++j) {
    const uint64_t o = s[j];
    r += (o < mine || (o == mine && j < i)) ? 1u : 0u;
  }
  part[threadIdx.x] = r;
  __syncthreads();
  if (w == 0 && i < len) {
    uint32_t rank = 0;
#pragma unroll
    for (int v = 0; v < kRankW; ++v) rank += part[v * 64 + lane];
    out[base + rank] = mine;
  }
}

// One merge pass: sorted runs of `width` keys pairwise into runs of 2 *
// width.  Key p of its run goes to (p - run start) + its rank in the partner
// run; ties across the pair put the left run first (left counts partner keys
// < it, right counts partner keys <= it), so the result is a stable
// permutation.
__global__ __launch_bounds__(256) void merge_runs_kernel(const uint64_t* __restrict__ in,
                                                         uint64_t* __restrict__ out,
                                                         const int32_t* __restrict__ lens, int cap,
                                                         int width) {
  const int seg = blockIdx.y;
  const int len = min(lens[seg], cap);
  const uint64_t* src = in + (size_t)seg * cap;
  uint64_t* dst = out + (size_t)seg * cap;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < len; p += gridDim.x * blockDim.x) {
    const int run = p / width;
    const int lo = run * width;
    const bool left = (run & 1) == 0;
    const int pb = left ? lo + width : lo - width;  // partner run [pb, pe)
    const int pe = min(pb + width, len);
    const uint64_t key = src[p];
    int a = pb, b = max(pb, pe);  // first partner index with key (< or <=) partner key
    while (a < b) {
      const int m = (a + b) >> 1;
      const uint64_t o = src[m];
      if (left ? (o < key) : (o <= key)) a = m + 1;
      else b = m;
    }
    const int merged0 = left ? lo : pb;
    dst[merged0 + (p - lo) + (a - pb)] = key;
  }
}

constexpr int kTile = kLdsSortCap;

int merge_passes(int cap) {
  int n = 0;
  for (long long w = kTile; w < cap; w *= 2) ++n;
  return n;
}

}  // namespace

size_t sort_workspace_size(int S, int cap) {
  if (cap <= kLdsSortCap) return 0;
  WorkspaceSizer z;
  z.take<uint64_t>((size_t)S * cap);  // the other ping-pong buffer
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
  uint64_t* tmp = w.take<uint64_t>((size_t)S * cap);
  D2MI_REQUIRE(w.ok(), "sort workspace too small (%zu < %zu)", ws_bytes, w.off);
  const int nt = (cap + kTile - 1) / kTile;
  D2MI_REQUIRE((long long)S * nt < 65536, "segmented sort: %d segments x %d tiles too many", S, nt);
  // the passes alternate buffers; start so that the last one writes keys_out
  const int passes = merge_passes(cap);
  uint64_t* bufs[2] = {keys_out, tmp};
  int cur = passes % 2;  // buffer the tile sort writes
  hipLaunchKernelGGL(rank_sort_tiles_kernel, dim3(kTile / kRankI, S * nt), dim3(kRankT),
                     kTile * sizeof(uint64_t), stream, keys_in, bufs[cur], lens, cap, kTile, nt);
  D2MI_LAUNCH_CHECK();
  const int gx = std::max(1, std::min((cap + 255) / 256, 1024));
  for (long long width = kTile; width < cap; width *= 2) {
    hipLaunchKernelGGL(merge_runs_kernel, dim3(gx, S), dim3(256), 0, stream, bufs[cur],
                       bufs[cur ^ 1], lens, cap, (int)width);
    D2MI_LAUNCH_CHECK();
    cur ^= 1;
  }
  return 0;
}

}  // namespace d2mi
