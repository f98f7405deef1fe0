// Exact segmented top-k (TF TopKV2, sorted=True: value desc, ties lowest index
// first) as a radix select on gfx950.
//
// Reference call sites: rpn_outputs.py:70 (per-level pre-NMS top-k over up to
// 201,600 logits), rpn_outputs.py:106, retinanet.py:326 (up to 12.1 M sigmoid
// scores per level per image).
//
// The selection is a most-significant-digit radix select on the order-preserving
// uint32 image of the key (11 + 11 + 10 bits):
//   hist   multi-workgroup LDS histogram per segment, merged with global atomics
//   select one workgroup per segment finds the digit holding the k-th key and
//          stops as soon as (keys above it) + (keys in it) fit the 8192-key LDS sort
//   collect elements at or above the threshold digit are appended (unordered)
//          as (key, index) sort keys; index order is restored by the final sort
//   sort   one workgroup per segment, in-LDS bitonic sort, writes the first k.
// A segment whose k-th key is tied with more than 8192 others (all digits
// exhausted) takes the ordered path: one workgroup appends the tied keys in
// index order until k is reached — the TF tie rule, at the cost of one serial pass.
// Every kernel is launched unconditionally and reads the per-segment state, so
// the whole select is a fixed launch sequence (no host synchronisation).
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kBins = 2048;
constexpr int kCap = kLdsSortCap;  // candidates sortable in LDS

struct SegState {
  uint32_t prefix;     // selected high bits so far
  int32_t bits;        // number of resolved high bits
  int32_t k_rem;       // k minus keys strictly above the current prefix
  int32_t mode;        // 0 refine, 1 collect >= prefix, 2 collect all, 3 ordered ties, 4 empty
  int32_t ncand;       // appended candidates
  int32_t k;           // effective k
  int32_t need_eq;     // mode 3: tied keys still to take (in index order)
  int32_t pad;
};

__device__ __forceinline__ uint32_t value_key(float v, int key_mode) {
  if (key_mode == 1) v = 1.f / (1.f + expf(-v));
  return orderable(v);
}

__device__ __forceinline__ void digit_of(int pass, int& shift, int& nbits) {
  if (pass == 0) { shift = 21; nbits = 11; }
  else if (pass == 1) { shift = 10; nbits = 11; }
  else { shift = 0; nbits = 10; }
}

__global__ void topk_init_kernel(SegState* st, uint32_t* hist, const int32_t* seg_len,
                                 const int32_t* seg_k, int S, int k) {
  const int s = blockIdx.x;
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) hist[(size_t)s * kBins + i] = 0;
  if (threadIdx.x == 0) {
    const int len = max(seg_len[s], 0);
    int kk = seg_k ? min(seg_k[s], k) : k;
    kk = min(kk, len);
    SegState x;
    x.prefix = 0;
    x.bits = 0;
    x.k_rem = kk;
    x.k = kk;
    x.ncand = 0;
    x.need_eq = 0;
    x.pad = 0;
    x.mode = kk == 0 ? 4 : (len <= kCap ? 2 : 0);
    st[s] = x;
  }
}

__global__ __launch_bounds__(256) void topk_hist_kernel(const float* __restrict__ values,
                                                        const int64_t* __restrict__ seg_start,
                                                        const int32_t* __restrict__ seg_len,
                                                        const SegState* __restrict__ st,
                                                        uint32_t* __restrict__ hist, int pass,
                                                        int key_mode) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode != 0) return;
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  int shift, nbits;
  digit_of(pass, shift, nbits);
  const float* v = values + seg_start[s];
  const int len = seg_len[s];
  const int hs = shift + nbits;  // bits above this digit
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const uint32_t key = value_key(v[i], key_mode);
    if (hs == 32 || (key >> hs) == x.prefix) atomicAdd(&h[(key >> shift) & ((1u << nbits) - 1u)], 1u);
  }
  __syncthreads();
  uint32_t* g = hist + (size_t)s * kBins;
  for (int i = threadIdx.x; i < kBins; i += blockDim.x)
    if (h[i]) atomicAdd(&g[i], h[i]);
}

__global__ __launch_bounds__(256) void topk_select_kernel(SegState* st, uint32_t* hist,
                                                          int pass) {
  const int s = blockIdx.x;
  SegState x = st[s];
  if (x.mode != 0) return;
  int shift, nbits;
  digit_of(pass, shift, nbits);
  const int nb = 1 << nbits;
  uint32_t* g = hist + (size_t)s * kBins;
  // suffix sums from the top bin: thread t owns bins [nb-1-8t-7, nb-1-8t] (top first)
  __shared__ uint32_t part[256];
  const int per = nb / 256;
  const int t = threadIdx.x;
  uint32_t loc = 0;
  for (int j = 0; j < per; ++j) loc += g[nb - 1 - (t * per + j)];
  part[t] = loc;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t add = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  const uint32_t before = part[t] - loc;  // keys in bins above my range
  __shared__ int found_bin;
  __shared__ uint32_t found_gt, found_eq;
  if (t == 0) found_bin = -1;
  __syncthreads();
  if ((uint32_t)x.k_rem > before && (uint32_t)x.k_rem <= part[t]) {
    uint32_t acc = before;
    for (int j = 0; j < per; ++j) {
      const int b = nb - 1 - (t * per + j);
      const uint32_t c = g[b];
      if ((uint32_t)x.k_rem <= acc + c) {
        found_bin = b;
        found_gt = acc;
        found_eq = c;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  // reset histogram for the next pass
  for (int i = t; i < kBins; i += blockDim.x) g[i] = 0;
  if (t == 0) {
    if (found_bin < 0) {
      x.mode = 2;  // should not happen (counts inconsistent); fall back to "all"
    } else {
      x.prefix = (x.prefix << nbits) | (uint32_t)found_bin;
      x.bits += nbits;
      const int gt_total = (x.k - x.k_rem) + (int)found_gt;  // keys strictly above prefix
      x.k_rem -= (int)found_gt;
      if (gt_total + (int)found_eq <= kCap) x.mode = 1;
      else if (x.bits == 32) {
        x.mode = 3;
        x.need_eq = x.k_rem;
      }
    }
    st[s] = x;
  }
}

__global__ __launch_bounds__(256) void topk_collect_kernel(const float* __restrict__ values,
                                                           const int64_t* __restrict__ seg_start,
                                                           const int32_t* __restrict__ seg_len,
                                                           SegState* __restrict__ st,
                                                           uint64_t* __restrict__ cand,
                                                           int key_mode) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode == 0 || x.mode == 4) return;
  const float* v = values + seg_start[s];
  const int len = seg_len[s];
  uint64_t* c = cand + (size_t)s * kCap;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const float val = v[i];
    const uint32_t key = value_key(val, key_mode);
    bool take;
    if (x.mode == 2) take = true;
    else if (x.mode == 1) take = (key >> (32 - x.bits)) >= x.prefix;
    else take = key > x.prefix;  // mode 3: strictly greater; ties appended in order below
    if (take) {
      const int pos = atomicAdd(&st[s].ncand, 1);
      if (pos < kCap) c[pos] = ((uint64_t)(~key) << 32) | (uint32_t)i;
    }
  }
}

// mode 3 only: append the first need_eq keys equal to prefix, in index order.
__global__ __launch_bounds__(1024) void topk_ties_kernel(const float* __restrict__ values,
                                                         const int64_t* __restrict__ seg_start,
                                                         const int32_t* __restrict__ seg_len,
                                                         SegState* __restrict__ st,
                                                         uint64_t* __restrict__ cand,
                                                         int key_mode) {
  const int s = blockIdx.x;
  const SegState x = st[s];
  if (x.mode != 3) return;
  const float* v = values + seg_start[s];
  const int len = seg_len[s];
  uint64_t* c = cand + (size_t)s * kCap;
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = st[s].ncand;
  int need = x.need_eq;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int c0 = 0; c0 < len && need > 0; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    const bool eq = i < len && value_key(v[i], key_mode) == x.prefix;
    const uint64_t b = __ballot(eq);
    const int wrank = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(b);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      if (w < wv) before += wsum[w];
      total += wsum[w];
    }
    const int rank = before + wrank;
    if (eq && rank < need) c[base + rank] = ((uint64_t)(~x.prefix) << 32) | (uint32_t)i;
    __syncthreads();
    const int took = min(total, need);
    if (threadIdx.x == 0) base += took;
    need -= took;
    __syncthreads();
  }
  if (threadIdx.x == 0) st[s].ncand = base;
}

__global__ __launch_bounds__(1024) void topk_final_kernel(const uint64_t* __restrict__ cand,
                                                          const SegState* __restrict__ st,
                                                          int kmax, int key_mode,
                                                          float* __restrict__ vals_out,
                                                          int32_t* __restrict__ idx_out,
                                                          int32_t* __restrict__ count_out,
                                                          int32_t* err) {
  extern __shared__ uint64_t sk[];
  const int s = blockIdx.x;
  const SegState x = st[s];
  int len = x.mode == 4 ? 0 : x.ncand;
  if (len > kCap) {
    if (threadIdx.x == 0) atomicOr(err, kErrTopkCapacity);
    len = kCap;
  }
  int n = 1;
  while (n < len) n <<= 1;
  const uint64_t* src = cand + (size_t)s * kCap;
  for (int i = threadIdx.x; i < n; i += blockDim.x) sk[i] = i < len ? src[i] : ~0ull;
  __syncthreads();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = sk[i], b = sk[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) { sk[i] = b; sk[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  const int kk = min(x.k, len);
  for (int i = threadIdx.x; i < kmax; i += blockDim.x) {
    if (i < kk) {
      const uint64_t key = sk[i];
      vals_out[(size_t)s * kmax + i] = from_orderable(~(uint32_t)(key >> 32));
      idx_out[(size_t)s * kmax + i] = (int32_t)(key & 0xffffffffu);
    } else {
      vals_out[(size_t)s * kmax + i] = 0.f;
      idx_out[(size_t)s * kmax + i] = -1;
    }
  }
  if (threadIdx.x == 0) count_out[s] = kk;
  (void)key_mode;
}

}  // namespace

size_t topk_workspace_size(int S, int k) {
  (void)k;
  WorkspaceSizer z;
  z.take<SegState>(S);
  z.take<uint32_t>((size_t)S * kBins);
  z.take<uint64_t>((size_t)S * kCap);
  return z.off;
}

int topk_core_ex(const float* values, const int64_t* seg_start, const int32_t* seg_len,
                 const int32_t* seg_k, int S, int max_len, int k, int key_mode, float* vals_out,
                 int32_t* idx_out, int32_t* count_out, void* ws, size_t ws_bytes,
                 hipStream_t stream) {
  D2MI_REQUIRE(k >= 0 && k <= kCap, "top-k k=%d must be in [0, %d]", k, kCap);
  D2MI_REQUIRE(key_mode == 0 || key_mode == 1, "key_mode must be 0 or 1");
  if (S == 0) return 0;
  Workspace w(ws, ws_bytes);
  SegState* st = w.take<SegState>(S);
  uint32_t* hist = w.take<uint32_t>((size_t)S * kBins);
  uint64_t* cand = w.take<uint64_t>((size_t)S * kCap);
  D2MI_REQUIRE(w.ok(), "top-k workspace too small (%zu < %zu)", ws_bytes, w.off);
  const int per_block = 256 * 16;
  const int gx = std::max(1, std::min((max_len + per_block - 1) / per_block, 4096));
  hipLaunchKernelGGL(topk_init_kernel, dim3(S), dim3(256), 0, stream, st, hist, seg_len, seg_k, S,
                     k);
  D2MI_LAUNCH_CHECK();
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(topk_hist_kernel, dim3(gx, S), dim3(256), 0, stream, values, seg_start,
                       seg_len, st, hist, pass, key_mode);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(topk_select_kernel, dim3(S), dim3(256), 0, stream, st, hist, pass);
    D2MI_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(topk_collect_kernel, dim3(gx, S), dim3(256), 0, stream, values, seg_start,
                     seg_len, st, cand, key_mode);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(topk_ties_kernel, dim3(S), dim3(1024), 0, stream, values, seg_start, seg_len,
                     st, cand, key_mode);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(topk_final_kernel, dim3(S), dim3(1024), kCap * sizeof(uint64_t), stream, cand,
                     st, k, key_mode, vals_out, idx_out, count_out, error_word());
  D2MI_LAUNCH_CHECK();
  return 0;
}

int topk_core(const float* values, const int64_t* seg_start, const int32_t* seg_len, int S,
              int max_len, int k, int key_mode, float* vals_out, int32_t* idx_out,
              int32_t* count_out, void* ws, size_t ws_bytes, hipStream_t stream) {
  return topk_core_ex(values, seg_start, seg_len, nullptr, S, max_len, k, key_mode, vals_out,
                      idx_out, count_out, ws, ws_bytes, stream);
}

}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_topk_workspace_size(int num_segs, int k_max) {
  return topk_workspace_size(num_segs, k_max);
}

extern "C" int d2mi_topk(const float* values, const int64_t* seg_start, const int32_t* seg_len,
                         int num_segs, int max_seg_len, int k, int key_mode, float* values_out,
                         int32_t* idx_out, int32_t* count_out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  return topk_core(values, seg_start, seg_len, num_segs, max_seg_len, k, key_mode, values_out,
                   idx_out, count_out, workspace, workspace_bytes, as_stream(stream));
}
