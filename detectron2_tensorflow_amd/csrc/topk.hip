// Exact segmented top-k (TF TopKV2, sorted=True: value desc, ties lowest index
// first) as a radix select on gfx950.
//
// Reference call sites: rpn_outputs.py:70 (per-level pre-NMS top-k over up to
// 201,600 logits), rpn_outputs.py:106, retinanet.py:326 (top-k of the SIGMOID
// of up to 12.1 M logits per level per image, key_mode 1).
//
// The select runs on the order-preserving uint32 image of the RAW value, for
// both key modes: sigmoid is monotone, so the k-th largest sigmoid is the
// sigmoid of the k-th largest logit, and the scan passes need no expf (at
// 32 M scores per call the per-element sigmoid of every pass was the cost).
// Only the few collected candidates are ranked on their sigmoid keys.
//
//   hist     (3 passes, 12 + 12 + 8 bits) per-workgroup LDS histogram of a
//            16 K-element chunk (float4 loads, all in flight), flushed into 4
//            replicated global histograms (low same-address atomic traffic)
//   select   one workgroup per segment: suffix sums, the digit holding the
//            k-th key; stops refining once (keys above) + (keys in it) fit the
//            8192-key candidate buffer.  For key_mode 1 it also solves the
//            sigmoid tie interval of the bin's lower edge (binary search over
//            the key space): logits below the edge whose sigmoid equals the
//            edge's sigmoid may still belong to the top-k (TF ranks the
//            sigmoid values, ties by index).
//   collect  one pass: keys >= edge -> buffer A; keys in the tie window below
//            the edge whose sigmoid reaches the edge's -> buffer B.  One
//            atomic per workgroup reserves its slots (no per-element atomics).
//   resolve  one workgroup per segment: A + B when they fit; otherwise (a
//            saturated sigmoid, or more than 8192 equal keys) the exact
//            ordered path: keys strictly above the tie group, then the tied
//            keys in index order until k (the TF tie rule).
//   rank     counting rank of every candidate among all candidates on the
//            final 64-bit (score desc, index asc) key, spread over many
//            workgroups; rank < k scatters straight to the sorted output.
// Every kernel is launched unconditionally and reads the per-segment state,
// so the select is a fixed launch sequence (no host synchronisation).
//
// Sampled floor (key_mode 1, segments longer than the candidate buffer; the
// RetinaNet levels: top-1000 of up to 12.1 M scores).  The three histogram
// passes above cost far more than their reads: every element is an LDS atomic,
// and detection logits pile into a few 12-bit bins (same-address conflicts).
// The floor path replaces them with ONE read in the common case:
//   sample   12-bit histogram of 1/16 of the segment (1,024 contiguous keys out
//            of every 16,384)
//   floor    one workgroup per segment: the highest bin whose sampled suffix
//            count reaches 2 k scaled by the sampling rate; its lowest key,
//            lowered to the lowest key with the same sigmoid (nothing below
//            the floor ties with anything above it)
//   fcollect one pass: every key >= floor -> one of 16 spread slots (block-
//            aggregated; workgroup b appends to slot b % 16)
//   decide   k <= |A| <= 8192 (A = the slots compacted): A holds the whole top-k (at least k keys at or
//            above the floor, all strictly above everything below it in
//            sigmoid) -> straight to rank; otherwise back to the radix passes,
//            which then run exactly as without the floor.
// Exact either way; the sample only decides how often the fallback runs.
#include "detect.h"

namespace d2mi {
namespace {

constexpr int kBins = 4096;     // 12-bit digits
constexpr int kRep = 4;         // replicated global histograms
constexpr int kCap = kLdsSortCap;  // candidates (8192)
constexpr int kThreads = 256;

struct SegState {
  uint32_t prefix;   // selected high bits so far
  int32_t bits;      // number of resolved high bits
  int32_t k_rem;     // k minus keys strictly above the current prefix
  int32_t mode;      // 0 refine, 1 collect >= edge, 2 collect all, 3 resolved tie group, 4 empty
  int32_t k;         // effective k
  uint32_t edge;     // collect A: key >= edge (mode 1/3: lowest key of the prefix bin)
  uint32_t win_lo;   // key_mode 1: keys in [win_lo, edge) are tested on their sigmoid
  uint32_t tie_hi;   // key_mode 1: highest key whose sigmoid equals s_edge (mode 1/3)
  float s_edge;      // sigmoid of the edge value (key_mode 1)
  int32_t nA, nB;    // candidates appended to A / B
  int32_t ncand;     // candidates after resolve (ranked)
  int32_t pre;       // sampled floor: 2 floor chosen, 1 A is final (skip collect), 0 off
  uint32_t floor_key;
  int32_t nF[16];    // sampled floor: candidates per spread slot (fcollect)
};

__device__ __forceinline__ float key_value(float v, int key_mode) {
  return key_mode == 1 ? sigmoidf_tf(v) : v;
}

__device__ __forceinline__ void digit_of(int pass, int& shift, int& nbits) {
  if (pass == 0) { shift = 20; nbits = 12; }
  else if (pass == 1) { shift = 8; nbits = 12; }
  else { shift = 0; nbits = 8; }
}

// [lo, hi) element range of chunk b of a segment whose first element sits at
// p: chunks are aligned to 16 B in memory; chunk 0 also owns the unaligned head.
struct Chunk {
  int head;  // elements before the first 16-B boundary
  int64_t begin, end;
};
__device__ __forceinline__ Chunk chunk_of(const float* p, int len, int b, int per) {
  Chunk c;
  c.head = (int)((4 - (((uintptr_t)p >> 2) & 3)) & 3);
  if (c.head > len) c.head = len;
  c.begin = (int64_t)c.head + (int64_t)b * per;
  c.end = c.begin + per;
  if (c.end > len) c.end = len;
  return c;
}

// The workgroup's chunk held in registers: the float4 body (all loads of a
// thread issued before any use), plus at most one head element (chunk 0,
// before the first 16-B boundary) and one tail element (last chunk) per thread.
template <int V>
struct ChunkRegs {
  float4 v[V];
  int64_t begin;
  int n4;
  float hv, tv;
  int hi, ti;
  bool has_h, has_t, empty;

  __device__ __forceinline__ void load(const float* __restrict__ p, int len, int b) {
    constexpr int per = kThreads * V * 4;
    const Chunk c = chunk_of(p, len, b, per);
    begin = c.begin;
    empty = c.begin >= c.end && !(b == 0 && c.head > 0);
    has_h = b == 0 && (int)threadIdx.x < c.head;
    hi = threadIdx.x;
    hv = has_h ? p[hi] : 0.f;
    const int64_t n = c.end > c.begin ? c.end - c.begin : 0;
    n4 = (int)(n >> 2);
    const int nt = (int)(n - 4 * (int64_t)n4);
    has_t = (int)threadIdx.x < nt;
    ti = (int)(c.begin + 4 * (int64_t)n4) + threadIdx.x;
    tv = has_t ? p[ti] : 0.f;
    const float4* p4 = reinterpret_cast<const float4*>(p + c.begin);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int q = u * kThreads + threadIdx.x;
      v[u] = q < n4 ? p4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // f(index, value) for every element this thread holds
  template <typename F>
  __device__ __forceinline__ void visit(F f) const {
    if (has_h) f(hi, hv);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int q = u * kThreads + threadIdx.x;
      if (q < n4) {
        const int i = (int)(begin + 4 * (int64_t)q);
        f(i, v[u].x);
        f(i + 1, v[u].y);
        f(i + 2, v[u].z);
        f(i + 3, v[u].w);
      }
    }
    if (has_t) f(ti, tv);
  }
};

__global__ void topk_init_kernel(SegState* st, uint32_t* hist, const int32_t* seg_len,
                                 const int32_t* seg_k, int k) {
  const int s = blockIdx.y;
  uint32_t* h = hist + ((size_t)s * kRep + blockIdx.x) * kBins;
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int len = max(seg_len[s], 0);
    int kk = seg_k ? min(seg_k[s], k) : k;
    kk = max(min(kk, len), 0);
    SegState x = {};
    x.k_rem = kk;
    x.k = kk;
    x.mode = kk == 0 ? 4 : (len <= kCap ? 2 : 0);
    st[s] = x;
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void topk_hist_kernel(
    const float* __restrict__ values, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_len, const SegState* __restrict__ st,
    uint32_t* __restrict__ hist, int pass) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode != 0) return;
  const int len = seg_len[s];
  const int b = blockIdx.x;
  const float* p = values + seg_start[s];
  ChunkRegs<V> cr;
  cr.load(p, len, b);
  if (cr.empty) return;
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += kThreads) h[i] = 0;
  __syncthreads();
  int shift, nbits;
  digit_of(pass, shift, nbits);
  const int hs = shift + nbits;  // bits above this digit
  const uint32_t mask = (1u << nbits) - 1u;
  cr.visit([&](int, float v) {
    const uint32_t key = orderable(v);
    if (hs == 32 || (key >> hs) == x.prefix) atomicAdd(&h[(key >> shift) & mask], 1u);
  });
  __syncthreads();
  uint32_t* g = hist + ((size_t)s * kRep + (b & (kRep - 1))) * kBins;
  for (int i = threadIdx.x; i < kBins; i += kThreads)
    if (h[i]) atomicAdd(&g[i], h[i]);
}


__device__ void finish_state(SegState& x, int key_mode) {
  // x.edge: lowest key of the prefix bin (mode 1) or the resolved key (mode 3)
  x.win_lo = x.edge;
  x.tie_hi = x.edge;
  x.s_edge = 0.f;
  if (key_mode == 1 && x.edge > kKeyNegInf && x.edge <= kKeyPosInf) {
    const float se = sigmoidf_tf(from_orderable(x.edge));
    x.s_edge = se;
    const uint32_t lo = lower_bound_sig(kKeyNegInf, x.edge, se);
    x.win_lo = lo > kKeyNegInf + kWindowMargin ? lo - kWindowMargin : kKeyNegInf;
    x.tie_hi = upper_bound_sig(x.edge, kKeyPosInf, se);
  }
}

__global__ __launch_bounds__(kThreads) void topk_select_kernel(SegState* st, uint32_t* hist,
                                                               int pass, int key_mode) {
  const int s = blockIdx.x;
  SegState x = st[s];
  if (x.mode != 0) return;
  int shift, nbits;
  digit_of(pass, shift, nbits);
  const int nb = 1 << nbits;
  uint32_t* g = hist + (size_t)s * kRep * kBins;
  // suffix sums from the top bin: thread t owns bins [nb-1-per*t-(per-1), nb-1-per*t]
  __shared__ uint32_t part[kThreads];
  __shared__ uint32_t cnt[kBins];
  const int per = nb / kThreads;
  const int t = threadIdx.x;
  uint32_t loc = 0;
  for (int j = 0; j < per; ++j) {
    const int bin = nb - 1 - (t * per + j);
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) c += g[(size_t)r * kBins + bin];
    cnt[bin] = c;
    loc += c;
  }
  part[t] = loc;
  __syncthreads();
  for (int o = 1; o < kThreads; o <<= 1) {
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
      const int bin = nb - 1 - (t * per + j);
      const uint32_t c = cnt[bin];
      if ((uint32_t)x.k_rem <= acc + c) {
        found_bin = bin;
        found_gt = acc;
        found_eq = c;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  // reset the replicas for the next pass
  for (int i = t; i < kRep * kBins; i += kThreads) g[i] = 0;
  if (t == 0) {
    if (found_bin < 0) {
      x.mode = 2;  // counts inconsistent (cannot happen): take everything, resolve decides
      x.edge = 0;
    } else {
      x.prefix = (x.prefix << nbits) | (uint32_t)found_bin;
      x.bits += nbits;
      const int gt_total = (x.k - x.k_rem) + (int)found_gt;  // keys strictly above the bin
      x.k_rem -= (int)found_gt;
      if (gt_total + (int)found_eq <= kCap || x.bits == 32) {
        x.mode = gt_total + (int)found_eq <= kCap ? 1 : 3;
        x.edge = x.prefix << (32 - x.bits);
        finish_state(x, key_mode);
      }
    }
    st[s] = x;
  }
}

// Block-aggregated append: every thread contributes c items; returns the
// thread's first slot (one atomic per workgroup on *counter).
__device__ __forceinline__ int block_reserve(int c, int32_t* counter) {
  __shared__ int wsum[kThreads / 64];
  __shared__ int base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int wbefore = 0, total = 0;
#pragma unroll
  for (int j = 0; j < kThreads / 64; ++j) {
    if (j < w) wbefore += wsum[j];
    total += wsum[j];
  }
  if (threadIdx.x == 0) base = total ? atomicAdd(counter, total) : 0;
  __syncthreads();
  return base + wbefore + incl - c;
}

template <int V>
__global__ __launch_bounds__(kThreads) void topk_collect_kernel(
    const float* __restrict__ values, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_len, SegState* __restrict__ st,
    uint64_t* __restrict__ candA, uint64_t* __restrict__ candB, int key_mode) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode == 0 || x.mode == 4 || x.pre == 1) return;
  const int len = seg_len[s];
  const int b = blockIdx.x;
  const float* p = values + seg_start[s];
  ChunkRegs<V> cr;
  cr.load(p, len, b);
  if (cr.empty) return;
  // mode 2: all; mode 1: >= edge; mode 3: above the tie group (ties come in
  // index order in resolve; tie_hi == UINT32_MAX: nothing is above it)
  const bool none_above = x.mode == 3 && x.tie_hi == 0xffffffffu;
  const uint32_t a_lo = x.mode == 2 ? 0u : (x.mode == 3 ? x.tie_hi + 1u : x.edge);
  const bool win = key_mode == 1 && x.mode == 1 && x.win_lo < x.edge;
  int na = 0, nb = 0;
  cr.visit([&](int, float v) {
    const uint32_t key = orderable(v);
    if (none_above) return;
    if (key >= a_lo) ++na;
    else if (win && key >= x.win_lo && sigmoidf_tf(v) >= x.s_edge) ++nb;
  });
  int oa = block_reserve(na, &st[s].nA);
  int ob = block_reserve(nb, &st[s].nB);
  uint64_t* A = candA + (size_t)s * kCap;
  uint64_t* B = candB + (size_t)s * kCap;
  cr.visit([&](int i, float v) {
    const uint32_t key = orderable(v);
    if (none_above) return;
    const uint64_t e = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)i;
    if (key >= a_lo) {
      if (oa < kCap) A[oa] = e;
      ++oa;
    } else if (win && key >= x.win_lo && sigmoidf_tf(v) >= x.s_edge) {
      if (ob < kCap) B[ob] = e;
      ++ob;
    }
  });
}

// A + B when they fit; else the ordered path (module comment).
__global__ __launch_bounds__(1024) void topk_resolve_kernel(
    const float* __restrict__ values, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_len, SegState* __restrict__ st, uint64_t* __restrict__ candA,
    const uint64_t* __restrict__ candB, int key_mode) {
  const int s = blockIdx.x;
  SegState x = st[s];
  __shared__ int wsum[16];
  __shared__ int base_sh;
  if (x.mode == 0 || x.mode == 4) {
    if (threadIdx.x == 0) st[s].ncand = 0;
    return;
  }
  uint64_t* A = candA + (size_t)s * kCap;
  const uint64_t* B = candB + (size_t)s * kCap;
  const int nA = min(x.nA, kCap), nB = x.nB;
  if (x.mode != 3 && nA + nB <= kCap) {
    for (int i = threadIdx.x; i < nB; i += blockDim.x) A[nA + i] = B[i];
    if (threadIdx.x == 0) st[s].ncand = nA + nB;
    return;
  }
  // ordered path.  Tie group: keys in [tie_lo, tie_hi] whose key value equals
  // the edge's (key_mode 1: sigmoid == s_edge, tested exactly).  1. keep the
  // A entries strictly above the group, in place (order is irrelevant: ranked).
  const uint32_t tie_hi = x.tie_hi;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) base_sh = 0;
  __syncthreads();
  for (int c0 = 0; c0 < nA; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    uint64_t e = 0;
    bool keep = false;
    if (i < nA) {
      e = A[i];
      keep = orderable(__uint_as_float((uint32_t)(e >> 32))) > tie_hi;
    }
    const uint64_t bal = __ballot(keep);
    const int wrank = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < nw; ++w) {
      if (w < wv) before += wsum[w];
      total += wsum[w];
    }
    const int pos = base_sh + before + wrank;
    __syncthreads();  // every read of A[c0..] precedes the compacting writes
    if (keep) A[pos] = e;
    __syncthreads();
    if (threadIdx.x == 0) base_sh += total;
    __syncthreads();
  }
  int have = base_sh;
  int need = x.k - have;
  // 2. the tied keys in index order until k
  const float* v = values + seg_start[s];
  const int len = seg_len[s];
  const uint32_t tie_lo = key_mode == 1 ? x.win_lo : x.edge;
  for (int c0 = 0; c0 < len && need > 0; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    bool eq = false;
    float val = 0.f;
    if (i < len) {
      val = v[i];
      const uint32_t key = orderable(val);
      if (key >= tie_lo && key <= tie_hi)
        eq = key_mode == 1 ? sigmoidf_tf(val) == x.s_edge : key == x.edge;
    }
    const uint64_t bal = __ballot(eq);
    const int wrank = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < nw; ++w) {
      if (w < wv) before += wsum[w];
      total += wsum[w];
    }
    const int rank = before + wrank;
    if (eq && rank < need) A[have + rank] = ((uint64_t)__float_as_uint(val) << 32) | (uint32_t)i;
    const int took = min(total, need);
    have += took;
    need -= took;
    __syncthreads();
  }
  if (threadIdx.x == 0) st[s].ncand = min(have, kCap);
}

// Counting rank on the final key (~orderable(score) << 32 | index): a block
// ranks 64 candidates against all of its segment's, each of its 16 waves a sixteenth of them.
constexpr int kRankI = 64, kRankT = 1024, kRankW = kRankT / 64;  // 16 waves split the keys
__global__ __launch_bounds__(kRankT) void topk_rank_kernel(
    const uint64_t* __restrict__ candA, const SegState* __restrict__ st, int kmax, int key_mode,
    float* __restrict__ vals_out, int32_t* __restrict__ idx_out, int32_t* __restrict__ count_out) {
  extern __shared__ uint64_t sk[];
  __shared__ uint32_t part[kRankT];
  const int s = blockIdx.y;
  const SegState x = st[s];
  const int n = x.mode == 4 ? 0 : x.ncand;
  const int kk = min(x.k, n);
  const int i0 = blockIdx.x * kRankI;
  if (blockIdx.x == 0) {
    for (int i = kk + threadIdx.x; i < kmax; i += kRankT) {
      vals_out[(size_t)s * kmax + i] = 0.f;
      idx_out[(size_t)s * kmax + i] = -1;
    }
    if (threadIdx.x == 0) count_out[s] = kk;
  }
  if (i0 >= n) return;
  const uint64_t* A = candA + (size_t)s * kCap;
  // 8 loads in flight per thread (a dependent load per entry was the cost)
  for (int j0 = 0; j0 < n; j0 += 8 * kRankT) {
    uint64_t e[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * kRankT + threadIdx.x;
      e[u] = j < n ? A[j] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * kRankT + threadIdx.x;
      const float sc = key_value(__uint_as_float((uint32_t)(e[u] >> 32)), key_mode);
      if (j < n) sk[j] = ((uint64_t)(~orderable(sc)) << 32) | (uint32_t)e[u];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = i0 + lane;
  const uint64_t mine = i < n ? sk[i] : ~0ull;
  const int q = (n + kRankW - 1) / kRankW;
  const int j0 = w * q, j1 = min(n, j0 + q);
  uint32_t r = 0;
  int j = j0;
  for (; j + 8 <= j1; j += 8) {  // 8 broadcast reads in flight
    uint64_t c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) c[u] = sk[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) r += c[u] < mine ? 1u : 0u;
  }
  for (; j < j1; ++j) r += sk[j] < mine ? 1u : 0u;
  part[threadIdx.x] = r;
  __syncthreads();
  if (w == 0 && i < n) {
    uint32_t rank = 0;
#pragma unroll
    for (int v = 0; v < kRankW; ++v) rank += part[v * 64 + lane];
    if ((int)rank < kk) {
      // the value itself, from the candidate's raw bits (not rebuilt from the
      // key: orderable() gives -0.0 the key of +0.0, and TF's top_k returns
      // a -0.0 input as -0.0)
      const float v = key_value(__uint_as_float((uint32_t)(A[i] >> 32)), key_mode);
      vals_out[(size_t)s * kmax + rank] = v;
      idx_out[(size_t)s * kmax + rank] = (int32_t)(uint32_t)mine;
    }
  }
}


// ------------------------------------------------------------ sampled floor
constexpr int kSampleStride = 16384, kSampleRun = 1024, kSampleRunsPerWg = 16;
// fcollect appends into 16 slots per segment (workgroup b -> slot b % 16), each
// with its own counter: one counter per segment took every workgroup's atomic
// on one address (measured 39 us for the pass vs 14 us for a histogram pass)
constexpr int kFloorSlots = 16, kFloorSlotCap = 2048;

// 12-bit histogram of the sampled keys (1,024 contiguous out of every 16,384).
__global__ __launch_bounds__(kThreads) void topk_sample_kernel(
    const float* __restrict__ values, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_len, const SegState* __restrict__ st,
    uint32_t* __restrict__ hist) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode != 0) return;
  const int len = seg_len[s];
  const int64_t run0 = (int64_t)blockIdx.x * kSampleRunsPerWg;
  if (run0 * kSampleStride >= len) return;
  const float* p = values + seg_start[s];
  constexpr int U = kSampleRun / kThreads;
  float v[kSampleRunsPerWg][U];
  bool ok[kSampleRunsPerWg][U];
#pragma unroll
  for (int r = 0; r < kSampleRunsPerWg; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = (run0 + r) * kSampleStride + u * kThreads + threadIdx.x;
      ok[r][u] = i < len;
      v[r][u] = ok[r][u] ? p[i] : 0.f;
    }
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += kThreads) h[i] = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSampleRunsPerWg; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (ok[r][u]) atomicAdd(&h[orderable(v[r][u]) >> 20], 1u);
  __syncthreads();
  uint32_t* g = hist + ((size_t)s * kRep + (blockIdx.x & (kRep - 1))) * kBins;
  for (int i = threadIdx.x; i < kBins; i += kThreads)
    if (h[i]) atomicAdd(&g[i], h[i]);
}

// Floor from the sampled histogram (module comment); clears the replicas.
__global__ __launch_bounds__(kThreads) void topk_floor_kernel(SegState* st, uint32_t* hist,
                                                              const int32_t* seg_len) {
  const int s = blockIdx.x;
  const SegState x = st[s];
  if (x.mode != 0) return;
  uint32_t* g = hist + (size_t)s * kRep * kBins;
  __shared__ uint32_t part[kThreads];
  __shared__ uint32_t cnt[kBins];
  constexpr int per = kBins / kThreads;
  const int t = threadIdx.x;
  uint32_t loc = 0;
  for (int j = 0; j < per; ++j) {  // thread t owns bins from the top, as topk_select_kernel
    const int bin = kBins - 1 - (t * per + j);
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) c += g[(size_t)r * kBins + bin];
    cnt[bin] = c;
    loc += c;
  }
  part[t] = loc;
  __syncthreads();
  for (int o = 1; o < kThreads; o <<= 1) {
    const uint32_t add = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  const uint32_t total = part[kThreads - 1];
  const uint32_t before = part[t] - loc;
  // sampled suffix count that stands for 2 k keys of the whole segment
  const int len = seg_len[s];
  const uint32_t target =
      (uint32_t)max(1.0, ceil(2.0 * (double)x.k * (double)total / (double)max(len, 1)));
  __shared__ int found_bin;
  if (t == 0) found_bin = -1;
  __syncthreads();
  if (target > before && target <= part[t]) {
    uint32_t acc = before;
    for (int j = 0; j < per; ++j) {
      const int bin = kBins - 1 - (t * per + j);
      acc += cnt[bin];
      if (acc >= target) {
        found_bin = bin;
        break;
      }
    }
  }
  __syncthreads();
  for (int i = t; i < kRep * kBins; i += kThreads) g[i] = 0;  // clean for the fallback passes
  if (t == 0) {
    SegState y = x;
    if (found_bin < 0) {
      y.pre = 0;
    } else {
      uint32_t f = (uint32_t)found_bin << 20;
      if (f > kKeyNegInf && f <= kKeyPosInf) {  // no sigmoid tie across the floor
        f = lower_bound_sig(kKeyNegInf, f, sigmoidf_tf(from_orderable(f)));
        f = f > kKeyNegInf + kWindowMargin ? f - kWindowMargin : kKeyNegInf;  // as finish_state
      }
      y.floor_key = f;
      y.pre = 2;
    }
    st[s] = y;
  }
}

// Every key >= the floor -> its workgroup's spread slot (counted past the
// slot's end: decide reads the counts).
template <int V>
__global__ __launch_bounds__(kThreads) void topk_floor_collect_kernel(
    const float* __restrict__ values, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ seg_len, SegState* __restrict__ st,
    uint64_t* __restrict__ fbuf) {
  const int s = blockIdx.y;
  const SegState x = st[s];
  if (x.mode != 0 || x.pre != 2) return;
  const int len = seg_len[s];
  const float* p = values + seg_start[s];
  ChunkRegs<V> cr;
  cr.load(p, len, blockIdx.x);
  if (cr.empty) return;
  const uint32_t f = x.floor_key;
  int na = 0;
  cr.visit([&](int, float v) { na += orderable(v) >= f ? 1 : 0; });
  const int slot = blockIdx.x & (kFloorSlots - 1);
  int oa = block_reserve(na, &st[s].nF[slot]);
  uint64_t* A = fbuf + ((size_t)s * kFloorSlots + slot) * kFloorSlotCap;
  cr.visit([&](int i, float v) {
    if (orderable(v) >= f) {
      if (oa < kFloorSlotCap) A[oa] = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)i;
      ++oa;
    }
  });
}

// One workgroup per segment: every slot fits and k <= total <= 8192 -> the
// slots compacted into A (order is irrelevant: ranked), mode 1; otherwise the
// radix passes run as without the floor.
__global__ __launch_bounds__(kThreads) void topk_floor_decide_kernel(
    SegState* st, const uint64_t* __restrict__ fbuf, uint64_t* __restrict__ candA) {
  const int s = blockIdx.x;
  const SegState x = st[s];
  if (x.mode != 0 || x.pre != 2) return;
  int off[kFloorSlots + 1];
  bool fits = true;
  off[0] = 0;
#pragma unroll
  for (int j = 0; j < kFloorSlots; ++j) {
    fits = fits && x.nF[j] <= kFloorSlotCap;
    off[j + 1] = off[j] + x.nF[j];
  }
  const int total = off[kFloorSlots];
  const bool take = fits && total >= x.k && total <= kCap;
  if (take) {
    uint64_t* A = candA + (size_t)s * kCap;
    for (int j = 0; j < kFloorSlots; ++j) {
      const uint64_t* src = fbuf + ((size_t)s * kFloorSlots + j) * kFloorSlotCap;
      for (int i = threadIdx.x; i < x.nF[j]; i += kThreads) A[off[j] + i] = src[i];
    }
  }
  if (threadIdx.x == 0) {
    SegState y = x;
    if (take) {
      y.mode = 1;
      y.edge = y.floor_key;
      y.win_lo = y.floor_key;  // no tie window: nothing below the floor ties (floor kernel)
      y.tie_hi = y.floor_key;
      y.s_edge = 0.f;
      y.nA = total;
      y.nB = 0;
      y.pre = 1;
    } else {
      y.pre = 0;  // the radix passes run as without the floor
    }
    st[s] = y;
  }
}
}  // namespace

size_t topk_workspace_size(int S, int k) {
  (void)k;
  WorkspaceSizer z;
  z.take<SegState>(S);
  z.take<uint32_t>((size_t)S * kRep * kBins);
  z.take<uint64_t>((size_t)S * kCap);
  z.take<uint64_t>((size_t)S * kCap);
  z.take<uint64_t>((size_t)S * kFloorSlots * kFloorSlotCap);
  return z.off;
}

int topk_core_ex(const float* values, const int64_t* seg_start, const int32_t* seg_len,
                 const int32_t* seg_k, int S, int max_len, int k, int key_mode, float* vals_out,
                 int32_t* idx_out, int32_t* count_out, void* ws, size_t ws_bytes,
                 hipStream_t stream, bool sampled_floor) {
  D2MI_REQUIRE(k >= 0 && k <= kCap, "top-k k=%d must be in [0, %d]", k, kCap);
  D2MI_REQUIRE(key_mode == 0 || key_mode == 1, "key_mode must be 0 or 1");
  if (S == 0) return 0;
  Workspace w(ws, ws_bytes);
  SegState* st = w.take<SegState>(S);
  uint32_t* hist = w.take<uint32_t>((size_t)S * kRep * kBins);
  uint64_t* candA = w.take<uint64_t>((size_t)S * kCap);
  uint64_t* candB = w.take<uint64_t>((size_t)S * kCap);
  uint64_t* fbuf = w.take<uint64_t>((size_t)S * kFloorSlots * kFloorSlotCap);
  D2MI_REQUIRE(w.ok(), "top-k workspace too small (%zu < %zu)", ws_bytes, w.off);
  // chunk per workgroup: 16 K elements for the dense RetinaNet levels, 4 K
  // for RPN-sized segments (more workgroups over a smaller scan)
  const bool big = max_len >= (1 << 20);
  const int per = kThreads * 4 * (big ? 16 : 4);
  const int gx = std::max(1, (max_len + 3 + per - 1) / per);
  hipLaunchKernelGGL(topk_init_kernel, dim3(kRep, S), dim3(256), 0, stream, st, hist, seg_len,
                     seg_k, k);
  D2MI_LAUNCH_CHECK();
  static const char* floor_env = getenv("D2MI_TOPK_FLOOR");  // "0": radix passes only (A/B)
  if (sampled_floor && key_mode == 1 && max_len > kCap && !(floor_env && floor_env[0] == '0')) {
    const int runs = (max_len + kSampleStride - 1) / kSampleStride;
    hipLaunchKernelGGL(topk_sample_kernel, dim3((runs + kSampleRunsPerWg - 1) / kSampleRunsPerWg, S),
                       dim3(kThreads), 0, stream, values, seg_start, seg_len, st, hist);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(topk_floor_kernel, dim3(S), dim3(kThreads), 0, stream, st, hist, seg_len);
    D2MI_LAUNCH_CHECK();
    if (big)
      hipLaunchKernelGGL(topk_floor_collect_kernel<16>, dim3(gx, S), dim3(kThreads), 0, stream,
                         values, seg_start, seg_len, st, fbuf);
    else
      hipLaunchKernelGGL(topk_floor_collect_kernel<4>, dim3(gx, S), dim3(kThreads), 0, stream,
                         values, seg_start, seg_len, st, fbuf);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(topk_floor_decide_kernel, dim3(S), dim3(kThreads), 0, stream, st, fbuf,
                       candA);
    D2MI_LAUNCH_CHECK();
  }
  for (int pass = 0; pass < 3; ++pass) {
    if (big)
      hipLaunchKernelGGL(topk_hist_kernel<16>, dim3(gx, S), dim3(kThreads), 0, stream, values,
                         seg_start, seg_len, st, hist, pass);
    else
      hipLaunchKernelGGL(topk_hist_kernel<4>, dim3(gx, S), dim3(kThreads), 0, stream, values,
                         seg_start, seg_len, st, hist, pass);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(topk_select_kernel, dim3(S), dim3(kThreads), 0, stream, st, hist, pass,
                       key_mode);
    D2MI_LAUNCH_CHECK();
  }
  if (big)
    hipLaunchKernelGGL(topk_collect_kernel<16>, dim3(gx, S), dim3(kThreads), 0, stream, values,
                       seg_start, seg_len, st, candA, candB, key_mode);
  else
    hipLaunchKernelGGL(topk_collect_kernel<4>, dim3(gx, S), dim3(kThreads), 0, stream, values,
                       seg_start, seg_len, st, candA, candB, key_mode);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(topk_resolve_kernel, dim3(S), dim3(1024), 0, stream, values, seg_start,
                     seg_len, st, candA, candB, key_mode);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(topk_rank_kernel, dim3(kCap / kRankI, S), dim3(kRankT),
                     kCap * sizeof(uint64_t), stream, candA, st, k, key_mode, vals_out, idx_out,
                     count_out);
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
