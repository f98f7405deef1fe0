// Fused subsample_labels (lib/modeling/sampling.py subsample_labels as
// rpn_outputs.py:278-283 and roi_heads.py:160-216 call it): per row of
// labels, a uniformly random subset of min(num_pos, #positive) positives
// (label not -1 and not bg) and min(num_samples - that, #negative) negatives
// (label == bg), plus -- for the ROI heads -- the selected indices in
// fg-first, index order.  The reference shuffles (tf.random_shuffle) and
// takes the first k; here each masked element's rank r among its kind (a
// scan) is mapped through a keyed pseudo-random bijection of [0, n) (a
// 6-round Feistel network on the next power of 4, cycle-walked into range)
// and kept iff perm(r) < k: exactly k of the n, a different uniform draw.
// Three launches per call (block counts, selection + selected counts, order)
// replace ~50 small torch / top-k launches per training step.
#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kSampleBlock = 1024;  // elements per workgroup (256 threads x 4)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // lowbias32 finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Keyed bijection of [0, n) (n >= 1): a 6-round Feistel network on 2 * hb
// bits (2^(2 hb) >= n) whose round keys come from the whole 64-bit seed and
// the row (round_keys), cycle-walked into range (expected < 4 steps: the
// domain is < 4n).  Six rounds (Luby-Rackoff needs 4 for a pseudo-random
// permutation; the extra two cost a few VALU per element) with independent
// round keys, not one 32-bit key replayed per round.
constexpr int kFeistelRounds = 6;
struct RoundKeys {
  uint32_t k[kFeistelRounds];
};
__device__ __forceinline__ RoundKeys round_keys(uint64_t seed, uint32_t stream) {
  RoundKeys rk;
  const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < kFeistelRounds; ++i)
    rk.k[i] = mix32(lo ^ mix32(hi + 0x9e3779b9u * (uint32_t)(i + 1) + mix32(stream)));
  return rk;
}
__device__ __forceinline__ uint32_t perm(uint32_t x, uint32_t n, const RoundKeys& rk) {
  int hb = 1;
  while ((1u << (2 * hb)) < n) ++hb;
  const uint32_t mask = (1u << hb) - 1u;
  do {
    uint32_t l = x >> hb, r = x & mask;
#pragma unroll
    for (int k = 0; k < kFeistelRounds; ++k) {
      const uint32_t t = l ^ (mix32(r ^ rk.k[k]) & mask);
      l = r;
      r = t;
    }
    x = (l << hb) | r;
  } while (x >= n);
  return x;
}

__device__ __forceinline__ int kind_of(int64_t lab, int64_t bg) {  // 1 pos, 2 neg, 0 neither
  return lab == bg ? 2 : (lab != -1 ? 1 : 0);
}

// Block-wide exclusive prefix of (a, b) over the 256 threads; returns the
// thread's offsets and the block totals.
__device__ __forceinline__ void block_scan2(int a, int b, int& oa, int& ob, int& ta, int& tb,
                                            int* s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int xa = a, xb = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int ya = __shfl_up(xa, d), yb = __shfl_up(xb, d);
    if (lane >= d) {
      xa += ya;
      xb += yb;
    }
  }
  if (lane == 63) {
    s[w] = xa;
    s[4 + w] = xb;
  }
  __syncthreads();
  int pa = 0, pb = 0;
  ta = tb = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < w) {
      pa += s[k];
      pb += s[4 + k];
    }
    ta += s[k];
    tb += s[4 + k];
  }
  oa = pa + xa - a;
  ob = pb + xb - b;
  __syncthreads();
}

// Pass 1: positives / negatives per block.
__global__ __launch_bounds__(256) void sample_count_kernel(const int64_t* __restrict__ labels,
                                                           int P, int64_t bg, int nblk,
                                                           int2* __restrict__ cnt) {
  __shared__ int s[8];
  const int row = blockIdx.y, blk = blockIdx.x;
  const int64_t* lab = labels + (size_t)row * P;
  int a = 0, b = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = blk * kSampleBlock + u * 256 + threadIdx.x;
    if (i < P) {
      const int k = kind_of(lab[i], bg);
      a += k == 1;
      b += k == 2;
    }
  }
  int oa, ob, ta, tb;
  block_scan2(a, b, oa, ob, ta, tb, s);
  if (threadIdx.x == 0) cnt[(size_t)row * nblk + blk] = make_int2(ta, tb);
}

// The row's offsets before block blk and its totals (every block re-sums
// the row's block counts: nblk is a few hundred at most).
__device__ __forceinline__ void row_offsets(const int2* __restrict__ cnt, int nblk, int blk,
                                            int& ba, int& bb, int& na, int& nb, int* s) {
  int pa = 0, pb = 0, ta = 0, tb = 0;
  for (int j = threadIdx.x; j < nblk; j += 256) {
    const int2 c = cnt[j];
    ta += c.x;
    tb += c.y;
    if (j < blk) {
      pa += c.x;
      pb += c.y;
    }
  }
  int o0, o1;
  block_scan2(pa, pb, o0, o1, ba, bb, s);
  block_scan2(ta, tb, o0, o1, na, nb, s);
}

// Pass 2: each element's rank among its kind -> selected iff perm(rank) < k;
// the masks, and the selected counts per block (for the order pass).
__global__ __launch_bounds__(256) void sample_select_kernel(
    const int64_t* __restrict__ labels, int P, int64_t bg, int nblk, int num_samples,
    int num_pos, const int64_t* __restrict__ seed, const int2* __restrict__ cnt,
    uint8_t* __restrict__ pos_out, uint8_t* __restrict__ neg_out, int2* __restrict__ sel_cnt) {
  __shared__ int s[8];
  const int row = blockIdx.y, blk = blockIdx.x;
  const int64_t* lab = labels + (size_t)row * P;
  int ba, bb, na, nb;
  row_offsets(cnt + (size_t)row * nblk, nblk, blk, ba, bb, na, nb, s);
  const int kp = min(num_pos, na);
  const int kn = min(num_samples - kp, nb);
  const uint64_t sd = (uint64_t)seed[0];
  const RoundKeys key_p = round_keys(sd, 2u * row), key_n = round_keys(sd, 2u * row + 1u);
  int kind[4];
  int a = 0, b = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = blk * kSampleBlock + threadIdx.x * 4 + u;  // 4 consecutive per thread
    kind[u] = i < P ? kind_of(lab[i], bg) : 0;
    a += kind[u] == 1;
    b += kind[u] == 2;
  }
  int oa, ob, ta, tb;
  block_scan2(a, b, oa, ob, ta, tb, s);
  int ra = ba + oa, rb = bb + ob;
  int sa = 0, sb = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = blk * kSampleBlock + threadIdx.x * 4 + u;
    bool p = false, q = false;
    if (kind[u] == 1) {
      p = na <= kp || perm((uint32_t)ra, (uint32_t)na, key_p) < (uint32_t)kp;
      ++ra;
    } else if (kind[u] == 2) {
      q = nb <= kn || perm((uint32_t)rb, (uint32_t)nb, key_n) < (uint32_t)kn;
      ++rb;
    }
    sa += p;
    sb += q;
    if (i < P) {
      pos_out[(size_t)row * P + i] = p;
      neg_out[(size_t)row * P + i] = q;
    }
  }
  int o0, o1, t0, t1;
  block_scan2(sa, sb, o0, o1, t0, t1, s);
  if (threadIdx.x == 0 && sel_cnt) sel_cnt[(size_t)row * nblk + blk] = make_int2(t0, t1);
}

// Pass 3 (optional): order[row][slot] = the selected indices, positives first,
// each kind in index order; slots past the selection: index 0, valid 0.
__global__ __launch_bounds__(256) void sample_order_kernel(
    const uint8_t* __restrict__ pos, const uint8_t* __restrict__ neg, int P, int nblk, int S,
    const int2* __restrict__ sel_cnt, int64_t* __restrict__ order, uint8_t* __restrict__ valid) {
  __shared__ int s[8];
  const int row = blockIdx.y, blk = blockIdx.x;
  int ba, bb, na, nb;
  row_offsets(sel_cnt + (size_t)row * nblk, nblk, blk, ba, bb, na, nb, s);
  bool p[4], q[4];
  int a = 0, b = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = blk * kSampleBlock + threadIdx.x * 4 + u;
    p[u] = i < P && pos[(size_t)row * P + i];
    q[u] = i < P && neg[(size_t)row * P + i];
    a += p[u];
    b += q[u];
  }
  int oa, ob, ta, tb;
  block_scan2(a, b, oa, ob, ta, tb, s);
  int ra = ba + oa, rb = na + bb + ob;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = blk * kSampleBlock + threadIdx.x * 4 + u;
    int slot = -1;
    if (p[u]) slot = ra++;
    else if (q[u]) slot = rb++;
    if (slot >= 0 && slot < S) {
      order[(size_t)row * S + slot] = i;
      valid[(size_t)row * S + slot] = 1;
    }
  }
  // the unfilled tail (one block per row writes it)
  if (blk == 0)
    for (int j = na + nb + threadIdx.x; j < S; j += 256) {
      order[(size_t)row * S + j] = 0;
      valid[(size_t)row * S + j] = 0;
    }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_subsample_workspace_size(int N, int P) {
  if (N <= 0 || P <= 0) return 0;
  const size_t nblk = (size_t)(P + kSampleBlock - 1) / kSampleBlock;
  return 2 * (size_t)N * nblk * sizeof(int2) + 16;
}

extern "C" int d2mi_subsample(const int64_t* labels, int N, int P, long long bg_label,
                              int num_samples, int num_pos, const int64_t* seed, uint8_t* pos_out,
                              uint8_t* neg_out, int64_t* order_out, uint8_t* order_valid, int S,
                              void* workspace, size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N >= 0 && P >= 0 && num_samples >= 0 && num_pos >= 0 && num_pos <= num_samples,
               "subsample: bad sizes (N=%d P=%d num_samples=%d num_pos=%d)", N, P, num_samples,
               num_pos);
  D2MI_REQUIRE(!order_out || (order_valid && S >= 0), "subsample: order needs its valid mask");
  if (N == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (P == 0) {
    if (order_out && S > 0) {
      D2MI_REQUIRE(fill_bytes(order_out, (size_t)N * S * sizeof(int64_t), 0, st) == 0, "fill failed");
      D2MI_REQUIRE(fill_bytes(order_valid, (size_t)N * S, 0, st) == 0, "fill failed");
    }
    return 0;
  }
  D2MI_REQUIRE(labels && seed && pos_out && neg_out, "subsample: null operand");
  const int nblk = (P + kSampleBlock - 1) / kSampleBlock;
  D2MI_REQUIRE(workspace && workspace_bytes >= d2mi_subsample_workspace_size(N, P),
               "subsample workspace too small");
  int2* cnt = static_cast<int2*>(workspace);
  int2* sel = cnt + (size_t)N * nblk;
  const dim3 grid(nblk, N);
  hipLaunchKernelGGL(sample_count_kernel, grid, dim3(256), 0, st, labels, P, (int64_t)bg_label,
                     nblk, cnt);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(sample_select_kernel, grid, dim3(256), 0, st, labels, P, (int64_t)bg_label,
                     nblk, num_samples, num_pos, seed, cnt, pos_out, neg_out,
                     order_out ? sel : nullptr);
  D2MI_LAUNCH_CHECK();
  if (order_out && S > 0) {
    hipLaunchKernelGGL(sample_order_kernel, grid, dim3(256), 0, st, pos_out, neg_out, P, nblk, S,
                       sel, order_out, order_valid);
    D2MI_LAUNCH_CHECK();
  }
  return 0;
}
