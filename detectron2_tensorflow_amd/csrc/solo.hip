// SOLOv2 inference tail (lib/modeling/single_stage_heads/solo_v2.py:476-627)
// and the TF ResizeBilinear kernel its head resamples with
// (lib/layers/functional.py:9-36 -> tf.compat.v2.image.resize, bilinear).
//
// Pipeline (one host read of the live-cell counts between stage 1 and 2):
//   1 d2mi_solo_cells        sigmoid + point NMS of every category map
//                            (solo_v2.py:29-40, :267-269) into the dense
//                            [N, T, K] score array the reference flattens
//                            (:567-586), and the "live" grid cells (any score
//                            > SCORE_THRESH_TEST), compacted in cell order.
//   - the dynamic 1x1 conv (:499-511) runs on the MFMA GEMM (caller), ONE row
//     per live cell instead of one per (cell, class) candidate: the mask of a
//     candidate depends on its cell only, so the rows are shared.
//   2 d2mi_solo_mask_stats   per row: sum_masks = #(sigmoid > MASK_THRESH)
//                            (:513-517), sum of those sigmoids (:529-531).
//   3 d2mi_solo_select       candidate scores score * (sum_sig / sum_masks)
//                            where score > SCORE_THRESH and sum_masks >
//                            stride (:482-532), -inf elsewhere; exact top-k
//                            (tf.nn.top_k, ties by candidate order
//                            (cell, class)) (:535-539); the top-k binary masks,
//                            bit-packed (64 pixels per word), for Matrix NMS.
//   - d2mi_solo_matrix_nms   (:541-545, nms.py:29-83) on the bits: the
//                            intersection GEMM of 0/1 masks is AND + popcount
//                            (exact integers, 1/32 of the f32 bytes).
//   4 d2mi_solo_finalize     decayed score > UPDATE_SCORE_THRESH, in order,
//                            pad / clip to DETECTIONS_PER_IMAGE (:547-557);
//                            masks resized to the padded image with TF
//                            bilinear, > MASK_THRESH (:598-602), written as
//                            uint8; boxes from the masks (:604-623).
// Every float expression follows the reference's op order (compiled with
// -ffp-contract=off).
#include <limits.h>
#include <math.h>

#include <algorithm>

#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

// ------------------------------------------------------------ ResizeBilinear
// TF 1.15 resize_bilinear_op.cc: compute_interpolation_weights with
// HalfPixelScaler ((x + 0.5) * scale - 0.5) or LegacyScaler (x * scale);
// lower = max(floor(in), 0), upper = min(ceil(in), in_size - 1),
// lerp = in - floor(in); compute_lerp: top = tl + (tr - tl) * xl,
// bottom = bl + (br - bl) * xl, out = top + (bottom - top) * yl.
struct Interp {
  int lo, hi;
  float lerp;
};

__device__ __forceinline__ Interp interp_at(int i, float scale, int in_size, int half_pixel) {
  const float in = half_pixel ? ((float)i + 0.5f) * scale - 0.5f : (float)i * scale;
  const float in_f = floorf(in);
  Interp r;
  r.lo = max((int)in_f, 0);
  r.hi = min((int)ceilf(in), in_size - 1);
  r.lerp = in - in_f;
  return r;
}

__device__ __forceinline__ float tf_lerp(float tl, float tr, float bl, float br, float xl,
                                         float yl) {
  const float top = tl + (tr - tl) * xl;
  const float bottom = bl + (br - bl) * xl;
  return top + (bottom - top) * yl;
}

template <bool VEC4>
__global__ __launch_bounds__(256) void resize_bilinear_kernel(const float* __restrict__ x,
                                                              float* __restrict__ y, int N, int H,
                                                              int W, int C, int OH, int OW,
                                                              float sh, float sw, int half_pixel) {
  const int CV = VEC4 ? C / 4 : C;
  const size_t total = (size_t)N * OH * OW * CV;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
       e += (size_t)gridDim.x * blockDim.x) {
    const int cv = (int)(e % CV);
    size_t r = e / CV;
    const int ox = (int)(r % OW);
    r /= OW;
    const int oy = (int)(r % OH);
    const int n = (int)(r / OH);
    const Interp iy = interp_at(oy, sh, H, half_pixel);
    const Interp ix = interp_at(ox, sw, W, half_pixel);
    const float* b = x + (size_t)n * H * W * C;
    const size_t tl = ((size_t)iy.lo * W + ix.lo) * C, tr = ((size_t)iy.lo * W + ix.hi) * C;
    const size_t bl = ((size_t)iy.hi * W + ix.lo) * C, br = ((size_t)iy.hi * W + ix.hi) * C;
    if (VEC4) {
      const int c = cv * 4;
      const float4 a = *(const float4*)(b + tl + c), bb = *(const float4*)(b + tr + c);
      const float4 cc = *(const float4*)(b + bl + c), d = *(const float4*)(b + br + c);
      float4 o;
      o.x = tf_lerp(a.x, bb.x, cc.x, d.x, ix.lerp, iy.lerp);
      o.y = tf_lerp(a.y, bb.y, cc.y, d.y, ix.lerp, iy.lerp);
      o.z = tf_lerp(a.z, bb.z, cc.z, d.z, ix.lerp, iy.lerp);
      o.w = tf_lerp(a.w, bb.w, cc.w, d.w, ix.lerp, iy.lerp);
      *(float4*)(y + e * 4) = o;
    } else {
      y[e] = tf_lerp(b[tl + cv], b[tr + cv], b[bl + cv], b[br + cv], ix.lerp, iy.lerp);
    }
  }
}

// CalculateResizeScale (TF image_resizer_state.h), float division.
static float resize_scale(int in, int out, int align_corners) {
  return (align_corners && out > 1) ? (float)(in - 1) / (float)(out - 1)
                                    : (float)in / (float)out;
}

__device__ __forceinline__ float sigmoidf_tf(float v) { return 1.f / (1.f + expf(-v)); }

// --------------------------------------------------------------- level table
constexpr int kMaxLevels = 8;
struct SoloLevels {
  const float* cate[kMaxLevels];  // [N, S, S, K] logits
  int S[kMaxLevels];
  int off[kMaxLevels + 1];        // first cell of each level; off[L] = T
  float stride[kMaxLevels];
  int L;
};

__device__ __forceinline__ int level_of(const SoloLevels& lv, int c) {
  int l = 0;
  while (l + 1 < lv.L && c >= lv.off[l + 1]) ++l;
  return l;
}

// ------------------------------------------------------------------- stage 1
// One wave per (image, cell): sigmoid of the cell's K logits and of its up,
// left and up-left neighbours (out-of-range = the zero padding, never above a
// sigmoid), keep = (p == 2x2 window max) (point_nms, solo_v2.py:29-40),
// probs = p * keep.  live_row[n, c] = any kept prob > thr (0 / 1 flag for
// the compaction that follows).
__global__ __launch_bounds__(256) void solo_cells_kernel(SoloLevels lv, int N, int K, float thr,
                                                         float* __restrict__ probs,
                                                         int32_t* __restrict__ flag) {
  const int T = lv.off[lv.L];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= N * T) return;
  const int n = wave / T, c = wave % T;
  const int l = level_of(lv, c);
  const int S = lv.S[l];
  const int loc = c - lv.off[l];
  const int i = loc / S, j = loc % S;
  const float* base = lv.cate[l] + (size_t)n * S * S * K;
  bool any = false;
  for (int k = lane; k < K; k += 64) {
    const float v = sigmoidf_tf(base[((size_t)i * S + j) * K + k]);
    float m = v;
    if (i > 0) m = fmaxf(m, sigmoidf_tf(base[((size_t)(i - 1) * S + j) * K + k]));
    if (j > 0) m = fmaxf(m, sigmoidf_tf(base[((size_t)i * S + j - 1) * K + k]));
    if (i > 0 && j > 0) m = fmaxf(m, sigmoidf_tf(base[((size_t)(i - 1) * S + j - 1) * K + k]));
    const float out = v * (v == m ? 1.f : 0.f);
    probs[((size_t)n * T + c) * K + k] = out;
    any |= out > thr;
  }
  const uint64_t b = __ballot(any);
  if (lane == 0) flag[(size_t)n * T + c] = b ? 1 : 0;
}

// One block per image: stable compaction of the live cells.
__global__ __launch_bounds__(1024) void solo_live_kernel(int T, int32_t* __restrict__ live_row,
                                                         int32_t* __restrict__ live_cells,
                                                         int32_t* __restrict__ live_count) {
  __shared__ int wsum[16];
  __shared__ int base_sh;
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) base_sh = 0;
  __syncthreads();
  for (int c0 = 0; c0 < T; c0 += blockDim.x) {
    const int c = c0 + threadIdx.x;
    const bool live = c < T && live_row[(size_t)n * T + c] != 0;
    const uint64_t bal = __ballot(live);
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int before = base_sh, total = 0;
    for (int w = 0; w < nw; ++w) {
      if (w < wv) before += wsum[w];
      total += wsum[w];
    }
    const int pos = before + __popcll(bal & ((1ull << lane) - 1ull));
    if (c < T) {
      live_row[(size_t)n * T + c] = live ? pos : -1;
      if (live) live_cells[(size_t)n * T + pos] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) base_sh += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) live_count[n] = base_sh;
}

// ------------------------------------------------------------------- stage 2
// One block per dynamic-conv row: the count of sigmoid(logit) > thr and the
// sum of those sigmoids, fixed-order (deterministic) reduction.
__global__ __launch_bounds__(256) void solo_mask_stats_kernel(const float* __restrict__ logits,
                                                              int P, float thr,
                                                              float* __restrict__ sum_masks,
                                                              float* __restrict__ sum_scores) {
  __shared__ int rc[256];
  __shared__ float rs[256];
  const size_t r = blockIdx.x;
  const float* row = logits + r * P;
  int cnt = 0;
  float acc = 0.f;
  if ((P & 3) == 0) {
    // four float4 loads in flight per thread, consumed in the same order
    const int step = blockDim.x * 4;
    for (int p0 = threadIdx.x * 4; p0 < P; p0 += 4 * step) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = p0 + u * step;
        v[u] = p < P ? *(const float4*)(row + p) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (p0 + u * step >= P) break;
        const float s[4] = {sigmoidf_tf(v[u].x), sigmoidf_tf(v[u].y), sigmoidf_tf(v[u].z),
                            sigmoidf_tf(v[u].w)};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (s[q] > thr) {
            ++cnt;
            acc += s[q];
          }
      }
    }
  } else {
    for (int p = threadIdx.x; p < P; p += blockDim.x) {
      const float s = sigmoidf_tf(row[p]);
      if (s > thr) {
        ++cnt;
        acc += s;
      }
    }
  }
  rc[threadIdx.x] = cnt;
  rs[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      rc[threadIdx.x] += rc[threadIdx.x + o];
      rs[threadIdx.x] += rs[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sum_masks[r] = (float)rc[0];
    sum_scores[r] = rs[0];
  }
}

// ------------------------------------------------------------------- stage 3
// Dense candidate scores [N, T*K]: the reference's keep_inds (score > thr, in
// (cell, class) order) filtered by sum_masks > stride and rescored by the
// mask score; everything else -inf (never selected: the top-k takes at most
// the per-image valid count).
__global__ __launch_bounds__(256) void solo_cand_kernel(
    SoloLevels lv, const float* __restrict__ probs, const int32_t* __restrict__ live_row,
    const int32_t* __restrict__ row_off, const float* __restrict__ sum_masks,
    const float* __restrict__ sum_scores, int N, int K, float thr, float* __restrict__ dense,
    int32_t* __restrict__ valid_count, int64_t* __restrict__ seg_start,
    int32_t* __restrict__ seg_len) {
  const int T = lv.off[lv.L];
  const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (e < (size_t)N) {
    seg_start[e] = (int64_t)e * T * K;
    seg_len[e] = T * K;
  }
  if (e >= (size_t)N * T * K) return;
  const int n = (int)(e / ((size_t)T * K));
  const int c = (int)((e / K) % T);
  const int row = live_row[(size_t)n * T + c];
  float out = -INFINITY;
  bool valid = false;
  if (row >= 0) {
    const float p = probs[e];
    const int gr = row_off[n] + row;
    const float sm = sum_masks[gr];
    const float stride = lv.stride[level_of(lv, c)];
    if (p > thr && sm > stride) {
      valid = true;
      out = p * (sum_scores[gr] / sm);
    }
  }
  dense[e] = out;
  const uint64_t b = __ballot(valid);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&valid_count[n], (int)__popcll(b));
}

// Bit-packed binary masks, classes and sum_masks of the top-k candidates
// (the Matrix NMS inputs): bit p of word p / 64 of row t is
// sigmoid(logit[p]) > thr; one wave builds a 64-pixel word with one ballot
// over 64 coalesced logits.  Rows past the image's count are zero masks with
// classes -1 - t (distinct from every real class and from each other: their
// IoU with any row is zero, so they decay nothing and the real rows are
// unchanged).
__global__ __launch_bounds__(256) void solo_gather_kernel(
    const int32_t* __restrict__ top_idx, const int32_t* __restrict__ top_count,
    const int32_t* __restrict__ live_row, const int32_t* __restrict__ row_off,
    const float* __restrict__ logits, const float* __restrict__ sum_masks, int T, int K, int P,
    int k, int W64, float thr, int64_t* __restrict__ classes, float* __restrict__ top_sum,
    uint64_t* __restrict__ bits) {
  const int t = blockIdx.x, n = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = t < top_count[n];
  uint64_t* dst = bits + ((size_t)n * k + t) * W64;
  if (!live) {
    for (int w = threadIdx.x; w < W64; w += blockDim.x) dst[w] = 0ull;
    if (threadIdx.x == 0) {
      classes[(size_t)n * k + t] = -1 - t;
      top_sum[(size_t)n * k + t] = 0.f;
    }
    return;
  }
  const int idx = top_idx[(size_t)n * k + t];
  const int cell = idx / K, cls = idx % K;
  const int gr = row_off[n] + live_row[(size_t)n * T + cell];
  const float* src = logits + (size_t)gr * P;
  // 8 words per wave per step, all loads in flight before the sigmoids (one
  // dependent load per word made this latency-bound)
  const int nw = blockDim.x >> 6;
  for (int w0 = wv * 8; w0 < W64; w0 += nw * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = (w0 + u) * 64 + lane;
      v[u] = (w0 + u < W64 && p < P) ? src[p] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = (w0 + u) * 64 + lane;
      const bool on = w0 + u < W64 && p < P && sigmoidf_tf(v[u]) > thr;
      const uint64_t b = __ballot(on);
      if (lane == 0 && w0 + u < W64) dst[w0 + u] = b;
    }
  }
  if (threadIdx.x == 0) {
    classes[(size_t)n * k + t] = cls;
    top_sum[(size_t)n * k + t] = sum_masks[gr];
  }
}

// ---------------------------------------------------------- Matrix NMS (0/1)
// matrix_nms (lib/layers/nms.py:29-83) on bit-packed binary masks: the
// intersection counts inter = M M^T are popcounts of AND-ed words (exact
// integers; the reference's float matmul of 0/1 masks gives the same
// values), tiled 64 x 64 rows per workgroup over a slice of the words, the
// slices summed with integer atomics (exact in any order).  Only the upper
// triangle (i < j) is used by the IoU.
constexpr int kMT = 64, kMW = 32;  // rows per tile side, words per LDS stage

__global__ __launch_bounds__(256) void solo_inter_kernel(const uint64_t* __restrict__ bits, int k,
                                                         int W64, int words_per_split,
                                                         int32_t* __restrict__ inter) {
  __shared__ uint64_t As[kMW][kMT + 1];
  __shared__ uint64_t Bs[kMW][kMT + 1];
  const int ti = blockIdx.x, tj = blockIdx.y;  // tile row / column
  const int n = blockIdx.z / ((W64 + words_per_split - 1) / words_per_split);
  const int split = blockIdx.z % ((W64 + words_per_split - 1) / words_per_split);
  if (ti > tj) return;  // lower tiles never read
  const int w0 = split * words_per_split, w1 = min(W64, w0 + words_per_split);
  const uint64_t* base = bits + (size_t)n * k * W64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16 threads, 4 x 4 outputs each
  int acc[4][4] = {};
  for (int ws = w0; ws < w1; ws += kMW) {
    for (int e = threadIdx.x; e < kMW * kMT; e += 256) {
      const int r = e / kMW, w = e % kMW;
      const int ra = ti * kMT + r, rb = tj * kMT + r, ww = ws + w;
      As[w][r] = (ra < k && ww < w1) ? base[(size_t)ra * W64 + ww] : 0ull;
      Bs[w][r] = (rb < k && ww < w1) ? base[(size_t)rb * W64 + ww] : 0ull;
    }
    __syncthreads();
#pragma unroll 4
    for (int w = 0; w < kMW; ++w) {
      uint64_t a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = As[w][ty * 4 + q];
        b[q] = Bs[w][tx * 4 + q];
      }
#pragma unroll
      for (int qi = 0; qi < 4; ++qi)
#pragma unroll
        for (int qj = 0; qj < 4; ++qj) acc[qi][qj] += __popcll(a[qi] & b[qj]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int qi = 0; qi < 4; ++qi)
#pragma unroll
    for (int qj = 0; qj < 4; ++qj) {
      const int i = ti * kMT + ty * 4 + qi, j = tj * kMT + tx * 4 + qj;
      if (i < k && j < k && i < j && acc[qi][qj])
        atomicAdd(&inter[((size_t)n * k + i) * k + j], acc[qi][qj]);
    }
}

// r6: the same counts on the int8 MFMA (v_mfma_i32_32x32x32_i8: exact i32
// accumulation of 0/1 products).  One wave owns a 64 x 64 output tile of an
// upper-triangle tile pair (ti <= tj) over a slice of the pixel words (2 x 2
// MFMA tiles of 32 x 32); a k-step is 32 pixels.  Lane l (row r = l & 31,
// half h = l >> 5) expands bits 16h .. 16h+15 of its row's 32-pixel chunk to
// 16 bytes of 0 / 1 for both operands: the A and B fragments use the same
// lane / element -> k assignment, so every product pairs one pixel of row i
// with the SAME pixel of row j and the sum over the 32 is popcount(a & b),
// whatever the hardware's k order inside the step.
//
// The wave's 128 rows (64 A, 64 B) come in chunks of 16 words (1,024
// pixels, one 128-B line per row): 32 coalesced 8-B loads per lane (4 whole
// lines per instruction) land in registers while the previous chunk is
// multiplied out of the wave's LDS image (rows padded to 136 B: the 32 rows a
// read touches fall on distinct banks), then go to LDS.  Partials per pixel
// slice go to a workspace slab (ints: summed exactly in the reduce launch).
constexpr int kIT = 64;                        // output tile side per wave
constexpr int kIWords = 16;                    // pixel words per chunk
constexpr int kIRowB = kIWords * 8 + 8;        // LDS bytes per row (padded)
constexpr int kIWaveB = 2 * kIT * kIRowB;      // LDS bytes per wave
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 16 bits -> 16 bytes of 0 / 1 (bit b -> byte b): per nibble x,
// x * (1 + 2^7 + 2^14 + 2^21) puts bit i at bit 8i with no carries.
__device__ __forceinline__ v4i expand16(uint32_t x) {
  v4i r;
  r[0] = (int)(__umul24(x & 0xFu, 0x204081u) & 0x01010101u);
  r[1] = (int)(__umul24((x >> 4) & 0xFu, 0x204081u) & 0x01010101u);
  r[2] = (int)(__umul24((x >> 8) & 0xFu, 0x204081u) & 0x01010101u);
  r[3] = (int)(__umul24((x >> 12) & 0xFu, 0x204081u) & 0x01010101u);
  return r;
}

// The same by table (r6): an LDS table of the 256 byte values' 8-byte
// expansions, two lookups per 16 bits (4 VALU + 2 LDS reads instead of 12 VALU)
__device__ __forceinline__ v4i expand16_lut(uint32_t x, const uint2* __restrict__ lut) {
  const uint2 lo = lut[x & 0xFFu], hi = lut[(x >> 8) & 0xFFu];
  v4i r;
  r[0] = (int)lo.x;
  r[1] = (int)lo.y;
  r[2] = (int)hi.x;
  r[3] = (int)hi.y;
  return r;
}

// upper-triangle tile pair u -> (ti, tj), ti <= tj, row-major over ti
__device__ __forceinline__ void tri_pair(int u, int T, int& ti, int& tj) {
  int i = 0, left = T;
  while (u >= left) {
    u -= left;
    ++i;
    --left;
  }
  ti = i;
  tj = i + u;
}

// Workgroup: kIWaves waves on ONE tile pair, each over its own run of chunks
// (two waves per SIMD: one wave's expansions beside the other's MFMAs); their
// accumulators are summed in LDS (integer adds: exact in any order) and one
// partial tile per workgroup goes to the workspace.
constexpr int kIWaves = 8;

template <bool LUT>
__global__ __launch_bounds__(64 * kIWaves) void solo_inter_mfma_kernel(
    const uint64_t* __restrict__ bits, int N, int k, int W64, int T, int groups,
    int words_per_wave, int32_t* __restrict__ part, float* __restrict__ comp) {
  extern __shared__ __align__(16) unsigned char ism[];
  __shared__ uint2 lut[256];
  if (LUT) {
    for (int v = threadIdx.x; v < 256; v += 64 * kIWaves) {
      const v4i e = expand16((uint32_t)v);
      lut[v] = make_uint2((uint32_t)e[0], (uint32_t)e[1]);
    }
    __syncthreads();
  }
  if (blockIdx.x == 0)  // (the reduce launch max-folds the compensation into it)
    for (int e = threadIdx.x; e < N * k; e += 64 * kIWaves) comp[e] = 0.f;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int tri = T * (T + 1) / 2;
  const int grp = blockIdx.x % groups, u = (blockIdx.x / groups) % tri, n = blockIdx.x / (groups * tri);
  unsigned char* img = ism + (size_t)wv * kIWaveB;
  int ti, tj;
  tri_pair(u, T, ti, tj);
  const int r = lane & 31, h = lane >> 5;
  const uint64_t* base = bits + (size_t)n * k * W64;
  // load slot q (0..31) of a chunk: image row 4q + (lane >> 4), word lane & 15
  // (image rows 0..63 = A rows ti * 64 + ..., 64..127 = B rows tj * 64 + ...)
  const int lw = lane & 15;
  const int slice = grp * kIWaves + wv;
  const int w0 = min(W64, slice * words_per_wave), w1 = min(W64, w0 + words_per_wave);
  auto src_of = [&](int q) -> const uint64_t* {
    const int ir = 4 * q + (lane >> 4);
    const int row = (ir < kIT ? ti * kIT + ir : tj * kIT + ir - kIT);
    return row < k ? base + (size_t)row * W64 : nullptr;
  };
  v16i acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0;
  uint64_t pre[32];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const uint64_t* p = src_of(q);
      const int w = c0 + lw;
      pre[q] = (p != nullptr && w < w1) ? p[w] : 0ull;
    }
  };
  load_chunk(w0);
  for (int c0 = w0; c0 < w1; c0 += kIWords) {
    // the chunk's words into the wave's image, then the next chunk's loads
#pragma unroll
    for (int q = 0; q < 32; ++q)
      *reinterpret_cast<uint64_t*>(img + (size_t)(4 * q + (lane >> 4)) * kIRowB + 8 * lw) = pre[q];
    __builtin_amdgcn_wave_barrier();
    if (c0 + kIWords < w1) load_chunk(c0 + kIWords);
    const int nks = min(kIWords, w1 - c0) * 2;  // 32-pixel k-steps in this chunk
#pragma unroll 2
    for (int ks = 0; ks < nks; ks += 2) {
      uint64_t d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)  // rows r, 32 + r (A), 64 + r, 96 + r (B)
        d[q] = *reinterpret_cast<const uint64_t*>(img + (size_t)(32 * q + r) * kIRowB + 4 * ks);
#pragma unroll
      for (int half32 = 0; half32 < 2; ++half32) {
        v4i fr[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          fr[q] = LUT ? expand16_lut((uint32_t)(d[q] >> (32 * half32 + 16 * h)) & 0xFFFFu, lut)
                      : expand16((uint32_t)(d[q] >> (32 * half32 + 16 * h)) & 0xFFFFu);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[a], fr[2 + b], acc[a][b], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  // the waves' tiles summed in LDS (the staging images are free now), then
  // stored row-major.  C / D layout (dtype-independent on gfx950):
  // col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
  int32_t* red = reinterpret_cast<int32_t*>(ism);
  __syncthreads();
  for (int e = threadIdx.x; e < kIT * kIT; e += 64 * kIWaves) red[e] = 0;
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h, col = 32 * b + r;
        atomicAdd(&red[row * kIT + col], acc[a][b][e]);
      }
  __syncthreads();
  int32_t* out = part + (((size_t)grp * N + n) * tri + u) * (kIT * kIT);
  for (int e = threadIdx.x; e < kIT * kIT; e += 64 * kIWaves) out[e] = red[e];
}

// The groups' partial tiles summed (ints: exact in any order) into the IoU
// matrix TRANSPOSED, iouT[n][j][i] = iou(i, j) of solo_iou below (0 unless
// i < j and the classes match), so that the compensation / decay passes read
// rows.  A workgroup takes 16 columns j of one (image, tile pair): the
// partials are read row-major (coalesced), transposed through LDS and stored
// as rows of iouT; a pair ti < tj also zeroes its mirror (i > j).
constexpr int kRedCols = 16;
template <int TS>
__global__ __launch_bounds__(256) void solo_inter_reduce_kernel(
    const int32_t* __restrict__ part, int N, int k, int T, int groups,
    const float* __restrict__ sums, const int64_t* __restrict__ cls, float* __restrict__ iouT,
    float* __restrict__ comp) {
  __shared__ float tile[kRedCols][TS + 1];
  const int tri = T * (T + 1) / 2;
  const int cb = blockIdx.x % (TS / kRedCols);
  const int u = (blockIdx.x / (TS / kRedCols)) % tri, n = blockIdx.x / ((TS / kRedCols) * tri);
  int ti, tj;
  tri_pair(u, T, ti, tj);
  const size_t per = (size_t)N * tri * TS * TS;
  const size_t at0 = ((size_t)n * tri + u) * (TS * TS);
  const float* sn = sums + (size_t)n * k;
  const int64_t* cn = cls + (size_t)n * k;
  for (int e = threadIdx.x; e < TS * kRedCols; e += 256) {
    const int ii = e / kRedCols, jj = cb * kRedCols + e % kRedCols;  // part row i, column j
    const int i = ti * TS + ii, j = tj * TS + jj;
    float v = 0.f;
    if (i < j && j < k && cn[i] == cn[j]) {
      int it = 0;
      for (int q = 0; q < groups; ++q) it += part[(size_t)q * per + at0 + (size_t)ii * TS + jj];
      const float fit = (float)it;
      const float uni = (sn[j] + sn[i]) - fit;  // sum_matrix + sum_matrix^T - inter
      v = fit / uni;
    }
    tile[jj - cb * kRedCols][ii] = v;
  }
  __syncthreads();
  // comp[j] = max_i iou(i, j) (the reference's column max, nms.py:66-69): this
  // block's part of row j of iouT, folded in with an integer atomicMax on the
  // IoU's bits (IoU >= 0: the bit patterns order as the values; exact in any
  // order).  One wave per four rows of the block's 16.
  {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int jl = wv; jl < kRedCols; jl += 4) {
      float mx = tile[jl][lane];
      if (TS > 64) mx = fmaxf(mx, tile[jl][64 + lane]);
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      const int j = tj * TS + cb * kRedCols + jl;
      if (lane == 0 && j < k && mx > 0.f)
        atomicMax(reinterpret_cast<int*>(comp) + (size_t)n * k + j, __float_as_int(mx));
    }
  }
  for (int e = threadIdx.x; e < TS * kRedCols; e += 256) {
    const int jl = e / TS, ii = e % TS, jj = cb * kRedCols + jl;
    const int i = ti * TS + ii, j = tj * TS + jj;
    if (i < k && j < k) iouT[((size_t)n * k + j) * k + i] = tile[jl][ii];
    // the mirror (rows j' of tile ti, columns i' of tile tj: i' > j')
    const int i2 = tj * TS + ii, j2 = ti * TS + jj;
    if (ti < tj && i2 < k && j2 < k) iouT[((size_t)n * k + j2) * k + i2] = 0.f;
  }
}

// out[j] = scores[j] * min_i decay(iou[i][j], comp[i]) over row j of iouT:
// one wave per (row, image); the decay formula of solo_decay_kernel
__global__ __launch_bounds__(256) void solo_decay_rows_kernel(
    const float* __restrict__ iouT, const float* __restrict__ comp,
    const float* __restrict__ scores, int N, int k, int kernel, float sigma,
    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N * k) return;
  const int n = row / k;
  const float* p = iouT + (size_t)row * k;
  const float* cp = comp + (size_t)n * k;
  const float ns = -1.f * sigma;
  float mn = INFINITY;
  for (int i = lane; i < k; i += 64) {
    const float v = p[i], ci = cp[i];
    const float d = kernel == 0 ? expf(ns * (v * v - ci * ci)) : (1.f - v) / (1.f - ci);
    mn = fminf(mn, d);
  }
  for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o));
  if (lane == 0) out[row] = scores[row] * mn;
}

__device__ __forceinline__ float solo_iou(const int32_t* inter, const float* s, const int64_t* cls,
                                          int k, int i, int j) {
  if (i >= j || cls[i] != cls[j]) return 0.f;  // band part removed, class-specific
  const float it = (float)inter[(size_t)i * k + j];
  const float uni = (s[j] + s[i]) - it;        // sum_matrix + sum_matrix^T - inter
  return it / uni;
}

// comp[j] = max_i iou[i][j]: one 256-thread workgroup per (column, image),
// threads over the rows, tree max (exact in any order).
__global__ __launch_bounds__(256) void solo_comp_kernel(const int32_t* __restrict__ inter,
                                                        const float* __restrict__ sums,
                                                        const int64_t* __restrict__ cls, int k,
                                                        float* __restrict__ comp) {
  __shared__ float red[256];
  const int j = blockIdx.x, n = blockIdx.y;
  const int32_t* in = inter + (size_t)n * k * k;
  const float* s = sums + (size_t)n * k;
  const int64_t* c = cls + (size_t)n * k;
  float mx = 0.f;  // the i >= j entries of the column are 0
  for (int i = threadIdx.x; i < j; i += blockDim.x) mx = fmaxf(mx, solo_iou(in, s, c, k, i, j));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) comp[(size_t)n * k + j] = red[0];
}

// out[j] = scores[j] * min_i decay[i][j], decay = exp(-sigma (iou^2 - comp_i^2))
// (gaussian) or (1 - iou) / (1 - comp_i) (linear); one workgroup per
// (column, image), tree min (exact in any order).
__global__ __launch_bounds__(256) void solo_decay_kernel(
    const int32_t* __restrict__ inter, const float* __restrict__ sums,
    const int64_t* __restrict__ cls, const float* __restrict__ comp,
    const float* __restrict__ scores, int k, int kernel, float sigma, float* __restrict__ out) {
  __shared__ float red[256];
  const int j = blockIdx.x, n = blockIdx.y;
  const int32_t* in = inter + (size_t)n * k * k;
  const float* s = sums + (size_t)n * k;
  const int64_t* c = cls + (size_t)n * k;
  const float* cp = comp + (size_t)n * k;
  const float ns = -1.f * sigma;
  float mn = INFINITY;
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const float v = solo_iou(in, s, c, k, i, j);
    const float ci = cp[i];
    const float d = kernel == 0 ? expf(ns * (v * v - ci * ci)) : (1.f - v) / (1.f - ci);
    mn = fminf(mn, d);
  }
  red[threadIdx.x] = mn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fminf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[(size_t)n * k + j] = scores[(size_t)n * k + j] * red[0];
}

// ------------------------------------------------------------------- stage 4
struct BoxAcc {
  unsigned long long sy, sx;
  int cnt, miny, maxy, minx, maxx, pad;
};

// One block per image: keep decayed > thr in candidate order, pad / clip to
// max_det (pad_or_clip_tensor: zeros).
__global__ __launch_bounds__(512) void solo_keep_kernel(
    const float* __restrict__ nms_scores, const int64_t* __restrict__ top_classes,
    const int32_t* __restrict__ top_count, int k, float thr, int max_det,
    int32_t* __restrict__ det_src, float* __restrict__ out_scores,
    int64_t* __restrict__ out_classes, uint8_t* __restrict__ out_valid) {
  __shared__ int wsum[8];
  __shared__ int base_sh;
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int cnt = top_count[n];
  if (threadIdx.x == 0) base_sh = 0;
  for (int d = threadIdx.x; d < max_det; d += blockDim.x) {
    det_src[(size_t)n * max_det + d] = -1;
    out_scores[(size_t)n * max_det + d] = 0.f;
    out_classes[(size_t)n * max_det + d] = 0;
    out_valid[(size_t)n * max_det + d] = 0;
  }
  __syncthreads();
  for (int t0 = 0; t0 < cnt; t0 += blockDim.x) {
    const int t = t0 + threadIdx.x;
    const float s = t < cnt ? nms_scores[(size_t)n * k + t] : 0.f;
    const bool keep = t < cnt && s > thr;
    const uint64_t bal = __ballot(keep);
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int before = base_sh, total = 0;
    for (int w = 0; w < nw; ++w) {
      if (w < wv) before += wsum[w];
      total += wsum[w];
    }
    const int pos = before + __popcll(bal & ((1ull << lane) - 1ull));
    if (keep && pos < max_det) {
      const size_t o = (size_t)n * max_det + pos;
      det_src[o] = t;
      out_scores[o] = s;
      out_classes[o] = top_classes[(size_t)n * k + t];
      out_valid[o] = 1;
    }
    __syncthreads();
    if (threadIdx.x == 0) base_sh += total;
    __syncthreads();
  }
}

__device__ __forceinline__ int wave_min(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float mask_bit(const uint64_t* m, size_t p) {
  return (float)((m[p >> 6] >> (p & 63)) & 1ull);
}

constexpr int kPasteRows = 16;   // output rows per workgroup
constexpr int kPasteWords = 512; // mask words staged in LDS per workgroup

// Masks of the kept detections resized from [Hm, Wm] to the padded image
// [OH, OW] (TF bilinear, half-pixel centres), > thr, uint8.  A workgroup
// owns kPasteRows output rows of one detection, four pixels per thread per
// step.  The column interpolation (lo, hi, lerp: the same for every row) is
// tabled in LDS once per workgroup, and the mask words under its source rows
// (about 3 rows x Wm bits) are staged in LDS; a pixel whose four source bits
// agree is that bit (tf_lerp of four equal 0 / 1 values is exact), the rest
// run tf_lerp.  Box statistics (integers: exact in any order) — mask count,
// coordinate sums, min / max of the coordinates > 0 — go to the workgroup's
// own partial slot (no atomics), reduced per detection by solo_boxes_kernel.
// Dynamic LDS: kPasteWords * 8 + OW * 8 bytes.
__global__ __launch_bounds__(256) void solo_paste_kernel(
    const uint64_t* __restrict__ bits, const int32_t* __restrict__ det_src, int k, int W64, int Hm,
    int Wm, int OH, int OW, float sh, float sw, float thr, int max_det, uint8_t* __restrict__ out,
    BoxAcc* __restrict__ part) {
  extern __shared__ uint64_t psm[];
  uint64_t* wbuf = psm;
  uint32_t* xidx = reinterpret_cast<uint32_t*>(psm + kPasteWords);  // lo | hi << 16
  float* xlr = reinterpret_cast<float*>(xidx + OW);
  const int d = blockIdx.y, n = blockIdx.z;
  const int src = det_src[(size_t)n * max_det + d];
  const int r0 = blockIdx.x * kPasteRows, r1 = min(OH, r0 + kPasteRows);
  const int qrow = OW / 4;
  const int nq = (r1 - r0) * qrow;
  uint8_t* dst = out + ((size_t)n * max_det + d) * OH * OW + (size_t)r0 * OW;
  if (src < 0) {
    for (int q = threadIdx.x; q < nq; q += blockDim.x)
      *(uchar4*)(dst + (size_t)q * 4) = make_uchar4(0, 0, 0, 0);
    return;
  }
  const uint64_t* m = bits + ((size_t)n * k + src) * W64;
  const uint32_t* m32 = reinterpret_cast<const uint32_t*>(m);  // little-endian halves
  for (int ox = threadIdx.x; ox < OW; ox += blockDim.x) {
    const Interp ix = interp_at(ox, sw, Wm, 1);
    xidx[ox] = (uint32_t)ix.lo | ((uint32_t)ix.hi << 16);
    xlr[ox] = ix.lerp;
  }
  const int ylo = interp_at(r0, sh, Hm, 1).lo, yhi = interp_at(r1 - 1, sh, Hm, 1).hi;
  const uint32_t w0 = (uint32_t)(((size_t)ylo * Wm) >> 5);
  const uint32_t w1 = (uint32_t)((((size_t)yhi + 1) * Wm - 1) >> 5);
  const bool staged = w1 - w0 + 1 <= 2u * kPasteWords;  // workgroup-uniform
  uint32_t* wb32 = reinterpret_cast<uint32_t*>(wbuf);
  if (staged)
    for (int i = threadIdx.x; i <= (int)(w1 - w0); i += blockDim.x) wb32[i] = m32[w0 + i];
  __syncthreads();
  auto bit = [&](uint32_t p) -> uint32_t {
    const uint32_t wd = staged ? wb32[(p >> 5) - w0] : m32[p >> 5];
    return (wd >> (p & 31u)) & 1u;
  };
  int cnt = 0, miny = INT_MAX, maxy = INT_MIN, minx = INT_MAX, maxx = INT_MIN;
  unsigned long long sy = 0, sx = 0;
  // (row, quad) of q stepped incrementally (no per-step division), the row's
  // interpolation recomputed only when the row changes
  int qr = (int)threadIdx.x / qrow, qc = (int)threadIdx.x - qr * qrow;
  int cur_row = -1;
  Interp iy = {0, 0, 0.f};
  uint32_t a0 = 0, a1 = 0;
  for (int q = threadIdx.x; q < nq; q += blockDim.x) {
    const int oy = r0 + qr, ox0 = qc * 4;
    qc += blockDim.x;
    while (qc >= qrow) {
      qc -= qrow;
      ++qr;
    }
    if (oy != cur_row) {
      cur_row = oy;
      iy = interp_at(oy, sh, Hm, 1);
      a0 = (uint32_t)iy.lo * (uint32_t)Wm;
      a1 = (uint32_t)iy.hi * (uint32_t)Wm;
    }
    const uint4 xi4 = *reinterpret_cast<const uint4*>(&xidx[ox0]);
    const float4 xl4 = *reinterpret_cast<const float4*>(&xlr[ox0]);
    const uint32_t xi[4] = {xi4.x, xi4.y, xi4.z, xi4.w};
    const float xl[4] = {xl4.x, xl4.y, xl4.z, xl4.w};
    uint32_t on4 = 0;  // bit e: pixel ox0 + e is on
    // the four pixels' source bits of each row sit in one 64-bit window
    // (two words) when the columns span < 32 (upsampling: a few bits)
    const uint32_t lo0 = xi[0] & 0xffffu, hi3 = xi[3] >> 16;
    const bool win = hi3 - lo0 < 32u;  // columns are monotone in ox
    const uint32_t b0 = (a0 + lo0) & ~31u, b1 = (a1 + lo0) & ~31u;
    uint64_t r0w = 0, r1w = 0;
    if (win) {
      r0w = (uint64_t)(staged ? wb32[(b0 >> 5) - w0] : m32[b0 >> 5]);
      r1w = (uint64_t)(staged ? wb32[(b1 >> 5) - w0] : m32[b1 >> 5]);
      if (((a0 + hi3) >> 5) != (b0 >> 5))
        r0w |= (uint64_t)(staged ? wb32[(b0 >> 5) + 1 - w0] : m32[(b0 >> 5) + 1]) << 32;
      if (((a1 + hi3) >> 5) != (b1 >> 5))
        r1w |= (uint64_t)(staged ? wb32[(b1 >> 5) + 1 - w0] : m32[(b1 >> 5) + 1]) << 32;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = xi[e] & 0xffffu, hi = xi[e] >> 16;
      uint32_t tl, tr, bl, br;
      if (win) {
        tl = (uint32_t)(r0w >> (a0 + lo - b0)) & 1u;
        tr = (uint32_t)(r0w >> (a0 + hi - b0)) & 1u;
        bl = (uint32_t)(r1w >> (a1 + lo - b1)) & 1u;
        br = (uint32_t)(r1w >> (a1 + hi - b1)) & 1u;
      } else {
        tl = bit(a0 + lo);
        tr = bit(a0 + hi);
        bl = bit(a1 + lo);
        br = bit(a1 + hi);
      }
      const uint32_t all = tl & tr & bl & br, any = tl | tr | bl | br;
      const float v = (all | (any ^ 1u)) ? (float)tl
                                         : tf_lerp((float)tl, (float)tr, (float)bl, (float)br,
                                                   xl[e], iy.lerp);
      on4 |= (v > thr ? 1u : 0u) << e;
    }
    // the four pixels' bytes, and their statistics from the 4-bit mask
    *(uint32_t*)(dst + (size_t)q * 4) =
        (on4 & 1u) | ((on4 & 2u) << 7) | ((on4 & 4u) << 14) | ((on4 & 8u) << 21);
    const int c4 = __popc(on4);
    cnt += c4;
    sy += (unsigned long long)c4 * (unsigned long long)oy;
    sx += (unsigned long long)c4 * (unsigned long long)ox0 + (unsigned)__popc(on4 & 0xAu) +
          2u * (unsigned)__popc(on4 & 0xCu);
    if (on4 && oy > 0) {
      miny = min(miny, oy);
      maxy = max(maxy, oy);
    }
    const uint32_t onx = ox0 == 0 ? on4 & ~1u : on4;  // coordinates > 0 only
    if (onx) {
      minx = min(minx, ox0 + __ffs((int)onx) - 1);
      maxx = max(maxx, ox0 + 31 - __clz((int)onx));
    }
  }
  __shared__ int s_i[4][5];
  __shared__ unsigned long long s_l[4][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  cnt = (int)wave_sum((unsigned long long)cnt);
  sy = wave_sum(sy);
  sx = wave_sum(sx);
  miny = wave_min(miny);
  maxy = wave_max(maxy);
  minx = wave_min(minx);
  maxx = wave_max(maxx);
  if (lane == 0) {
    s_i[wv][0] = cnt;
    s_i[wv][1] = miny;
    s_i[wv][2] = maxy;
    s_i[wv][3] = minx;
    s_i[wv][4] = maxx;
    s_l[wv][0] = sy;
    s_l[wv][1] = sx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    BoxAcc a;
    a.cnt = s_i[0][0];
    a.miny = s_i[0][1];
    a.maxy = s_i[0][2];
    a.minx = s_i[0][3];
    a.maxx = s_i[0][4];
    a.sy = s_l[0][0];
    a.sx = s_l[0][1];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      a.cnt += s_i[w][0];
      a.miny = min(a.miny, s_i[w][1]);
      a.maxy = max(a.maxy, s_i[w][2]);
      a.minx = min(a.minx, s_i[w][3]);
      a.maxx = max(a.maxx, s_i[w][4]);
      a.sy += s_l[w][0];
      a.sx += s_l[w][1];
    }
    a.pad = 0;
    part[((size_t)n * max_det + d) * gridDim.x + blockIdx.x] = a;
  }
}

// Boxes from masks (solo_v2.py:604-623), one wave per detection over its
// row-strip partials: yy_mean = sum(y * mask) / (sum_masks + 1e-5) replaces
// every zero of y * mask (all pixels off the mask and the mask's row 0), so
// ymin = min(yy_mean, min mask y > 0) and likewise for ymax / x; an empty
// (or padded) mask gives 0 / 1e-5 = 0.
__global__ __launch_bounds__(64) void solo_boxes_kernel(const BoxAcc* __restrict__ part,
                                                        const int32_t* __restrict__ det_src,
                                                        int nparts, float* __restrict__ boxes) {
  const int i = blockIdx.x, lane = threadIdx.x;
  if (det_src[i] < 0) {
    if (lane == 0) *(float4*)(boxes + (size_t)i * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  int cnt = 0, miny = INT_MAX, maxy = INT_MIN, minx = INT_MAX, maxx = INT_MIN;
  unsigned long long sy = 0, sx = 0;
  for (int j = lane; j < nparts; j += 64) {
    const BoxAcc a = part[(size_t)i * nparts + j];
    cnt += a.cnt;
    sy += a.sy;
    sx += a.sx;
    miny = min(miny, a.miny);
    maxy = max(maxy, a.maxy);
    minx = min(minx, a.minx);
    maxx = max(maxx, a.maxx);
  }
  cnt = (int)wave_sum((unsigned long long)cnt);
  sy = wave_sum(sy);
  sx = wave_sum(sx);
  miny = wave_min(miny);
  maxy = wave_max(maxy);
  minx = wave_min(minx);
  maxx = wave_max(maxx);
  if (lane == 0) {
    const float den = (float)cnt + 1e-5f;
    const float ym = (float)sy / den;
    const float xm = (float)sx / den;
    float4 b;
    b.x = miny != INT_MAX ? fminf(ym, (float)miny) : ym;
    b.y = minx != INT_MAX ? fminf(xm, (float)minx) : xm;
    b.z = maxy != INT_MIN ? fmaxf(ym, (float)maxy) : ym;
    b.w = maxx != INT_MIN ? fmaxf(xm, (float)maxx) : xm;
    *(float4*)(boxes + (size_t)i * 4) = b;
  }
}

static int fill_levels(SoloLevels& lv, const float* const* cate, const int32_t* grids,
                       const float* strides, int L) {
  D2MI_REQUIRE(L >= 1 && L <= kMaxLevels, "SOLO: 1..%d levels (got %d)", kMaxLevels, L);
  lv.L = L;
  lv.off[0] = 0;
  for (int l = 0; l < L; ++l) {
    D2MI_REQUIRE(grids[l] > 0, "SOLO: grid %d must be positive", l);
    lv.cate[l] = cate ? cate[l] : nullptr;
    lv.S[l] = grids[l];
    lv.stride[l] = strides ? strides[l] : 0.f;
    lv.off[l + 1] = lv.off[l] + grids[l] * grids[l];
  }
  return 0;
}

static inline int grid_for(size_t n, int threads, int cap = 1 << 20) {
  return (int)std::min<size_t>((n + threads - 1) / threads, (size_t)cap);
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_resize_bilinear(const float* x, int N, int H, int W, int C, int OH, int OW,
                                    int align_corners, int half_pixel_centers, float* y,
                                    void* stream) {
  D2MI_REQUIRE(N >= 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, "bad resize sizes");
  D2MI_REQUIRE(!(align_corners && half_pixel_centers),
               "align_corners and half_pixel_centers are exclusive (TF)");
  if (N == 0) return 0;
  const float sh = resize_scale(H, OH, align_corners), sw = resize_scale(W, OW, align_corners);
  const bool vec = (C & 3) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0;
  const size_t total = (size_t)N * OH * OW * (vec ? C / 4 : C);
  const int g = grid_for(total, 256, 65536);
  if (vec)
    hipLaunchKernelGGL(resize_bilinear_kernel<true>, dim3(g), dim3(256), 0, as_stream(stream), x,
                       y, N, H, W, C, OH, OW, sh, sw, half_pixel_centers);
  else
    hipLaunchKernelGGL(resize_bilinear_kernel<false>, dim3(g), dim3(256), 0, as_stream(stream),
                       x, y, N, H, W, C, OH, OW, sh, sw, half_pixel_centers);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_solo_cells(const float* const* cate, const int32_t* grids, int L, int N,
                               int K, float score_thr, float* probs, int32_t* live_cells,
                               int32_t* live_row, int32_t* live_count, void* stream) {
  SoloLevels lv;
  if (fill_levels(lv, cate, grids, nullptr, L)) return -1;
  D2MI_REQUIRE(N >= 0 && K > 0, "bad SOLO cell sizes");
  if (N == 0) return 0;
  const int T = lv.off[L];
  hipStream_t st = as_stream(stream);
  const size_t waves = (size_t)N * T;
  hipLaunchKernelGGL(solo_cells_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, lv,
                     N, K, score_thr, probs, live_row);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(solo_live_kernel, dim3(N), dim3(1024), 0, st, T, live_row, live_cells,
                     live_count);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_solo_mask_stats(const float* logits, int R, int P, float mask_thr,
                                    float* sum_masks, float* sum_scores, void* stream) {
  D2MI_REQUIRE(R >= 0 && P > 0, "bad SOLO mask-stat sizes");
  D2MI_REQUIRE(((uintptr_t)logits & 15) == 0, "SOLO mask logits must be 16-B aligned");
  if (R == 0) return 0;
  hipLaunchKernelGGL(solo_mask_stats_kernel, dim3(R), dim3(256), 0, as_stream(stream), logits, P,
                     mask_thr, sum_masks, sum_scores);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_solo_select_workspace_size(int N, int T, int K, int k) {
  WorkspaceSizer z;
  z.take<float>((size_t)N * T * K);
  z.take<int32_t>(N);
  z.take<int64_t>(N);
  z.take<int32_t>(N);
  z.take<int32_t>((size_t)N * k);
  z.off += topk_workspace_size(N, k) + 256;
  return z.off;
}

extern "C" int d2mi_solo_select(const float* probs, const int32_t* live_row,
                                const int32_t* row_off, const float* logits,
                                const float* sum_masks, const float* sum_scores,
                                const int32_t* grids, const float* strides, int L, int N, int K,
                                int P, float score_thr, float mask_thr, int k, float* top_scores,
                                int64_t* top_classes, float* top_sum_masks, int32_t* top_count,
                                uint64_t* mask_bits, void* workspace, size_t workspace_bytes,
                                void* stream) {
  SoloLevels lv;
  if (fill_levels(lv, nullptr, grids, strides, L)) return -1;
  D2MI_REQUIRE(N >= 0 && K > 0 && P > 0, "bad SOLO select sizes");
  D2MI_REQUIRE(k > 0, "pre-NMS top-k must be positive");
  if (N == 0) return 0;
  const int T = lv.off[L];
  const int W64 = (P + 63) / 64;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  float* dense = w.take<float>((size_t)N * T * K);
  int32_t* valid = w.take<int32_t>(N);
  int64_t* seg_start = w.take<int64_t>(N);
  int32_t* seg_len = w.take<int32_t>(N);
  int32_t* top_idx = w.take<int32_t>((size_t)N * k);
  const size_t tk_bytes = topk_workspace_size(N, k);
  void* tk_ws = w.take<char>(tk_bytes);
  D2MI_REQUIRE(w.ok(), "SOLO select workspace too small (%zu < %zu)", workspace_bytes, w.off);
  D2MI_REQUIRE(fill_bytes(valid, sizeof(int32_t) * N, 0, st) == 0, "fill failed");
  const size_t total = (size_t)N * T * K;
  hipLaunchKernelGGL(solo_cand_kernel, dim3(grid_for(std::max(total, (size_t)N), 256)),
                     dim3(256), 0, st, lv, probs, live_row, row_off, sum_masks, sum_scores, N, K,
                     score_thr, dense, valid, seg_start, seg_len);
  D2MI_LAUNCH_CHECK();
  int rc = topk_core_ex(dense, seg_start, seg_len, valid, N, T * K, k, 0, top_scores, top_idx,
                        top_count, tk_ws, tk_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(solo_gather_kernel, dim3(k, N), dim3(256), 0, st, top_idx, top_count,
                     live_row, row_off, logits, sum_masks, T, K, P, k, W64, mask_thr, top_classes,
                     top_sum_masks, mask_bits);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// workgroups per tile pair of the MFMA intersection: about one per CU over
// the upper-triangle 64 x 64 tile pairs of all images (each workgroup's
// kIWaves waves split its pixel words)
static int solo_mfma_groups(int N, int k, int W64) {
  const int T = (k + kIT - 1) / kIT, tri = T * (T + 1) / 2;
  const int want = std::max(1, 256 / std::max(1, N * tri));
  const int most = std::max(1, (W64 + kIWaves * kIWords - 1) / (kIWaves * kIWords));
  return std::min(want, most);
}

extern "C" size_t d2mi_solo_matrix_nms_workspace_size(int N, int k) {
  WorkspaceSizer z;
  z.take<int32_t>((size_t)N * k * k);
  z.take<float>((size_t)N * k);
  // (the MFMA path's partial tiles, sized for the most groups any P gives)
  const int T = (k + kIT - 1) / kIT, tri = T * (T + 1) / 2;
  const int gmax = std::max(1, 256 / std::max(1, N * tri));
  z.take<int32_t>((size_t)gmax * N * tri * kIT * kIT);
  return z.off;
}

extern "C" int d2mi_solo_matrix_nms(const uint64_t* mask_bits, const int64_t* classes,
                                    const float* scores, const float* sum_masks, int N, int k,
                                    int P, int kernel, float sigma, float* out_scores,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(N >= 0 && k > 0 && P > 0, "bad SOLO Matrix-NMS sizes");
  D2MI_REQUIRE(kernel == 0 || kernel == 1, "NMS kernel must be gaussian (0) or linear (1)");
  if (N == 0) return 0;
  const int W64 = (P + 63) / 64;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  int32_t* inter = w.take<int32_t>((size_t)N * k * k);
  float* comp = w.take<float>((size_t)N * k);
  D2MI_REQUIRE(w.ok(), "SOLO Matrix-NMS workspace too small (%zu < %zu)", workspace_bytes, w.off);
  if (tuning(kTuneSoloMfma) != 0) {
    // (inter's bytes hold the transposed IoU matrix: float, N * k * k)
    float* iouT = reinterpret_cast<float*>(inter);
    const int T = (k + kIT - 1) / kIT, tri = T * (T + 1) / 2;
    const int groups = solo_mfma_groups(N, k, W64);
    const int slices = groups * kIWaves;
    const int wpw = ((W64 + slices - 1) / slices + kIWords - 1) / kIWords * kIWords;
    int32_t* part = w.take<int32_t>((size_t)groups * N * tri * kIT * kIT);
    D2MI_REQUIRE(w.ok(), "SOLO Matrix-NMS workspace too small (%zu < %zu)", workspace_bytes,
                 w.off);
    // tuning "solo_mfma": 2 (default) = bits expanded by an LDS table (r6:
    // intersections 38.1 -> 31.9 us per call, profiles/r6m_stats_*.csv), 1 = by
    // arithmetic
    if (tuning(kTuneSoloMfma) == 2)
      hipLaunchKernelGGL(solo_inter_mfma_kernel<true>, dim3(N * tri * groups), dim3(64 * kIWaves),
                         kIWaves * kIWaveB, st, mask_bits, N, k, W64, T, groups, wpw, part, comp);
    else
      hipLaunchKernelGGL(solo_inter_mfma_kernel<false>, dim3(N * tri * groups), dim3(64 * kIWaves),
                         kIWaves * kIWaveB, st, mask_bits, N, k, W64, T, groups, wpw, part, comp);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(solo_inter_reduce_kernel<kIT>, dim3(N * tri * (kIT / kRedCols)), dim3(256), 0,
                       st, part, N, k, T, groups, sum_masks, classes, iouT, comp);
    D2MI_LAUNCH_CHECK();
    const unsigned rows_grid = (unsigned)(((size_t)N * k + 3) / 4);
    hipLaunchKernelGGL(solo_decay_rows_kernel, dim3(rows_grid), dim3(256), 0, st, iouT, comp,
                       scores, N, k, kernel, sigma, out_scores);
    D2MI_LAUNCH_CHECK();
    return 0;
  } else {
  D2MI_REQUIRE(fill_bytes(inter, sizeof(int32_t) * (size_t)N * k * k, 0, st) == 0, "fill failed");
  const int tiles = (k + kMT - 1) / kMT;
  // word slices: enough workgroups to fill the chip (>= ~4 per CU over the
  // upper-triangle tiles), at least one LDS stage each
  const int tri = tiles * (tiles + 1) / 2;
  int splits = std::max(1, std::min((W64 + kMW - 1) / kMW, (1024 + tri * N - 1) / (tri * N)));
  const int wps = ((W64 + splits - 1) / splits + kMW - 1) / kMW * kMW;
  splits = (W64 + wps - 1) / wps;
  hipLaunchKernelGGL(solo_inter_kernel, dim3(tiles, tiles, N * splits), dim3(256), 0, st,
                     mask_bits, k, W64, wps, inter);
  D2MI_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(solo_comp_kernel, dim3(k, N), dim3(256), 0, st, inter, sum_masks, classes, k,
                     comp);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(solo_decay_kernel, dim3(k, N), dim3(256), 0, st, inter, sum_masks, classes,
                     comp, scores, k, kernel, sigma, out_scores);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t d2mi_solo_finalize_workspace_size(int N, int max_det, int OH) {
  WorkspaceSizer z;
  z.take<int32_t>((size_t)N * max_det);
  z.take<BoxAcc>((size_t)N * max_det * ((OH + kPasteRows - 1) / kPasteRows));
  return z.off;
}

extern "C" int d2mi_solo_finalize(const float* nms_scores, const int64_t* top_classes,
                                  const int32_t* top_count, const uint64_t* mask_bits, int N,
                                  int k, int Hm, int Wm, float update_thr, int max_det,
                                  float mask_thr, int OH, int OW, uint8_t* out_masks,
                                  float* out_boxes, float* out_scores, int64_t* out_classes,
                                  uint8_t* out_valid, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  D2MI_REQUIRE(N >= 0 && k > 0 && Hm > 0 && Wm > 0 && max_det > 0 && OH > 0 && OW > 0,
               "bad SOLO finalize sizes");
  D2MI_REQUIRE(OW % 4 == 0, "SOLO output width must be a multiple of 4 (got %d)", OW);
  D2MI_REQUIRE(((uintptr_t)out_masks & 3) == 0 && ((uintptr_t)out_boxes & 15) == 0,
               "SOLO outputs misaligned");
  if (N == 0) return 0;
  const int W64 = (Hm * Wm + 63) / 64;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  const int nparts = (OH + kPasteRows - 1) / kPasteRows;
  int32_t* det_src = w.take<int32_t>((size_t)N * max_det);
  BoxAcc* part = w.take<BoxAcc>((size_t)N * max_det * nparts);
  D2MI_REQUIRE(w.ok(), "SOLO finalize workspace too small (%zu < %zu)", workspace_bytes, w.off);
  hipLaunchKernelGGL(solo_keep_kernel, dim3(N), dim3(512), 0, st, nms_scores, top_classes,
                     top_count, k, update_thr, max_det, det_src, out_scores, out_classes,
                     out_valid);
  D2MI_LAUNCH_CHECK();
  const float sh = resize_scale(Hm, OH, 0), sw = resize_scale(Wm, OW, 0);
  D2MI_REQUIRE(Wm <= 65535, "SOLO mask width %d exceeds the 16-bit column table", Wm);
  const size_t paste_lds = (size_t)kPasteWords * 8 + (size_t)OW * 8;
  D2MI_REQUIRE(paste_lds <= 160 * 1024, "SOLO output width %d too large for the paste table", OW);
  hipLaunchKernelGGL(solo_paste_kernel, dim3(nparts, max_det, N), dim3(256), paste_lds, st, mask_bits,
                     det_src, k, W64, Hm, Wm, OH, OW, sh, sw, mask_thr, max_det, out_masks, part);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(solo_boxes_kernel, dim3(N * max_det), dim3(64), 0, st, part, det_src, nparts,
                     out_boxes);
  D2MI_LAUNCH_CHECK();
  return 0;
}
