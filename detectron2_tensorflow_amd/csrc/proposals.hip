// Anchor generation, box decoding and the three detection post-processing
// pipelines of the reference, fused around the segmented top-k and NMS cores:
//
//   d2mi_grid_anchors          anchor_generator.py:31-40, :92-109
//   d2mi_apply_deltas          box_regression.py:76-123
//   d2mi_rpn_proposals         rpn_outputs.py:29-132 (+ :403-440 predict_proposals /
//                              predict_objectness_logits, anchor_generator.py:92-109)
//   d2mi_fast_rcnn_inference   fast_rcnn.py:28-187 (+ :359-379 predict_boxes/probs)
//   d2mi_retinanet_inference   retinanet.py:285-387
//
// The reference decodes every anchor (268,569 per image for R-CNN FPN at
// 1333x800) and then keeps <= 1000 per level; decoding is elementwise, so
// selecting first and decoding only the selected anchors (regenerated from
// the flat index) gives identical results for a fraction of the traffic.
#include "detect.h"

namespace d2mi {
namespace {

__device__ __forceinline__ void atomic_max_ordered(uint32_t* p, float v) {
  atomicMax(p, orderable(v));
}

// ------------------------------------------------------------- simple ops
__global__ void grid_anchors_kernel(int H, int W, int stride, Levels lv, float4* out) {
  const int A = lv.A;
  const int total = H * W * A;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int hw = i / A, a = i - hw * A;
    out[i] = anchor_at(lv, 0, hw, a);
  }
}

__global__ void apply_deltas_kernel(const float4* __restrict__ deltas,
                                    const float4* __restrict__ boxes, int N, int K, DeltaCfg dc,
                                    float4* __restrict__ out) {
  const int64_t total = (int64_t)N * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / K;
    out[i] = apply_delta(boxes[n], deltas[i], dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
  }
}

// ------------------------------------------------------------ RPN proposals
__global__ void seg_setup_kernel(Levels lv, int N, int K, int topk, int64_t* seg_start,
                                 int32_t* seg_len, int32_t* seg_k) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= N * lv.L) return;
  const int n = s / lv.L, l = s - n * lv.L;
  const int64_t hwa = (int64_t)lv.H[l] * lv.W[l] * lv.A;
  seg_start[s] = lv.off_a[l] + n * lv.img_a[l] * K;
  seg_len[s] = (int32_t)(hwa * K);
  if (seg_k) seg_k[s] = (int32_t)min((int64_t)topk, hwa);
}

__global__ void rpn_decode_kernel(const float* __restrict__ base_d, Levels lv, int N, int k,
                                  const float* __restrict__ tvals, const int32_t* __restrict__ tidx,
                                  const int32_t* __restrict__ tcount,
                                  const int32_t* __restrict__ image_hw, DeltaCfg dc,
                                  float min_size, float4* __restrict__ dec,
                                  uint64_t* __restrict__ keys, int32_t* __restrict__ lens) {
  const int s = blockIdx.y;
  const int n = s / lv.L, l = s - n * lv.L;
  const int cnt = tcount[s];
  if (blockIdx.x == 0 && threadIdx.x == 0) lens[s] = cnt;
  const float hmax = (float)image_hw[2 * n], wmax = (float)image_hw[2 * n + 1];
  const int HW = lv.H[l] * lv.W[l];
  const float4* d4 = reinterpret_cast<const float4*>(base_d + lv.off_b[l]);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
    const size_t o = (size_t)s * k + j;
    const int id = tidx[o];
    const int hw = id / lv.A, a = id - hw * lv.A;
    const float4 anc = anchor_at(lv, l, hw, a);
    const float4 d = d4[(size_t)n * lv.img_b[l] + (size_t)hw * lv.A + a];
    float4 b = apply_delta(anc, d, dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
    b = clip_box(b, hmax, wmax);
    bool ok = true;
    if (min_size > 0.f) {
      const float bh = b.z - b.x, bw = b.w - b.y;
      ok = (bw >= min_size) && (bh >= min_size);  // prune_small_boxes (box_list_ops.py:515)
    }
    dec[o] = b;
    keys[o] = ok ? desc_key(tvals[o], (uint32_t)j) : ~0ull;
  }
}

// r5 (tuning "rpn_compact" = 1): decode AND the NMS input in one launch, one
// workgroup per segment.  The top-k list is already in the NMS order (score
// descending, list position ascending -- desc_key's order, -0.0 tied with
// +0.0 in both), so the NMS's segmented sort is the identity on the valid
// entries: a stable compaction of them (prune_small_boxes, NaN / -inf scores
// dropped, as desc_key drops them) gives exactly the sorted boxes, positions
// and count that keys -> sort -> gather produced (three launches, ~25 us per
// RPN step).  dec keeps every decoded box at its list position for the merge.
__global__ __launch_bounds__(1024) void rpn_decode_compact_kernel(
    const float* __restrict__ base_d, Levels lv, int N, int k, const float* __restrict__ tvals,
    const int32_t* __restrict__ tidx, const int32_t* __restrict__ tcount,
    const int32_t* __restrict__ image_hw, DeltaCfg dc, float min_size, float4* __restrict__ dec,
    float4* __restrict__ sboxes, int32_t* __restrict__ sidx, int32_t* __restrict__ scount) {
  __shared__ int s_wave[16];
  const int s = blockIdx.x;
  const int n = s / lv.L, l = s - n * lv.L;
  const int cnt = tcount[s];
  const float hmax = (float)image_hw[2 * n], wmax = (float)image_hw[2 * n + 1];
  const float4* d4 = reinterpret_cast<const float4*>(base_d + lv.off_b[l]);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int run = 0;
  for (int j0 = 0; j0 < cnt; j0 += blockDim.x) {
    const int j = j0 + (int)threadIdx.x;
    const size_t o = (size_t)s * k + j;
    bool valid = false;
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < cnt) {
      const int id = tidx[o];
      const int hw = id / lv.A, a = id - hw * lv.A;
      const float4 anc = anchor_at(lv, l, hw, a);
      const float4 d = d4[(size_t)n * lv.img_b[l] + (size_t)hw * lv.A + a];
      b = apply_delta(anc, d, dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
      b = clip_box(b, hmax, wmax);
      bool ok = true;
      if (min_size > 0.f) {
        const float bh = b.z - b.x, bw = b.w - b.y;
        ok = (bw >= min_size) && (bh >= min_size);  // prune_small_boxes (box_list_ops.py:515)
      }
      dec[o] = b;
      valid = ok && tvals[o] > -INFINITY;  // (desc_key: NaN / -inf never selected)
    }
    const unsigned long long bal = __ballot(valid);
    if (lane == 0) s_wave[w] = __popcll(bal);
    __syncthreads();
    int before = 0, tot = 0;
    for (int q = 0; q < nw; ++q) {
      const int v = s_wave[q];
      before += q < w ? v : 0;
      tot += v;
    }
    if (valid) {
      const int pos = run + before + __popcll(bal & ((1ull << lane) - 1ull));
      sboxes[(size_t)s * k + pos] = b;
      sidx[(size_t)s * k + pos] = j;
    }
    run += tot;
    __syncthreads();  // (s_wave reused)
  }
  if (threadIdx.x == 0) scount[s] = run;
}

// One workgroup per image: concat the per-level NMS survivors, top_k(post,
// sorted=True) with the concat position as tie-break, zero-pad.
__global__ __launch_bounds__(1024) void rpn_merge_kernel(
    const float4* __restrict__ dec, const float* __restrict__ tvals,
    const int32_t* __restrict__ keep, const int32_t* __restrict__ num_keep, int L, int k,
    int post, float4* __restrict__ out_boxes, float* __restrict__ out_scores,
    uint8_t* __restrict__ out_valid) {
  extern __shared__ uint64_t sk[];
  const int n = blockIdx.x;
  __shared__ int base_l[D2MI_MAX_LEVELS + 1];
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      base_l[l] = acc;
      acc += num_keep[n * L + l];
    }
    base_l[L] = acc;
  }
  __syncthreads();
  const int total = base_l[L];
  int m = 1;
  while (m < total) m <<= 1;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    uint64_t key = ~0ull;
    if (i < total) {
      int l = 0;
      while (i >= base_l[l + 1]) ++l;
      const int t = i - base_l[l];
      const int s = n * L + l;
      const int j = keep[(size_t)s * post + t];
      key = desc_key(tvals[(size_t)s * k + j], (uint32_t)(l * post + t));
    }
    sk[i] = key;
  }
  __syncthreads();
  for (int kk = 2; kk <= m; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = sk[i], b = sk[ixj];
          const bool up = (i & kk) == 0;
          if ((a > b) == up) { sk[i] = b; sk[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < post; i += blockDim.x) {
    const size_t o = (size_t)n * post + i;
    if (i < total && sk[i] != ~0ull) {
      const uint32_t p = (uint32_t)(sk[i] & 0xffffffffu);
      const int l = p / post, t = p - l * post;
      const int s = n * L + l;
      const int j = keep[(size_t)s * post + t];
      out_boxes[o] = dec[(size_t)s * k + j];
      out_scores[o] = tvals[(size_t)s * k + j];
      out_valid[o] = 1;
    } else {
      out_boxes[o] = make_float4(0.f, 0.f, 0.f, 0.f);
      out_scores[o] = 0.f;
      out_valid[o] = 0;
    }
  }
}

// r5: the same concat + top_k(post) as a merge rank over the per-level NMS
// survivor lists, which are already in key order (score desc, keep position
// asc): an entry's position = its own position + the earlier levels' entries
// whose key is not above its own + the later levels' entries strictly above
// it -- the desc_key(score, l * post + t) order of rpn_merge_kernel, scores
// compared as orderable words (-0.0 and +0.0 share one word, so they tie and
// the concat position decides, as TF compares values).  Many workgroups per
// image (one entry per thread, every list's score words in LDS) instead of
// one workgroup's bitonic sort of up to 8,192 keys (61 us per training step).
constexpr int kMergeT = 256;
__global__ __launch_bounds__(kMergeT) void rpn_merge_rank_kernel(
    const float4* __restrict__ dec, const float* __restrict__ tvals,
    const int32_t* __restrict__ keep, const int32_t* __restrict__ num_keep, int L, int k,
    int post, float4* __restrict__ out_boxes, float* __restrict__ out_scores,
    uint8_t* __restrict__ out_valid) {
  extern __shared__ uint32_t sw[];  // [L * post] orderable score words
  __shared__ int cnt[D2MI_MAX_LEVELS], cum[D2MI_MAX_LEVELS + 1];
  const int n = blockIdx.y, t = threadIdx.x;
  if (t == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      cnt[l] = num_keep[n * L + l];
      cum[l] = acc;
      acc += cnt[l];
    }
    cum[L] = acc;
  }
  __syncthreads();
  // every level's kept score words into LDS: 8 entries per thread per round,
  // their keep indices loaded together and then their scores (two dependent
  // load rounds per 8 entries instead of per entry)
  for (int q0 = t; q0 < L * post; q0 += 8 * kMergeT) {
    int ix[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = q0 + u * kMergeT;
      const int l = q / post, i = q - l * post;
      ix[u] = (q < L * post && i < cnt[l]) ? keep[(size_t)(n * L + l) * post + i] : -1;
    }
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = q0 + u * kMergeT;
      const int l = q / post;
      w[u] = ix[u] >= 0 ? orderable(tvals[(size_t)(n * L + l) * k + ix[u]]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (q0 + u * kMergeT < L * post) sw[q0 + u * kMergeT] = w[u];
  }
  __syncthreads();
  const int r = blockIdx.x * kMergeT + t;
  const int total = cum[L];
  if (r >= max(total, post)) return;
  if (r >= total) {  // zero padding past the survivors
    const size_t o = (size_t)n * post + r;
    out_boxes[o] = make_float4(0.f, 0.f, 0.f, 0.f);
    out_scores[o] = 0.f;
    out_valid[o] = 0;
    return;
  }
  int l = 0;
  while (l + 1 < L && cum[l + 1] <= r) ++l;
  const int i = r - cum[l];
  const uint32_t me = sw[l * post + i];
  int lo[D2MI_MAX_LEVELS], hi[D2MI_MAX_LEVELS];
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
    lo[m] = 0;
    // (only positions < post are kept: a level searched over its first post
    // entries -- a count of post already puts this entry past the cut -- in
    // ceil(log2(post + 1)) rounds, kept as a loop: r6, 14 unrolled rounds
    // before; the same cut for every entry whose position is < post)
    hi[m] = (m < L && m != l) ? min(cnt[m], post) : 0;
  }
  const int rounds = 32 - __clz(post);
  // earlier levels: entries with word >= mine come first; later: word > mine
#pragma unroll 1
  for (int step = 0; step < rounds; ++step) {
    uint32_t pv[D2MI_MAX_LEVELS];
#pragma unroll
    for (int m = 0; m < D2MI_MAX_LEVELS; ++m)
      pv[m] = m < L ? sw[m * post + min((lo[m] + hi[m]) >> 1, post - 1)] : 0u;
#pragma unroll
    for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
      if (lo[m] < hi[m]) {
        const int mid = (lo[m] + hi[m]) >> 1;
        if (m < l ? pv[m] >= me : pv[m] > me) lo[m] = mid + 1;
        else hi[m] = mid;
      }
    }
  }
  int pos = i;
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) pos += lo[m];
  if (pos < post) {
    const int s = n * L + l;
    const int j = keep[(size_t)s * post + i];
    const size_t o = (size_t)n * post + pos;
    out_boxes[o] = dec[(size_t)s * k + j];
    out_scores[o] = tvals[(size_t)s * k + j];
    out_valid[o] = 1;
  }
}

// --------------------------------------------------------- Fast R-CNN
__global__ void slot_map_kernel(const int32_t* roi_img, const int32_t* roi_slot, int R, int P,
                                int N, int32_t* slot2roi, int32_t* err) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int n = roi_img[r], s = roi_slot[r];
  if (s < 0) return;  // ignored row (an invalid / padded proposal)
  if (n < 0 || n >= N || s >= P) {
    atomicOr(err, kErrBoxInd);
    return;
  }
  slot2roi[n * P + s] = r;
}

__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One wave per ROI: softmax over K+1 logits, class-specific decode + clip,
// per-image max coordinate, candidate append (score > thresh).
__global__ __launch_bounds__(256) void frcnn_score_kernel(
    const float* __restrict__ logits, const float4* __restrict__ deltas,
    const float4* __restrict__ props, const int32_t* __restrict__ roi_img,
    const int32_t* __restrict__ roi_slot, int R, int N, int P, int K, int agnostic,
    const int32_t* __restrict__ image_hw, DeltaCfg dc, float thresh, int cap,
    uint32_t* __restrict__ maxc, int32_t* __restrict__ cnt, uint64_t* __restrict__ keys,
    float4* __restrict__ cbox, float* __restrict__ cscore, int32_t* err) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const int n = roi_img[r], slot = roi_slot[r];
  if (n < 0 || n >= N || slot < 0 || slot >= P) return;
  const float* lg = logits + (size_t)r * (K + 1);
  float mx = -INFINITY;
  for (int c = lane; c <= K; c += 64) mx = fmaxf(mx, lg[c]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int c = lane; c <= K; c += 64) sum += expf(lg[c] - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;  // TF softmax: exp(x - max) * (1 / sum)
  const float hmax = (float)image_hw[2 * n], wmax = (float)image_hw[2 * n + 1];
  const float4 pb = props[r];
  float bmax = 0.f;
  for (int c = lane; c < K; c += 64) {
    const float p = expf(lg[c] - mx) * inv;
    const float4 d = deltas[(size_t)r * (agnostic ? 1 : K) + (agnostic ? 0 : c)];
    float4 b = apply_delta(pb, d, dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
    b = clip_box(b, hmax, wmax);
    bmax = fmaxf(bmax, fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
    if (p > thresh) {
      const int pos = atomicAdd(&cnt[n], 1);
      if (pos < cap) {
        const size_t o = (size_t)n * cap + pos;
        keys[o] = desc_key(p, (uint32_t)(c * P + slot));  // class-major tf.where order
        cbox[o] = b;
        cscore[o] = p;
      } else {
        atomicOr(err, kErrNmsCapacity);
      }
    }
  }
  bmax = wave_max(bmax);
  if (lane == 0) atomic_max_ordered(&maxc[n], bmax);
}

__global__ void clamp_lens_kernel(int32_t* cnt, int N, int cap) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < N) cnt[n] = min(cnt[n], cap);
}

// After the sort the key no longer says where the candidate's box is, so the
// candidate slot rides in a parallel lookup: keys were appended at position
// pos with payload (c*P + slot); we rebuild pos by a second "flat -> pos" map.
__global__ void frcnn_posmap_kernel(const uint64_t* __restrict__ keys,
                                    const int32_t* __restrict__ lens, int cap, int P, int K,
                                    int32_t* __restrict__ flat2pos) {
  const int n = blockIdx.y;
  const int len = lens[n];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const uint32_t flat = (uint32_t)(keys[(size_t)n * cap + i] & 0xffffffffu);
    flat2pos[(size_t)n * P * K + flat] = i;
  }
}

__global__ void frcnn_gather_kernel(const uint64_t* __restrict__ sorted,
                                    const int32_t* __restrict__ lens,
                                    const int32_t* __restrict__ flat2pos,
                                    const float4* __restrict__ cbox,
                                    const uint32_t* __restrict__ maxc, int cap, int P, int K,
                                    int agnostic_nms, float4* __restrict__ sboxes,
                                    int32_t* __restrict__ sidx, int32_t* __restrict__ count) {
  const int n = blockIdx.y;
  const int len = lens[n];
  if (blockIdx.x == 0 && threadIdx.x == 0) count[n] = len;
  // nms_cls_agnostic (fast_rcnn.py:138-139): the filtered boxes as they are
  const float off1 = agnostic_nms ? 0.f : from_orderable(maxc[n]) + 1.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const size_t o = (size_t)n * cap + i;
    const uint32_t flat = (uint32_t)(sorted[o] & 0xffffffffu);
    const int c = flat / P;
    const int pos = flat2pos[(size_t)n * P * K + flat];
    const float4 b = cbox[(size_t)n * cap + pos];
    const float off = (float)c * off1;  // tf.cast(cls, f32) * (max_coord + 1)
    sboxes[o] = agnostic_nms ? b : make_float4(b.x + off, b.y + off, b.z + off, b.w + off);
    sidx[o] = pos;
  }
}

__global__ void frcnn_output_kernel(const int32_t* __restrict__ keep,
                                    const int32_t* __restrict__ num_keep,
                                    const uint64_t* __restrict__ unsorted_keys,
                                    const float4* __restrict__ cbox,
                                    const float* __restrict__ cscore,
                                    const int32_t* __restrict__ slot2roi, int cap, int P,
                                    int max_det, int N, float4* __restrict__ ob,
                                    float* __restrict__ os, int64_t* __restrict__ oc,
                                    uint8_t* __restrict__ ov, int32_t* __restrict__ oroi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * max_det) return;
  const int n = i / max_det, j = i - n * max_det;
  if (j < num_keep[n]) {
    const int pos = keep[i];
    const size_t o = (size_t)n * cap + pos;
    const uint32_t flat = (uint32_t)(unsorted_keys[o] & 0xffffffffu);
    const int c = flat / P, slot = flat - c * P;
    ob[i] = cbox[o];
    os[i] = cscore[o];
    oc[i] = c;
    ov[i] = 1;
    oroi[i] = slot2roi[n * P + slot];
  } else {
    ob[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    os[i] = 0.f;
    oc[i] = 0;
    ov[i] = 0;
    oroi[i] = -1;
  }
}

// ----------------------------------------------------------- RetinaNet
__global__ void retina_decode_kernel(const float* __restrict__ base_b, Levels lv, int N, int K,
                                     int k, const float* __restrict__ tvals,
                                     const int32_t* __restrict__ tidx,
                                     const int32_t* __restrict__ tcount, float thresh,
                                     DeltaCfg dc, int cap, uint64_t* __restrict__ keys,
                                     float4* __restrict__ cbox, float* __restrict__ cscore,
                                     int32_t* __restrict__ ccls, uint32_t* __restrict__ maxc) {
  const int s = blockIdx.y;
  const int n = s / lv.L, l = s - n * lv.L;
  const int cnt = tcount[s];
  const int HW = lv.H[l] * lv.W[l];
  const float4* d4 = reinterpret_cast<const float4*>(base_b + lv.off_b[l]);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < k; j += gridDim.x * blockDim.x) {
    const int q = l * k + j;
    const size_t o = (size_t)n * cap + q;
    const size_t t = (size_t)s * k + j;
    if (j < cnt && tvals[t] > thresh) {
      const int id = tidx[t];
      const int aidx = id / K, cls = id - aidx * K;
      const int hw = aidx / lv.A, a = aidx - hw * lv.A;
      const float4 anc = anchor_at(lv, l, hw, a);
      const float4 d = d4[(size_t)n * HW * lv.A + aidx];
      const float4 b = apply_delta(anc, d, dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
      keys[o] = desc_key(tvals[t], (uint32_t)q);
      cbox[o] = b;
      cscore[o] = tvals[t];
      ccls[o] = cls;
      atomic_max_ordered(&maxc[n], fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
    } else {
      keys[o] = ~0ull;
    }
  }
}

__global__ void fill_kernel(int32_t* p, int n, int v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
__global__ void fill_u32_kernel(uint32_t* p, int n, uint32_t v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void retina_gather_kernel(const uint64_t* __restrict__ sorted, const int32_t* lens,
                                     const float4* __restrict__ cbox,
                                     const int32_t* __restrict__ ccls,
                                     const uint32_t* __restrict__ maxc, int cap,
                                     float4* __restrict__ sboxes, int32_t* __restrict__ sidx,
                                     int32_t* __restrict__ count) {
  const int n = blockIdx.y;
  const int len = lens[n];
  const size_t base = (size_t)n * cap;
  const float off1 = from_orderable(maxc[n]) + 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0 && len > 0 && sorted[base] == ~0ull) count[n] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && len == 0) count[n] = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const uint64_t key = sorted[base + i];
    const bool valid = key != ~0ull;
    const uint32_t q = (uint32_t)(key & 0xffffffffu);
    if (valid) {
      const float4 b = cbox[base + q];
      const float off = (float)ccls[base + q] * off1;
      sboxes[base + i] = make_float4(b.x + off, b.y + off, b.z + off, b.w + off);
      sidx[base + i] = (int32_t)q;
    }
    const bool next_valid = (i + 1 < len) && sorted[base + i + 1] != ~0ull;
    if (valid && !next_valid) count[n] = i + 1;
  }
}

__global__ void retina_output_kernel(const int32_t* __restrict__ keep,
                                     const int32_t* __restrict__ num_keep,
                                     const float4* __restrict__ cbox,
                                     const float* __restrict__ cscore,
                                     const int32_t* __restrict__ ccls, int cap, int max_det,
                                     int N, float4* __restrict__ ob, float* __restrict__ os,
                                     int32_t* __restrict__ oc, uint8_t* __restrict__ ov) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * max_det) return;
  const int n = i / max_det, j = i - n * max_det;
  if (j < num_keep[n]) {
    const size_t o = (size_t)n * cap + keep[i];
    ob[i] = cbox[o];
    os[i] = cscore[o];
    oc[i] = ccls[o];
    ov[i] = 1;
  } else {
    ob[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    os[i] = 0.f;
    oc[i] = 0;
    ov[i] = 0;
  }
}

inline int grid1(size_t n, int block = 256, int cap = 4096) {
  return (int)std::max<size_t>(1, std::min<size_t>((n + block - 1) / block, cap));
}

int frcnn_cap(int P, int K, float thresh) {
  int per = K;
  if (thresh > 0.f) per = std::min(K, (int)std::ceil(1.0 / (double)thresh) + 1);
  return std::max(1, P * per);
}

}  // namespace

int make_levels(Levels& lv, const float* const* a_ptrs, const float* const* b_ptrs,
                const int32_t* level_hw, const float* strides, const float* cell, int L, int A) {
  D2MI_REQUIRE(L >= 1 && L <= D2MI_MAX_LEVELS, "L=%d out of range", L);
  D2MI_REQUIRE(A >= 1 && A <= kMaxA, "A=%d out of range [1,%d]", A, kMaxA);
  lv.L = L;
  lv.A = A;
  for (int l = 0; l < L; ++l) {
    lv.H[l] = level_hw[2 * l];
    lv.W[l] = level_hw[2 * l + 1];
    D2MI_REQUIRE(lv.H[l] > 0 && lv.W[l] > 0, "level %d is empty", l);
    lv.stride[l] = (int)strides[l];
    D2MI_REQUIRE((float)lv.stride[l] == strides[l], "anchor strides must be integers");
    lv.off_a[l] = a_ptrs ? (int64_t)((const float*)a_ptrs[l] - (const float*)a_ptrs[0]) : 0;
    lv.off_b[l] = b_ptrs ? (int64_t)((const float*)b_ptrs[l] - (const float*)b_ptrs[0]) : 0;
    lv.img_a[l] = lv.img_b[l] = (int64_t)lv.H[l] * lv.W[l] * A;
    if (b_ptrs) D2MI_REQUIRE(((uintptr_t)b_ptrs[l] & 15) == 0, "delta tensors must be 16B aligned");
    for (int a = 0; a < A; ++a)
      for (int c = 0; c < 4; ++c) lv.cell[l][a][c] = cell[(l * A + a) * 4 + c];
  }
  return 0;
}

DeltaCfg make_dc(const float* w4, float clamp) {
  DeltaCfg d;
  d.wy = w4[0];
  d.wx = w4[1];
  d.wh = w4[2];
  d.ww = w4[3];
  d.clamp = clamp;
  return d;
}

}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_grid_anchors(int H, int W, float stride, const float* cell_anchors_host,
                                 int A, float* out, void* stream) {
  Levels lv = {};
  int32_t hw[2] = {H, W};
  int rc = make_levels(lv, nullptr, nullptr, hw, &stride, cell_anchors_host, 1, A);
  if (rc) return rc;
  hipLaunchKernelGGL(grid_anchors_kernel, dim3(grid1((size_t)H * W * A)), dim3(256), 0,
                     as_stream(stream), H, W, (int)stride, lv, reinterpret_cast<float4*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_apply_deltas(const float* deltas, const float* boxes, int N, int K,
                                 const float* weights4_host, float scale_clamp, float* out,
                                 void* stream) {
  D2MI_REQUIRE(N >= 0 && K >= 1, "bad apply_deltas sizes");
  if (N == 0) return 0;
  hipLaunchKernelGGL(apply_deltas_kernel, dim3(grid1((size_t)N * K)), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const float4*>(deltas),
                     reinterpret_cast<const float4*>(boxes), N, K, make_dc(weights4_host, scale_clamp),
                     reinterpret_cast<float4*>(out));
  D2MI_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------ RPN
namespace {
struct RpnWs {
  int64_t* seg_start;
  int32_t* seg_len;
  float* tvals;
  int32_t* tidx;
  int32_t* tcount;
  void* topk_ws;
  size_t topk_bytes;
  float4* dec;
  uint64_t* keys;
  int32_t* lens;
  int32_t* keep;
  int32_t* num_keep;
  void* nms_ws;
  size_t nms_bytes;
};

template <typename WS>
void rpn_layout(WS& w, RpnWs* o, int N, int L, int k, int post) {
  const int S = N * L;
  auto p0 = w.template take<int64_t>(S);
  auto p1 = w.template take<int32_t>(S);
  auto p2 = w.template take<float>((size_t)S * k);
  auto p3 = w.template take<int32_t>((size_t)S * k);
  auto p4 = w.template take<int32_t>(S);
  const size_t tb = topk_workspace_size(S, k);
  auto p5 = w.template take<char>(tb);
  auto p6 = w.template take<float4>((size_t)S * k);
  auto p7 = w.template take<uint64_t>((size_t)S * k);
  auto p8 = w.template take<int32_t>(S);
  auto p9 = w.template take<int32_t>((size_t)S * post);
  auto p10 = w.template take<int32_t>(S);
  const size_t nb = nms_core_workspace_size(S, k);
  auto p11 = w.template take<char>(nb);
  if (o) {
    *o = RpnWs{(int64_t*)p0, (int32_t*)p1, (float*)p2, (int32_t*)p3, (int32_t*)p4, (void*)p5, tb,
               (float4*)p6, (uint64_t*)p7, (int32_t*)p8, (int32_t*)p9, (int32_t*)p10, (void*)p11, nb};
  }
}

struct SizerPtr {
  WorkspaceSizer z;
  template <typename T>
  T* take(size_t n) {
    z.take<T>(n);
    return nullptr;
  }
};
}  // namespace

extern "C" size_t d2mi_rpn_proposals_workspace_size(int N, int L, const int32_t* level_hw, int A,
                                                    int pre_nms_topk, int post_nms_topk) {
  int maxlen = 0;
  for (int l = 0; l < L; ++l) maxlen = std::max(maxlen, level_hw[2 * l] * level_hw[2 * l + 1] * A);
  const int k = std::max(1, std::min(pre_nms_topk, maxlen));
  SizerPtr s;
  rpn_layout(s, nullptr, N, L, k, post_nms_topk);
  return s.z.off;
}

extern "C" int d2mi_rpn_proposals(const float* const* logits, const float* const* deltas,
                                  const int32_t* level_hw, const float* strides,
                                  const float* cell_anchors, int L, int A, int N,
                                  const int32_t* image_hw, int pre_nms_topk, int post_nms_topk,
                                  float nms_thresh, float min_box_side_len,
                                  const float* weights4_host, float scale_clamp, float* out_boxes,
                                  float* out_scores, uint8_t* out_valid, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  return d2mi_rpn_proposals_ex(logits, deltas, nullptr, nullptr, level_hw, strides, cell_anchors,
                               L, A, N, image_hw, pre_nms_topk, post_nms_topk, nms_thresh,
                               min_box_side_len, weights4_host, scale_clamp, out_boxes, out_scores,
                               out_valid, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_rpn_proposals_ex(const float* const* logits, const float* const* deltas,
                                     const int64_t* logits_image_stride,
                                     const int64_t* deltas_image_stride,
                                     const int32_t* level_hw, const float* strides,
                                     const float* cell_anchors, int L, int A, int N,
                                     const int32_t* image_hw, int pre_nms_topk,
                                     int post_nms_topk, float nms_thresh,
                                     float min_box_side_len, const float* weights4_host,
                                     float scale_clamp, float* out_boxes, float* out_scores,
                                     uint8_t* out_valid, void* workspace, size_t workspace_bytes,
                                     void* stream) {
  hipStream_t st = as_stream(stream);
  D2MI_REQUIRE(N >= 1 && pre_nms_topk >= 1 && post_nms_topk >= 1, "bad RPN sizes");
  D2MI_REQUIRE(L * post_nms_topk <= kLdsSortCap, "L*post_nms_topk=%d exceeds %d", L * post_nms_topk,
               kLdsSortCap);
  Levels lv = {};
  int rc = make_levels(lv, logits, deltas, level_hw, strides, cell_anchors, L, A);
  if (rc) return rc;
  for (int l = 0; l < L; ++l) {  // strided levels (views of one concatenated buffer)
    if (logits_image_stride) {
      D2MI_REQUIRE(logits_image_stride[l] >= lv.img_a[l], "logits image stride too small");
      lv.img_a[l] = logits_image_stride[l];
    }
    if (deltas_image_stride) {
      D2MI_REQUIRE(deltas_image_stride[l] % 4 == 0 && deltas_image_stride[l] / 4 >= lv.img_b[l],
                   "deltas image stride must be a multiple of 4 covering the level");
      lv.img_b[l] = deltas_image_stride[l] / 4;
    }
  }
  int maxlen = 0;
  for (int l = 0; l < L; ++l) maxlen = std::max(maxlen, lv.H[l] * lv.W[l] * A);
  const int k = std::max(1, std::min(pre_nms_topk, maxlen));
  D2MI_REQUIRE(k <= kLdsSortCap, "pre_nms_topk=%d exceeds %d", k, kLdsSortCap);
  const int S = N * L;
  Workspace w(workspace, workspace_bytes);
  RpnWs o;
  rpn_layout(w, &o, N, L, k, post_nms_topk);
  D2MI_REQUIRE(w.ok(), "RPN workspace too small (%zu < %zu)", workspace_bytes, w.off);
  hipLaunchKernelGGL(seg_setup_kernel, dim3((S + 63) / 64), dim3(64), 0, st, lv, N, 1, k,
                     o.seg_start, o.seg_len, (int32_t*)nullptr);
  D2MI_LAUNCH_CHECK();
  rc = topk_core_ex(logits[0], o.seg_start, o.seg_len, nullptr, S, maxlen, k, 0, o.tvals, o.tidx,
                    o.tcount, o.topk_ws, o.topk_bytes, st);
  if (rc) return rc;
  if (tuning(kTuneRpnCompact) != 0) {
    // the NMS workspace carved as nms_core carves it (its sort keys unused)
    Workspace nw(o.nms_ws, o.nms_bytes);
    nw.take<uint64_t>((size_t)S * k);
    float4* sboxes = nw.take<float4>((size_t)S * k);
    int32_t* sidx = nw.take<int32_t>((size_t)S * k);
    int32_t* scount = nw.take<int32_t>(S);
    const size_t mask_bytes = nms_sorted_workspace_size(S, k);
    void* mask_ws = nw.take<char>(mask_bytes);
    D2MI_REQUIRE(nw.ok(), "RPN NMS workspace too small");
    hipLaunchKernelGGL(rpn_decode_compact_kernel, dim3(S), dim3(1024), 0, st, deltas[0], lv, N, k,
                       o.tvals, o.tidx, o.tcount, image_hw, make_dc(weights4_host, scale_clamp),
                       min_box_side_len, o.dec, sboxes, sidx, scount);
    D2MI_LAUNCH_CHECK();
    rc = nms_sorted(sboxes, sidx, scount, S, k, post_nms_topk, nms_thresh, o.keep, o.num_keep,
                    mask_ws, mask_bytes, st);
    if (rc) return rc;
  } else {  // decode -> keys -> nms_core's sort + gather (A/B)
    hipLaunchKernelGGL(rpn_decode_kernel, dim3(grid1(k, 256, 64), S), dim3(256), 0, st, deltas[0],
                       lv, N, k, o.tvals, o.tidx, o.tcount, image_hw,
                       make_dc(weights4_host, scale_clamp), min_box_side_len, o.dec, o.keys, o.lens);
    D2MI_LAUNCH_CHECK();
    rc = nms_core(o.keys, o.lens, o.dec, nullptr, S, k, post_nms_topk, nms_thresh, o.keep,
                  o.num_keep, o.nms_ws, o.nms_bytes, st);
    if (rc) return rc;
  }
  // tuning "rpn_merge": 1 the merge rank (r5), 0 the one-workgroup bitonic sort (A/B)
  if (tuning(kTuneRpnMerge) != 0) {
    const int span = std::max(L * post_nms_topk, post_nms_topk);
    hipLaunchKernelGGL(rpn_merge_rank_kernel, dim3((span + kMergeT - 1) / kMergeT, N),
                       dim3(kMergeT), (size_t)L * post_nms_topk * sizeof(uint32_t), st, o.dec,
                       o.tvals, o.keep, o.num_keep, L, k, post_nms_topk,
                       reinterpret_cast<float4*>(out_boxes), out_scores, out_valid);
    D2MI_LAUNCH_CHECK();
    return 0;
  }
  int m = 1;
  while (m < L * post_nms_topk) m <<= 1;
  hipLaunchKernelGGL(rpn_merge_kernel, dim3(N), dim3(1024), m * sizeof(uint64_t), st, o.dec,
                     o.tvals, o.keep, o.num_keep, L, k, post_nms_topk,
                     reinterpret_cast<float4*>(out_boxes), out_scores, out_valid);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// ----------------------------------------------------------- Fast R-CNN
namespace {
struct FrcnnWs {
  int32_t* slot2roi;
  uint32_t* maxc;
  int32_t* cnt;
  uint64_t* keys;
  float4* cbox;
  float* cscore;
  int32_t* flat2pos;
  uint64_t* sorted;
  float4* sboxes;
  int32_t* sidx;
  int32_t* count;
  int32_t* keep;
  int32_t* num_keep;
  void* sort_ws;
  size_t sort_bytes;
  void* nms_ws;
  size_t nms_bytes;
};
template <typename WS>
void frcnn_layout(WS& w, FrcnnWs* o, int N, int P, int K, int cap, int max_det) {
  auto a0 = w.template take<int32_t>((size_t)N * P);
  auto a1 = w.template take<uint32_t>(N);
  auto a2 = w.template take<int32_t>(N);
  auto a3 = w.template take<uint64_t>((size_t)N * cap);
  auto a4 = w.template take<float4>((size_t)N * cap);
  auto a5 = w.template take<float>((size_t)N * cap);
  auto a6 = w.template take<int32_t>((size_t)N * P * K);
  auto a7 = w.template take<uint64_t>((size_t)N * cap);
  auto a8 = w.template take<float4>((size_t)N * cap);
  auto a9 = w.template take<int32_t>((size_t)N * cap);
  auto a10 = w.template take<int32_t>(N);
  auto a11 = w.template take<int32_t>((size_t)N * max_det);
  auto a12 = w.template take<int32_t>(N);
  const size_t sb = sort_workspace_size(N, cap);
  auto a13 = w.template take<char>(sb);
  const size_t nb = nms_sorted_workspace_size(N, cap);
  auto a14 = w.template take<char>(nb);
  if (o)
    *o = FrcnnWs{(int32_t*)a0, (uint32_t*)a1, (int32_t*)a2, (uint64_t*)a3, (float4*)a4, (float*)a5,
                 (int32_t*)a6, (uint64_t*)a7, (float4*)a8, (int32_t*)a9, (int32_t*)a10,
                 (int32_t*)a11, (int32_t*)a12, (void*)a13, sb, (void*)a14, nb};
}
}  // namespace

extern "C" size_t d2mi_fast_rcnn_workspace_size(int N, int P, int K, float score_thresh,
                                                int max_det) {
  SizerPtr s;
  frcnn_layout(s, nullptr, N, std::max(1, P), K, frcnn_cap(std::max(1, P), K, score_thresh),
               max_det);
  return s.z.off;
}

extern "C" int d2mi_fast_rcnn_inference(const float* logits, const float* deltas,
                                        const float* proposals, const int32_t* roi_img,
                                        const int32_t* roi_slot, int R, int N, int P, int K,
                                        int cls_agnostic, const int32_t* image_hw,
                                        const float* weights4_host, float scale_clamp,
                                        float score_thresh, float nms_thresh, int max_det,
                                        float* out_boxes, float* out_scores, int64_t* out_classes,
                                        uint8_t* out_valid, int32_t* out_roi, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  D2MI_REQUIRE(N >= 1 && P >= 1 && K >= 1 && R >= 0 && max_det >= 1 && max_det <= 1000,
               "bad fast_rcnn_inference sizes");
  D2MI_REQUIRE(((uintptr_t)deltas & 15) == 0 && ((uintptr_t)proposals & 15) == 0,
               "deltas/proposals must be 16B aligned");
  // cls_agnostic: bit 0 = one class-agnostic box per ROI (deltas [R, 4]),
  // bit 1 = class-agnostic NMS (NMS_CLS_AGNOSTIC: no class offsets)
  D2MI_REQUIRE((cls_agnostic & ~3) == 0, "bad cls_agnostic flags %d", cls_agnostic);
  const int agnostic_box = cls_agnostic & 1, agnostic_nms = (cls_agnostic >> 1) & 1;
  const int cap = frcnn_cap(P, K, score_thresh);
  Workspace w(workspace, workspace_bytes);
  FrcnnWs o;
  frcnn_layout(w, &o, N, P, K, cap, max_det);
  D2MI_REQUIRE(w.ok(), "fast_rcnn workspace too small (%zu < %zu)", workspace_bytes, w.off);
  int32_t* err = error_word();
  D2MI_REQUIRE(fill_bytes(o.slot2roi, (size_t)N * P * 4, 0xff, st) == 0, "fill failed");
  D2MI_REQUIRE(fill_bytes(o.cnt, (size_t)N * 4, 0, st) == 0, "fill failed");
  hipLaunchKernelGGL(fill_u32_kernel, dim3((N + 255) / 256), dim3(256), 0, st, o.maxc, N,
                     0x80000000u /* orderable(+0.0f) */);
  D2MI_LAUNCH_CHECK();
  if (R > 0) {
    hipLaunchKernelGGL(slot_map_kernel, dim3((R + 255) / 256), dim3(256), 0, st, roi_img, roi_slot,
                       R, P, N, o.slot2roi, err);
    D2MI_LAUNCH_CHECK();
    hipLaunchKernelGGL(frcnn_score_kernel, dim3((R + 3) / 4), dim3(256), 0, st, logits,
                       reinterpret_cast<const float4*>(deltas),
                       reinterpret_cast<const float4*>(proposals), roi_img, roi_slot, R, N, P, K,
                       agnostic_box, image_hw, make_dc(weights4_host, scale_clamp), score_thresh,
                       cap, o.maxc, o.cnt, o.keys, o.cbox, o.cscore, err);
    D2MI_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(clamp_lens_kernel, dim3((N + 255) / 256), dim3(256), 0, st, o.cnt, N, cap);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(frcnn_posmap_kernel, dim3(grid1(cap, 256, 64), N), dim3(256), 0, st, o.keys,
                     o.cnt, cap, P, K, o.flat2pos);
  D2MI_LAUNCH_CHECK();
  int rc = sort_keys_segmented(o.keys, o.sorted, o.cnt, N, cap, o.sort_ws, o.sort_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(frcnn_gather_kernel, dim3(grid1(cap, 256, 64), N), dim3(256), 0, st, o.sorted,
                     o.cnt, o.flat2pos, o.cbox, o.maxc, cap, P, K, agnostic_nms, o.sboxes, o.sidx,
                     o.count);
  D2MI_LAUNCH_CHECK();
  rc = nms_sorted(o.sboxes, o.sidx, o.count, N, cap, max_det, nms_thresh, o.keep, o.num_keep,
                  o.nms_ws, o.nms_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(frcnn_output_kernel, dim3((N * max_det + 255) / 256), dim3(256), 0, st, o.keep,
                     o.num_keep, o.keys, o.cbox, o.cscore, o.slot2roi, cap, P, max_det, N,
                     reinterpret_cast<float4*>(out_boxes), out_scores, out_classes, out_valid,
                     out_roi);
  D2MI_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------ RetinaNet
namespace {
struct RetinaWs {
  int64_t* seg_start;
  int32_t* seg_len;
  int32_t* seg_k;
  float* tvals;
  int32_t* tidx;
  int32_t* tcount;
  void* topk_ws;
  size_t topk_bytes;
  uint64_t* keys;
  float4* cbox;
  float* cscore;
  int32_t* ccls;
  uint32_t* maxc;
  int32_t* lens;
  uint64_t* sorted;
  float4* sboxes;
  int32_t* sidx;
  int32_t* count;
  int32_t* keep;
  int32_t* num_keep;
  void* sort_ws;
  size_t sort_bytes;
  void* nms_ws;
  size_t nms_bytes;
};
template <typename WS>
void retina_layout(WS& w, RetinaWs* o, int N, int L, int k, int max_det) {
  const int S = N * L, cap = L * k;
  auto a0 = w.template take<int64_t>(S);
  auto a1 = w.template take<int32_t>(S);
  auto a2 = w.template take<int32_t>(S);
  auto a3 = w.template take<float>((size_t)S * k);
  auto a4 = w.template take<int32_t>((size_t)S * k);
  auto a5 = w.template take<int32_t>(S);
  const size_t tb = topk_workspace_size(S, k);
  auto a6 = w.template take<char>(tb);
  auto a7 = w.template take<uint64_t>((size_t)N * cap);
  auto a8 = w.template take<float4>((size_t)N * cap);
  auto a9 = w.template take<float>((size_t)N * cap);
  auto a10 = w.template take<int32_t>((size_t)N * cap);
  auto a11 = w.template take<uint32_t>(N);
  auto a12 = w.template take<int32_t>(N);
  auto a13 = w.template take<uint64_t>((size_t)N * cap);
  auto a14 = w.template take<float4>((size_t)N * cap);
  auto a15 = w.template take<int32_t>((size_t)N * cap);
  auto a16 = w.template take<int32_t>(N);
  auto a17 = w.template take<int32_t>((size_t)N * max_det);
  auto a18 = w.template take<int32_t>(N);
  const size_t sb = sort_workspace_size(N, cap);
  auto a19 = w.template take<char>(sb);
  const size_t nb = nms_sorted_workspace_size(N, cap);
  auto a20 = w.template take<char>(nb);
  if (o)
    *o = RetinaWs{(int64_t*)a0, (int32_t*)a1, (int32_t*)a2, (float*)a3, (int32_t*)a4,
                  (int32_t*)a5, (void*)a6, tb, (uint64_t*)a7, (float4*)a8, (float*)a9,
                  (int32_t*)a10, (uint32_t*)a11, (int32_t*)a12, (uint64_t*)a13, (float4*)a14,
                  (int32_t*)a15, (int32_t*)a16, (int32_t*)a17, (int32_t*)a18, (void*)a19, sb,
                  (void*)a20, nb};
}
}  // namespace

extern "C" size_t d2mi_retinanet_workspace_size(int N, int L, const int32_t* level_hw, int A,
                                                int K, int topk_candidates) {
  SizerPtr s;
  retina_layout(s, nullptr, N, L, std::max(1, topk_candidates), 1000);
  size_t z = s.z.off;
  if (retina_fused_eligible(L, topk_candidates, 1000))
    z = std::max(z, retina_fused_workspace_size(N, L, level_hw, A, K, topk_candidates));
  return z;
}

extern "C" int d2mi_retinanet_inference(const float* const* cls, const float* const* box,
                                        const int32_t* level_hw, const float* strides,
                                        const float* cell_anchors, int L, int A, int K, int N,
                                        int topk_candidates, float score_thresh, float nms_thresh,
                                        int max_det, const float* weights4_host, float scale_clamp,
                                        float* out_boxes, float* out_scores, int32_t* out_classes,
                                        uint8_t* out_valid, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  hipStream_t st = as_stream(stream);
  D2MI_REQUIRE(N >= 1 && K >= 1 && topk_candidates >= 1 && max_det >= 1 && max_det <= 1000,
               "bad retinanet sizes");
  Levels lv = {};
  int rc = make_levels(lv, cls, box, level_hw, strides, cell_anchors, L, A);
  if (rc) return rc;
  const int k = topk_candidates;
  D2MI_REQUIRE(k <= kLdsSortCap, "topk_candidates=%d exceeds %d", k, kLdsSortCap);
  int64_t maxlen = 0;
  for (int l = 0; l < L; ++l) maxlen = std::max<int64_t>(maxlen, (int64_t)lv.H[l] * lv.W[l] * A * K);
  D2MI_REQUIRE(maxlen < (1ll << 31), "level too large");
  const int mode = tuning(kTuneRetinaFused);
  if (mode != 0 && retina_fused_eligible(L, k, max_det))
    return retinanet_fused(cls, box, lv, level_hw, K, N, k, score_thresh, nms_thresh, max_det,
                           make_dc(weights4_host, scale_clamp), out_boxes, out_scores, out_classes,
                           out_valid, workspace, workspace_bytes, st, mode == 2);
  const int S = N * L, cap = L * k;
  Workspace w(workspace, workspace_bytes);
  RetinaWs o;
  retina_layout(w, &o, N, L, k, max_det);
  D2MI_REQUIRE(w.ok(), "retinanet workspace too small (%zu < %zu)", workspace_bytes, w.off);
  hipLaunchKernelGGL(seg_setup_kernel, dim3((S + 63) / 64), dim3(64), 0, st, lv, N, K, k,
                     o.seg_start, o.seg_len, o.seg_k);
  D2MI_LAUNCH_CHECK();
  // sampled floor: exact, and the decode below keeps j < tcount only
  rc = topk_core_ex(cls[0], o.seg_start, o.seg_len, o.seg_k, S, (int)maxlen, k, 1, o.tvals, o.tidx,
                    o.tcount, o.topk_ws, o.topk_bytes, st, /*sampled_floor=*/true);
  if (rc) return rc;
  hipLaunchKernelGGL(fill_u32_kernel, dim3((N + 255) / 256), dim3(256), 0, st, o.maxc, N,
                     0x007fffffu /* orderable(-inf) */);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(fill_kernel, dim3((N + 255) / 256), dim3(256), 0, st, o.lens, N, cap);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(retina_decode_kernel, dim3(grid1(k, 256, 64), S), dim3(256), 0, st, box[0], lv,
                     N, K, k, o.tvals, o.tidx, o.tcount, score_thresh,
                     make_dc(weights4_host, scale_clamp), cap, o.keys, o.cbox, o.cscore, o.ccls,
                     o.maxc);
  D2MI_LAUNCH_CHECK();
  rc = sort_keys_segmented(o.keys, o.sorted, o.lens, N, cap, o.sort_ws, o.sort_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(retina_gather_kernel, dim3(grid1(cap, 256, 64), N), dim3(256), 0, st, o.sorted,
                     o.lens, o.cbox, o.ccls, o.maxc, cap, o.sboxes, o.sidx, o.count);
  D2MI_LAUNCH_CHECK();
  rc = nms_sorted(o.sboxes, o.sidx, o.count, N, cap, max_det, nms_thresh, o.keep, o.num_keep,
                  o.nms_ws, o.nms_bytes, st);
  if (rc) return rc;
  hipLaunchKernelGGL(retina_output_kernel, dim3((N * max_det + 255) / 256), dim3(256), 0, st,
                     o.keep, o.num_keep, o.cbox, o.cscore, o.ccls, cap, max_det, N,
                     reinterpret_cast<float4*>(out_boxes), out_scores, out_classes, out_valid);
  D2MI_LAUNCH_CHECK();
  return 0;
}
