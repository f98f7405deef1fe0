// Segmented greedy NMS with TF NonMaxSuppressionV3 semantics on gfx950.
//
// Reference call sites: lib/layers/nms.py:23 (batch_nms),
// lib/modeling/proposal_generator/rpn_outputs.py:90, roi_heads/fast_rcnn.py:145,
// single_stage_heads/retinanet.py:353.  TF's CPU kernel pops candidates from a
// max-heap (score desc, lowest index first on ties) and drops a candidate when
// IoU(candidate, any selected) > threshold.  That is exactly a scan of the
// score-sorted list against an upper-triangular "row i suppresses col j" bit
// matrix, which is what runs here:
//
//   1. keys   desc_key(score, local index) per candidate (NaN / -inf never selected)
//   2. sort   segmented counting-rank sort in LDS (<= 8192), else 8192-key tiles + merge passes (sort.hip)
//   3. gather boxes into sorted order, count selectable candidates
//   4. mask   one wave per (segment, 64-row tile, 64-col tile): every lane holds one
//             column box, the 64 row boxes are broadcast from LDS and
//             __ballot(IoU > thr) yields one 64-bit word per row
//   5. scan   one wave per segment: the diagonal words of a 64-row tile are
//             resolved serially in scalar registers (v_readlane), the kept rows'
//             words are OR-ed into the removal bits of the later tiles; stops at
//             max_output_size.
// IoU is the float32 expression of TF's IOU() in the same evaluation order
// (compiled with -ffp-contract=off), so the kept indices are bit-exact.
#include "internal.h"

namespace d2mi {
namespace {

__global__ void nms_keys_kernel(const float* __restrict__ scores,
                                const int32_t* __restrict__ seg_offsets, int S, int cap,
                                uint64_t* __restrict__ keys, int32_t* __restrict__ lens,
                                int32_t* err) {
  const int s = blockIdx.y;
  const int begin = seg_offsets[s];
  int len = seg_offsets[s + 1] - begin;
  if (len > cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, kErrNmsCapacity);
    len = cap;
  }
  if (len < 0) len = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) lens[s] = len;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x)
    keys[(size_t)s * cap + i] = desc_key(scores[begin + i], (uint32_t)i);
}

// Gathers boxes in sorted order and counts selectable candidates.
__global__ void nms_prep_kernel(const uint64_t* __restrict__ sorted, const int32_t* lens,
                                const float4* __restrict__ boxes, const int32_t* box_off,
                                int cap, float4* __restrict__ sboxes, int32_t* __restrict__ idx,
                                int32_t* __restrict__ count) {
  const int s = blockIdx.y;
  const int len = lens[s];
  const size_t base = (size_t)s * cap;
  const int off = box_off ? box_off[s] : (int)base;
  if (len == 0 && blockIdx.x == 0 && threadIdx.x == 0) count[s] = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
    const uint64_t k = sorted[base + i];
    const bool valid = k != ~0ull;
    const uint32_t li = (uint32_t)(k & 0xffffffffu);
    idx[base + i] = valid ? (int32_t)li : -1;
    sboxes[base + i] = valid ? boxes[off + li] : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool next_valid = (i + 1 < len) && sorted[base + i + 1] != ~0ull;
    if (valid && !next_valid) count[s] = i + 1;
    if (i == 0 && !valid) count[s] = 0;
  }
}

// grid (colTile, rowTile, seg), 64 threads.
__global__ __launch_bounds__(64) void nms_mask_kernel(const float4* __restrict__ sboxes,
                                                      const int32_t* __restrict__ count, int cap,
                                                      int T, float thr,
                                                      uint64_t* __restrict__ mask) {
  const int ct = blockIdx.x, rt = blockIdx.y, s = blockIdx.z;
  if (ct < rt) return;
  const int n = count[s];
  const int row0 = rt * 64, col0 = ct * 64;
  if (row0 >= n || col0 >= n) return;
  const int lane = threadIdx.x;
  __shared__ float4 rows[64];
  const size_t base = (size_t)s * cap;
  const int rmax = min(64, n - row0);
  if (lane < rmax) rows[lane] = sboxes[base + row0 + lane];
  __syncthreads();
  const int col = col0 + lane;
  const bool cvalid = col < n;
  const float4 cb = cvalid ? sboxes[base + col] : make_float4(0.f, 0.f, 0.f, 0.f);
  uint64_t mine = 0;
  for (int r = 0; r < rmax; ++r) {
    const bool sup = cvalid && (col > row0 + r) && (tf_iou(rows[r], cb) > thr);
    const uint64_t word = __ballot(sup);
    if (lane == r) mine = word;
  }
  if (lane < rmax) mask[(base + row0 + lane) * T + ct] = mine;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// One workgroup of four waves per segment; removed[] lives in LDS (T words).
// Wave 0 resolves each 64-row tile serially (the diagonal words in scalar
// registers via v_readlane); then all four waves propagate the kept rows
// into the removal words of the later tiles, each wave a quarter of the rows
// (16 mask loads in flight per lane: one round of load latency per tile
// instead of four), combined with an LDS atomic OR (order-free: exact).
constexpr int kScanWaves = 4;
__global__ __launch_bounds__(64 * kScanWaves) void nms_scan_kernel(
    const uint64_t* __restrict__ mask, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ count, int cap, int T, int max_out, int32_t* __restrict__ keep,
    int32_t* __restrict__ num_keep) {
  extern __shared__ uint64_t removed[];
  __shared__ uint64_t s_keptm;
  __shared__ int s_kept;
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = count[s];
  const int nt = (n + 63) / 64;
  for (int t = threadIdx.x; t < nt; t += blockDim.x) removed[t] = 0;
  __syncthreads();
  const size_t base = (size_t)s * cap;
  int32_t* out = keep + (size_t)s * max_out;
  int kept = 0;
  constexpr int RW = 64 / kScanWaves;  // propagation rows per wave
  const int r0 = wave * RW;
  // wave 0 holds the next tile's diagonal words and output indices in flight
  // while the current tile resolves and propagates (neither depends on
  // removed[]).  (Issuing the propagation loads before the resolve too
  // measured slower: 157 vs 144 us per RPN scan.)
  uint64_t diag_next = 0;
  int32_t idx_next = 0;
  if (wave == 0 && nt > 0) {
    diag_next = lane < n ? mask[(base + lane) * T] : 0ull;
    idx_next = lane < n ? idx[base + lane] : 0;
  }
  for (int t = 0; t < nt && kept < max_out; ++t) {
    const int t2a = t + 1 + lane;  // this lane's first later tile
    if (wave == 0) {
      const int row = t * 64 + lane;
      const uint64_t diag = diag_next;
      const int32_t my_idx = idx_next;
      if (t + 1 < nt) {
        const int nrow = row + 64;
        diag_next = nrow < n ? mask[(base + nrow) * T + t + 1] : 0ull;
        idx_next = nrow < n ? idx[base + nrow] : 0;
      }
      const int rem = n - t * 64;
      uint64_t w = removed[t];
      if (rem < 64) w |= ~((1ull << rem) - 1ull);
      uint64_t keptm = 0;
      for (int r = 0; r < 64; ++r) {
        if (kept >= max_out) break;
        if (!((w >> r) & 1ull)) {
          keptm |= 1ull << r;
          ++kept;
          w |= readlane64(diag, r);
        }
      }
      if ((keptm >> lane) & 1ull) {
        const int pos = (kept - __popcll(keptm)) + __popcll(keptm & ((1ull << lane) - 1ull));
        out[pos] = my_idx;
      }
      if (lane == 0) {
        s_keptm = keptm;
        s_kept = kept;
      }
    }
    __syncthreads();
    const uint64_t keptm = s_keptm;
    kept = s_kept;
    if (kept >= max_out) break;  // uniform: every wave read the same s_kept
    // propagate the kept rows of tile t (not the last, so all 64 rows exist)
    // into the removal words of the later tiles: wave v takes rows 16v..16v+15
    if ((keptm >> r0) & ((1ull << RW) - 1ull)) {
      for (int t2 = t2a; t2 < nt; t2 += 64) {
        const uint64_t* col = mask + (base + (size_t)t * 64 + r0) * T + t2;
        uint64_t v[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) v[r] = col[(size_t)r * T];
        uint64_t acc = 0;
#pragma unroll
        for (int r = 0; r < RW; ++r) acc |= ((keptm >> (r0 + r)) & 1ull) ? v[r] : 0ull;
        if (acc) atomicOr(reinterpret_cast<unsigned long long*>(&removed[t2]),
                          (unsigned long long)acc);
      }
    }
    __syncthreads();
  }
  for (int i = kept + (int)threadIdx.x; i < max_out; i += blockDim.x) out[i] = -1;
  if (threadIdx.x == 0) num_keep[s] = kept;
}

}  // namespace

size_t nms_sorted_workspace_size(int S, int cap) {
  const int T = (cap + 63) / 64;
  WorkspaceSizer z;
  z.take<uint64_t>((size_t)S * cap * T);  // mask
  return z.off;
}

int nms_sorted(const float4* sboxes, const int32_t* sidx, const int32_t* count, int S, int cap,
               int max_out, float iou_thr, int32_t* keep, int32_t* num_keep, void* ws,
               size_t ws_bytes, hipStream_t stream) {
  if (S == 0) return 0;
  D2MI_REQUIRE(max_out >= 0, "max_output_size must be >= 0");
  if (cap == 0 || max_out == 0) {
    D2MI_REQUIRE(fill_bytes(num_keep, S * sizeof(int32_t), 0, stream) == 0, "fill failed");
    if (max_out > 0)
      D2MI_REQUIRE(fill_bytes(keep, (size_t)S * max_out * 4, 0xff, stream) == 0, "fill failed");
    return 0;
  }
  const int T = (cap + 63) / 64;
  Workspace w(ws, ws_bytes);
  uint64_t* mask = w.take<uint64_t>((size_t)S * cap * T);
  D2MI_REQUIRE(w.ok(), "NMS mask workspace too small (%zu < %zu)", ws_bytes, w.off);
  hipLaunchKernelGGL(nms_mask_kernel, dim3(T, T, S), dim3(64), 0, stream, sboxes, count, cap, T,
                     iou_thr, mask);
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(nms_scan_kernel, dim3(S), dim3(64 * kScanWaves), T * sizeof(uint64_t), stream,
                     mask, sidx,
                     count, cap, T, max_out, keep, num_keep);
  D2MI_LAUNCH_CHECK();
  return 0;
}

size_t nms_core_workspace_size(int S, int cap) {
  WorkspaceSizer z;
  z.take<uint64_t>((size_t)S * cap);      // sorted keys
  z.take<float4>((size_t)S * cap);        // sorted boxes
  z.take<int32_t>((size_t)S * cap);       // sorted local idx
  z.take<int32_t>(S);                     // count
  z.take<char>(nms_sorted_workspace_size(S, cap));
  z.take<char>(sort_workspace_size(S, cap));
  return z.off;
}

int nms_core(const uint64_t* keys, const int32_t* lens, const float4* boxes,
             const int32_t* box_off, int S, int cap, int max_out, float iou_thr, int32_t* keep,
             int32_t* num_keep, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (S == 0) return 0;
  Workspace w(ws, ws_bytes);
  uint64_t* sorted = w.take<uint64_t>((size_t)S * cap);
  float4* sboxes = w.take<float4>((size_t)S * cap);
  int32_t* idx = w.take<int32_t>((size_t)S * cap);
  int32_t* count = w.take<int32_t>(S);
  const size_t mask_bytes = nms_sorted_workspace_size(S, cap);
  void* mask_ws = w.take<char>(mask_bytes);
  const size_t sort_bytes = sort_workspace_size(S, cap);
  void* sort_ws = w.take<char>(sort_bytes);
  D2MI_REQUIRE(w.ok(), "NMS workspace too small (%zu < %zu)", ws_bytes, w.off);
  if (cap > 0) {
    int rc = sort_keys_segmented(keys, sorted, lens, S, cap, sort_ws, sort_bytes, stream);
    if (rc) return rc;
    const int gx = std::min((cap + 255) / 256, 64);
    hipLaunchKernelGGL(nms_prep_kernel, dim3(gx, S), dim3(256), 0, stream, sorted, lens, boxes,
                       box_off, cap, sboxes, idx, count);
    D2MI_LAUNCH_CHECK();
  }
  return nms_sorted(sboxes, idx, count, S, cap, max_out, iou_thr, keep, num_keep, mask_ws,
                    mask_bytes, stream);
}

}  // namespace d2mi

using namespace d2mi;

extern "C" size_t d2mi_nms_workspace_size(int num_segs, int seg_capacity) {
  WorkspaceSizer z;
  z.take<uint64_t>((size_t)num_segs * seg_capacity);
  z.take<int32_t>(num_segs);
  z.take<char>(nms_core_workspace_size(num_segs, seg_capacity));
  return z.off;
}

extern "C" int d2mi_nms(const float* boxes, const float* scores, const int32_t* seg_offsets,
                        int num_segs, int seg_capacity, int max_out, float iou_threshold,
                        int32_t* keep, int32_t* num_keep, void* workspace,
                        size_t workspace_bytes, void* stream) {
  D2MI_REQUIRE(num_segs >= 0 && seg_capacity >= 0, "bad NMS sizes");
  D2MI_REQUIRE(iou_threshold >= 0.f && iou_threshold <= 1.f,
               "iou_threshold must be in [0, 1], got %f", (double)iou_threshold);
  D2MI_REQUIRE(max_out >= 0, "max_output_size must be >= 0, got %d", max_out);
  D2MI_REQUIRE(((uintptr_t)boxes & 15) == 0, "boxes must be 16-byte aligned");
  if (num_segs == 0) return 0;
  hipStream_t st = as_stream(stream);
  Workspace w(workspace, workspace_bytes);
  uint64_t* keys = w.take<uint64_t>((size_t)num_segs * seg_capacity);
  int32_t* lens = w.take<int32_t>(num_segs);
  const size_t core = nms_core_workspace_size(num_segs, seg_capacity);
  void* core_ws = w.take<char>(core);
  D2MI_REQUIRE(w.ok(), "NMS workspace too small (%zu < %zu)", workspace_bytes, w.off);
  int32_t* err = error_word();
  const int gx = std::max(1, std::min((seg_capacity + 255) / 256, 64));
  hipLaunchKernelGGL(nms_keys_kernel, dim3(gx, num_segs), dim3(256), 0, st, scores, seg_offsets,
                     num_segs, seg_capacity, keys, lens, err);
  D2MI_LAUNCH_CHECK();
  // segment boxes start at seg_offsets[s]
  return nms_core(keys, lens, reinterpret_cast<const float4*>(boxes), seg_offsets, num_segs,
                  seg_capacity, max_out, iou_threshold, keep, num_keep, core_ws, core, st);
}
