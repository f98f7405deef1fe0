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
//   4. mask   one wave per (segment, 64-row tile, 64-col tile), four column tiles
//             per workgroup: every lane holds one column box, the 64 row boxes are
//             broadcast from LDS and __ballot(IoU > thr) yields one 64-bit word per row
//   5. scan   one workgroup per segment: each 64-row tile's kept set is the fixed
//             point of a ballot over its column words (r5; serially in scalar
//             registers before), the kept rows' words are OR-ed into the removal
//             bits of the later tiles; stops at max_output_size.
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

// grid (column-tile group, row tile, seg), 4 waves: wave w takes column tile
// 4 * blockIdx.x + w (>= the row tile), the row tile's 64 boxes staged in LDS
// once per workgroup (normalised corners and area) -- a quarter of r4's
// 64-thread workgroups (one per tile pair, half of them exiting at once);
// one wave per column tile keeps the occupancy that hides the IoU's division
// and LDS latency (a workgroup per row tile looping over its column tiles
// measured 1.9x slower).  Each lane holds one column box; __ballot(IoU > thr)
// over the lanes gives row r's word.  IoU is tf_iou's float32 expression
// term by term (the row side's min / max / area computed once), so the
// words are the same bits.
constexpr int kMaskWaves = 4;
__global__ __launch_bounds__(64 * kMaskWaves) void nms_mask_kernel(
    const float4* __restrict__ sboxes, const int32_t* __restrict__ count, int cap, int T,
    float thr, uint64_t* __restrict__ mask, uint64_t* __restrict__ colw) {
  const int rt = blockIdx.y, s = blockIdx.z;
  const int n = count[s];
  const int row0 = rt * 64;
  const int ntc = (n + 63) / 64;
  if (row0 >= n || kMaskWaves * (int)blockIdx.x + kMaskWaves - 1 < rt) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float4 rlo[64];  // ymin, xmin, ymax, xmax
  __shared__ float rarea[64];
  const size_t base = (size_t)s * cap;
  const int rmax = min(64, n - row0);
  if (threadIdx.x < rmax) {
    const float4 a = sboxes[base + row0 + threadIdx.x];
    const float ymin = fminf(a.x, a.z), xmin = fminf(a.y, a.w);
    const float ymax = fmaxf(a.x, a.z), xmax = fmaxf(a.y, a.w);
    rlo[threadIdx.x] = make_float4(ymin, xmin, ymax, xmax);
    rarea[threadIdx.x] = (ymax - ymin) * (xmax - xmin);
  }
  __syncthreads();
  const int ct = kMaskWaves * blockIdx.x + wave;
  if (ct >= rt && ct < ntc) {
    const int col0 = ct * 64;
    const int col = col0 + lane;
    const bool cvalid = col < n;
    const float4 b = cvalid ? sboxes[base + col] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float ymin_j = fminf(b.x, b.z), xmin_j = fminf(b.y, b.w);
    const float ymax_j = fmaxf(b.x, b.z), xmax_j = fmaxf(b.y, b.w);
    const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
    const bool want_col = colw && ct - rt <= 1;
    uint64_t mine = 0, colword = 0;
#pragma unroll 4
    for (int r = 0; r < rmax; ++r) {
      const float4 a = rlo[r];
      const float area_i = rarea[r];
      bool sup = false;
      if (cvalid && col > row0 + r && !(area_i <= 0.f || area_j <= 0.f)) {
        const float iymin = fmaxf(a.x, ymin_j), ixmin = fmaxf(a.y, xmin_j);
        const float iymax = fminf(a.z, ymax_j), ixmax = fminf(a.w, xmax_j);
        const float inter = fmaxf(iymax - iymin, 0.f) * fmaxf(ixmax - ixmin, 0.f);
        sup = inter / ((area_i + area_j) - inter) > thr;
      }
      const uint64_t word = __ballot(sup);
      if (lane == r) mine = word;
      colword |= sup ? 1ull << r : 0ull;
    }
    if (lane < rmax) mask[(base + row0 + lane) * T + ct] = mine;
    if (want_col) colw[(((size_t)s * T + rt) * 2 + (ct - rt)) * 64 + lane] = colword;
  }
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


// r5 scan (tuning "nms_scan" = 1, for T <= 64 tiles): the serial 64-row
// resolve of nms_scan_kernel (one dependent v_readlane / branch round per row,
// ~4 us per tile) becomes a fixed point over the tile, and no global load
// latency sits between two tiles' resolves:
//  * wave 0 resolves tile t: lane c is row c, alive unless removed;
//    K <- ballot(alive && !(colD[c] & K)) from K = ballot(alive) until K
//    repeats.  Row c's decision depends only on rows < c, so row c is final
//    after c + 1 rounds and the only fixed point is the greedy kept set (bit
//    for bit); the rounds needed are the length of the longest chain of
//    flipping decisions -- a few for real boxes.
//  * the rows tile t suppresses in tile t + 1 come from the block's column
//    words too (one ballot: the "carry" register), so tile t + 1 never waits
//    on tile t's propagation;
//  * waves 1..8 OR the kept rows of tile t - 1 into the removal words of tiles
//    >= t + 1 (LDS atomics, order-free) from row words they loaded two tiles
//    earlier, while wave 0 resolves tile t; one barrier per tile.  Waves 1..4
//    take the even tiles' rows, 5..8 the odd ones' (16 rows each).
//  * wave 0 loads a tile's column words and output indices two tiles ahead.
// Load placement: every load is issued unconditionally (clamped addresses --
// the waitcnt analysis counts a conditional load as possibly absent and then
// waits for everything); wave 0's two operand sets are used in a loop written
// out twice, so no register holding an in-flight load is moved (a move waits
// for the load); a propagation wave holds ONE set (a second set in the same
// wave made the compiler's waits cover both); wave 0 and the propagation
// waves run separate loops with one barrier per tile each (a hardware barrier
// counts waves, not code locations); the kept indices collect in LDS and are
// written out at the end (global stores count in the same vmcnt).
constexpr int kFpProp = 4;          // propagation waves per tile parity, 16 rows each
constexpr int kFpRows = 64 / kFpProp;
struct FpTile {
  uint64_t d, nx;  // column words of the diagonal block, of the next block
  int32_t ix;      // the row's output index
};
__global__ __launch_bounds__(64 * (1 + 2 * kFpProp)) void nms_scan_fp_kernel(
    const uint64_t* __restrict__ mask, const uint64_t* __restrict__ colw,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ count, int cap, int T,
    int max_out, int32_t* __restrict__ keep, int32_t* __restrict__ num_keep) {
  extern __shared__ int32_t s_out[];  // min(max_out, cap) kept indices
  __shared__ uint64_t removed[64];
  __shared__ uint64_t s_keptm[2];
  __shared__ int s_kept[2];  // (double-buffered: wave 0 may publish tile t + 1's
                             // count before a slow wave has read tile t's)
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = count[s];
  const int nt = (n + 63) / 64;
  if (threadIdx.x < 64) removed[threadIdx.x] = 0;
  const size_t base = (size_t)s * cap;
  const uint64_t* cw = colw + (size_t)s * T * 2 * 64;
  __syncthreads();
  int kept = 0;
  if (wave == 0) {
    auto load_tile = [&](int t, FpTile& f) {
      const int tc = min(t, max(nt - 1, 0));
      f.d = cw[((size_t)tc * 2) * 64 + lane];
      f.nx = cw[((size_t)tc * 2 + 1) * 64 + lane];  // (unused when tc is the last tile)
      f.ix = idx[base + min(t * 64 + lane, max(n - 1, 0))];
    };
    FpTile fa, fb;
    load_tile(0, fa);
    load_tile(1, fb);
    uint64_t carry = 0;
    auto resolve = [&](int t, FpTile& f) {
      uint64_t w = removed[t] | carry;
      const int rem = n - t * 64;
      if (rem < 64) w |= ~((1ull << rem) - 1ull);
      const bool alive = !((w >> lane) & 1ull);
      const uint64_t colD = f.d;
      uint64_t K = __ballot(alive);
      for (int it = 0; it <= 64; ++it) {
        const uint64_t K2 = __ballot(alive && (colD & K) == 0ull);
        if (K2 == K) break;
        K = K2;
      }
      const int room = max_out - kept;
      if (__popcll(K) > room) {  // the greedy stops at max_output_size
        uint64_t k2 = 0, rest = K;
        for (int q = 0; q < room; ++q) {
          const uint64_t low = rest & (~rest + 1ull);
          k2 |= low;
          rest ^= low;
        }
        K = k2;
      }
      if ((K >> lane) & 1ull) s_out[kept + __popcll(K & ((1ull << lane) - 1ull))] = f.ix;
      kept += __popcll(K);
      carry = t + 1 < nt ? __ballot((f.nx & K) != 0ull) : 0ull;
      if (lane == 0) {
        s_keptm[t & 1] = K;
        s_kept[t & 1] = kept;
      }
      load_tile(t + 2, f);
      __syncthreads();
    };
    for (int t = 0; t < nt; t += 2) {
      resolve(t, fa);
      if (kept >= max_out || t + 1 >= nt) break;
      resolve(t + 1, fb);
      if (kept >= max_out) break;
    }
  } else {
    // propagation waves 1..4 take the even tiles' rows, 5..8 the odd ones':
    // each wave's one set of row words is used two tiles after its load (a
    // second set in the same wave makes the compiler's waits cover both)
    const int par = (wave - 1) / kFpProp;
    const int r0 = ((wave - 1) % kFpProp) * kFpRows;  // rows r0 .. r0 + 15 of a tile
    auto load_rows = [&](int j, uint64_t* v) {  // clamped: always issued
      const int jc = min(j, max(nt - 1, 0));
      const int t2 = min(j + 2 + lane, T - 1);
#pragma unroll
      for (int r = 0; r < kFpRows; ++r)  // (rows past cap only on clamped, unused loads)
        v[r] = mask[(base + (size_t)min(jc * 64 + r0 + r, cap - 1)) * T + t2];
    };
    uint64_t p[kFpRows];
    load_rows(par, p);
    for (int t = 0; t < nt; ++t) {
      const int j = t - 1;  // tile j's kept rows into the removal words of tiles >= t + 1
      if (j >= 0 && (j & 1) == par) {
        const uint64_t Kj = s_keptm[j & 1];
        const int t2 = j + 2 + lane;
        if ((Kj >> r0) & ((1ull << kFpRows) - 1ull) && t2 < nt) {
          uint64_t acc = 0;
#pragma unroll
          for (int r = 0; r < kFpRows; ++r) acc |= ((Kj >> (r0 + r)) & 1ull) ? p[r] : 0ull;
          if (acc) atomicOr(reinterpret_cast<unsigned long long*>(&removed[t2]),
                            (unsigned long long)acc);
        }
        load_rows(j + 2, p);
      }
      __syncthreads();
      kept = s_kept[t & 1];
      if (kept >= max_out) break;
    }
  }
  __syncthreads();  // (every wave's kept is the final count: wave 0's own, the
                    // others' read after each tile's barrier)
  int32_t* out = keep + (size_t)s * max_out;
  for (int i = threadIdx.x; i < max_out; i += blockDim.x) out[i] = i < kept ? s_out[i] : -1;
  if (threadIdx.x == 0) num_keep[s] = kept;
}

}  // namespace

size_t nms_sorted_workspace_size(int S, int cap) {
  const int T = (cap + 63) / 64;
  WorkspaceSizer z;
  z.take<uint64_t>((size_t)S * cap * T);  // mask
  z.take<uint64_t>((size_t)S * T * 2 * 64);  // column words (the fixed-point scan)
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
  uint64_t* colw = w.take<uint64_t>((size_t)S * T * 2 * 64);
  D2MI_REQUIRE(w.ok(), "NMS mask workspace too small (%zu < %zu)", ws_bytes, w.off);
  // tuning "nms_scan": 1 the fixed-point scan (r5) where its removal words
  // fit one propagation lane per tile (T <= 64: <= 4,096 candidates), 0 the
  // serial-resolve scan (A/B)
  const bool fp = tuning(kTuneNmsScan) != 0 && T <= 64;
  hipLaunchKernelGGL(nms_mask_kernel, dim3((T + kMaskWaves - 1) / kMaskWaves, T, S),
                     dim3(64 * kMaskWaves), 0, stream, sboxes, count, cap, T, iou_thr, mask,
                     fp ? colw : nullptr);
  D2MI_LAUNCH_CHECK();
  if (fp)
    hipLaunchKernelGGL(nms_scan_fp_kernel, dim3(S), dim3(64 * (1 + 2 * kFpProp)),
                       (size_t)std::max(1, std::min(max_out, cap)) * sizeof(int32_t), stream, mask, colw,
                       sidx, count, cap, T, max_out, keep, num_keep);
  else
    hipLaunchKernelGGL(nms_scan_kernel, dim3(S), dim3(64 * kScanWaves), T * sizeof(uint64_t),
                       stream, mask, sidx, count, cap, T, max_out, keep, num_keep);
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
