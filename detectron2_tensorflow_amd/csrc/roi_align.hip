// Multi-level ROIAlign / crop_and_resize forward + backward for gfx950.
//
// Restates, per output element, the exact float32 sequence of
//   lib/modeling/poolers.py:11-49        assign_boxes_to_levels
//   lib/layers/roi_align.py:45-66        ROIAlign.call (boxes * spatial_scale, SR crop,
//                                         avg_pool SR x SR)
//   lib/layers/functional.py:100-166     crop_and_resize wrapper (SYMMETRIC pad 1 + box
//                                         re-normalisation, aligned / unaligned)
//   TF 1.15 CropAndResize CPU kernel     bilinear, extrapolation value 0
// The SYMMETRIC pad is never materialised: padded index p maps to the source
// row clamp(p - 1, 0, H - 1), which is exactly what MirrorPad(SYMMETRIC, 1) holds.
//
// Data layout: NHWC feature maps, C contiguous. One wave owns one output bin
// (all C channels): for C = 256 each lane moves one float4 per corner, so every
// corner fetch is a fully coalesced 1 KiB wave-instruction and every output bin
// one 1 KiB store. A 256-thread workgroup = 4 waves walks up to 64 bins of one
// ROI, so the per-ROI geometry (level, normalised box) stays in scalar registers.
#include "common.h"
#include "internal.h"

#include <climits>

namespace d2mi {
namespace {

struct RoiArgs {
  const float* feat[D2MI_MAX_LEVELS];
  float* gfeat[D2MI_MAX_LEVELS];
  int N[D2MI_MAX_LEVELS], H[D2MI_MAX_LEVELS], W[D2MI_MAX_LEVELS];
  float scale[D2MI_MAX_LEVELS];
  int L, C;
  const float* boxes;
  const int32_t* box_ind;
  int R;
  int out_h, out_w, sr, box_mode, pad_border, assign;
  int min_level, max_level, canon_size, canon_level;
  int32_t* level_out;
  float* out;
  const float* gout;
  int32_t* err;
  int bpb;  // forward: output bins per workgroup (16, 32 or 64)
  int xcd_remap;  // forward: ROIs spread XCD-contiguously (roi_fwd tuning bit 8)
  // backward over one or two ROI sets of the same maps (Contrib::set picks):
  // each set's grad_out and its sampling ratio (the avg-pool divisor)
  const float* gout_s[2];
  int sr_s[2];
  int acc_mask;  // backward: bit l = level l's map already holds a gradient to add to
};

struct RoiGeom {
  int lvl, n, Hp, Wp, H, W, ch, cw;
  float y1, x1, y2, x2, hs, ws;
  bool ok;
};

// assign_boxes_to_levels (poolers.py:37-48), float32 throughout.
__device__ __forceinline__ int assign_level(float4 b, const RoiArgs& a) {
  const float area = (b.z - b.x) * (b.w - b.y);              // box_list_ops.area
  const float size = sqrtf(area);                              // tf.sqrt
  const float t = size / (float)a.canon_size + 2.220446049250313e-16f;  // + eps
  const float v = (float)a.canon_level + logf(t) / 0.6931471805599453f; // / math.log(2)
  const float fl = floorf(v);
  long long lv;
  // tf.cast(float -> int64) of NaN/inf/out-of-range gives INT64_MIN on x86,
  // which clip_by_value then maps to min_level.
  if (!(fl >= -9.2e18f && fl <= 9.2e18f)) lv = (long long)a.min_level;
  else lv = (long long)fl;
  if (lv < a.min_level) lv = a.min_level;
  if (lv > a.max_level) lv = a.max_level;
  return (int)(lv - a.min_level);
}

__device__ __forceinline__ RoiGeom roi_geom(const RoiArgs& a, int r) {
  RoiGeom g;
  const float4 b0 = reinterpret_cast<const float4*>(a.boxes)[r];
  g.lvl = (a.assign && a.L > 1) ? assign_level(b0, a) : 0;
  g.n = a.box_ind[r];
  g.ok = (g.n >= 0 && g.n < a.N[g.lvl]);
  g.H = a.H[g.lvl];
  g.W = a.W[g.lvl];
  const int S = a.sr > 0 ? a.sr : 1;
  g.ch = a.out_h * S;
  g.cw = a.out_w * S;
  float ymin = b0.x, xmin = b0.y, ymax = b0.z, xmax = b0.w;
  if (a.box_mode != 0) {
    // ROIAlign.call: boxes * spatial_scale (roi_align.py:55)
    const float s = a.scale[g.lvl];
    ymin = ymin * s; xmin = xmin * s; ymax = ymax * s; xmax = xmax * s;
  }
  g.Hp = g.H; g.Wp = g.W;
  if (a.pad_border) {  // functional.py:123-126
    g.Hp = g.H + 2; g.Wp = g.W + 2;
    ymin = ymin + 1.f; xmin = xmin + 1.f; ymax = ymax + 1.f; xmax = xmax + 1.f;
  }
  if (a.box_mode == 1) {  // aligned, functional.py:138-152
    const float sh = (ymax - ymin) / (float)g.ch;
    const float sw = (xmax - xmin) / (float)g.cw;
    const float i0 = (float)(g.Hp - 1), i1 = (float)(g.Wp - 1);
    const float ny = ((ymin + sh / 2.f) - 0.5f) / i0;
    const float nx = ((xmin + sw / 2.f) - 0.5f) / i1;
    const float nh = (sh * (float)(g.ch - 1)) / i0;
    const float nw = (sw * (float)(g.cw - 1)) / i1;
    g.y1 = ny; g.x1 = nx; g.y2 = ny + nh; g.x2 = nx + nw;
  } else if (a.box_mode == 2) {  // unaligned, functional.py:153-159
    const float i0 = (float)g.Hp, i1 = (float)g.Wp;
    g.y1 = ymin / i0; g.y2 = ymax / i0; g.x1 = xmin / i1; g.x2 = xmax / i1;
  } else {  // raw normalised boxes
    g.y1 = ymin; g.x1 = xmin; g.y2 = ymax; g.x2 = xmax;
  }
  // TF CropAndResize: height_scale / width_scale
  g.hs = g.ch > 1 ? ((g.y2 - g.y1) * (float)(g.Hp - 1)) / (float)(g.ch - 1) : 0.f;
  g.ws = g.cw > 1 ? ((g.x2 - g.x1) * (float)(g.Wp - 1)) / (float)(g.cw - 1) : 0.f;
  return g;
}

__device__ __forceinline__ float in_coord(float c1, float c2, float scale, int i, int crop,
                                          int img) {
  if (crop > 1) return c1 * (float)(img - 1) + (float)i * scale;
  // 0.5 * (y1 + y2) * (image_height - 1) is evaluated in double by the C++ kernel
  return (float)(0.5 * (double)(c1 + c2) * (double)(img - 1));
}

// One bilinear sample position of the padded map, mapped to source rows/cols.
struct Tap {
  int r0, r1;      // source rows (top, bottom)
  float lerp;      // y_lerp / x_lerp
  bool valid;
};

__device__ __forceinline__ Tap make_tap(float in, int img_p, int img, bool pad) {
  Tap t;
  t.valid = in >= 0.f && in <= (float)(img_p - 1);  // NaN -> extrapolate (TF: UB)
  const float fl = floorf(in);
  const int lo = (int)fl;
  const int hi = (int)ceilf(in);
  t.lerp = in - (float)lo;
  if (pad) {
    t.r0 = min(max(lo - 1, 0), img - 1);
    t.r1 = min(max(hi - 1, 0), img - 1);
  } else {
    t.r0 = min(max(lo, 0), img - 1);
    t.r1 = min(max(hi, 0), img - 1);
  }
  return t;
}

__device__ __forceinline__ float4 lerp4(float4 a, float4 b, float t) {
  return make_float4(a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t, a.z + (b.z - a.z) * t,
                     a.w + (b.w - a.w) * t);
}

// Forward grid: (R, ceil(bins / bpb)); bpb = 64 bins per 4-wave workgroup,
// halved (down to 16) while the grid has fewer than 2048 workgroups, so the
// few-ROI launches (the mask pooler's foreground ROIs) still fill 256 CUs.
constexpr int kMaxBinsPerBlock = 64, kMinBinsPerBlock = 16, kFwdMinBlocks = 2048;

// U: bins per wave iteration in the C = 256 path (their 4U corner loads are
// in flight together); NT: output rows stored non-temporally (streamed past
// the L2 the feature maps are being gathered through); XCD: ROI r taken from
// a bijective XCD-contiguous remap of blockIdx.x (ROIs that neighbour in the
// sampled layout -- foreground proposals of one GT -- share an XCD's L2).
template <bool NTL>
__device__ __forceinline__ float4 ld_row4(const float4* p) {
  if constexpr (NTL) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

template <bool VEC4, int U = 4, bool NT = false, bool NTL = false>
__global__ __launch_bounds__(256) void roi_align_fwd_kernel(RoiArgs a) {
  int r = blockIdx.x;
  if (a.xcd_remap) {
    const int nwg = gridDim.x, q = nwg / 8, r8 = nwg % 8, xcd = r % 8;
    r = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + r / 8;
  }
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const RoiGeom g = roi_geom(a, r);
  if (threadIdx.x == 0 && blockIdx.y == 0) {
    if (a.level_out) a.level_out[r] = g.lvl;
    if (!g.ok) atomicOr(a.err, kErrBoxInd);
  }
  const int nbins = a.out_h * a.out_w;
  const int S = a.sr > 0 ? a.sr : 1;
  const float inv = a.sr > 0 ? (float)(a.sr * a.sr) : 1.f;
  const float* base = a.feat[g.lvl] + (size_t)(g.ok ? g.n : 0) * g.H * g.W * a.C;
  const int C = a.C;
  const bool pad = a.pad_border != 0;
  const int b_end = min(nbins, (int)(blockIdx.y + 1) * a.bpb);
  if (VEC4 && S == 1 && C == 256) {
    // Common case (C = 256, one sample per bin): U bins per wave iteration with
    // all 4U corner loads issued before any is consumed (the taps are clamped
    // to valid rows, so the loads are unconditional; invalid samples are zeroed
    // after) — memory-level parallelism instead of one latency per bin.
    const float4* p = reinterpret_cast<const float4*>(base);
    for (int bb = blockIdx.y * a.bpb + wave; bb < b_end; bb += 4 * U) {
      float4 c00[U], c01[U], c10[U], c11[U];
      float ly[U], lx[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int bin = min(bb + 4 * u, b_end - 1);
        const int oy = bin / a.out_w, ox = bin - oy * a.out_w;
        const Tap ty = make_tap(in_coord(g.y1, g.y2, g.hs, oy, g.ch, g.Hp), g.Hp, g.H, pad);
        const Tap tx = make_tap(in_coord(g.x1, g.x2, g.ws, ox, g.cw, g.Wp), g.Wp, g.W, pad);
        ok[u] = g.ok && ty.valid && tx.valid;
        ly[u] = ty.lerp;
        lx[u] = tx.lerp;
        c00[u] = ld_row4<NTL>(p + ((size_t)ty.r0 * g.W + tx.r0) * 64 + lane);
        c01[u] = ld_row4<NTL>(p + ((size_t)ty.r0 * g.W + tx.r1) * 64 + lane);
        c10[u] = ld_row4<NTL>(p + ((size_t)ty.r1 * g.W + tx.r0) * 64 + lane);
        c11[u] = ld_row4<NTL>(p + ((size_t)ty.r1 * g.W + tx.r1) * 64 + lane);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int bin = bb + 4 * u;
        if (bin >= b_end) break;
        const float4 top = lerp4(c00[u], c01[u], lx[u]);
        const float4 bot = lerp4(c10[u], c11[u], lx[u]);
        const float4 v = ok[u] ? lerp4(top, bot, ly[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
        float4* dst = reinterpret_cast<float4*>(a.out + ((size_t)r * nbins + bin) * C) + lane;
        if (NT) {
          typedef float f4v __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(dst));
        } else
          *dst = v;
      }
    }
    return;
  }
  for (int bin = blockIdx.y * a.bpb + wave; bin < b_end; bin += 4) {
    const int oy = bin / a.out_w, ox = bin - oy * a.out_w;
    float* dst = a.out + ((size_t)r * nbins + bin) * C;
    if (VEC4) {
      for (int c4 = lane; c4 * 4 < C; c4 += 64) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g.ok) {
          for (int sy = 0; sy < S; ++sy) {
            const Tap ty = make_tap(in_coord(g.y1, g.y2, g.hs, oy * S + sy, g.ch, g.Hp), g.Hp,
                                    g.H, pad);
            for (int sx = 0; sx < S; ++sx) {
              const Tap tx = make_tap(in_coord(g.x1, g.x2, g.ws, ox * S + sx, g.cw, g.Wp),
                                      g.Wp, g.W, pad);
              float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
              if (ty.valid && tx.valid) {
                const float4* p = reinterpret_cast<const float4*>(base);
                const float4 tl = p[((size_t)ty.r0 * g.W + tx.r0) * (C / 4) + c4];
                const float4 tr = p[((size_t)ty.r0 * g.W + tx.r1) * (C / 4) + c4];
                const float4 bl = p[((size_t)ty.r1 * g.W + tx.r0) * (C / 4) + c4];
                const float4 br = p[((size_t)ty.r1 * g.W + tx.r1) * (C / 4) + c4];
                const float4 top = lerp4(tl, tr, tx.lerp);
                const float4 bot = lerp4(bl, br, tx.lerp);
                v = lerp4(top, bot, ty.lerp);
              }
              if (S == 1) {
                acc = v;
              } else {
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
              }
            }
          }
          if (S > 1) { acc.x /= inv; acc.y /= inv; acc.z /= inv; acc.w /= inv; }
        }
        reinterpret_cast<float4*>(dst)[c4] = acc;
      }
    } else {
      for (int c = lane; c < C; c += 64) {
        float acc = 0.f;
        if (g.ok) {
          for (int sy = 0; sy < S; ++sy) {
            const Tap ty = make_tap(in_coord(g.y1, g.y2, g.hs, oy * S + sy, g.ch, g.Hp), g.Hp,
                                    g.H, pad);
            for (int sx = 0; sx < S; ++sx) {
              const Tap tx = make_tap(in_coord(g.x1, g.x2, g.ws, ox * S + sx, g.cw, g.Wp),
                                      g.Wp, g.W, pad);
              float v = 0.f;
              if (ty.valid && tx.valid) {
                const float tl = base[((size_t)ty.r0 * g.W + tx.r0) * C + c];
                const float tr = base[((size_t)ty.r0 * g.W + tx.r1) * C + c];
                const float bl = base[((size_t)ty.r1 * g.W + tx.r0) * C + c];
                const float br = base[((size_t)ty.r1 * g.W + tx.r1) * C + c];
                const float top = tl + (tr - tl) * tx.lerp;
                const float bot = bl + (br - bl) * tx.lerp;
                v = top + (bot - top) * ty.lerp;
              }
              acc = (S == 1) ? v : acc + v;
            }
          }
          if (S > 1) acc = acc / inv;
        }
        dst[c] = acc;
      }
    }
  }
}

// ---------------------------------------------------------------- backward
// TF CropAndResizeGradImage (+ AvgPoolGrad's 1/count and MirrorPadGrad folding
// the pad rows onto the edge rows, implicit in the clamped taps) as a GATHER:
// device-scope float atomics on gfx950 resolve beyond the XCD-private L2 and a
// scatter of them ran at ~120 GB/s.  Instead, a hand-written counting sort of
// the contributions by (pixel, set) -- r1/r2 ran a rocPRIM onesweep radix sort
// here, ~87 us of its ~11 launches per step:
//   1. emit: for every (ROI, sample, corner) contribution, slot = (roi *
//      samples + sample) * 4 + corner, its (grad_out row, y_lerp, x_lerp)
//      record at slot >> 2 and an integer atomic on its pair's counter, whose
//      old value is the contribution's arrival rank in the pair (a wave whose
//      live lanes all hit one pair -- collapsed boxes -- takes one atomic);
//   2. runs (one thread per pixel): each touched pair gets a contiguous range
//      of the arrival array (workgroup-aggregated cursor: ranges are
//      independent, so their placement order does not matter), the pixel goes
//      on the touched list, and a run longer than kSeg gets a block of
//      kSeg-long segments plus the tasks of its long sort;
//   3. place (one thread per contribution): arrival[start + rank] = slot;
//   4. a run's arrival order is not deterministic, its slot order (the TF
//      loop order) is: runs up to kSeg are ranked by slot inside the pixel
//      pass (a few LDS / shuffle compares per lane); longer runs are ranked by
//      `roi_bwd_long_kernel` (1,024 elements per task, each ranked
//      against the whole run through LDS tiles) into sorted_long;
//   5. segment partials of the long runs (one wave per kSeg slots), then the
//      grad maps -- zero-filled by the clear launch -- get their touched
//      pixels summed by waves striding over the touched list.
// Two ROI sets of the same maps (the box and mask poolers, d2mi_roi_align_bwd2)
// share one pass: pairs are (pixel, set), each set's run is summed apart and
// the two sums added.
// Summation order per pixel is (box, y, x, corner), the TF kernel's loop order
// (partials regroup it for pixels past kSeg): deterministic run to run, and
// bit-identical to the TF scatter for pixels with at most kSeg contributions
// and no folded pad row.
constexpr int kSeg = 64;    // contributions per wave before a pixel is split
constexpr int kBatch = 2;   // contributions in flight per wave (r1 sweep, pixel kernel avg: 16 -> 103 us, 8 -> 64, 4 -> 49.5, 2 -> 46.7: occupancy, not loads in flight, binds)
constexpr int kLongTask = 1024;  // run elements ranked per long-sort task (one workgroup)
constexpr int kLongTile = 4096;  // run elements per LDS tile of the long sort

struct PixMap {
  long long base[D2MI_MAX_LEVELS + 1];  // first global pixel id per level
  // the touched-pixel list, partitioned by level: level l's entries start at
  // tbase[l] (capacity tbase[l + 1] - tbase[l] = min(samples x 4, its pixels)),
  // so a level's pixel pass walks its own pixels only
  int32_t tbase[D2MI_MAX_LEVELS + 1];
  int L;
};

struct Contrib {
  int32_t row;  // grad_out row index r * nbins + bin (of its set's grad_out)
  float yl, xl;
  int32_t set;  // ROI set (0 / 1) of a merged backward
};

// A contribution in its run's arrival order (r5): the place launch writes
// the slot AND the sample's record next to each other, so the C = 256 pixel
// pass reads a run's records in one coalesced load round instead of a slot
// and then a record per contribution (one dependent load fewer per
// contribution, and the row addresses of a run all known after its slot sort).
struct RunRec {
  int32_t slot;  // ((sample) << 2) | corner
  int32_t row;   // grad_out row of the sample's bin (its set's grad_out)
  float yl, xl;
};

// Device-side bookkeeping of one backward (cleared by the clear launch).
struct BwdCounters {
  int32_t touched, segs, tasks, cursor;
  int32_t touched_lv[D2MI_MAX_LEVELS];  // touched pixels per level (light: from the front)
  int32_t touched_hv[D2MI_MAX_LEVELS];  // ... heavy (> roi_heavy contributions: from the back)
  int32_t lsdone;  // workgroups of the long-sort launch that finished
};

// The touched pixels of levels [lo, hi]: their count, and the t-th of them
// (the level segments of the list in level order).
// r5: a level's segment of the touched list holds its light pixels from the
// front and its heavy ones (> roi_heavy contributions) from the back, and entry
// order puts a level's heavy pixels first: the first waves of a pass take the
// longest load chains, the light pixels fill in behind them (a pass's time was
// its longest runs' row batches behind everything else).  The threshold is
// tuning "roi_heavy" (default 16; 0: every pixel light, the r5b order).
struct TouchedRange {
  // (every index below is a compile-time constant after unrolling: a
  // dynamically indexed register array lives in scratch memory)
  int32_t pre[D2MI_MAX_LEVELS + 1];
  int32_t hv[D2MI_MAX_LEVELS];
  int lo, hi;
  __device__ __forceinline__ void init(const PixMap& pm, const BwdCounters* ctr, int lv_lo,
                                       int lv_hi) {
    lo = lv_lo;
    hi = lv_hi;
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < D2MI_MAX_LEVELS; ++j) {
      const bool in = j <= hi - lo;
      hv[j] = in ? ctr->touched_hv[lo + j] : 0;
      pre[j + 1] = pre[j] + (in ? ctr->touched_lv[lo + j] + hv[j] : 0);
    }
  }
  __device__ __forceinline__ int total() const {
    int v = 0;
#pragma unroll
    for (int j = 0; j <= D2MI_MAX_LEVELS; ++j) v = j == hi - lo + 1 ? pre[j] : v;
    return v;
  }
  // global pixel id and level of entry t < total()
  __device__ __forceinline__ long long at(const PixMap& pm, const int32_t* touched, int t,
                                          int& l) const {
    return touched[index(pm, t, l)];
  }
  // the touched-list index of entry t < total(), and its level: a level's
  // heavy pixels (its segment's back, last-allocated first) then its light ones
  __device__ __forceinline__ int index(const PixMap& pm, int t, int& l) const {
    int k = 0, base = 0, h = hv[0];
#pragma unroll
    for (int j = 1; j < D2MI_MAX_LEVELS; ++j)
      if (j <= hi - lo && t >= pre[j]) {
        k = j;
        base = pre[j];
        h = hv[j];
      }
    l = lo + k;
    const int kk = t - base;
    return kk < h ? pm.tbase[l + 1] - 1 - kk : pm.tbase[l] + (kk - h);
  }
};

// One launch clears every buffer the backward starts from (the per-level grad
// maps to 0, the pair counters and the bookkeeping counters to 0) instead of a
// hipMemsetAsync per buffer: each memset is its own ~5 us dispatch.
constexpr int kMaxClear = D2MI_MAX_LEVELS + 2;
struct ClearList {
  uint32_t* ptr[kMaxClear];
  long long words[kMaxClear];
  uint32_t value[kMaxClear];
  int n;
};

__global__ __launch_bounds__(256) void roi_bwd_clear_kernel(ClearList cl) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (int k = 0; k < cl.n; ++k) {
    uint32_t* p = cl.ptr[k];
    const long long n = cl.words[k];
    const uint32_t v = cl.value[k];
    // 16-byte aligned body as uint4 stores, the unaligned head / tail as words
    const long long head = std::min<long long>(n, (long long)((16 - ((uintptr_t)p & 15)) & 15) / 4);
    const long long quads = (n - head) / 4;
    uint4* q = reinterpret_cast<uint4*>(p + head);
    const uint4 v4 = make_uint4(v, v, v, v);
    for (long long i = tid; i < quads; i += stride) q[i] = v4;
    const long long tail0 = head + quads * 4;
    if (tid < head) p[tid] = v;
    if (tid < n - tail0) p[tail0 + tid] = v;
  }
}

// The ROI geometry is recomputed per sample (a few dozen flops against the
// 48 B the thread stores) rather than staged by a separate launch.
// set / sample_base: a merged backward emits its second ROI set after the
// first (samples from sample_base on) with pairs pixel * 2 + set
// (set_bits = 1): each set's contributions of a pixel form their own run.
// ent[slot] = pair << 32 | arrival rank, ~0 for a contribution outside the map.
__device__ __forceinline__ void emit_samples(const RoiArgs& a, const PixMap& pm, int set,
                                             int set_bits, long long sample_base, long long tl,
                                             int32_t* __restrict__ count,
                                             uint64_t* __restrict__ ent,
                                             Contrib* __restrict__ rec) {
  const int S = a.sr > 0 ? a.sr : 1;
  const long long nsamp = (long long)a.out_h * a.out_w * S * S;
  const bool in_range = tl < (long long)a.R * nsamp;
  const int r = in_range ? (int)(tl / nsamp) : 0;
  const int s = in_range ? (int)(tl - (long long)r * nsamp) : 0;
  const RoiGeom g = roi_geom(a, in_range ? r : 0);
  const long long t = sample_base + tl;
  const uint64_t slot = (uint64_t)t * 4u;
  bool ok = in_range && g.ok;
  Tap ty = {}, tx = {};
  int iy = 0, ix = 0;
  if (ok) {
    const bool pad = a.pad_border != 0;
    iy = s / g.cw;
    ix = s - iy * g.cw;
    ty = make_tap(in_coord(g.y1, g.y2, g.hs, iy, g.ch, g.Hp), g.Hp, g.H, pad);
    tx = make_tap(in_coord(g.x1, g.x2, g.ws, ix, g.cw, g.Wp), g.Wp, g.W, pad);
    ok = ty.valid && tx.valid;
  }
  uint32_t q[4] = {0u, 0u, 0u, 0u};
  if (ok) {
    Contrib c;
    c.row = r * (a.out_h * a.out_w) + (iy / S) * a.out_w + ix / S;
    c.yl = ty.lerp;
    c.xl = tx.lerp;
    c.set = set;
    rec[t] = c;  // shared by the 4 corners: slot >> 2
    const uint64_t img = (uint64_t)pm.base[g.lvl] + (uint64_t)g.n * g.H * g.W;
    const uint32_t sb = (uint32_t)set;
    q[0] = (uint32_t)((img + (uint64_t)ty.r0 * g.W + tx.r0) << set_bits) | sb;
    q[1] = (uint32_t)((img + (uint64_t)ty.r0 * g.W + tx.r1) << set_bits) | sb;
    q[2] = (uint32_t)((img + (uint64_t)ty.r1 * g.W + tx.r0) << set_bits) | sb;
    q[3] = (uint32_t)((img + (uint64_t)ty.r1 * g.W + tx.r1) << set_bits) | sb;
  }
  // the four corners' arrival ranks (live lanes only), all four atomics in
  // flight before any result is used (r5; one round trip per corner before).
  // When every live lane of the wave hits the same pair -- degenerate boxes
  // collapsed onto one point, where hundreds of ROIs pile onto a pixel -- one
  // atomic takes the whole wave's ranks: same-address device atomics serialise.
  uint32_t rk[4] = {0u, 0u, 0u, 0u};
  const unsigned long long lm = __ballot(ok);
  if (lm != 0) {
    const int lane = threadIdx.x & 63;
    const int lead = __ffsll((long long)lm) - 1;
    bool coll[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t q0 = (uint32_t)__shfl((int)q[k], lead);
      coll[k] = __ballot(ok && q[k] == q0) == lm;  // the whole wave on one pair
    }
    uint32_t base[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (coll[k]) {
        if (lane == lead) base[k] = (uint32_t)atomicAdd(&count[q[k]], __popcll(lm));
      } else if (ok) {
        rk[k] = (uint32_t)atomicAdd(&count[q[k]], 1);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (coll[k])
        rk[k] = (uint32_t)__shfl((int)base[k], lead) + (uint32_t)__popcll(lm & ((1ull << lane) - 1ull));
  }
  uint64_t e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = ok ? ((uint64_t)q[k] << 32) | rk[k] : ~0ull;
  if (in_range) {
    uint64_t* d = ent + slot;
    d[0] = e[0];
    d[1] = e[1];
    d[2] = e[2];
    d[3] = e[3];
  }
}

// Both ROI sets' samples in one launch (r5: a launch per set before): the
// first nb0 workgroups take set 0, the rest set 1 (from sample ns0 on).
__global__ __launch_bounds__(256) void roi_bwd_emit_kernel(RoiArgs a0, RoiArgs a1, int nb0,
                                                           long long ns0, PixMap pm, int set_bits,
                                                           int32_t* __restrict__ count,
                                                           uint64_t* __restrict__ ent,
                                                           Contrib* __restrict__ rec) {
  if ((int)blockIdx.x < nb0)
    emit_samples(a0, pm, 0, set_bits, 0, (long long)blockIdx.x * blockDim.x + threadIdx.x, count,
                 ent, rec);
  else
    emit_samples(a1, pm, 1, set_bits, ns0,
                 (long long)(blockIdx.x - nb0) * blockDim.x + threadIdx.x, count, ent, rec);
}

// Workgroup-aggregated allocation from a global counter: returns this
// thread's offset for `want` items (one device atomic per workgroup --
// same-address atomics serialise, one per wave cost ~20 us per launch).
template <int NT>
__device__ __forceinline__ int wg_alloc(int want, int32_t* __restrict__ counter, int* s_wave,
                                        int* s_base) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // inclusive wave scan
  int x = want;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_wave[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int k = 0; k < NT / 64; ++k) {
      const int v = s_wave[k];
      s_wave[k] = tot;
      tot += v;
    }
    *s_base = tot ? atomicAdd(counter, tot) : 0;
  }
  __syncthreads();
  const int off = *s_base + s_wave[w] + x - want;
  __syncthreads();  // s_wave / s_base reusable by the caller's next allocation
  return off;
}

// K allocations from K global counters in ONE workgroup round (r5): the K
// wave scans run together, then K threads issue their atomics at once (one
// round trip, two barriers) -- the runs launch made five wg_alloc rounds in a
// row, each its own barriers and atomic latency.  Counter k's total is skipped
// (no atomic) when it is zero; ctr[k] may be null when want[k] is always 0.
template <int NT, int K>
__device__ __forceinline__ void wg_alloc_multi(const int (&want)[K], int32_t* const (&ctr)[K],
                                               int (&off)[K], int (*s_wave)[NT / 64],
                                               int* s_base) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x[K];
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = want[k];
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int y = __shfl_up(x[k], d);
      if (lane >= d) x[k] += y;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < K; ++k) s_wave[k][w] = x[k];
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    int tot = 0;
    for (int j = 0; j < NT / 64; ++j) {
      const int v = s_wave[k][j];
      s_wave[k][j] = tot;
      tot += v;
    }
    s_base[k] = tot ? atomicAdd(ctr[k], tot) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) off[k] = s_base[k] + s_wave[k][w] + x[k] - want[k];
}

// One thread per pixel: each touched (pixel, set) pair gets its range of the
// arrival array, the pixel goes on the touched list, and a pair with more
// than kSeg contributions gets its segment slots (owner = pair) and the tasks
// of its long sort.  The list / range orders vary run to run; every per-pixel
// sum does not.
__global__ __launch_bounds__(1024) void roi_bwd_runs_kernel(
    const int32_t* __restrict__ count, long long total_pixels, int set_bits,
    int32_t* __restrict__ run_start, int32_t* __restrict__ seg_first,
    int32_t* __restrict__ seg_pixel, int2* __restrict__ tasks, int32_t* __restrict__ touched,
    int4* __restrict__ trun, BwdCounters* __restrict__ ctr, PixMap pm, int heavy_min) {
  __shared__ int s_wave[16], s_base;
  __shared__ int s_wave7[7][16], s_base7[7];
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < total_pixels;
  const int nsets = 1 << set_bits;
  int c[2] = {0, 0};
  for (int s = 0; s < nsets; ++s) c[s] = live ? count[(p << set_bits) | s] : 0;
  const int tot = c[0] + c[1];
  int nseg[2] = {0, 0}, ntask[2] = {0, 0};
  for (int s = 0; s < nsets; ++s) {
    if (c[s] > kSeg) {
      nseg[s] = (c[s] + kSeg - 1) / kSeg;
      ntask[s] = (c[s] + kLongTask - 1) / kLongTask;
    }
  }
  // the pixel's slot in its level's segment of the touched list (the
  // workgroup's pixels span levels lf..ll; the first two in the one round
  // with the arrival range, the segments and the tasks, any further level --
  // maps smaller than a workgroup -- one round each, uniform)
  const long long p0 = (long long)blockIdx.x * blockDim.x;
  const long long p1 = min(p0 + (long long)blockDim.x, total_pixels) - 1;
  int lf = 0, ll = 0, lp = 0;
  while (lf + 1 < pm.L && p0 >= pm.base[lf + 1]) ++lf;
  while (ll + 1 < pm.L && p1 >= pm.base[ll + 1]) ++ll;
  while (lp + 1 < pm.L && p >= pm.base[lp + 1]) ++lp;
  const int l2 = min(lf + 1, ll);
  const bool heavy = heavy_min > 0 && tot > heavy_min, light = tot > 0 && !heavy;
  const int want[7] = {tot, light && lp == lf ? 1 : 0, l2 > lf && light && lp == l2 ? 1 : 0,
                       nseg[0] + nseg[1], ntask[0] + ntask[1], heavy && lp == lf ? 1 : 0,
                       l2 > lf && heavy && lp == l2 ? 1 : 0};
  int32_t* const ctrs[7] = {&ctr->cursor, &ctr->touched_lv[lf], &ctr->touched_lv[l2], &ctr->segs,
                            &ctr->tasks, &ctr->touched_hv[lf], &ctr->touched_hv[l2]};
  int off[7];
  wg_alloc_multi<1024, 7>(want, ctrs, off, s_wave7, s_base7);
  const int pos = off[0], sf = off[3], tf = off[4];
  // light pixels from the level segment's front, heavy ones from its back
  auto slot_of = [&](int lv, int o_light, int o_heavy) {
    return heavy ? pm.tbase[lv + 1] - 1 - o_heavy : pm.tbase[lv] + o_light;
  };
  int tix = lp == lf ? slot_of(lf, off[1], off[5]) : (lp == l2 ? slot_of(l2, off[2], off[6]) : 0);
  for (int lv = l2 + 1; lv <= ll; ++lv) {
    __syncthreads();  // (s_wave / s_base reused)
    const int ol = wg_alloc<1024>(light && lp == lv ? 1 : 0, &ctr->touched_lv[lv], s_wave, &s_base);
    const int oh = wg_alloc<1024>(heavy && lp == lv ? 1 : 0, &ctr->touched_hv[lv], s_wave, &s_base);
    if (lp == lv) tix = slot_of(lv, ol, oh);
  }
  if (tot == 0) return;
  touched[tix] = (int32_t)p;
  int o = pos, so = sf, to = tf;
  for (int s = 0; s < nsets; ++s) {
    const int q = (int)((p << set_bits) | s);
    // the touched entry's run of this set (pixel, count, start, first segment):
    // the C = 256 pixel pass reads it with the entry, no count / start lookup
    if (trun) trun[((long long)tix << set_bits) | s] = make_int4((int)p, c[s], o, nseg[s] ? so : -1);
    if (c[s] == 0) continue;
    run_start[q] = o;
    o += c[s];
    if (nseg[s]) {
      seg_first[q] = so;
      for (int k = 0; k < nseg[s]; ++k) seg_pixel[so + k] = q;
      so += nseg[s];
      for (int k = 0; k < ntask[s]; ++k) tasks[to + k] = make_int2(q, k);
      to += ntask[s];
    }
  }
}

// One thread per contribution: its slot at its arrival rank in its pair's
// range, and (runrec non-null) its run record there too.
__global__ __launch_bounds__(256) void roi_bwd_place_kernel(const uint64_t* __restrict__ ent,
                                                            long long n,
                                                            const int32_t* __restrict__ run_start,
                                                            int32_t* __restrict__ arrival,
                                                            const Contrib* __restrict__ rec,
                                                            RunRec* __restrict__ runrec) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t e = ent[i];
  if (e == ~0ull) return;
  const int q = (int)(e >> 32);
  const int pos = run_start[q] + (int)(uint32_t)e;
  arrival[pos] = (int32_t)i;
  if (runrec) {
    const Contrib c = rec[i >> 2];
    runrec[pos] = RunRec{(int32_t)i, c.row, c.yl, c.xl};
  }
}

// g / (sr * sr), the avg-pool divisor TF applies to each grad_out value.  When
// sr * sr is a power of two the product by its (exact) reciprocal is the same
// single rounding of the same exact quotient -- bit-identical -- and costs one
// multiply instead of a ~10-instruction IEEE division per channel (r5: the
// C = 256 pixel pass 101 -> 99 us per step; it is bound by its load chains,
// not by VALU).
struct BinDiv {
  float inv, rcp;
  bool pow2;
};
__device__ __forceinline__ BinDiv bin_div(int sr) {
  const int n = sr * sr;
  return BinDiv{(float)n, 1.f / (float)n, n > 0 && (n & (n - 1)) == 0};
}
__device__ __forceinline__ float4 div4(float4 g, const BinDiv& d) {
  if (d.pow2) return make_float4(g.x * d.rcp, g.y * d.rcp, g.z * d.rcp, g.w * d.rcp);
  return make_float4(g.x / d.inv, g.y / d.inv, g.z / d.inv, g.w / d.inv);
}

// TF order of operations: dtop = (1 - y_lerp) * g, dbot = y_lerp * g, then
// (1 - x_lerp) * d or x_lerp * d.
__device__ __forceinline__ float weigh(int corner, float yl, float xl, float v) {
  const float d = (corner < 2) ? (1.f - yl) * v : yl * v;
  return (corner & 1) ? xl * d : (1.f - xl) * d;
}

// Sum of the contributions slots[0, n) (slot order) for the lane's channel(s) c.
template <bool VEC4>
__device__ __forceinline__ float4 sum_slots(const RoiArgs& a, const int32_t* slots,
                                            const Contrib* __restrict__ rec, int n, int c,
                                            bool live) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int C = a.C;
  for (int i = 0; i < n; i += kBatch) {
    int corner[kBatch];
    Contrib e[kBatch];
    const int m = min(kBatch, n - i);
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      if (u < m) {
        const int slot = slots[i + u];
        corner[u] = slot & 3;
        e[u] = rec[slot >> 2];
      }
    }
    float4 v[kBatch] = {};  // dead lanes accumulate zeros, never uninitialised registers
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      if (u < m && live) {
        const float* src = a.gout_s[e[u].set] + (size_t)e[u].row * C + c;
        if (VEC4) v[u] = *reinterpret_cast<const float4*>(src);
        else v[u].x = *src;
      }
    }
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      if (u < m) {
        float4 g = v[u];
        const int sr = a.sr_s[e[u].set];
        if (sr > 0) g = div4(g, bin_div(sr));  // the avg-pool divisor of the set's sampling ratio
        acc.x += weigh(corner[u], e[u].yl, e[u].xl, g.x);
        if (VEC4) {
          acc.y += weigh(corner[u], e[u].yl, e[u].xl, g.y);
          acc.z += weigh(corner[u], e[u].yl, e[u].xl, g.z);
          acc.w += weigh(corner[u], e[u].yl, e[u].xl, g.w);
        }
      }
    }
  }
  return acc;
}

// Slot order of a short run (n <= kSeg) by the G lanes of one group (G = 64
// or 16, `sub` = the lane's index in it): each lane holds kSeg / G of the
// run's arrival-ordered slots, ranks them against all n (slots are distinct)
// and stores them at their ranks in the group's LDS row `out`; `in` is a
// second row of scratch.  Wave-local: LDS operations of one wave complete in
// order.
template <int G>
__device__ __forceinline__ void order_run(const int32_t* __restrict__ arrival, int i0, int n,
                                          int sub, int32_t* in, int32_t* out) {
  constexpr int K = kSeg / G;
  int v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int idx = sub + k * G;
    v[k] = idx < n ? arrival[i0 + idx] : INT_MAX;
    if (idx < n) in[idx] = v[k];
  }
  __builtin_amdgcn_wave_barrier();
  int rank[K] = {};
  for (int j = 0; j < n; ++j) {
    const int o = in[j];
#pragma unroll
    for (int k = 0; k < K; ++k) rank[k] += o < v[k] ? 1 : 0;
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (sub + k * G < n) out[rank[k]] = v[k];
  __builtin_amdgcn_wave_barrier();
}

// Long runs (> kSeg contributions), then their segment partials, in ONE
// launch (r5; two before, each a dispatch that only reads zero counts and
// exits in an ordinary step):
//   1. a task ranks kLongTask of a run's elements against the whole run
//      (slots are distinct), streamed through LDS in kLongTile tiles -- O(len^2)
//      compares per run over len / 1024 workgroups; only degenerate piles of
//      boxes make runs this long;
//   2. the workgroup that finishes last (device counter, fences on both sides)
//      writes every segment's partial[seg] (C floats, one wave per segment,
//      slot order within it).
template <bool VEC4>
__global__ __launch_bounds__(1024) void roi_bwd_long_kernel(
    RoiArgs a, const int32_t* __restrict__ arrival, const int32_t* __restrict__ count,
    const int32_t* __restrict__ run_start, const int2* __restrict__ tasks,
    BwdCounters* __restrict__ ctr, int32_t* __restrict__ sorted_long,
    const Contrib* __restrict__ rec, const int32_t* __restrict__ seg_first,
    const int32_t* __restrict__ seg_pixel, float* __restrict__ partial) {
  __shared__ int32_t tile[kLongTile];
  __shared__ int s_last;
  const int ntasks = ctr->tasks;
  for (int tk = blockIdx.x; tk < ntasks; tk += gridDim.x) {
    const int2 task = tasks[tk];
    const int i0 = run_start[task.x], len = count[task.x];
    const int e = task.y * kLongTask + (int)threadIdx.x;
    const int mine = e < len ? arrival[i0 + e] : INT_MAX;
    int rank = 0;
    for (int j0 = 0; j0 < len; j0 += kLongTile) {
      const int m = min(kLongTile, len - j0);
      __syncthreads();
      for (int j = threadIdx.x; j < m; j += blockDim.x) tile[j] = arrival[i0 + j0 + j];
      __syncthreads();
      int j = 0;
      for (; j + 8 <= m; j += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += tile[j + u] < mine ? 1 : 0;
      }
      for (; j < m; ++j) rank += tile[j] < mine ? 1 : 0;
    }
    if (e < len) sorted_long[i0 + rank] = mine;
    __syncthreads();
  }
  // the last workgroup to finish computes the segment partials
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this workgroup's sorted_long stores before its arrival
    s_last = atomicAdd(&ctr->lsdone, 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int nsegs = ctr->segs;
  const int step = VEC4 ? 256 : 64;
  for (int seg = threadIdx.x >> 6; seg < nsegs; seg += nw) {
    const int q = seg_pixel[seg];
    const int k = seg - seg_first[q];
    const int i0 = run_start[q] + k * kSeg;
    const int n = min(kSeg, count[q] - k * kSeg);
    for (int c0 = 0; c0 < a.C; c0 += step) {
      const int c = c0 + (VEC4 ? lane * 4 : lane);
      const bool live = c < a.C;
      const float4 acc = sum_slots<VEC4>(a, sorted_long + i0, rec, n, c, live);
      if (live) {
        float* dst = partial + (size_t)seg * a.C + c;
        if (VEC4) *reinterpret_cast<float4*>(dst) = acc;
        else *dst = acc.x;
      }
    }
  }
}

// Touched pixels only (the grad maps were zero-filled at full bandwidth
// first): waves stride over the compact touched-pixel list, one pixel per wave
// iteration, so the dependent load chain of a pixel (run bounds -> slots ->
// records -> grad_out rows) overlaps across waves instead of a wave per
// feature-map pixel (most of which only stored zeros) -- that launch was bound
// by wave start-up and latency, at ~1/4 of its store bandwidth.
template <bool VEC4>
__global__ __launch_bounds__(256) void roi_bwd_pixel_kernel(
    RoiArgs a, PixMap pm, const int32_t* __restrict__ arrival, const Contrib* __restrict__ rec,
    int set_bits, const int32_t* __restrict__ count, const int32_t* __restrict__ run_start,
    const int32_t* __restrict__ seg_first, const float* __restrict__ partial,
    const int32_t* __restrict__ touched, const BwdCounters* __restrict__ ctr, int lv_lo,
    int lv_hi) {
  __shared__ int32_t lds[4][2][kSeg];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int C = a.C;
  const int step = VEC4 ? 256 : 64;
  TouchedRange tr;
  tr.init(pm, ctr, lv_lo, lv_hi);  // the levels of this pass (bwd2 phase 2: one)
  const int nt = tr.total();
  const int nsets = 1 << set_bits;
  for (int t = blockIdx.x * 4 + w; t < nt; t += gridDim.x * 4) {
    int l;
    const long long pix = tr.at(pm, touched, t, l);
    float* dst = a.gfeat[l] + (size_t)(pix - pm.base[l]) * C;
    const bool acc_lv = (a.acc_mask >> l) & 1;
    // each set's run in slot order once per pixel (the channel loop reuses it)
    for (int c0 = 0; c0 < C; c0 += step) {
      const int c = c0 + (VEC4 ? lane * 4 : lane);
      const bool live = c < C;
      float4 res = make_float4(0.f, 0.f, 0.f, 0.f);
      bool any = false;
      // each set's contributions summed apart (its own TF-order run), then
      // set 0 + set 1: the rounding of the sum of two separate backwards
      for (int sidx = 0; sidx < nsets; ++sidx) {
        const long long q = (pix << set_bits) | sidx;
        const int n = count[q];
        if (n == 0) continue;
        const int i0 = run_start[q];
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n <= kSeg) {
          order_run<64>(arrival, i0, n, lane, lds[w][0], lds[w][1]);
          acc = sum_slots<VEC4>(a, lds[w][1], rec, n, c, live);
        } else if (live) {
          const int f = seg_first[q];
          const int ns = (n + kSeg - 1) / kSeg;
          for (int j = 0; j < ns; ++j) {
            const float* src = partial + (size_t)(f + j) * C + c;
            if (VEC4) {
              const float4 v = *reinterpret_cast<const float4*>(src);
              acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            } else {
              acc.x += *src;
            }
          }
        }
        if (any) {
          res.x = res.x + acc.x; res.y = res.y + acc.y; res.z = res.z + acc.z; res.w = res.w + acc.w;
        } else {
          res = acc;
          any = true;
        }
      }
      if (live) {
        // accumulate: the level's map already holds another gradient of the
        // same features (a hand-off between backward calls): old + new, the
        // rounding of autograd's sum of the two maps
        if (VEC4) {
          if (acc_lv) {
            const float4 o = *reinterpret_cast<const float4*>(dst + c);
            res.x = o.x + res.x;
            res.y = o.y + res.y;
            res.z = o.z + res.z;
            res.w = o.w + res.w;
          }
          *reinterpret_cast<float4*>(dst + c) = res;
        } else {
          dst[c] = acc_lv ? dst[c] + res.x : res.x;
        }
      }
    }
  }
}

// r4 form of roi_bwd_pixel_c256_kernel (tuning "roi_bwd_rec" = 0, A/B): the
// run's slots ordered in LDS, then a record and a row per contribution.
// C == 256 form of roi_bwd_pixel_kernel: a wave sums FOUR touched pixels at
// once, 16 lanes per pixel, 16 channels (4 float4) per lane -- four
// independent load chains (run bounds -> slots -> records -> grad_out rows)
// in flight per wave instead of one, the same per-pixel order and rounding.
template <int PPW>
__global__ __launch_bounds__(256) void roi_bwd_pixel_c256_slots_kernel(
    RoiArgs a, PixMap pm, const int32_t* __restrict__ arrival, const Contrib* __restrict__ rec,
    int set_bits, const int32_t* __restrict__ count, const int32_t* __restrict__ run_start,
    const int32_t* __restrict__ seg_first, const float* __restrict__ partial,
    const int32_t* __restrict__ touched, const BwdCounters* __restrict__ ctr, int lv_lo,
    int lv_hi) {
  constexpr int C = 256;
  constexpr int LPP = 64 / PPW;     // lanes per pixel
  constexpr int F = C / LPP / 4;    // float4 per lane
  __shared__ int32_t lds[4][PPW][2][kSeg];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / LPP, sub = lane % LPP;
  const int c = sub * 4 * F;  // this lane's channels
  TouchedRange tr;
  tr.init(pm, ctr, lv_lo, lv_hi);
  const int nt = tr.total();
  const int nsets = 1 << set_bits;
  int32_t* lin = lds[w][grp][0];
  int32_t* lout = lds[w][grp][1];
  const int wave = blockIdx.x * 4 + w;
  for (int tb = wave * PPW; tb < nt; tb += gridDim.x * 4 * PPW) {
    const int t = tb + grp;
    if (t >= nt) continue;
    int l;
    const long long pix = tr.at(pm, touched, t, l);
    float* dst = a.gfeat[l] + (size_t)(pix - pm.base[l]) * C + c;
    float4* d4 = reinterpret_cast<float4*>(dst);
    // accumulate: the map's old value is loaded first, its latency hidden
    // behind the contribution sums (r4: the deferred per-level passes into
    // the RPN head's dgrad output waited on it at the end)
    const bool acc_lv = (a.acc_mask >> l) & 1;
    float4 old[F];
    if (acc_lv) {
#pragma unroll
      for (int k = 0; k < F; ++k) old[k] = d4[k];
    }
    float4 res[F];
    bool any = false;
    for (int sidx = 0; sidx < nsets; ++sidx) {
      const long long q = (pix << set_bits) | sidx;
      const int n = count[q];
      if (n == 0) continue;
      const int i0 = run_start[q];
      float4 acc[F];
#pragma unroll
      for (int k = 0; k < F; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n <= kSeg) {
        order_run<LPP>(arrival, i0, n, sub, lin, lout);
        for (int i = 0; i < n; ++i) {
          const int slot = lout[i];
          const int corner = slot & 3;
          const Contrib e = rec[slot >> 2];
          const float4* src =
              reinterpret_cast<const float4*>(a.gout_s[e.set] + (size_t)e.row * C + c);
          float4 v[F];
#pragma unroll
          for (int k = 0; k < F; ++k) v[k] = src[k];
          const int sr = a.sr_s[e.set];
          const BinDiv bd = bin_div(sr);
#pragma unroll
          for (int k = 0; k < F; ++k) {
            float4 g = v[k];
            if (sr > 0) g = div4(g, bd);
            acc[k].x += weigh(corner, e.yl, e.xl, g.x);
            acc[k].y += weigh(corner, e.yl, e.xl, g.y);
            acc[k].z += weigh(corner, e.yl, e.xl, g.z);
            acc[k].w += weigh(corner, e.yl, e.xl, g.w);
          }
        }
      } else {
        const int f = seg_first[q];
        const int ns = (n + kSeg - 1) / kSeg;
        for (int j = 0; j < ns; ++j) {
          const float4* src = reinterpret_cast<const float4*>(partial + (size_t)(f + j) * C + c);
#pragma unroll
          for (int k = 0; k < F; ++k) {
            const float4 v = src[k];
            acc[k].x += v.x; acc[k].y += v.y; acc[k].z += v.z; acc[k].w += v.w;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < F; ++k) {
        if (any) {
          res[k].x = res[k].x + acc[k].x; res[k].y = res[k].y + acc[k].y;
          res[k].z = res[k].z + acc[k].z; res[k].w = res[k].w + acc[k].w;
        } else {
          res[k] = acc[k];
        }
      }
      any = true;
    }
    if (!any) continue;
#pragma unroll
    for (int k = 0; k < F; ++k) {
      if (acc_lv) {
        const float4 o = old[k];
        res[k].x = o.x + res[k].x; res[k].y = o.y + res[k].y;
        res[k].z = o.z + res[k].z; res[k].w = o.w + res[k].w;
      }
      d4[k] = res[k];
    }
  }
}

// C == 256 form of roi_bwd_pixel_kernel: a wave sums PPW touched pixels at
// once, 64 / PPW lanes per pixel -- PPW independent load chains (run bounds
// -> run records -> grad_out rows) in flight per wave instead of one, the
// same per-pixel order and rounding (r4: four pixels).
// r5: a short run's records come from runrec in one coalesced round (each
// lane kSeg / 16 of them), are put in slot order in LDS, and their grad_out
// rows are then loaded kRowBatch at a time (the row addresses are all known
// after the sort) and summed in that order -- the slot -> record -> row chain
// per contribution of r4 (one dependent global load per step) is gone.
// r5b: the touched entry carries each set's (pixel, count, run start, first
// segment) (trun, written by the runs launch), so a pixel's chain is entry ->
// run records -> rows; RB rows in flight per lane.
// r5c: TWO pixels per wave (32 lanes, 8 channels each), 4 rows in flight: a
// launch's time is set by its longest runs' dependent row batches (a pixel
// with n contributions waits n / RB load round trips; the widest launch of a
// step ran 55 us against a 25 us mean), so a lane's registers buy more rows
// of ONE pixel in flight instead of more pixels: 99.3 -> 85.2 us per step
// (profiles/r5_roi_ppw2_timed_kernel_stats.csv), in-step -0.43 %
// (profiles/r5_ab_roi_ppw2_rb4.log); one pixel per wave with 8 rows and two
// with 2 rows measured the same (r5_ab_roi_ppw1_vs_ppw2.log, _rb2_vs_rb4.log).
template <int PPW, int kRowBatch>
__global__ __launch_bounds__(256) void roi_bwd_pixel_c256_kernel(
    RoiArgs a, PixMap pm, const RunRec* __restrict__ runrec, int set_bits,
    const int4* __restrict__ trun, const float* __restrict__ partial,
    const BwdCounters* __restrict__ ctr, int lv_lo, int lv_hi) {
  constexpr int C = 256;
  constexpr int LPP = 64 / PPW;     // lanes per pixel
  constexpr int F = C / LPP / 4;    // float4 per lane
  constexpr int KR = kSeg / LPP;    // run records per lane
  __shared__ int32_t lslot[4][PPW][kSeg];
  __shared__ int4 lrec[4][PPW][kSeg];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / LPP, sub = lane % LPP;
  const int c = sub * 4 * F;  // this lane's channels
  TouchedRange tr;
  tr.init(pm, ctr, lv_lo, lv_hi);
  const int nt = tr.total();
  const int nsets = 1 << set_bits;
  int32_t* lin = lslot[w][grp];
  int4* lout = lrec[w][grp];
  const int wave = blockIdx.x * 4 + w;
  for (int tb = wave * PPW; tb < nt; tb += gridDim.x * 4 * PPW) {
    const int t = tb + grp;
    if (t >= nt) continue;
    int l;
    const int ti = tr.index(pm, t, l);
    const int4 ru0 = trun[(long long)ti << set_bits];
    const int4 ru1 = set_bits ? trun[((long long)ti << set_bits) | 1] : make_int4(0, 0, 0, -1);
    const long long pix = ru0.x;
    float* dst = a.gfeat[l] + (size_t)(pix - pm.base[l]) * C + c;
    float4* d4 = reinterpret_cast<float4*>(dst);
    // accumulate: the map's old value is loaded first, its latency hidden
    // behind the contribution sums (r4: the deferred per-level passes into
    // the RPN head's dgrad output waited on it at the end)
    const bool acc_lv = (a.acc_mask >> l) & 1;
    float4 old[F];
    if (acc_lv) {
#pragma unroll
      for (int k = 0; k < F; ++k) old[k] = d4[k];
    }
    float4 res[F];
    bool any = false;
    for (int sidx = 0; sidx < nsets; ++sidx) {
      const int4 ru = sidx ? ru1 : ru0;  // (no dynamic register-array index: scratch)
      const int n = ru.y;
      if (n == 0) continue;
      const int i0 = ru.z;
      float4 acc[F];
#pragma unroll
      for (int k = 0; k < F; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n <= kSeg) {
        // the run's records (arrival order), ranked by slot: the TF loop order
        int4 v[KR];
#pragma unroll
        for (int k = 0; k < KR; ++k) {
          const int idx = sub + k * LPP;
          v[k] = idx < n ? *reinterpret_cast<const int4*>(runrec + i0 + idx)
                         : make_int4(INT_MAX, 0, 0, 0);
          if (idx < n) lin[idx] = v[k].x;
        }
        __builtin_amdgcn_wave_barrier();
        int rank[KR] = {};
        for (int j = 0; j < n; ++j) {
          const int o = lin[j];
#pragma unroll
          for (int k = 0; k < KR; ++k) rank[k] += o < v[k].x ? 1 : 0;
        }
#pragma unroll
        for (int k = 0; k < KR; ++k)
          if (sub + k * LPP < n) lout[rank[k]] = v[k];
        __builtin_amdgcn_wave_barrier();
        const float* gout = a.gout_s[sidx];
        const int sr = a.sr_s[sidx];
        const BinDiv bd = bin_div(sr);
        for (int i = 0; i < n; i += kRowBatch) {
          int4 e[kRowBatch];
          float4 vv[kRowBatch][F];
#pragma unroll
          for (int u = 0; u < kRowBatch; ++u) {
            if (i + u < n) {
              e[u] = lout[i + u];
              const float4* src = reinterpret_cast<const float4*>(gout + (size_t)e[u].y * C + c);
#pragma unroll
              for (int k = 0; k < F; ++k) vv[u][k] = src[k];
            }
          }
#pragma unroll
          for (int u = 0; u < kRowBatch; ++u) {
            if (i + u < n) {
              const int corner = e[u].x & 3;
              const float yl = __int_as_float(e[u].z), xl = __int_as_float(e[u].w);
#pragma unroll
              for (int k = 0; k < F; ++k) {
                float4 g = vv[u][k];
                if (sr > 0) g = div4(g, bd);
                acc[k].x += weigh(corner, yl, xl, g.x);
                acc[k].y += weigh(corner, yl, xl, g.y);
                acc[k].z += weigh(corner, yl, xl, g.z);
                acc[k].w += weigh(corner, yl, xl, g.w);
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();  // (lin / lout reused by the next run)
      } else {
        const int f = ru.w;
        const int ns = (n + kSeg - 1) / kSeg;
        for (int j = 0; j < ns; ++j) {
          const float4* src = reinterpret_cast<const float4*>(partial + (size_t)(f + j) * C + c);
#pragma unroll
          for (int k = 0; k < F; ++k) {
            const float4 v = src[k];
            acc[k].x += v.x; acc[k].y += v.y; acc[k].z += v.z; acc[k].w += v.w;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < F; ++k) {
        if (any) {
          res[k].x = res[k].x + acc[k].x; res[k].y = res[k].y + acc[k].y;
          res[k].z = res[k].z + acc[k].z; res[k].w = res[k].w + acc[k].w;
        } else {
          res[k] = acc[k];
        }
      }
      any = true;
    }
    if (!any) continue;
#pragma unroll
    for (int k = 0; k < F; ++k) {
      if (acc_lv) {
        const float4 o = old[k];
        res[k].x = o.x + res[k].x; res[k].y = o.y + res[k].y;
        res[k].z = o.z + res[k].z; res[k].w = o.w + res[k].w;
      }
      d4[k] = res[k];
    }
  }
}

int fill_args(RoiArgs& a, const int32_t* dims, const float* scales, int num_levels, int C,
              const float* boxes, const int32_t* box_ind, int R, int out_h, int out_w,
              int sampling_ratio, int box_mode, int pad_border, int assign, int min_level,
              int max_level, int canonical_box_size, int canonical_level) {
  D2MI_REQUIRE(num_levels >= 1 && num_levels <= D2MI_MAX_LEVELS, "num_levels=%d out of [1,%d]",
               num_levels, D2MI_MAX_LEVELS);
  D2MI_REQUIRE(C > 0 && R >= 0 && out_h > 0 && out_w > 0, "bad ROIAlign sizes C=%d R=%d out=%dx%d",
               C, R, out_h, out_w);
  D2MI_REQUIRE(sampling_ratio >= 0, "sampling_ratio must be >= 0, got %d", sampling_ratio);
  D2MI_REQUIRE(box_mode >= 0 && box_mode <= 2, "box_mode must be 0, 1 or 2");
  D2MI_REQUIRE(!(assign && num_levels > 1) || (max_level - min_level + 1 == num_levels),
               "level range %d..%d does not match num_levels=%d", min_level, max_level,
               num_levels);
  D2MI_REQUIRE(canonical_box_size > 0, "canonical_box_size must be > 0");
  D2MI_REQUIRE(((uintptr_t)boxes & 15) == 0, "boxes must be 16-byte aligned");
  a.L = num_levels;
  a.C = C;
  for (int l = 0; l < num_levels; ++l) {
    a.N[l] = dims[3 * l];
    a.H[l] = dims[3 * l + 1];
    a.W[l] = dims[3 * l + 2];
    a.scale[l] = scales[l];
    D2MI_REQUIRE(a.H[l] > 0 && a.W[l] > 0, "level %d has empty spatial size", l);
  }
  a.boxes = boxes;
  a.box_ind = box_ind;
  a.R = R;
  a.out_h = out_h;
  a.out_w = out_w;
  a.sr = sampling_ratio;
  a.box_mode = box_mode;
  a.pad_border = pad_border;
  a.assign = assign;
  a.min_level = min_level;
  a.max_level = max_level;
  a.canon_size = canonical_box_size;
  a.canon_level = canonical_level;
  a.err = error_word();
  D2MI_REQUIRE(a.err != nullptr, "device error word unavailable");
  return 0;
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_roi_align_fwd(const float* const* feats, const int32_t* dims,
                                  const float* scales, int num_levels, int C, const float* boxes,
                                  const int32_t* box_ind, int R, int out_h, int out_w,
                                  int sampling_ratio, int box_mode, int pad_border, int assign,
                                  int min_level, int max_level, int canonical_box_size,
                                  int canonical_level, int32_t* level_out, float* out,
                                  void* stream) {
  RoiArgs a = {};
  int rc = fill_args(a, dims, scales, num_levels, C, boxes, box_ind, R, out_h, out_w,
                     sampling_ratio, box_mode, pad_border, assign, min_level, max_level,
                     canonical_box_size, canonical_level);
  if (rc) return rc;
  bool vec4 = (C % 4) == 0 && ((uintptr_t)out & 15) == 0;
  for (int l = 0; l < num_levels; ++l) {
    a.feat[l] = feats[l];
    vec4 = vec4 && (((uintptr_t)feats[l] & 15) == 0);
  }
  a.level_out = level_out;
  a.out = out;
  if (R == 0) return 0;
  const int nbins = out_h * out_w;
  a.bpb = kMaxBinsPerBlock;
  while (a.bpb > kMinBinsPerBlock &&
         (long long)R * ((nbins + a.bpb - 1) / a.bpb) < kFwdMinBlocks)
    a.bpb /= 2;
  // tuning "roi_fwd" (A/B, tools/roi_ab.py): bit 1 = 2 bins per wave
  // iteration (fewer VGPRs, more resident waves), bit 2 = the blocks of a ROI
  // split its bins evenly, bit 4 = non-temporal output stores, bit 8 = XCD-
  // contiguous ROI order.  Default (-1): 2 | 4 | 8, and 1 from 256 ROIs up --
  // measured on the training step's own ROIs: the box pooler (1,024 ROIs)
  // 32.1 -> 26.3 us (XCD order alone 28.1: ROIs that neighbour in the sampled
  // layout share an L2), the mask pooler (32 ROIs x 14x14) 19.7 -> 18.9-19.6
  int tv = tuning(kTuneRoiFwd);
  if (tv < 0) tv = 2 | 4 | 8 | (R >= 256 ? 1 : 0);
  // r6, bit 16: ONE wave iteration per wave -- a workgroup takes 4 x U bins,
  // so every wave issues all of its corner loads in one round (the bins'
  // loads no longer wait on the previous bins' round trips); bit 32: U = 8
  const int U = (tv & 32) ? 8 : (tv & 1) ? 2 : 4;
  if (tv & 16) a.bpb = 4 * U;
  const int nby = (nbins + a.bpb - 1) / a.bpb;
  if (tv & 2) a.bpb = (nbins + nby - 1) / nby;
  a.xcd_remap = (tv & 8) ? 1 : 0;
  dim3 grid(R, nby);
  hipStream_t st = as_stream(stream);
  if (!vec4)
    hipLaunchKernelGGL((roi_align_fwd_kernel<false>), grid, dim3(256), 0, st, a);
  else if (tv & 64) {  // r6, bit 64: the corner rows loaded non-temporally
    if (U == 2)
      hipLaunchKernelGGL((roi_align_fwd_kernel<true, 2, true, true>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((roi_align_fwd_kernel<true, 4, true, true>), grid, dim3(256), 0, st, a);
  } else if (U == 8)
    hipLaunchKernelGGL((roi_align_fwd_kernel<true, 8, true>), grid, dim3(256), 0, st, a);
  else if ((tv & 5) == 0)
    hipLaunchKernelGGL((roi_align_fwd_kernel<true, 4, false>), grid, dim3(256), 0, st, a);
  else if ((tv & 5) == 1)
    hipLaunchKernelGGL((roi_align_fwd_kernel<true, 2, false>), grid, dim3(256), 0, st, a);
  else if ((tv & 5) == 4)
    hipLaunchKernelGGL((roi_align_fwd_kernel<true, 4, true>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((roi_align_fwd_kernel<true, 2, true>), grid, dim3(256), 0, st, a);
  D2MI_LAUNCH_CHECK();
  return 0;
}

namespace d2mi {
namespace {

struct BwdPlan {
  long long total_pixels, pairs, n_keys, n_samples, max_segs, max_touched, max_tasks;
  int set_bits;
  PixMap pm;
};

// n_samples: the sampling points of all ROI sets; set_bits: 1 for a merged
// two-set backward (runs per (pixel, set) pair), else 0.
int bwd_plan_n(const int32_t* dims, int num_levels, long long n_samples, int set_bits,
               BwdPlan* p) {
  p->n_samples = n_samples;
  p->n_keys = p->n_samples * 4;
  p->set_bits = set_bits;
  long long t = 0;
  for (int l = 0; l < num_levels; ++l) {
    p->pm.base[l] = t;
    t += (long long)dims[3 * l] * dims[3 * l + 1] * dims[3 * l + 2];
  }
  p->pm.base[num_levels] = t;
  p->pm.L = num_levels;
  p->total_pixels = t;
  p->pairs = t << set_bits;
  // every split run has > kSeg contributions: segments <= 2 * n / kSeg, and
  // long-sort tasks <= n / kLongTask + (number of long runs)
  p->max_segs = 2 * (p->n_keys / kSeg) + 1;
  p->max_tasks = p->n_keys / kLongTask + p->n_keys / (kSeg + 1) + 2;
  p->pm.tbase[0] = 0;
  for (int l = 0; l < num_levels; ++l)
    p->pm.tbase[l + 1] =
        p->pm.tbase[l] + (int32_t)std::min(p->n_keys, p->pm.base[l + 1] - p->pm.base[l]);
  p->max_touched = p->pm.tbase[num_levels];
  D2MI_REQUIRE(p->n_keys < (1LL << 31) && p->pairs < (1LL << 31) &&
                   p->n_keys * num_levels < (1LL << 31),
               "ROIAlign backward too large");
  return 0;
}

int bwd_plan(const int32_t* dims, int num_levels, int R, int out_h, int out_w, int sr,
             BwdPlan* p) {
  const long long S = sr > 0 ? sr : 1;
  return bwd_plan_n(dims, num_levels, (long long)R * out_h * out_w * S * S, 0, p);
}

template <class WS>
void bwd_layout(WS& w, int C, const BwdPlan& p) {
  w.template take<uint64_t>((size_t)p.n_keys + 1);          // ent: pair << 32 | arrival rank
  w.template take<int32_t>((size_t)p.n_keys + 1);           // arrival-ordered slots
  w.template take<RunRec>((size_t)p.n_keys + 1);            // arrival-ordered run records
  w.template take<int32_t>((size_t)p.n_keys + 1);           // long runs in slot order
  w.template take<Contrib>((size_t)p.n_samples + 1);        // records
  w.template take<int32_t>((size_t)p.pairs + 1);            // count
  w.template take<int32_t>((size_t)p.pairs + 1);            // run_start
  w.template take<int32_t>((size_t)p.pairs + 1);            // seg_first
  w.template take<int32_t>((size_t)p.max_segs);             // seg_pixel
  w.template take<float>((size_t)p.max_segs * C);           // partial rows
  w.template take<int32_t>((size_t)p.max_touched + 1);      // touched pixels
  w.template take<int4>(((size_t)p.max_touched + 1) * 2);   // their runs per set
  w.template take<int2>((size_t)p.max_tasks);               // long-sort tasks
  w.template take<BwdCounters>(1);
}

// The backward over nsets (1 or 2) ROI sets of the same maps; sets[k] holds
// each set's ROIs / crop / grad_out (everything else equal).
// phase bit 1 (prepare): the clear launch (pair counters, bookkeeping, and the
// maps of levels [lv_lo, lv_hi] not in acc_mask), emits, runs, place, long
// sort, segment partials -- everything but the pixel pass, its results left in
// the workspace; bit 2 (pixels): the pixel pass over the touched pixels of
// levels [lv_lo, lv_hi] only.  Phase 3 is the whole backward.  Split phases
// let the pixel pass of a level run later, into a map another backward has
// written in full (the RPN head conv's dgrad: no clear of that map, no second
// read of it): the workspace must then stay untouched in between.
int roi_bwd_core(const RoiArgs* sets, int nsets, const int32_t* dims, int num_levels, int C,
                 int acc_mask, bool vec4, void* workspace, size_t workspace_bytes,
                 hipStream_t st, int phase = 3, int lv_lo = 0, int lv_hi = -1) {
  if (lv_hi < 0) lv_hi = num_levels - 1;
  D2MI_REQUIRE(phase >= 1 && phase <= 3 && 0 <= lv_lo && lv_lo <= lv_hi && lv_hi < num_levels,
               "ROIAlign backward: bad phase %d / level range [%d, %d]", phase, lv_lo, lv_hi);
  RoiArgs a = sets[0];
  a.acc_mask = acc_mask;
  long long ns[2] = {0, 0};
  for (int k = 0; k < nsets; ++k) {
    const long long S = sets[k].sr > 0 ? sets[k].sr : 1;
    ns[k] = (long long)sets[k].R * sets[k].out_h * sets[k].out_w * S * S;
    a.gout_s[k] = sets[k].gout;
    a.sr_s[k] = sets[k].sr;
  }
  const int sb = nsets > 1 ? 1 : 0;
  BwdPlan p;
  int rc = bwd_plan_n(dims, num_levels, ns[0] + ns[1], sb, &p);
  if (rc) return rc;
  WorkspaceSizer z;
  bwd_layout(z, C, p);
  D2MI_REQUIRE(workspace_bytes >= z.off && (workspace || z.off == 0),
               "ROIAlign backward workspace too small: %zu < %zu", workspace_bytes, z.off);
  if (p.total_pixels == 0) return 0;
  Workspace w(workspace, workspace_bytes);
  uint64_t* ent = w.take<uint64_t>((size_t)p.n_keys + 1);
  int32_t* arrival = w.take<int32_t>((size_t)p.n_keys + 1);
  RunRec* runrec = w.take<RunRec>((size_t)p.n_keys + 1);
  int32_t* sorted_long = w.take<int32_t>((size_t)p.n_keys + 1);
  Contrib* rec = w.take<Contrib>((size_t)p.n_samples + 1);
  int32_t* count = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* run_start = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* seg_first = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* seg_pixel = w.take<int32_t>((size_t)p.max_segs);
  float* partial = w.take<float>((size_t)p.max_segs * C);
  int32_t* touched = w.take<int32_t>((size_t)p.max_touched + 1);
  int4* trun = w.take<int4>(((size_t)p.max_touched + 1) * 2);
  int2* tasks = w.take<int2>((size_t)p.max_tasks);
  BwdCounters* ctr = w.take<BwdCounters>(1);
  // r5: the C = 256 pixel pass reads run records (tuning "roi_bwd_rec", 1);
  // 0 = the r4 slot pass (A/B).  Phase 1 and phase 2 of one backward must
  // see the same value (a deferred pass reads what the prepare wrote).
  const bool use_runrec = vec4 && C == 256 && tuning(kTuneRoiBwdRec) != 0;
  if (phase & 1) {
  ClearList cl = {};
  long long clear_words = 0;
  auto clear = [&](void* ptr, long long words, uint32_t value) {
    cl.ptr[cl.n] = static_cast<uint32_t*>(ptr);
    cl.words[cl.n] = words;
    cl.value[cl.n] = value;
    ++cl.n;
    clear_words += words;
  };
  for (int l = lv_lo; l <= lv_hi; ++l)  // untouched pixels: zero (accumulated levels: kept)
    if (!((acc_mask >> l) & 1))
      clear(a.gfeat[l], (long long)dims[3 * l] * dims[3 * l + 1] * dims[3 * l + 2] * C, 0u);
  clear(count, p.pairs, 0u);
  clear(ctr, sizeof(BwdCounters) / 4, 0u);
  hipLaunchKernelGGL(roi_bwd_clear_kernel,
                     dim3((unsigned)std::max(1LL, std::min((clear_words / 4 + 255) / 256, 8192LL))),
                     dim3(256), 0, st, cl);
  D2MI_LAUNCH_CHECK();
  if (p.n_keys == 0) return 0;
  {
    const int nb0 = (int)((ns[0] + 255) / 256), nb1 = nsets > 1 ? (int)((ns[1] + 255) / 256) : 0;
    if (nb0 + nb1 > 0) {
      hipLaunchKernelGGL(roi_bwd_emit_kernel, dim3((unsigned)(nb0 + nb1)), dim3(256), 0, st,
                         sets[0], sets[nsets > 1 ? 1 : 0], nb0, ns[0], p.pm, sb, count, ent, rec);
      D2MI_LAUNCH_CHECK();
    }
  }
  hipLaunchKernelGGL(roi_bwd_runs_kernel, dim3((unsigned)((p.total_pixels + 1023) / 1024)),
                     dim3(1024), 0, st, count, p.total_pixels, sb, run_start, seg_first, seg_pixel,
                     tasks, touched, use_runrec ? trun : nullptr, ctr, p.pm,
                     tuning(kTuneRoiHeavy));
  D2MI_LAUNCH_CHECK();
  hipLaunchKernelGGL(roi_bwd_place_kernel, dim3((unsigned)((p.n_keys + 255) / 256)), dim3(256), 0,
                     st, ent, p.n_keys, run_start, arrival, rec, use_runrec ? runrec : nullptr);
  D2MI_LAUNCH_CHECK();
  // long runs (degenerate piles of boxes) in slot order, then their segment
  // partials: grid-stride loops over the device-side task / segment counts
  // (zero in an ordinary step: the launches exit at once)
  // (small grids: the dispatch of a large grid that only reads a zero count
  // and exits is most of these launches' cost in an ordinary step)
  hipLaunchKernelGGL((vec4 ? roi_bwd_long_kernel<true> : roi_bwd_long_kernel<false>),
                     dim3((unsigned)std::max(1LL, std::min<long long>(p.max_tasks, 64LL))),
                     dim3(1024), 0, st, a, arrival, count, run_start, tasks, ctr, sorted_long, rec,
                     seg_first, seg_pixel, partial);
  D2MI_LAUNCH_CHECK();
  }  // phase 1
  if (phase == 2) {  // a pixel pass alone: its non-accumulated maps start from zero
    ClearList cl = {};
    long long words = 0;
    for (int l = lv_lo; l <= lv_hi; ++l)
      if (!((acc_mask >> l) & 1)) {
        cl.ptr[cl.n] = reinterpret_cast<uint32_t*>(a.gfeat[l]);
        cl.words[cl.n] = (long long)dims[3 * l] * dims[3 * l + 1] * dims[3 * l + 2] * C;
        words += cl.words[cl.n++];
      }
    if (cl.n) {
      hipLaunchKernelGGL(roi_bwd_clear_kernel,
                         dim3((unsigned)std::max(1LL, std::min((words / 4 + 255) / 256, 8192LL))),
                         dim3(256), 0, st, cl);
      D2MI_LAUNCH_CHECK();
    }
  }
  if (!(phase & 2) || p.n_keys == 0) return 0;
  // fixed grid sized by the capacity of the pass's level segments (the
  // touched counts stay on the device): at most 8192 workgroups x 4 waves =
  // 32 waves per SIMD over 256 CUs x 4 SIMDs; waves beyond residency start
  // as earlier ones retire (the kBatch sweep above)
  // (tuning roi_pix_grid: the workgroup cap; the waves grid-stride)
  const long long cap = p.pm.tbase[lv_hi + 1] - p.pm.tbase[lv_lo];
  const long long wg_max = std::max(1, tuning(kTuneRoiPixGrid));
  const dim3 grid((unsigned)std::max(1LL, std::min((cap + 3) / 4, wg_max)));
  if (vec4 && C == 256) {
    static const int ppw = [] {
      const char* e = getenv("D2MI_ROI_BWD_PPW");
      return e && e[0] == '8' ? 8 : 0;
    }();
    // tuning "roi_bwd_rec" (the run-record pass): 1 two pixels per wave, 4
    // rows in flight per lane (r5c, default); 2 / 3 four pixels per wave with
    // 2 / 4 rows (r5b: 4); 5 one pixel per wave, 8 rows; D2MI_ROI_BWD_PPW=8
    // eight pixels per wave (A/B forms)
    const int tv = tuning(kTuneRoiBwdRec);
    const int pw = ppw == 8 ? 8 : tv == 5 ? 1 : (tv == 2 || tv == 3) ? 4 : 2;  // pixels per wave
    const dim3 g4((unsigned)std::max(1LL, std::min((cap + 4 * pw - 1) / (4 * pw), wg_max)));
    if (!use_runrec)  // the r4 pixel pass (A/B)
      hipLaunchKernelGGL(roi_bwd_pixel_c256_slots_kernel<4>, g4, dim3(256), 0, st, a, p.pm,
                         arrival, rec, sb, count, run_start, seg_first, partial, touched, ctr,
                         lv_lo, lv_hi);
    else if (ppw == 8)
      hipLaunchKernelGGL((roi_bwd_pixel_c256_kernel<8, 4>), g4, dim3(256), 0, st, a, p.pm, runrec,
                         sb, trun, partial, ctr, lv_lo, lv_hi);
    else if (tv == 2)
      hipLaunchKernelGGL((roi_bwd_pixel_c256_kernel<4, 2>), g4, dim3(256), 0, st, a, p.pm, runrec,
                         sb, trun, partial, ctr, lv_lo, lv_hi);
    else if (tv == 3)
      hipLaunchKernelGGL((roi_bwd_pixel_c256_kernel<4, 4>), g4, dim3(256), 0, st, a, p.pm, runrec,
                         sb, trun, partial, ctr, lv_lo, lv_hi);
    else if (tv == 5)
      hipLaunchKernelGGL((roi_bwd_pixel_c256_kernel<1, 8>), g4, dim3(256), 0, st, a, p.pm, runrec,
                         sb, trun, partial, ctr, lv_lo, lv_hi);
    else
      hipLaunchKernelGGL((roi_bwd_pixel_c256_kernel<2, 4>), g4, dim3(256), 0, st, a, p.pm, runrec,
                         sb, trun, partial, ctr, lv_lo, lv_hi);
  } else if (vec4) {
    hipLaunchKernelGGL(roi_bwd_pixel_kernel<true>, grid, dim3(256), 0, st, a, p.pm, arrival, rec,
                       sb, count, run_start, seg_first, partial, touched, ctr, lv_lo, lv_hi);
  } else {
    hipLaunchKernelGGL(roi_bwd_pixel_kernel<false>, grid, dim3(256), 0, st, a, p.pm, arrival, rec,
                       sb, count, run_start, seg_first, partial, touched, ctr, lv_lo, lv_hi);
  }
  D2MI_LAUNCH_CHECK();
  return 0;
}

}  // namespace
}  // namespace d2mi

extern "C" size_t d2mi_roi_align_bwd_workspace_size(const int32_t* dims, int num_levels, int C,
                                                    int R, int out_h, int out_w,
                                                    int sampling_ratio) {
  if (!dims || num_levels < 1 || num_levels > D2MI_MAX_LEVELS || R < 0 || C < 1) return 0;
  BwdPlan p;
  if (bwd_plan(dims, num_levels, R, out_h, out_w, sampling_ratio, &p)) return 0;
  WorkspaceSizer w;
  bwd_layout(w, C, p);
  return w.off;
}

extern "C" int d2mi_roi_align_bwd_ex(float* const* grad_feats, const int32_t* dims,
                                     const float* scales, int num_levels, int C,
                                     const float* boxes, const int32_t* box_ind, int R, int out_h,
                                     int out_w, int sampling_ratio, int box_mode, int pad_border,
                                     int assign, int min_level, int max_level,
                                     int canonical_box_size, int canonical_level,
                                     const float* grad_out, int accumulate, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  RoiArgs a = {};
  int rc = fill_args(a, dims, scales, num_levels, C, boxes, box_ind, R, out_h, out_w,
                     sampling_ratio, box_mode, pad_border, assign, min_level, max_level,
                     canonical_box_size, canonical_level);
  if (rc) return rc;
  bool vec4 = (C % 4) == 0 && ((uintptr_t)grad_out & 15) == 0;
  for (int l = 0; l < num_levels; ++l) {
    a.gfeat[l] = grad_feats[l];
    vec4 = vec4 && (((uintptr_t)grad_feats[l] & 15) == 0);
  }
  a.gout = grad_out;
  return roi_bwd_core(&a, 1, dims, num_levels, C, accumulate ? (1 << num_levels) - 1 : 0, vec4,
                      workspace, workspace_bytes, as_stream(stream));
}

extern "C" size_t d2mi_roi_align_bwd2_workspace_size(const int32_t* dims, int num_levels, int C,
                                                     int R0, int out_h0, int out_w0, int sr0,
                                                     int R1, int out_h1, int out_w1, int sr1) {
  if (!dims || num_levels < 1 || num_levels > D2MI_MAX_LEVELS || R0 < 0 || R1 < 0 || C < 1)
    return 0;
  const long long S0 = sr0 > 0 ? sr0 : 1, S1 = sr1 > 0 ? sr1 : 1;
  BwdPlan p;
  if (bwd_plan_n(dims, num_levels,
                 (long long)R0 * out_h0 * out_w0 * S0 * S0 + (long long)R1 * out_h1 * out_w1 * S1 * S1,
                 1, &p))
    return 0;
  WorkspaceSizer w;
  bwd_layout(w, C, p);
  return w.off;
}

extern "C" int d2mi_roi_align_bwd2_ex(float* const* grad_feats, const int32_t* dims,
                                      const float* scales, int num_levels, int C, int box_mode,
                                      int pad_border, int assign, int min_level, int max_level,
                                      int canonical_box_size, int canonical_level,
                                      const float* boxes0, const int32_t* box_ind0, int R0,
                                      int out_h0, int out_w0, int sr0, const float* grad_out0,
                                      const float* boxes1, const int32_t* box_ind1, int R1,
                                      int out_h1, int out_w1, int sr1, const float* grad_out1,
                                      int accumulate_mask, int phase, int level_lo, int level_hi,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  RoiArgs sets[2] = {};
  int rc = fill_args(sets[0], dims, scales, num_levels, C, boxes0, box_ind0, R0, out_h0, out_w0,
                     sr0, box_mode, pad_border, assign, min_level, max_level, canonical_box_size,
                     canonical_level);
  if (rc) return rc;
  rc = fill_args(sets[1], dims, scales, num_levels, C, boxes1, box_ind1, R1, out_h1, out_w1, sr1,
                 box_mode, pad_border, assign, min_level, max_level, canonical_box_size,
                 canonical_level);
  if (rc) return rc;
  bool vec4 = (C % 4) == 0 && ((uintptr_t)grad_out0 & 15) == 0 && ((uintptr_t)grad_out1 & 15) == 0;
  for (int l = 0; l < num_levels; ++l) {
    // (a map outside a phase's level range may be null)
    sets[0].gfeat[l] = sets[1].gfeat[l] = grad_feats ? grad_feats[l] : nullptr;
    vec4 = vec4 && (((uintptr_t)sets[0].gfeat[l] & 15) == 0);
  }
  sets[0].gout = grad_out0;
  sets[1].gout = grad_out1;
  D2MI_REQUIRE((accumulate_mask >> num_levels) == 0, "accumulate_mask has bits past the levels");
  for (int l = level_lo; l <= level_hi && l < num_levels; ++l)
    D2MI_REQUIRE(l < 0 || sets[0].gfeat[l] != nullptr ||
                     (phase == 1 && ((accumulate_mask >> l) & 1)),
                 "level %d's gradient map is needed by this phase", l);
  return roi_bwd_core(sets, 2, dims, num_levels, C, accumulate_mask, vec4, workspace,
                      workspace_bytes, as_stream(stream), phase, level_lo, level_hi);
}

extern "C" int d2mi_roi_align_bwd2(float* const* grad_feats, const int32_t* dims,
                                   const float* scales, int num_levels, int C, int box_mode,
                                   int pad_border, int assign, int min_level, int max_level,
                                   int canonical_box_size, int canonical_level,
                                   const float* boxes0, const int32_t* box_ind0, int R0,
                                   int out_h0, int out_w0, int sr0, const float* grad_out0,
                                   const float* boxes1, const int32_t* box_ind1, int R1,
                                   int out_h1, int out_w1, int sr1, const float* grad_out1,
                                   int accumulate_mask, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  return d2mi_roi_align_bwd2_ex(grad_feats, dims, scales, num_levels, C, box_mode, pad_border,
                                assign, min_level, max_level, canonical_box_size, canonical_level,
                                boxes0, box_ind0, R0, out_h0, out_w0, sr0, grad_out0, boxes1,
                                box_ind1, R1, out_h1, out_w1, sr1, grad_out1, accumulate_mask, 3, 0,
                                num_levels - 1, workspace, workspace_bytes, stream);
}

extern "C" int d2mi_roi_align_bwd(float* const* grad_feats, const int32_t* dims,
                                  const float* scales, int num_levels, int C, const float* boxes,
                                  const int32_t* box_ind, int R, int out_h, int out_w,
                                  int sampling_ratio, int box_mode, int pad_border, int assign,
                                  int min_level, int max_level, int canonical_box_size,
                                  int canonical_level, const float* grad_out, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  return d2mi_roi_align_bwd_ex(grad_feats, dims, scales, num_levels, C, boxes, box_ind, R, out_h,
                               out_w, sampling_ratio, box_mode, pad_border, assign, min_level,
                               max_level, canonical_box_size, canonical_level, grad_out, 0,
                               workspace, workspace_bytes, stream);
}
