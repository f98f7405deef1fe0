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
template <bool VEC4, int U = 4, bool NT = false>
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
        c00[u] = p[((size_t)ty.r0 * g.W + tx.r0) * 64 + lane];
        c01[u] = p[((size_t)ty.r0 * g.W + tx.r1) * 64 + lane];
        c10[u] = p[((size_t)ty.r1 * g.W + tx.r0) * 64 + lane];
        c11[u] = p[((size_t)ty.r1 * g.W + tx.r1) * 64 + lane];
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
// scatter of them ran at ~120 GB/s.  Instead:
//   1. emit: for every (ROI, sample, corner) contribution a 64-bit key
//      pixel << low_bits | slot, slot = (roi * samples + sample) * 4 + corner,
//      and its (grad_out row, y_lerp, x_lerp) record at index slot (the ROI
//      geometry is computed in place);
//   2. stable onesweep radix sort on the pixel bits only: pixel-major, and
//      within a pixel the emission (TF loop) order is kept;
//   3. runs (one kernel): the touched-pixel list, each run's bounds, and for
//      runs with more than kSeg contributions a block of kSeg-long segments
//      (slots from a counter) summed by one wave each into a partial row —
//      bounded work per wave however many ROIs pile onto one pixel (collapsed
//      proposals at the image border do);
//   4. the grad maps are zero-filled (one clear launch, full bandwidth) and
//      the touched pixels are summed by waves striding over that list, four
//      pixels per wave at C = 256 (16 lanes x 16 channels each): each sums its
//      contributions (or its segments' partials) in order and stores the
//      pixel once.
// Two ROI sets of the same maps (the box and mask poolers, d2mi_roi_align_bwd2)
// share one pass: keys carry (pixel, set), each set's run is summed apart and
// the two sums added.
// Summation order per pixel is (box, y, x, corner), the TF kernel's loop order
// (partials regroup it for pixels past kSeg): deterministic run to run, and
// bit-identical to the TF scatter for pixels with at most kSeg contributions
// and no folded pad row.
constexpr int kSeg = 64;    // contributions per wave before a pixel is split
constexpr int kBatch = 2;   // contributions in flight per wave (r1 sweep, pixel kernel avg: 16 -> 103 us, 8 -> 64, 4 -> 49.5, 2 -> 46.7: occupancy, not loads in flight, binds)

struct PixMap {
  long long base[D2MI_MAX_LEVELS + 1];  // first global pixel id per level
};

struct Contrib {
  int32_t row;  // grad_out row index r * nbins + bin (of its set's grad_out)
  float yl, xl;
  int32_t set;  // ROI set (0 / 1) of a merged backward
};

// One launch clears every buffer the backward starts from (the per-level grad
// maps to 0, run_start to -1, the touched counter to 0) instead of a
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
// 40 B the thread stores) rather than staged by a separate launch.
// set / sample_base: a merged backward emits its second ROI set after the
// first (samples from sample_base on) with pair keys pixel * 2 + set
// (set_bits = 1): each set's contributions of a pixel form their own run.
__global__ void roi_bwd_emit_kernel(RoiArgs a, PixMap pm, int low_bits, int set, int set_bits,
                                    long long sample_base, uint64_t* __restrict__ keys,
                                    Contrib* __restrict__ rec) {
  const int S = a.sr > 0 ? a.sr : 1;
  const long long nsamp = (long long)a.out_h * a.out_w * S * S;
  const long long tl = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tl >= (long long)a.R * nsamp) return;
  const int r = (int)(tl / nsamp);
  const int s = (int)(tl - (long long)r * nsamp);
  const RoiGeom g = roi_geom(a, r);
  const long long t = sample_base + tl;
  const uint64_t slot = (uint64_t)t * 4u;
  uint64_t* k = keys + slot;
  bool ok = g.ok;
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
  if (!ok) {
    k[0] = k[1] = k[2] = k[3] = ~0ull;
    return;
  }
  Contrib c;
  c.row = r * (a.out_h * a.out_w) + (iy / S) * a.out_w + ix / S;
  c.yl = ty.lerp;
  c.xl = tx.lerp;
  c.set = set;
  rec[t] = c;  // shared by the 4 corners: slot >> 2
  const uint64_t img = (uint64_t)pm.base[g.lvl] + (uint64_t)g.n * g.H * g.W;
  const int sh = low_bits + set_bits;
  const uint64_t sb = (uint64_t)set << low_bits;
  k[0] = ((img + (uint64_t)ty.r0 * g.W + tx.r0) << sh) | sb | (slot + 0);
  k[1] = ((img + (uint64_t)ty.r0 * g.W + tx.r1) << sh) | sb | (slot + 1);
  k[2] = ((img + (uint64_t)ty.r1 * g.W + tx.r0) << sh) | sb | (slot + 2);
  k[3] = ((img + (uint64_t)ty.r1 * g.W + tx.r1) << sh) | sb | (slot + 3);
}

// run_start[p] = first sorted index of pixel p (-1 untouched), run_end[p] = one past its last.
// Every touched pixel is also appended to touched[] (*n_touched entries; the
// list order varies run to run, the per-pixel sums do not).
// One thread per sorted key.  The first key of a pixel appends the pixel to
// touched[] (workgroup-aggregated counter); the first key of a (pixel, set)
// run (set_bits = 1: runs per pair, indexed pixel * 2 + set) records the run:
// start, end (found by walking the sorted keys: runs are a handful of keys),
// and for a run longer than kSeg its segment count, a block of segment slots
// taken from *n_segs and the slots' owner -- the split-run bookkeeping that
// took a per-pixel pass, a scan and a fill pass before.  Slot order varies run
// to run; each run's partials are summed in segment order (deterministic).
__global__ __launch_bounds__(1024) void roi_bwd_runs_kernel(const uint64_t* __restrict__ keys, long long n, int low_bits,
                                    int set_bits, long long total_pixels,
                                    int32_t* __restrict__ run_start,
                                    int32_t* __restrict__ run_end, int32_t* __restrict__ nseg,
                                    int32_t* __restrict__ seg_first,
                                    int32_t* __restrict__ seg_pixel, int32_t* __restrict__ n_segs,
                                    int32_t* __restrict__ touched,
                                    int32_t* __restrict__ n_touched) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t q = i < n ? keys[i] >> low_bits : ~0ull;  // pair
  const uint64_t p = q >> set_bits;                         // pixel
  const bool live = i < n && (long long)p < total_pixels;  // invalid contributions sort last
  const uint64_t qprev = (live && i > 0) ? keys[i - 1] >> low_bits : ~0ull;
  const bool first = live && (i == 0 || (qprev >> set_bits) != p);  // first of the pixel
  const bool first_pair = live && (i == 0 || qprev != q);
  // one global counter atomic per 1024-thread workgroup: same-address device
  // atomics serialise (one per wave still cost ~20 us per launch); the waves'
  // offsets come from an LDS counter
  __shared__ int wg_count, wg_base;
  if (threadIdx.x == 0) wg_count = 0;
  __syncthreads();
  const uint64_t m = __ballot(first);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (m && lane == 0) base = atomicAdd(&wg_count, __popcll(m));
  base = __shfl(base, 0);
  __syncthreads();
  if (threadIdx.x == 0) wg_base = wg_count ? atomicAdd(n_touched, wg_count) : 0;
  __syncthreads();
  base += wg_base;
  if (first) touched[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)p;
  if (first_pair) {
    long long j = i + 1;
    while (j < n && (keys[j] >> low_bits) == q) ++j;
    const int len = (int)(j - i);
    run_start[q] = (int32_t)i;
    run_end[q] = (int32_t)j;
    int ns = 0;
    if (len > kSeg) {
      ns = (len + kSeg - 1) / kSeg;
      const int f = atomicAdd(n_segs, ns);
      seg_first[q] = f;
      for (int k = 0; k < ns; ++k) seg_pixel[f + k] = (int32_t)q;
    }
    nseg[q] = ns;
  }
}

// TF order of operations: dtop = (1 - y_lerp) * g, dbot = y_lerp * g, then
// (1 - x_lerp) * d or x_lerp * d.
__device__ __forceinline__ float weigh(int corner, float yl, float xl, float v) {
  const float d = (corner < 2) ? (1.f - yl) * v : yl * v;
  return (corner & 1) ? xl * d : (1.f - xl) * d;
}

// Sum of sorted contributions [i0, i1) for the lane's channel(s) c.
template <bool VEC4>
__device__ __forceinline__ float4 sum_run(const RoiArgs& a, const uint64_t* __restrict__ keys,
                                          const Contrib* __restrict__ rec, uint64_t low_mask,
                                          int i0, int i1, int c, bool live) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int C = a.C;
  for (int i = i0; i < i1; i += kBatch) {
    int corner[kBatch];
    Contrib e[kBatch];
    const int m = min(kBatch, i1 - i);
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      if (u < m) {
        const uint64_t slot = keys[i + u] & low_mask;
        corner[u] = (int)(slot & 3u);
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
        if (sr > 0) {  // the avg-pool divisor of the set's sampling ratio
          const float inv = (float)(sr * sr);
          g.x = g.x / inv; g.y = g.y / inv; g.z = g.z / inv; g.w = g.w / inv;
        }
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

// One wave per split segment: partial[seg] (C floats).
template <bool VEC4>
__global__ __launch_bounds__(256) void roi_bwd_segment_kernel(
    RoiArgs a, const uint64_t* __restrict__ keys, const Contrib* __restrict__ rec, int low_bits,
    const int32_t* __restrict__ run_start, const int32_t* __restrict__ run_end,
    const int32_t* __restrict__ seg_first, const int32_t* __restrict__ seg_pixel,
    const int32_t* __restrict__ total_segs, float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int nsegs = *total_segs;
  const uint64_t low_mask = (1ull << low_bits) - 1ull;
  const int step = VEC4 ? 256 : 64;
  for (int seg = blockIdx.x * 4 + (threadIdx.x >> 6); seg < nsegs; seg += gridDim.x * 4) {
    const int p = seg_pixel[seg];
    const int k = seg - seg_first[p];
    const int i0 = run_start[p] + k * kSeg;
    const int i1 = min(i0 + kSeg, run_end[p]);
    for (int c0 = 0; c0 < a.C; c0 += step) {
      const int c = c0 + (VEC4 ? lane * 4 : lane);
      const bool live = c < a.C;
      const float4 acc = sum_run<VEC4>(a, keys, rec, low_mask, i0, i1, c, live);
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
// iteration, so the dependent load chain of a pixel (run bounds -> sorted keys
// -> records -> grad_out rows) overlaps across waves instead of a wave per
// feature-map pixel (most of which only stored zeros) -- that launch was bound
// by wave start-up and latency, at ~1/4 of its store bandwidth.
template <bool VEC4>
__global__ __launch_bounds__(256) void roi_bwd_pixel_kernel(
    RoiArgs a, PixMap pm, const uint64_t* __restrict__ keys, const Contrib* __restrict__ rec,
    int low_bits, int set_bits, const int32_t* __restrict__ run_start,
    const int32_t* __restrict__ run_end, const int32_t* __restrict__ nseg,
    const int32_t* __restrict__ seg_first, const float* __restrict__ partial,
    const int32_t* __restrict__ touched, const int32_t* __restrict__ n_touched) {
  const int lane = threadIdx.x & 63;
  const int C = a.C;
  const uint64_t low_mask = (1ull << low_bits) - 1ull;
  const int step = VEC4 ? 256 : 64;
  const int nt = *n_touched;
  const int nsets = 1 << set_bits;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < nt; t += gridDim.x * 4) {
    const long long pix = touched[t];
    int l = 0;
    while (l + 1 < a.L && pix >= pm.base[l + 1]) ++l;
    float* dst = a.gfeat[l] + (size_t)(pix - pm.base[l]) * C;
    const bool acc_lv = (a.acc_mask >> l) & 1;
    for (int c0 = 0; c0 < C; c0 += step) {
      const int c = c0 + (VEC4 ? lane * 4 : lane);
      const bool live = c < C;
      float4 res = make_float4(0.f, 0.f, 0.f, 0.f);
      bool any = false;
      // each set's contributions summed apart (its own TF-order run), then
      // set 0 + set 1: the rounding of the sum of two separate backwards
      for (int sidx = 0; sidx < nsets; ++sidx) {
        const long long q = (pix << set_bits) | sidx;
        const int i0 = run_start[q];
        if (i0 < 0) continue;
        const int i1 = run_end[q];
        const int ns = nseg[q];
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ns == 0) {
          acc = sum_run<VEC4>(a, keys, rec, low_mask, i0, i1, c, live);
        } else if (live) {
          const int f = seg_first[q];
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

// C == 256 form of roi_bwd_pixel_kernel: a wave sums FOUR touched pixels at
// once, 16 lanes per pixel, 16 channels (4 float4) per lane -- four
// independent load chains (run bounds -> keys -> records -> grad_out rows)
// in flight per wave instead of one, the same per-pixel order and rounding.
template <int PPW>
__global__ __launch_bounds__(256) void roi_bwd_pixel_c256_kernel(
    RoiArgs a, PixMap pm, const uint64_t* __restrict__ keys, const Contrib* __restrict__ rec,
    int low_bits, int set_bits, const int32_t* __restrict__ run_start,
    const int32_t* __restrict__ run_end, const int32_t* __restrict__ nseg,
    const int32_t* __restrict__ seg_first, const float* __restrict__ partial,
    const int32_t* __restrict__ touched, const int32_t* __restrict__ n_touched) {
  constexpr int C = 256;
  constexpr int LPP = 64 / PPW;     // lanes per pixel
  constexpr int F = C / LPP / 4;    // float4 per lane
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPP, sub = lane % LPP;
  const int c = sub * 4 * F;  // this lane's channels
  const uint64_t low_mask = (1ull << low_bits) - 1ull;
  const int nt = *n_touched;
  const int nsets = 1 << set_bits;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int tb = wave * PPW; tb < nt; tb += gridDim.x * 4 * PPW) {
    const int t = tb + grp;
    if (t >= nt) continue;
    const long long pix = touched[t];
    int l = 0;
    while (l + 1 < a.L && pix >= pm.base[l + 1]) ++l;
    float* dst = a.gfeat[l] + (size_t)(pix - pm.base[l]) * C + c;
    float4 res[F];
    bool any = false;
    for (int sidx = 0; sidx < nsets; ++sidx) {
      const long long q = (pix << set_bits) | sidx;
      const int i0 = run_start[q];
      if (i0 < 0) continue;
      const int i1 = run_end[q];
      const int ns = nseg[q];
      float4 acc[F];
#pragma unroll
      for (int k = 0; k < F; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ns == 0) {
        for (int i = i0; i < i1; ++i) {
          const uint64_t slot = keys[i] & low_mask;
          const int corner = (int)(slot & 3u);
          const Contrib e = rec[slot >> 2];
          const float4* src =
              reinterpret_cast<const float4*>(a.gout_s[e.set] + (size_t)e.row * C + c);
          float4 v[F];
#pragma unroll
          for (int k = 0; k < F; ++k) v[k] = src[k];
          const int sr = a.sr_s[e.set];
          const float inv = (float)(sr * sr);
#pragma unroll
          for (int k = 0; k < F; ++k) {
            float4 g = v[k];
            if (sr > 0) { g.x = g.x / inv; g.y = g.y / inv; g.z = g.z / inv; g.w = g.w / inv; }
            acc[k].x += weigh(corner, e.yl, e.xl, g.x);
            acc[k].y += weigh(corner, e.yl, e.xl, g.y);
            acc[k].z += weigh(corner, e.yl, e.xl, g.z);
            acc[k].w += weigh(corner, e.yl, e.xl, g.w);
          }
        }
      } else {
        const int f = seg_first[q];
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
    const bool acc_lv = (a.acc_mask >> l) & 1;
    float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll
    for (int k = 0; k < F; ++k) {
      if (acc_lv) {
        const float4 o = d4[k];
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
  const int nby = (nbins + a.bpb - 1) / a.bpb;
  if (tv & 2) a.bpb = (nbins + nby - 1) / nby;
  a.xcd_remap = (tv & 8) ? 1 : 0;
  dim3 grid(R, nby);
  hipStream_t st = as_stream(stream);
  if (!vec4)
    hipLaunchKernelGGL((roi_align_fwd_kernel<false>), grid, dim3(256), 0, st, a);
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

int bits_for(unsigned long long v) {  // smallest b with 2^b > v
  int b = 0;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

struct BwdPlan {
  long long total_pixels, pairs, n_keys, n_samples, max_segs, max_touched;
  int low_bits, end_bit, set_bits;
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
  p->total_pixels = t;
  p->pairs = t << set_bits;
  // every split run has > kSeg contributions: segments <= 2 * n / kSeg
  p->max_segs = 2 * (p->n_keys / kSeg) + 1;
  p->max_touched = std::min(p->n_keys, t);
  p->low_bits = max(1, bits_for(p->n_keys > 0 ? (unsigned long long)(p->n_keys - 1) : 0ull));
  p->end_bit = p->low_bits + set_bits + bits_for((unsigned long long)t);
  D2MI_REQUIRE(p->end_bit <= 64, "ROIAlign backward key space too large (%d bits)", p->end_bit);
  D2MI_REQUIRE(p->n_keys < (1LL << 31) && p->pairs < (1LL << 31), "ROIAlign backward too large");
  return 0;
}

int bwd_plan(const int32_t* dims, int num_levels, int R, int out_h, int out_w, int sr,
             BwdPlan* p) {
  const long long S = sr > 0 ? sr : 1;
  return bwd_plan_n(dims, num_levels, (long long)R * out_h * out_w * S * S, 0, p);
}

template <class WS>
void bwd_layout(WS& w, int C, const BwdPlan& p) {
  w.template take<uint64_t>((size_t)p.n_keys + 1);          // keys
  w.template take<uint64_t>((size_t)p.n_keys + 1);          // sorted keys
  w.template take<Contrib>((size_t)p.n_samples + 1);        // records
  w.template take<int32_t>((size_t)p.pairs + 1);            // run_start
  w.template take<int32_t>((size_t)p.pairs + 1);            // run_end
  w.template take<int32_t>((size_t)p.pairs + 1);            // nseg
  w.template take<int32_t>((size_t)p.pairs + 1);            // seg_first
  w.template take<int32_t>((size_t)p.max_segs);             // seg_pixel
  w.template take<float>((size_t)p.max_segs * C);           // partial rows
  w.template take<int32_t>((size_t)p.max_touched + 1);      // touched pixels
  w.template take<int32_t>(2);                              // their count, segment count
  w.template take<char>(radix_sort_u64_workspace_size((size_t)p.n_keys, p.low_bits, p.end_bit));
}

// The backward over nsets (1 or 2) ROI sets of the same maps; sets[k] holds
// each set's ROIs / crop / grad_out (everything else equal).
int roi_bwd_core(const RoiArgs* sets, int nsets, const int32_t* dims, int num_levels, int C,
                 int acc_mask, bool vec4, void* workspace, size_t workspace_bytes,
                 hipStream_t st) {
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
  uint64_t* keys = w.take<uint64_t>((size_t)p.n_keys + 1);
  uint64_t* sorted = w.take<uint64_t>((size_t)p.n_keys + 1);
  Contrib* rec = w.take<Contrib>((size_t)p.n_samples + 1);
  int32_t* run_start = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* run_end = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* nseg = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* seg_first = w.take<int32_t>((size_t)p.pairs + 1);
  int32_t* seg_pixel = w.take<int32_t>((size_t)p.max_segs);
  float* partial = w.take<float>((size_t)p.max_segs * C);
  int32_t* touched = w.take<int32_t>((size_t)p.max_touched + 1);
  int32_t* n_touched = w.take<int32_t>(2);  // [0] touched pixels, [1] segment slots
  int32_t* n_segs = n_touched + 1;
  const size_t tmp_bytes = radix_sort_u64_workspace_size((size_t)p.n_keys, p.low_bits, p.end_bit);
  void* tmp = w.take<char>(tmp_bytes);
  const long long TQ = p.pairs;
  ClearList cl = {};
  long long clear_words = 0;
  auto clear = [&](void* ptr, long long words, uint32_t value) {
    cl.ptr[cl.n] = static_cast<uint32_t*>(ptr);
    cl.words[cl.n] = words;
    cl.value[cl.n] = value;
    ++cl.n;
    clear_words += words;
  };
  for (int l = 0; l < num_levels; ++l)  // untouched pixels: zero (accumulated levels: kept)
    if (!((acc_mask >> l) & 1))
      clear(a.gfeat[l], (long long)dims[3 * l] * dims[3 * l + 1] * dims[3 * l + 2] * C, 0u);
  clear(run_start, TQ, 0xffffffffu);
  clear(n_touched, 2, 0u);
  hipLaunchKernelGGL(roi_bwd_clear_kernel,
                     dim3((unsigned)std::max(1LL, std::min((clear_words / 4 + 255) / 256, 8192LL))),
                     dim3(256), 0, st, cl);
  D2MI_LAUNCH_CHECK();
  if (p.n_keys > 0) {
    long long base = 0;
    for (int k = 0; k < nsets; ++k) {
      if (ns[k] > 0) {
        hipLaunchKernelGGL(roi_bwd_emit_kernel, dim3((unsigned)((ns[k] + 255) / 256)), dim3(256),
                           0, st, sets[k], p.pm, p.low_bits, k, sb, base, keys, rec);
        D2MI_LAUNCH_CHECK();
      }
      base += ns[k];
    }
    // pair bits only: the sort is stable and the keys are emitted in slot
    // (TF loop) order, so each (pixel, set) run stays in that order
    rc = radix_sort_u64(keys, sorted, (size_t)p.n_keys, p.low_bits, p.end_bit, tmp, tmp_bytes,
                        st);
    if (rc) return rc;
    hipLaunchKernelGGL(roi_bwd_runs_kernel, dim3((unsigned)((p.n_keys + 1023) / 1024)), dim3(1024),
                       0, st, sorted, p.n_keys, p.low_bits, sb, p.total_pixels, run_start, run_end,
                       nseg, seg_first, seg_pixel, n_segs, touched, n_touched);
    D2MI_LAUNCH_CHECK();
  }
  if (p.n_keys == 0) return 0;
  // segment partials of the split runs: a grid-stride loop over *n_segs
  // (usually a handful; bounded by max_segs)
  const dim3 sgrid((unsigned)std::max(1LL, std::min<long long>((p.max_segs + 3) / 4, 1024LL)));
  if (vec4)
    hipLaunchKernelGGL(roi_bwd_segment_kernel<true>, sgrid, dim3(256), 0, st, a, sorted, rec,
                       p.low_bits, run_start, run_end, seg_first, seg_pixel, n_segs, partial);
  else
    hipLaunchKernelGGL(roi_bwd_segment_kernel<false>, sgrid, dim3(256), 0, st, a, sorted, rec,
                       p.low_bits, run_start, run_end, seg_first, seg_pixel, n_segs, partial);
  D2MI_LAUNCH_CHECK();
  // fixed grid (the touched count stays on the device): at most 8192
  // workgroups x 4 waves = 32 waves per SIMD over 256 CUs x 4 SIMDs; waves
  // beyond residency start as earlier ones retire (the kBatch sweep above)
  const dim3 grid((unsigned)std::max(1LL, std::min((p.max_touched + 3) / 4, 8192LL)));
#define PIX(V)                                                                            \
  hipLaunchKernelGGL((roi_bwd_pixel_kernel<V>), grid, dim3(256), 0, st, a, p.pm, sorted, rec, \
                     p.low_bits, sb, run_start, run_end, nseg, seg_first, partial, touched,  \
                     n_touched)
  if (vec4 && C == 256) {
    static const int ppw = [] {
      const char* e = getenv("D2MI_ROI_BWD_PPW");
      return e && e[0] == '8' ? 8 : 4;
    }();
    const dim3 g4((unsigned)std::max(1LL, std::min((p.max_touched + 4 * ppw - 1) / (4 * ppw), 8192LL)));
    if (ppw == 8)
      hipLaunchKernelGGL(roi_bwd_pixel_c256_kernel<8>, g4, dim3(256), 0, st, a, p.pm, sorted, rec,
                         p.low_bits, sb, run_start, run_end, nseg, seg_first, partial, touched,
                         n_touched);
    else
      hipLaunchKernelGGL(roi_bwd_pixel_c256_kernel<4>, g4, dim3(256), 0, st, a, p.pm, sorted, rec,
                         p.low_bits, sb, run_start, run_end, nseg, seg_first, partial, touched,
                         n_touched);
  } else if (vec4) {
    PIX(true);
  } else {
    PIX(false);
  }
#undef PIX
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
    sets[0].gfeat[l] = sets[1].gfeat[l] = grad_feats[l];
    vec4 = vec4 && (((uintptr_t)grad_feats[l] & 15) == 0);
  }
  sets[0].gout = grad_out0;
  sets[1].gout = grad_out1;
  D2MI_REQUIRE((accumulate_mask >> num_levels) == 0, "accumulate_mask has bits past the levels");
  return roi_bwd_core(sets, 2, dims, num_levels, C, accumulate_mask, vec4, workspace,
                      workspace_bytes, as_stream(stream));
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
