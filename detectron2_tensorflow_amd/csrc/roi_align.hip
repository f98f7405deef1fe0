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
  t.valid = !(in < 0.f || in > (float)(img_p - 1));
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

constexpr int kBinsPerBlock = 64;

template <bool VEC4>
__global__ __launch_bounds__(256) void roi_align_fwd_kernel(RoiArgs a) {
  const int r = blockIdx.x;
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
  const int b_end = min(nbins, (int)(blockIdx.y + 1) * kBinsPerBlock);
  for (int bin = blockIdx.y * kBinsPerBlock + wave; bin < b_end; bin += 4) {
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

// Backward: TF CropAndResizeGradImage scatter (+ AvgPoolGrad's 1/count and
// MirrorPadGrad folding the pad rows onto the edge rows, both implicit here).
// Channel mapping c = lane + 64 k keeps every atomic wave-instruction on 256
// contiguous bytes (the full-rate atomic shape on gfx950).
__global__ __launch_bounds__(256) void roi_align_bwd_kernel(RoiArgs a) {
  const int r = blockIdx.x;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const RoiGeom g = roi_geom(a, r);
  if (!g.ok) return;
  const int nbins = a.out_h * a.out_w;
  const int S = a.sr > 0 ? a.sr : 1;
  const float inv = a.sr > 0 ? (float)(a.sr * a.sr) : 1.f;
  float* base = a.gfeat[g.lvl] + (size_t)g.n * g.H * g.W * a.C;
  const int C = a.C;
  const bool pad = a.pad_border != 0;
  const int b_end = min(nbins, (int)(blockIdx.y + 1) * kBinsPerBlock);
  for (int bin = blockIdx.y * kBinsPerBlock + wave; bin < b_end; bin += 4) {
    const int oy = bin / a.out_w, ox = bin - oy * a.out_w;
    const float* src = a.gout + ((size_t)r * nbins + bin) * C;
    for (int sy = 0; sy < S; ++sy) {
      const Tap ty = make_tap(in_coord(g.y1, g.y2, g.hs, oy * S + sy, g.ch, g.Hp), g.Hp, g.H,
                              pad);
      if (!ty.valid) continue;
      for (int sx = 0; sx < S; ++sx) {
        const Tap tx = make_tap(in_coord(g.x1, g.x2, g.ws, ox * S + sx, g.cw, g.Wp), g.Wp,
                                g.W, pad);
        if (!tx.valid) continue;
        float* tl = base + ((size_t)ty.r0 * g.W + tx.r0) * C;
        float* tr = base + ((size_t)ty.r0 * g.W + tx.r1) * C;
        float* bl = base + ((size_t)ty.r1 * g.W + tx.r0) * C;
        float* br = base + ((size_t)ty.r1 * g.W + tx.r1) * C;
        for (int c = lane; c < C; c += 64) {
          float gv = src[c];
          if (S > 1) gv = gv / inv;
          const float dtop = (1.f - ty.lerp) * gv;
          const float dbot = ty.lerp * gv;
          atomicAdd(tl + c, (1.f - tx.lerp) * dtop);
          atomicAdd(tr + c, tx.lerp * dtop);
          atomicAdd(bl + c, (1.f - tx.lerp) * dbot);
          atomicAdd(br + c, tx.lerp * dbot);
        }
      }
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
  dim3 grid(R, (nbins + kBinsPerBlock - 1) / kBinsPerBlock);
  if (vec4)
    hipLaunchKernelGGL(roi_align_fwd_kernel<true>, grid, dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(roi_align_fwd_kernel<false>, grid, dim3(256), 0, as_stream(stream), a);
  D2MI_LAUNCH_CHECK();
  return 0;
}

extern "C" int d2mi_roi_align_bwd(float* const* grad_feats, const int32_t* dims,
                                  const float* scales, int num_levels, int C, const float* boxes,
                                  const int32_t* box_ind, int R, int out_h, int out_w,
                                  int sampling_ratio, int box_mode, int pad_border, int assign,
                                  int min_level, int max_level, int canonical_box_size,
                                  int canonical_level, const float* grad_out, void* stream) {
  RoiArgs a = {};
  int rc = fill_args(a, dims, scales, num_levels, C, boxes, box_ind, R, out_h, out_w,
                     sampling_ratio, box_mode, pad_border, assign, min_level, max_level,
                     canonical_box_size, canonical_level);
  if (rc) return rc;
  for (int l = 0; l < num_levels; ++l) a.gfeat[l] = grad_feats[l];
  a.gout = grad_out;
  if (R == 0) return 0;
  const int nbins = out_h * out_w;
  dim3 grid(R, (nbins + kBinsPerBlock - 1) / kBinsPerBlock);
  hipLaunchKernelGGL(roi_align_bwd_kernel, grid, dim3(256), 0, as_stream(stream), a);
  D2MI_LAUNCH_CHECK();
  return 0;
}
