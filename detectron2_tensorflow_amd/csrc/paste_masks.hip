// Mask pasting for gfx950: per-detection box masks -> full-canvas uint8 masks.
//
// Restates, per output pixel, the exact float32 sequence of
//   lib/modeling/postprocessing.py:9-59   detector_postprocess ("conventional"
//                                          and "fixed"; "fixed" first scales the
//                                          boxes by output_shape / image_shape)
//   lib/structures/mask_ops.py:7-56       reframe_box_masks_to_image_masks:
//     boxes -> normalised (box_list_ops.to_normalized_coordinates: * (1/H), * (1/W)),
//     reverse box of the unit square ((0 - min) / (max - min), (1 - min) / (max - min)),
//     tf.image.crop_and_resize(box_masks, reverse boxes, crop = canvas, bilinear,
//     extrapolation 0), then tf.greater(., threshold) -> uint8.
// The reference materialises the float32 canvas [D, H, W, 1] (4 B/pixel) and
// thresholds it in a second pass; here the threshold is the epilogue and only
// the uint8 canvas is written (1 B/pixel): the launch is HBM-write-bound.
//
// Layout: box masks [D, mh, mw] f32 (the mask head's sigmoid output), boxes
// [D, 4] f32 yxyx absolute, out [D, H, W] u8.  One 256-thread workgroup owns
// kRows canvas rows of one detection; the (mh x mw) mask is staged in LDS; a
// thread produces 4 adjacent pixels per step (one 32-bit store).
#include "common.h"
#include "internal.h"

namespace d2mi {
namespace {

constexpr int kRows = 8;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxMaskElems = 64 * 64;

struct PasteArgs {
  const float* masks;
  const float* boxes;
  const float* yx_scale;   // [D, 2] or null ("fixed" format)
  const uint8_t* valid;    // [D] or null
  int D, mh, mw, H, W;
  float threshold;
  uint8_t* out;
};

// TF CropAndResize per-axis sample: source index pair + lerp, or invalid
// (extrapolation) when the coordinate leaves [0, img - 1].
struct Samp {
  int lo, hi;
  float lerp;
  bool ok;
};

__device__ __forceinline__ Samp sample(float c1, float scale, int i, int img) {
  Samp s;
  const float in = c1 * (float)(img - 1) + (float)i * scale;
  s.ok = in >= 0.f && in <= (float)(img - 1);  // NaN (degenerate box) -> extrapolate
  const float fl = floorf(in);
  s.lo = (int)fl;
  s.hi = (int)ceilf(in);
  s.lerp = in - fl;
  s.lo = min(max(s.lo, 0), img - 1);
  s.hi = min(max(s.hi, 0), img - 1);
  return s;
}

// Conservative index range [lo, hi] of the canvas rows / columns i in [0, n)
// whose sample c * (m - 1) + i * s can land inside [0, m - 1] (solved in
// double, widened by 2): outside it every pixel is the extrapolation value,
// inside it every pixel gets the exact per-pixel test.  Non-finite
// coordinates (degenerate boxes) sample nothing.
__device__ __forceinline__ void live_range(float c, float s, int m, int n, int& lo, int& hi) {
  const double a = (double)(c * (float)(m - 1)), sd = (double)s;
  if (!(isfinite(a) && isfinite(sd))) { lo = 1; hi = 0; return; }
  if (sd == 0.0) { lo = 0; hi = n - 1; return; }
  double t0 = -a / sd, t1 = ((double)(m - 1) - a) / sd;
  if (t0 > t1) { const double t = t0; t0 = t1; t1 = t; }
  t0 = fmax(t0, -4.0);
  t1 = fmin(t1, (double)n + 4.0);
  lo = max(0, (int)floor(t0) - 2);
  hi = min(n - 1, (int)ceil(t1) + 2);
}

__global__ __launch_bounds__(256) void paste_masks_kernel(PasteArgs a) {
  const int d = blockIdx.y;
  const int row0 = blockIdx.x * kRows;
  uint8_t* out = a.out + (size_t)d * a.H * a.W;
  const bool live = a.valid == nullptr || a.valid[d] != 0;
  const int row1 = min(row0 + kRows, a.H);
  // the workgroup's rows are one contiguous chunk: zero it with wide stores
  auto zero_fill = [&]() {
    uint8_t* p = out + (size_t)row0 * a.W;
    const size_t bytes = (size_t)(row1 - row0) * a.W;
    if ((a.W & 15) == 0) {
      // streaming (non-temporal) stores: the canvas is not re-read here
      for (size_t i = threadIdx.x * 16; i < bytes; i += blockDim.x * 16)
        __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, reinterpret_cast<u32x4*>(p + i));
    } else {
      for (size_t i = threadIdx.x; i < bytes; i += blockDim.x) p[i] = 0;
    }
  };
  if (!live) {  // padded detection slot: zeros (SparseBoxList.to_dense)
    zero_fill();
    return;
  }
  // box -> (fixed: * scale) -> normalised -> reverse box, in the reference's order
  float y1 = a.boxes[4 * d + 0], x1 = a.boxes[4 * d + 1];
  float y2 = a.boxes[4 * d + 2], x2 = a.boxes[4 * d + 3];
  if (a.yx_scale) {
    const float sy = a.yx_scale[2 * d], sx = a.yx_scale[2 * d + 1];
    y1 = sy * y1; y2 = sy * y2; x1 = sx * x1; x2 = sx * x2;
  }
  const float ih = 1.f / (float)a.H, iw = 1.f / (float)a.W;
  y1 = ih * y1; y2 = ih * y2; x1 = iw * x1; x2 = iw * x2;
  const float dy = y2 - y1, dx = x2 - x1;
  const float ry1 = (0.f - y1) / dy, rx1 = (0.f - x1) / dx;
  const float ry2 = (1.f - y1) / dy, rx2 = (1.f - x1) / dx;
  // crop = canvas (H, W) from the (mh, mw) mask
  const float hs = a.H > 1 ? ((ry2 - ry1) * (float)(a.mh - 1)) / (float)(a.H - 1) : 0.f;
  const float ws = a.W > 1 ? ((rx2 - rx1) * (float)(a.mw - 1)) / (float)(a.W - 1) : 0.f;
  const float cy = a.H > 1 ? ry1 : 0.f, cx = a.W > 1 ? rx1 : 0.f;

  const uint8_t ext = 0.f > a.threshold ? 1 : 0;  // extrapolation value 0, thresholded
  int ylo = 0, yhi = a.H - 1, xlo = 0, xhi = a.W - 1;
  if (!ext) {  // skip the exact test where it can only give the (zero) extrapolation
    if (a.H > 1) live_range(cy, hs, a.mh, a.H, ylo, yhi);
    if (a.W > 1) live_range(cx, ws, a.mw, a.W, xlo, xhi);
  }
  if (row0 > yhi || row1 - 1 < ylo || xlo > xhi) {  // no live sample in these rows
    zero_fill();
    return;
  }
  __shared__ float m[kMaxMaskElems];
  const int n = a.mh * a.mw;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m[i] = a.masks[(size_t)d * n + i];
  __syncthreads();

  const bool vec = (a.W & 3) == 0;
  const bool vec16 = (a.W & 15) == 0;
  for (int y = row0; y < row1; ++y) {
    uint8_t* orow = out + (size_t)y * a.W;
    if (y < ylo || y > yhi || xlo > xhi) {  // all-extrapolation row: plain zero stores
      if (vec16) {
        for (int x = threadIdx.x * 16; x < a.W; x += blockDim.x * 16)
          __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, reinterpret_cast<u32x4*>(orow + x));
      } else {
        for (int x = threadIdx.x; x < a.W; x += blockDim.x) orow[x] = 0;
      }
      continue;
    }
    Samp sy;
    if (a.H > 1) {
      sy = sample(cy, hs, y, a.mh);
    } else {  // crop height 1: 0.5 * (y1 + y2) * (image_height - 1), in double (TF)
      const float in = (float)(0.5 * (double)(ry1 + ry2) * (double)(a.mh - 1));
      sy.ok = in >= 0.f && in <= (float)(a.mh - 1);
      const float fl = floorf(in);
      sy.lo = min(max((int)fl, 0), a.mh - 1);
      sy.hi = min(max((int)ceilf(in), 0), a.mh - 1);
      sy.lerp = in - fl;
    }
    const float* mt = m + sy.lo * a.mw;
    const float* mb = m + sy.hi * a.mw;
    auto pix = [&](int x) -> uint8_t {
      if (!sy.ok) return ext;
      Samp sx;
      if (a.W > 1) {
        sx = sample(cx, ws, x, a.mw);
      } else {
        const float in = (float)(0.5 * (double)(rx1 + rx2) * (double)(a.mw - 1));
        sx.ok = in >= 0.f && in <= (float)(a.mw - 1);
        const float fl = floorf(in);
        sx.lo = min(max((int)fl, 0), a.mw - 1);
        sx.hi = min(max((int)ceilf(in), 0), a.mw - 1);
        sx.lerp = in - fl;
      }
      if (!sx.ok) return ext;
      const float tl = mt[sx.lo], tr = mt[sx.hi], bl = mb[sx.lo], br = mb[sx.hi];
      const float top = tl + (tr - tl) * sx.lerp;
      const float bot = bl + (br - bl) * sx.lerp;
      const float v = top + (bot - top) * sy.lerp;
      return v > a.threshold ? 1 : 0;
    };
    if (vec) {
      for (int x4 = threadIdx.x * 4; x4 < a.W; x4 += blockDim.x * 4) {
        uint32_t w = 0;
        if (x4 + 3 >= xlo && x4 <= xhi)
          w = (uint32_t)pix(x4) | ((uint32_t)pix(x4 + 1) << 8) | ((uint32_t)pix(x4 + 2) << 16) |
              ((uint32_t)pix(x4 + 3) << 24);
        __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(orow + x4));
      }
    } else {
      for (int x = threadIdx.x; x < a.W; x += blockDim.x)
        orow[x] = (x >= xlo && x <= xhi) ? pix(x) : 0;
    }
  }
}

}  // namespace
}  // namespace d2mi

using namespace d2mi;

extern "C" int d2mi_paste_masks(const float* box_masks, const float* boxes, const float* yx_scale,
                                const uint8_t* valid, int D, int mask_h, int mask_w, int out_h,
                                int out_w, float threshold, uint8_t* out, void* stream) {
  D2MI_REQUIRE(D >= 0 && mask_h > 0 && mask_w > 0 && out_h > 0 && out_w > 0,
               "bad paste_masks sizes D=%d mask=%dx%d out=%dx%d", D, mask_h, mask_w, out_h,
               out_w);
  D2MI_REQUIRE(mask_h * mask_w <= kMaxMaskElems, "box masks larger than %d elements",
               kMaxMaskElems);
  D2MI_REQUIRE(((uintptr_t)out & 3) == 0, "out must be 4-byte aligned");
  if (D == 0) return 0;
  PasteArgs a;
  a.masks = box_masks;
  a.boxes = boxes;
  a.yx_scale = yx_scale;
  a.valid = valid;
  a.D = D;
  a.mh = mask_h;
  a.mw = mask_w;
  a.H = out_h;
  a.W = out_w;
  a.threshold = threshold;
  a.out = out;
  D2MI_REQUIRE(D <= 65535, "at most 65535 detections per launch");
  const dim3 grid((unsigned)((out_h + kRows - 1) / kRows), (unsigned)D);
  hipLaunchKernelGGL(paste_masks_kernel, grid, dim3(256), 0, as_stream(stream), a);
  D2MI_LAUNCH_CHECK();
  return 0;
}
