// Shared device/host helpers for libd2mi_hip.so (gfx950 only).
// All translation units are compiled with -ffp-contract=off so that every
// float expression below rounds exactly like the TF 1.x CPU kernels it
// restates (no fused multiply-add unless written as one).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/d2mi.h"

namespace d2mi {

void set_error(const char* fmt, ...);
int32_t* error_word();

#define D2MI_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::d2mi::set_error(__VA_ARGS__);      \
      return -1;                           \
    }                                      \
  } while (0)

#define D2MI_HIP(expr)                                                             \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::d2mi::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                        __FILE__, __LINE__);                                       \
      return -2;                                                                   \
    }                                                                              \
  } while (0)

#define D2MI_LAUNCH_CHECK() D2MI_HIP(hipGetLastError())

enum ErrorBits : int32_t {
  kErrBoxInd = 1,
  kErrNmsCapacity = 2,
  kErrTopkCapacity = 4,
};

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-owned workspace.
struct Workspace {
  char* base;
  size_t cap;
  size_t off;
  Workspace(void* b, size_t c) : base((char*)b), cap(c), off(0) {}
  template <typename T>
  T* take(size_t n) {
    off = align_up(off, 256);
    T* p = (T*)(base + off);
    off += n * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

// Sizing twin of Workspace (same alignment rule) for *_workspace_size().
struct WorkspaceSizer {
  size_t off = 0;
  template <typename T>
  void take(size_t n) {
    off = align_up(off, 256);
    off += n * sizeof(T);
  }
};

// float -> uint32 whose unsigned order equals the float order.  -0.0 maps to
// +0.0's word: TF's top_k / NMS compare the values, so the two zeros tie (and
// the index decides), as in oracle/oracle.c's comparators.
__device__ __forceinline__ uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) == 0u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_orderable(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// Sort key: ascending order of the key == score descending, index ascending
// (TF NonMaxSuppressionV3 / TopKV2 tie rule). Scores that TF would never
// select (NaN, -inf with score_threshold=-inf) map to ~0ull.
__device__ __forceinline__ uint64_t desc_key(float score, uint32_t idx) {
  if (!(score > -INFINITY)) return ~0ull;
  return ((uint64_t)(~orderable(score)) << 32) | (uint64_t)idx;
}
__device__ __forceinline__ float key_score(uint64_t key) {
  return from_orderable(~(uint32_t)(key >> 32));
}

// TF non_max_suppression_op.cc IOU(): corners min/max-normalised, 0 when an
// area is <= 0, all float32, evaluated in exactly this order.
__device__ __forceinline__ float tf_iou(float4 a, float4 b) {
  const float ymin_i = fminf(a.x, a.z), xmin_i = fminf(a.y, a.w);
  const float ymax_i = fmaxf(a.x, a.z), xmax_i = fmaxf(a.y, a.w);
  const float ymin_j = fminf(b.x, b.z), xmin_j = fminf(b.y, b.w);
  const float ymax_j = fmaxf(b.x, b.z), xmax_j = fmaxf(b.y, b.w);
  const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
  const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
  if (area_i <= 0.f || area_j <= 0.f) return 0.f;
  const float iymin = fmaxf(ymin_i, ymin_j), ixmin = fmaxf(xmin_i, xmin_j);
  const float iymax = fminf(ymax_i, ymax_j), ixmax = fminf(xmax_i, xmax_j);
  const float inter = fmaxf(iymax - iymin, 0.f) * fmaxf(ixmax - ixmin, 0.f);
  return inter / ((area_i + area_j) - inter);
}

// Box2BoxTransform.apply_deltas for one (box, delta) pair
// (lib/modeling/box_regression.py:95-122), float32, no contraction.
// inv: wy, wx, wh, ww weights (division, as the reference divides).
__device__ __forceinline__ float4 apply_delta(float4 box, float4 d, float wy, float wx,
                                              float wh, float ww, float clamp) {
  const float h = box.z - box.x;
  const float w = box.w - box.y;
  const float cy = box.x + 0.5f * h;
  const float cx = box.y + 0.5f * w;
  const float dy = d.x / wy;
  const float dx = d.y / wx;
  float dh = d.z / wh;
  float dw = d.w / ww;
  dh = fminf(dh, clamp);
  dw = fminf(dw, clamp);
  const float pcy = dy * h + cy;
  const float pcx = dx * w + cx;
  const float ph = expf(dh) * h;
  const float pw = expf(dw) * w;
  return make_float4(pcy - 0.5f * ph, pcx - 0.5f * pw, pcy + 0.5f * ph, pcx + 0.5f * pw);
}

// clip_to_window with window [0, 0, hmax, wmax] (box_list_ops.py:112-147):
// max(min(v, win_max), win_min).
__device__ __forceinline__ float4 clip_box(float4 b, float hmax, float wmax) {
  return make_float4(fmaxf(fminf(b.x, hmax), 0.f), fmaxf(fminf(b.y, wmax), 0.f),
                     fmaxf(fminf(b.z, hmax), 0.f), fmaxf(fminf(b.w, wmax), 0.f));
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace d2mi
