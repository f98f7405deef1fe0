// Thread-local host error string + the device error word (see include/d2mi.h).
#include <algorithm>
#include <climits>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "internal.h"

namespace {
thread_local char g_msg[1024] = "";
__device__ int32_t g_error_word = 0;
}  // namespace

namespace d2mi {

namespace {
const char* const kTuneNames[kTuneCount] = {"conv_ws",   "roi_fwd",  "wgrad_ws",
                                            "conv_epi",  "wgrad_ws1", "wgrad_xcd",
                                            "conv_xcd",  "wgrad_inc", "conv_ws_mink",
                                            "roi_pix_grid", "conv_stream", "roi_bwd_rec",
                                            "retina_fused", "rpn_merge", "nms_scan", "roi_heavy", "rpn_compact", "conv_stream_nt", "conv_nt", "conv_tail_mink", "conv_ws_mintiles", "sgd_rev", "retina_rank", "solo_mfma", "retina_var"};
const char* const kTuneEnv[kTuneCount] = {"D2MI_CONV_WS",   "D2MI_ROI_FWD",   "D2MI_WGRAD_WS",
                                          "D2MI_CONV_EPI",  "D2MI_WGRAD_WS1", "D2MI_WGRAD_XCD",
                                          "D2MI_CONV_XCD",  "D2MI_WGRAD_INC", "D2MI_CONV_WS_MINK",
                                          "D2MI_ROI_PIX_GRID", "D2MI_CONV_STREAM",
                                          "D2MI_ROI_BWD_REC", "D2MI_RETINA_FUSED",
                                          "D2MI_RPN_MERGE", "D2MI_NMS_SCAN", "D2MI_ROI_HEAVY", "D2MI_RPN_COMPACT", "D2MI_CONV_STREAM_NT", "D2MI_CONV_NT", "D2MI_CONV_TAIL_MINK", "D2MI_CONV_WS_MINTILES", "D2MI_SGD_REV", "D2MI_RETINA_RANK", "D2MI_SOLO_MFMA", "D2MI_RETINA_VAR"};
// defaults: measured per shape and in the training step
// conv_stream: the streaming 1x1 for launches of >= 8192 output pixels (r5 in-step A/B:
// -0.85 %, profiles/r5_ab_inproc_conv_stream.log); roi_bwd_rec: run records (-0.41 %);
// retina_fused: RetinaNet inference in four launches (retina_post.hip; 0 the
// unfused pipeline, 2 the fused one with its in-workgroup exact select forced)
// rpn_merge: the RPN's per-image concat + top-k as a merge rank (proposals.hip)
// solo_mfma: the SOLOv2 Matrix-NMS intersections on int8 MFMA (solo.hip, r6):
// 2 = bits expanded by an LDS table (default), 1 = by arithmetic, 0 = the AND +
// popcount tiles; retina_var: the r6 RetinaNet post (compaction, early
// select bound, DPP / permlane bitonic and select, NMS IoU only where boxes
// meet, NMS tiles resolved as a ballot fixed point, the floor's radix select,
// the rank launch's rounds looped, small levels' floor samples spread over the
// level: 12018; 0 = the r5 form; + 4096, the rank
// inside the NMS per 128-candidate window, is faster on iid logits and slower
// on a model's head outputs, where the NMS needs several windows)
const int kTuneDefault[kTuneCount] = {2, -1, 1, 1, 6, 1, 1, 1, 16, 8192, 8192, 1, 1, 1, 1, 16, 1, 2, 0, 8, 0, 0, 0, 2, 12018};
int g_tune[kTuneCount];
bool g_tune_set[kTuneCount];
}  // namespace

int tuning(TuneKey k) {
  if (!g_tune_set[k]) {
    const char* e = getenv(kTuneEnv[k]);
    g_tune[k] = e ? atoi(e) : kTuneDefault[k];
    g_tune_set[k] = true;
  }
  return g_tune[k];
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_msg, sizeof(g_msg), fmt, ap);
  va_end(ap);
}

namespace {
__global__ void fill_u32_words_kernel(uint32_t* __restrict__ p, size_t n, uint32_t v) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}
__global__ void fill_u8_kernel(uint8_t* __restrict__ p, size_t n, uint8_t v) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}
}  // namespace

// A byte fill as a kernel on ``st`` (in place of hipMemsetAsync, r5): inside
// a captured hipGraph a memset becomes a memset node, and the graphed
// training step's replays diverged from the eager step only where a buffer
// zeroed by one fed an atomic accumulation (the matcher's per-GT best IoU)
// and only when the batch changed -- the node's ordering against the
// kernels around it is not what the stream order was.  A kernel node is
// ordered like every other launch of the capture.
int fill_bytes(void* p, size_t nbytes, uint8_t value, hipStream_t st) {
  if (nbytes == 0) return 0;
  if (((uintptr_t)p & 3) == 0 && (nbytes & 3) == 0) {
    const size_t n = nbytes / 4;
    const uint32_t v = 0x01010101u * value;
    hipLaunchKernelGGL(fill_u32_words_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)),
                       dim3(256), 0, st, (uint32_t*)p, n, v);
  } else {
    hipLaunchKernelGGL(fill_u8_kernel, dim3((unsigned)std::min<size_t>((nbytes + 255) / 256, 4096)),
                       dim3(256), 0, st, (uint8_t*)p, nbytes, value);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int32_t* error_word() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_error_word)) != hipSuccess) return nullptr;
  return (int32_t*)p;
}

}  // namespace d2mi

extern "C" {

int d2mi_version(void) { return 1; }

// Hash of the sources this library was built from (csrc/*.hip, csrc/*.h,
// include/d2mi.h; _build.source_hash), passed in by the build: _C.load
// refuses a library whose hash differs from the tree it is loaded from.
#ifndef D2MI_SOURCE_HASH
#define D2MI_SOURCE_HASH "unknown"
#endif
const char* d2mi_source_hash(void) { return D2MI_SOURCE_HASH; }

const char* d2mi_last_error(void) { return g_msg; }

int d2mi_set_tuning(const char* key, int value) {
  D2MI_REQUIRE(key != nullptr, "null tuning key");
  for (int k = 0; k < d2mi::kTuneCount; ++k) {
    if (strcmp(key, d2mi::kTuneNames[k]) == 0) {
      d2mi::g_tune[k] = value;
      d2mi::g_tune_set[k] = true;
      return 0;
    }
  }
  D2MI_REQUIRE(false, "unknown tuning key '%s'", key);
  return -1;
}

int d2mi_get_tuning(const char* key) {
  if (key == nullptr) return INT32_MIN;
  for (int k = 0; k < d2mi::kTuneCount; ++k)
    if (strcmp(key, d2mi::kTuneNames[k]) == 0) return d2mi::tuning((d2mi::TuneKey)k);
  return INT32_MIN;
}

int32_t* d2mi_error_word_dev(void) { return d2mi::error_word(); }

// Node census of a captured (not yet instantiated) hipGraph: counts[t] = the
// number of nodes of hipGraphNodeType t, for t < ntypes.  The graphed
// training step (engine/graphed.py) refuses a capture holding memset nodes
// while the runtime's graph packet capture is on: those are the nodes whose
// order against the kernels around them it does not keep (r5).
int d2mi_graph_census(void* graph, long long* counts, int ntypes) {
  D2MI_REQUIRE(graph != nullptr && counts != nullptr && ntypes > 0, "bad graph census arguments");
  for (int t = 0; t < ntypes; ++t) counts[t] = 0;
  size_t n = 0;
  D2MI_REQUIRE(hipGraphGetNodes((hipGraph_t)graph, nullptr, &n) == hipSuccess,
               "hipGraphGetNodes failed");
  if (n == 0) return 0;
  hipGraphNode_t* nodes = (hipGraphNode_t*)malloc(n * sizeof(hipGraphNode_t));
  D2MI_REQUIRE(nodes != nullptr, "out of host memory");
  int rc = 0;
  if (hipGraphGetNodes((hipGraph_t)graph, nodes, &n) != hipSuccess) {
    d2mi::set_error("hipGraphGetNodes failed");
    rc = -1;
  }
  for (size_t i = 0; rc == 0 && i < n; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) {
      d2mi::set_error("hipGraphNodeGetType failed");
      rc = -1;
    } else if ((int)t >= 0 && (int)t < ntypes) {
      ++counts[(int)t];
    }
  }
  free(nodes);
  return rc;
}

// The same census of the graph a stream is capturing into right now (a
// diagnosis: tools/graph_nodes.py runs it after every op of a capture to name
// the ops that add memset / memcpy nodes).  Returns 1 when the stream is not
// capturing (counts all 0).
int d2mi_capture_census(void* stream, long long* counts, int ntypes) {
  D2MI_REQUIRE(counts != nullptr && ntypes > 0, "bad capture census arguments");
  for (int t = 0; t < ntypes; ++t) counts[t] = 0;
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  D2MI_REQUIRE(hipStreamGetCaptureInfo_v2(d2mi::as_stream(stream), &status, &id, &graph, &deps,
                                          &ndeps) == hipSuccess,
               "hipStreamGetCaptureInfo_v2 failed");
  if (status != hipStreamCaptureStatusActive || graph == nullptr) return 1;
  return d2mi_graph_census((void*)graph, counts, ntypes);
}

int d2mi_clear_errors(void* stream) {
  int32_t* w = d2mi::error_word();
  D2MI_REQUIRE(w != nullptr, "cannot resolve the device error word");
  D2MI_REQUIRE(d2mi::fill_bytes(w, sizeof(int32_t), 0, d2mi::as_stream(stream)) == 0,
               "error word clear failed");
  return 0;
}

}  // extern "C"
