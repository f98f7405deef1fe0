// Library-internal host APIs shared between translation units.
#pragma once
#include "common.h"

namespace d2mi {

// Segmented ascending sort of 64-bit keys stored in "capacity layout":
// segment s owns keys[s*cap, s*cap + lens[s]).  Keys beyond lens[s] are
// ignored.  cap <= kLdsSortCap: the in-LDS counting-rank kernel; larger
// capacities: that kernel on kLdsSortCap-key tiles, then merge passes.
constexpr int kLdsSortCap = 8192;
size_t sort_workspace_size(int S, int cap);
int sort_keys_segmented(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* lens, int S,
                        int cap, void* ws, size_t ws_bytes, hipStream_t stream);

// Greedy NMS core over candidates already in capacity layout.
//   keys   [S*cap] sort keys (desc_key(score, local idx)); lens [S]
//   boxes  candidate boxes; candidate i of segment s is at
//          boxes[(box_off ? box_off[s] : s*cap) + i]
//   keep   [S*max_out] local candidate indices, -1 padded; num_keep [S]
size_t nms_core_workspace_size(int S, int cap);
int nms_core(const uint64_t* keys, const int32_t* lens, const float4* boxes,
             const int32_t* box_off, int S, int cap, int max_out, float iou_thr, int32_t* keep,
             int32_t* num_keep, void* ws, size_t ws_bytes, hipStream_t stream);

// Mask + scan only, over candidates already sorted and gathered in capacity
// layout: sboxes[s*cap + i] (boxes used for IoU, e.g. class-offset boxes),
// sidx[s*cap + i] (the value written to keep for that candidate), count[s]
// selectable candidates.
size_t nms_sorted_workspace_size(int S, int cap);
int nms_sorted(const float4* sboxes, const int32_t* sidx, const int32_t* count, int S, int cap,
               int max_out, float iou_thr, int32_t* keep, int32_t* num_keep, void* ws,
               size_t ws_bytes, hipStream_t stream);

// Exact segmented top-k (value desc, index asc).  See d2mi_topk.
size_t topk_workspace_size(int S, int k);
int topk_core(const float* values, const int64_t* seg_start, const int32_t* seg_len, int S,
              int max_len, int k, int key_mode, float* vals_out, int32_t* idx_out,
              int32_t* count_out, void* ws, size_t ws_bytes, hipStream_t stream);
// seg_k (device, nullable): per-segment k limit (effective k = min(k, seg_k[s], len)).
// sampled_floor (key_mode 1 only): try the one-pass sampled-floor select first
// (topk.hip module comment); the output is the same top-k either way.
int topk_core_ex(const float* values, const int64_t* seg_start, const int32_t* seg_len,
                 const int32_t* seg_k, int S, int max_len, int k, int key_mode, float* vals_out,
                 int32_t* idx_out, int32_t* count_out, void* ws, size_t ws_bytes,
                 hipStream_t stream, bool sampled_floor = false);

// Process-wide kernel-selection knobs (d2mi_set_tuning; initial values from
// the environment): in-process A/B timing of kernel variants (tools/).
enum TuneKey { kTuneConvWS = 0, kTuneRoiFwd = 1, kTuneWgradWS = 2, kTuneConvEpi = 3,
               kTuneWgradWS1 = 4, kTuneWgradXCD = 5, kTuneConvXCD = 6, kTuneWgradInc = 7,
               kTuneConvWSMinK = 8, kTuneRoiPixGrid = 9, kTuneConvStream = 10,
               kTuneRoiBwdRec = 11, kTuneRetinaFused = 12, kTuneRpnMerge = 13, kTuneNmsScan = 14, kTuneRoiHeavy = 15,
               kTuneRpnCompact = 16, kTuneConvStreamNt = 17, kTuneConvNt = 18,
               kTuneConvTailMinK = 19, kTuneConvWSMinTiles = 20,
               kTuneSgdRev = 21, kTuneRetinaRank = 22, kTuneSoloMfma = 23,
               kTuneRetinaVar = 24,
               kTuneCount };
int tuning(TuneKey k);

// Byte fill by a kernel launch on st (never hipMemsetAsync: errors.hip).
// 0 on success.
int fill_bytes(void* p, size_t nbytes, uint8_t value, hipStream_t st);

}  // namespace d2mi
