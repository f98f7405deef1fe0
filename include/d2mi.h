/*
 * d2mi.h — C ABI of libd2mi_hip.so, the MI355X (gfx950) hot path of the
 * detection stack (ROIAlign, batched greedy NMS, anchor/top-k/decode, FPN convs).
 *
 * Every entry point replaces a TensorFlow kernel (or a Python glue function
 * around one) that SimeonZhang/detectron2_tensorflow calls; the replaced
 * reference interface is cited above each declaration as path:line into the
 * reference tree.
 *
 * Conventions (all functions):
 *   - return 0 on success, a negative value on a host-detected argument error
 *     (message in d2mi_last_error(), thread-local);
 *   - every pointer argument named *_dev / listed as "device" is a device
 *     pointer owned by the CALLER (PyTorch allocates inputs, outputs and
 *     workspace; the library never hipMallocs); host arrays are plain host
 *     memory read during the call only;
 *   - `stream` is a hipStream_t passed as void* (torch's current stream);
 *     nothing synchronises, so every call is graph-capturable;
 *   - layouts follow the reference: NHWC activations, HWIO conv weights,
 *     boxes [ymin, xmin, ymax, xmax] (yxyx) in absolute pixels, deltas
 *     (dy, dx, dh, dw) — lib/data/fields.py, lib/layers/convolutional.py:175,
 *     lib/modeling/box_regression.py:53-73.
 *   - run-time data errors the reference raises inside a TF kernel (e.g.
 *     box_ind out of range in CropAndResize) are recorded in a device error
 *     word; d2mi_error_word_dev() returns it so the host can check lazily
 *     without a synchronisation on every call.
 */
#ifndef D2MI_H
#define D2MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define D2MI_MAX_LEVELS 8

/* ------------------------------------------------------------------ misc */
int d2mi_version(void);
/* sha256 prefix of the sources the library was built from (the csrc .hip
 * and .h files and this header): the loader checks it against its tree. */
const char* d2mi_source_hash(void);
const char* d2mi_last_error(void);
/* Process-wide kernel-selection knobs for in-process A/B timing (tools/);
 * each starts from its environment variable (D2MI_<KEY in capitals>).  No
 * reference counterpart (a tuning hook of this implementation).  Keys:
 *   "conv_ws"      warp-specialised 256x128 split conv for the long-K convs:
 *                  0 off, else on (default 2);
 *   "roi_fwd"      ROIAlign forward variant bits (-1 = default);
 *   "wgrad_ws"     warp-specialised split weight gradient for KxK convs
 *                  (Cin % 256 == 0, Cout % 128 == 0): 0 off, 1 (default) on;
 *   "conv_epi"     split-K partials stored from the accumulators (1, default)
 *                  or through the LDS epilogue (0);
 *   "wgrad_ws1"    the WS weight gradient on 1x1 convs of >= N GFLOP (6);
 *   "wgrad_xcd" / "conv_xcd"  XCD-contiguous grid remaps (1 on);
 *   "wgrad_inc"    incremental pixel cursor in the WS weight gradient (1 on);
 *   "conv_ws_mink" fewest k-steps that go to the WS conv (16);
 *   "roi_pix_grid" ROIAlign backward pixel-pass grid (8192);
 *   "conv_stream"  streaming short-K 1x1 conv (r5) for stride-1 1x1 launches
 *                  of at least this many output pixels; 0 = off;
 *   "roi_bwd_rec"  ROIAlign backward pixel pass over run records (r5, 1) or
 *                  the r4 slot pass (0); 2 / 3 / 5 other pixel x record shapes;
 *   "retina_fused" RetinaNet post-processing in five launches (1), the same
 *                  with the exact select forced (2), the unfused pipeline (0);
 *   "rpn_merge"    RPN proposals' level merge by merge rank (1) or the one-
 *                  workgroup bitonic sort (0);
 *   "nms_scan"     fixed-point NMS tile resolve when T <= 64 tiles (1);
 *   "roi_heavy"    ROIAlign backward: pixels with >= N runs go first (16);
 *   "rpn_compact"  RPN decode compacts the valid boxes before NMS (1);
 *   "conv_stream_nt" streaming 1x1's output stores non-temporal (2);
 *   "conv_nt"      tiled conv final stores non-temporal (0);
 *   "conv_tail_mink" fewest k-steps whose tail tiles are split along K (8);
 *   "conv_ws_mintiles" fewest 256x128 tiles that go to the WS conv (0);
 *   "sgd_rev"      SGD update over its chunks in reverse order (0);
 *   "retina_rank"  RetinaNet merge rank inside the NMS workgroup (0);
 *   "solo_mfma"    SOLOv2 Matrix-NMS intersections on int8 MFMA: 2 (default)
 *                  = bits expanded by an LDS table, 1 = by arithmetic; 0 = the
 *                  AND + popcount tiles;
 *   "retina_var"   RetinaNet fused-path variants (bits; default 12018, 0 = the
 *                  r5 form): 16 = the wave slots compacted by many workgroups
 *                  before the finish, 64 = the finish's k-th select stopped at
 *                  the first bound leaving <= 1,024 keys, 128 = its bitonic
 *                  exchanges in DPP / permlane lane permutations, 512 = its
 *                  k-th select's reductions and scans the same way, 1024 = the
 *                  NMS's IoU only where the boxes intersect, 2048 = the NMS
 *                  tiles resolved as a ballot fixed point over column words,
 *                  4096 = no rank launch (the NMS ranks each 128-candidate
 *                  window; off by default), 8192 = the floor's ts-th maximum
 *                  by a workgroup radix select, 32 = the rank launch's search
 *                  rounds capped and looped, 2 = a small level's floor
 *                  samples spread over the level, 4 = floor and finish
 *                  launched twice (measurement only). */
int d2mi_set_tuning(const char* key, int value);
/* Current value of a d2mi_set_tuning key (INT32_MIN for an unknown key). */
int d2mi_get_tuning(const char* key);
/* Device int32 error word. Bits: 1 = box_ind out of range (CropAndResize),
 * 2 = NMS segment longer than its declared capacity, 4 = top-k capacity. */
int32_t* d2mi_error_word_dev(void);
int d2mi_clear_errors(void* stream);
/* Node census of a captured, not yet instantiated hipGraph (hipGraph_t as
 * void*): counts[t] = nodes of hipGraphNodeType t for t < ntypes (0 kernel,
 * 1 memcpy, 2 memset, ...).  No reference counterpart: the graphed training
 * step (engine/graphed.py, replacing the loop of lib/engine/trainer.py:173-199)
 * checks its captures with it. */
int d2mi_graph_census(void* graph, long long* counts, int ntypes);
/* The same census of the graph `stream` is capturing into now; returns 1
 * (counts 0) when the stream is not capturing.  A diagnosis (tools/). */
int d2mi_capture_census(void* stream, long long* counts, int ntypes);

/* -------------------------------------------------------------- ROIAlign
 * Multi-level ROIAlign / crop_and_resize, one launch for all levels.
 * Replaces:
 *   lib/layers/roi_align.py:45-66       ROIAlign.call (scale, SR crop, avg_pool)
 *   lib/layers/functional.py:100-166    crop_and_resize (SYMMETRIC pad + box transform
 *                                        + tf.image.crop_and_resize bilinear)
 *   lib/modeling/poolers.py:11-49       assign_boxes_to_levels (when num_levels > 1)
 *   lib/modeling/poolers.py:134-180     ROIPooler.call (gather/concat/invert_permutation:
 *                                        output is written directly in input order)
 * feats[l]      device NHWC float [N, H_l, W_l, C] (C equal over levels)
 * dims          host int32 [num_levels][3] = (N, H_l, W_l)
 * scales        host float [num_levels] spatial_scale per level (1/stride)
 * boxes         device float [R,4] yxyx, image pixels (before spatial_scale)
 * box_ind       device int32 [R] image index of each box
 * box_mode      0 = raw normalised boxes (tf.image.crop_and_resize),
 *               1 = aligned fpcoor (ROIAlignV2), 2 = unaligned fpcoor (ROIAlign)
 * assign        1: level per box by the FPN heuristic (min_level..max_level,
 *               canonical_box_size, canonical_level); 0: every box on level 0
 * level_out     device int32 [R] (nullable): assigned level index
 * out           device float [R, out_h, out_w, C]
 */
int d2mi_roi_align_fwd(const float* const* feats, const int32_t* dims, const float* scales,
                       int num_levels, int C, const float* boxes, const int32_t* box_ind,
                       int R, int out_h, int out_w, int sampling_ratio, int box_mode,
                       int pad_border, int assign, int min_level, int max_level,
                       int canonical_box_size, int canonical_level, int32_t* level_out,
                       float* out, void* stream);

/* Gradient of d2mi_roi_align_fwd w.r.t. the feature maps (TF
 * CropAndResizeGradImage + the pad/avg_pool chain rule; boxes get no gradient,
 * lib/layers/functional.py:120). Every element of every grad_feats[l] is
 * WRITTEN (not accumulated; no zero-fill needed): the scatter is computed as a
 * gather — contributions radix-sorted by destination pixel, one wave per pixel
 * summing them in the TF kernel's (box, y, x, corner) order (pixels with more
 * than 64 contributions are split into 64-long partial sums first).
 * Deterministic, no atomics. Workspace from d2mi_roi_align_bwd_workspace_size
 * (same dims / C / R / crop arguments). */
size_t d2mi_roi_align_bwd_workspace_size(const int32_t* dims, int num_levels, int C, int R,
                                         int out_h, int out_w, int sampling_ratio);
int d2mi_roi_align_bwd(float* const* grad_feats, const int32_t* dims, const float* scales,
                       int num_levels, int C, const float* boxes, const int32_t* box_ind,
                       int R, int out_h, int out_w, int sampling_ratio, int box_mode,
                       int pad_border, int assign, int min_level, int max_level,
                       int canonical_box_size, int canonical_level, const float* grad_out,
                       void* workspace, size_t workspace_bytes, void* stream);
/* d2mi_roi_align_bwd_ex with accumulate = 1: the maps already hold another
 * ROI set's gradient of the same features (the box pooler's, when the mask
 * pooler's backward runs second: lib/modeling/roi_heads/roi_heads.py:545-605
 * pool the same p2..p5 twice, and TF's AddN sums the two
 * CropAndResizeGradImage maps); touched pixels become old + new, untouched
 * ones are left unwritten (no clear, no separate add pass). */
int d2mi_roi_align_bwd_ex(float* const* grad_feats, const int32_t* dims, const float* scales,
                          int num_levels, int C, const float* boxes, const int32_t* box_ind,
                          int R, int out_h, int out_w, int sampling_ratio, int box_mode,
                          int pad_border, int assign, int min_level, int max_level,
                          int canonical_box_size, int canonical_level, const float* grad_out,
                          int accumulate, void* workspace, size_t workspace_bytes, void* stream);

/* One backward over TWO ROI sets pooled from the same maps -- the box (7x7)
 * and mask (14x14) poolers of a training step (roi_heads.py:497-605), whose
 * CropAndResizeGradImage maps TF sums (AddN): one emit per set, ONE sort on
 * (pixel, set) keys, one gather pass that sums each set's contributions in
 * its TF order and writes set0 + set1 (untouched pixels 0).  Every element
 * of grad_feats is written, except for the levels whose bit is set in
 * accumulate_mask: their maps already hold another gradient of the same
 * features (the RPN head's input gradient, rpn.py:83-96 reading the same
 * p2..p5) and get old + (set0 + set1) at touched pixels only (no clear, no
 * separate add).  Geometry / level parameters are shared; each set has its
 * ROIs, crop size, sampling ratio and grad_out. */
size_t d2mi_roi_align_bwd2_workspace_size(const int32_t* dims, int num_levels, int C, int R0,
                                          int out_h0, int out_w0, int sr0, int R1, int out_h1,
                                          int out_w1, int sr1);
int d2mi_roi_align_bwd2(float* const* grad_feats, const int32_t* dims, const float* scales,
                        int num_levels, int C, int box_mode, int pad_border, int assign,
                        int min_level, int max_level, int canonical_box_size, int canonical_level,
                        const float* boxes0, const int32_t* box_ind0, int R0, int out_h0,
                        int out_w0, int sr0, const float* grad_out0, const float* boxes1,
                        const int32_t* box_ind1, int R1, int out_h1, int out_w1, int sr1,
                        const float* grad_out1, int accumulate_mask, void* workspace,
                        size_t workspace_bytes, void* stream);
/* The same backward in phases (r4).  phase 1 (prepare): every step but the
 * pixel pass -- the counting sort of the contributions by (pixel, set) and
 * the long-run partials -- with the maps of levels [level_lo, level_hi] not
 * in accumulate_mask zeroed; its results stay in the workspace.  phase 2
 * (pixels): the pixel pass over the touched pixels of levels [level_lo,
 * level_hi] only, adding into the maps whose accumulate_mask bit is set
 * (others zeroed first).  phase 3 = d2mi_roi_align_bwd2.  Between a phase 1
 * and its phase-2 calls the workspace must not be reused; a level's map may
 * be null in a phase that does not touch it.  Lets a level's pixel pass run
 * after another backward wrote that map in full (the RPN head conv's dgrad
 * of the same FPN level): no clear of the map, no second pass over it. */
int d2mi_roi_align_bwd2_ex(float* const* grad_feats, const int32_t* dims, const float* scales,
                           int num_levels, int C, int box_mode, int pad_border, int assign,
                           int min_level, int max_level, int canonical_box_size,
                           int canonical_level, const float* boxes0, const int32_t* box_ind0,
                           int R0, int out_h0, int out_w0, int sr0, const float* grad_out0,
                           const float* boxes1, const int32_t* box_ind1, int R1, int out_h1,
                           int out_w1, int sr1, const float* grad_out1, int accumulate_mask,
                           int phase, int level_lo, int level_hi, void* workspace,
                           size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------- NMS
 * Segmented greedy NMS with TF NonMaxSuppressionV3 semantics
 * (score_threshold = -inf; IoU with min/max-normalised corners, 0 when an
 * area <= 0; suppress when IoU > iou_threshold; score desc, ties lowest index
 * first; stop at max_output_size).
 * Replaces tf.image.non_max_suppression at lib/layers/nms.py:23 (batch_nms),
 * lib/modeling/proposal_generator/rpn_outputs.py:90,
 * lib/modeling/roi_heads/fast_rcnn.py:145, single_stage_heads/retinanet.py:353.
 * boxes [total,4], scores [total] device; seg_offsets device int32 [num_segs+1];
 * seg_capacity = host upper bound of any segment length.
 * keep device int32 [num_segs, max_out] (segment-relative indices in selection
 * order, -1 padded); num_keep device int32 [num_segs].
 */
size_t d2mi_nms_workspace_size(int num_segs, int seg_capacity);
int d2mi_nms(const float* boxes, const float* scores, const int32_t* seg_offsets, int num_segs,
             int seg_capacity, int max_out, float iou_threshold, int32_t* keep,
             int32_t* num_keep, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------ top-k (segmented)
 * Exact segmented top-k with TF TopKV2 sorted=True order (value desc, ties
 * lowest index first).  key_mode 0: keys are the values; 1: keys are
 * sigmoid(values) (RetinaNet, retinanet.py:321-326); values_out receives the keys.
 * Segment s = values[seg_start[s] : seg_start[s] + seg_len[s]] (device int64
 * start, int32 len).  Replaces tf.nn.top_k at rpn_outputs.py:70/:106,
 * retinanet.py:326.  Output idx is segment-relative. */
size_t d2mi_topk_workspace_size(int num_segs, int k_max);
int d2mi_topk(const float* values, const int64_t* seg_start, const int32_t* seg_len,
              int num_segs, int max_seg_len, int k, int key_mode, float* values_out,
              int32_t* idx_out, int32_t* count_out, void* workspace, size_t workspace_bytes,
              void* stream);

/* ---------------------------------------------------------- subsampling
 * subsample_labels (lib/modeling/sampling.py, called at rpn_outputs.py:278-283
 * and roi_heads.py:160-216) over labels [N, P] int64: pos_out / neg_out [N, P]
 * (uint8) mark a uniformly random min(num_pos, #positive) of the positives
 * (label not -1 and not bg_label) and min(num_samples - that, #negative) of
 * the negatives (label == bg_label).  The draw: each element's rank among its
 * kind through a keyed pseudo-random bijection of [0, n), kept iff < k (the
 * reference shuffles and takes the first k: the same distribution, another
 * stream); seed [1] int64 on the device.  order_out [N, S] (nullable, with
 * order_valid [N, S] uint8): the selected indices positives first, each kind
 * in index order, then 0 / invalid -- the ROI heads' fg-first batch. */
size_t d2mi_subsample_workspace_size(int N, int P);
int d2mi_subsample(const int64_t* labels, int N, int P, long long bg_label, int num_samples,
                   int num_pos, const int64_t* seed, uint8_t* pos_out, uint8_t* neg_out,
                   int64_t* order_out, uint8_t* order_valid, int S, void* workspace,
                   size_t workspace_bytes, void* stream);

/* -------------------------------------------------------- anchors/deltas
 * DefaultAnchorGenerator.grid_anchors for one level (anchor_generator.py:92-109):
 * out[(h*W + w)*A + a] = cell[a] + (h*stride, w*stride, h*stride, w*stride). */
int d2mi_grid_anchors(int H, int W, float stride, const float* cell_anchors_host, int A,
                      float* out, void* stream);

/* Box2BoxTransform.apply_deltas (box_regression.py:76-123):
 * deltas [N, K*4] (dy,dx,dh,dw), boxes [N,4] -> out [N, K*4]. */
int d2mi_apply_deltas(const float* deltas, const float* boxes, int N, int K,
                      const float* weights4_host, float scale_clamp, float* out, void* stream);

/* ------------------------------------------------------ RPN proposals
 * Fused find_top_rpn_proposals (rpn_outputs.py:29-132) +
 * predict_proposals (:403-426) + anchors (anchor_generator.py:92-109):
 * per (image, level) exact top-k of the objectness logits, decode ONLY the
 * selected anchors (anchors regenerated from the index), clip to the image,
 * prune small boxes, per-level NMS, then per-image top-k(post) and zero pad.
 * logits[l]  device float [N, H_l, W_l, A]; deltas[l] device [N, H_l, W_l, A*4]
 * level_hw   host int32 [L][2]; strides host float [L]; cell_anchors host [L][A][4]
 * image_hw   device int32 [N,2] (true image height, width)
 * out_boxes  device [N, post, 4]; out_scores [N, post]; out_valid uint8 [N, post]
 */
size_t d2mi_rpn_proposals_workspace_size(int N, int L, const int32_t* level_hw, int A,
                                         int pre_nms_topk, int post_nms_topk);
int d2mi_rpn_proposals(const float* const* logits, const float* const* deltas,
                       const int32_t* level_hw, const float* strides,
                       const float* cell_anchors, int L, int A, int N, const int32_t* image_hw,
                       int pre_nms_topk, int post_nms_topk, float nms_thresh,
                       float min_box_side_len, const float* weights4_host, float scale_clamp,
                       float* out_boxes, float* out_scores, uint8_t* out_valid,
                       void* workspace, size_t workspace_bytes, void* stream);
/* d2mi_rpn_proposals over strided levels: level l of image n starts
 * logits_image_stride[l] elements (deltas: deltas_image_stride[l], a multiple
 * of 4) after image n - 1's, i.e. per-level views of ONE concatenated
 * [N, sum_l H_l W_l A] (x4) buffer -- the training path's RPN head output
 * (d2mi_rpn_head_gather), with no per-level copies.  Null strides: dense. */
int d2mi_rpn_proposals_ex(const float* const* logits, const float* const* deltas,
                          const int64_t* logits_image_stride, const int64_t* deltas_image_stride,
                          const int32_t* level_hw, const float* strides,
                          const float* cell_anchors, int L, int A, int N, const int32_t* image_hw,
                          int pre_nms_topk, int post_nms_topk, float nms_thresh,
                          float min_box_side_len, const float* weights4_host, float scale_clamp,
                          float* out_boxes, float* out_scores, uint8_t* out_valid,
                          void* workspace, size_t workspace_bytes, void* stream);
/* RPN head outputs of a training step in the RPNOutputs layout
 * (rpn_outputs.py:346-357: per-image level-major concatenation): ys[l]
 * device [N, HW_l, C] (the fused objectness / anchor-delta 1x1 output,
 * C >= 5A channels: A logits then 4A deltas, the rest padding) ->
 * logits [N, T*A], deltas [N, T*A, 4], T = sum_l HW_l.  One launch instead
 * of a slice copy per level and head and two concatenations. */
int d2mi_rpn_head_gather(const float* const* ys, const int32_t* level_hw_flat, int L, int N,
                         int A, int C, float* logits, float* deltas, void* stream);
/* Its adjoint: g_logits [N, T*A], g_deltas [N, T*A, 4] (either nullable =
 * zero) -> gys[l] [N, HW_l, C], every element written (padding channels 0). */
int d2mi_rpn_head_scatter(const float* g_logits, const float* g_deltas,
                          const int32_t* level_hw_flat, int L, int N, int A, int C,
                          float* const* gys, void* stream);

/* --------------------------------------------------- Fast R-CNN inference
 * FastRCNNOutputs.predict_boxes/predict_probs + fast_rcnn_inference
 * (fast_rcnn.py:28-187, :359-379): softmax, class-specific decode, clip to the
 * true image shape, score > thresh in class-major order, class-offset NMS
 * (offset = cls * (max clipped coord of the image + 1)), top-k, pad.
 * logits [R, K+1] (background last), deltas [R, K*4] (or [R,4] when
 * bit 0 of cls_agnostic is set), proposals [R,4]; bit 1 of cls_agnostic =
 * NMS_CLS_AGNOSTIC (fast_rcnn.py:138-139: plain NMS, no class offsets); roi_img/roi_slot int32 [R] = (image, dense
 * slot) of each ROI (SparseBoxList.indices); P = dense slots per image.
 * Outputs [N, max_det] boxes/scores/classes(int64)/valid(uint8) and
 * out_roi int32 [N, max_det] (kept ROI row, -1 pad).
 */
size_t d2mi_fast_rcnn_workspace_size(int N, int P, int K, float score_thresh, int max_det);
int d2mi_fast_rcnn_inference(const float* logits, const float* deltas, const float* proposals,
                             const int32_t* roi_img, const int32_t* roi_slot, int R, int N, int P,
                             int K, int cls_agnostic, const int32_t* image_hw,
                             const float* weights4_host, float scale_clamp, float score_thresh,
                             float nms_thresh, int max_det, float* out_boxes, float* out_scores,
                             int64_t* out_classes, uint8_t* out_valid, int32_t* out_roi,
                             void* workspace, size_t workspace_bytes, void* stream);

/* --------------------------------------------------- RetinaNet inference
 * RetinaNetHead.inference (retinanet.py:285-387): per level sigmoid,
 * top_k(min(topk_candidates, H*W*A*K)), score > thresh, decode the chosen
 * anchors (no clipping), concat levels, class-offset NMS, pad to max_det.
 * cls[l] device [N, H_l, W_l, A*K]; box[l] device [N, H_l, W_l, A*4].
 */
size_t d2mi_retinanet_workspace_size(int N, int L, const int32_t* level_hw, int A, int K,
                                     int topk_candidates);
int d2mi_retinanet_inference(const float* const* cls, const float* const* box,
                             const int32_t* level_hw, const float* strides,
                             const float* cell_anchors, int L, int A, int K, int N,
                             int topk_candidates, float score_thresh, float nms_thresh,
                             int max_det, const float* weights4_host, float scale_clamp,
                             float* out_boxes, float* out_scores, int32_t* out_classes,
                             uint8_t* out_valid, void* workspace, size_t workspace_bytes,
                             void* stream);

/* ------------------------------------------------------------ Matrix NMS
 * lib/layers/nms.py:29-83 (SOLOv2 Matrix-NMS).  masks [M, HW] float,
 * classes int64 [M], scores [M], sum_masks [M] (nullable: computed);
 * kernel 0 = gaussian, 1 = linear.  out_scores [M]. */
size_t d2mi_matrix_nms_workspace_size(int M);
int d2mi_matrix_nms(const float* masks, const int64_t* classes, const float* scores,
                    const float* sum_masks, int M, int HW, int kernel, float sigma,
                    float* out_scores, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------- ResizeBilinear
 * tf.compat.v2.image.resize(method="bilinear") as the reference's
 * resize_images calls it (lib/layers/functional.py:9-36; TF >= 1.14 takes the
 * v2 branch, which drops align_corners: half-pixel centres, no antialias),
 * TF 1.15 resize_bilinear_op.cc arithmetic.  x [N,H,W,C] -> y [N,OH,OW,C]. */
int d2mi_resize_bilinear(const float* x, int N, int H, int W, int C, int OH, int OW,
                         int align_corners, int half_pixel_centers, float* y, void* stream);

/* ------------------------------------------------- SOLOv2 inference tail
 * MaskKernelBranch.inference (lib/modeling/single_stage_heads/solo_v2.py:476-627)
 * in four stages around the caller's dynamic-conv GEMM and d2mi_matrix_nms.
 *
 * d2mi_solo_cells: cate[l] device float [N, S_l, S_l, K] category logits
 * (grids host int32 [L] = S_l, T = sum S_l^2 cells) -> probs [N, T, K] =
 * point_nms(sigmoid(cate)) (solo_v2.py:29-40, :267-269) in the reference's
 * flattened order (:567-586); live_cells [N, T]: the cells with any prob >
 * score_thr in cell order, first live_count[n] valid; live_row [N, T]: a live
 * cell's position in live_cells, -1 otherwise.  cate is a host array of L
 * device pointers. */
int d2mi_solo_cells(const float* const* cate, const int32_t* grids, int L, int N, int K,
                    float score_thr, float* probs, int32_t* live_cells, int32_t* live_row,
                    int32_t* live_count, void* stream);

/* d2mi_solo_mask_stats: logits [R, P] (one dynamic-conv row per live cell,
 * :509-511) -> sum_masks[r] = #(sigmoid > mask_thr) (:513-517) and
 * sum_scores[r] = sum of those sigmoids (:529-531).  16-B aligned. */
int d2mi_solo_mask_stats(const float* logits, int R, int P, float mask_thr, float* sum_masks,
                         float* sum_scores, void* stream);

/* d2mi_solo_select: candidates (cell, class) with prob > score_thr and
 * sum_masks > stride of the cell's level (:482-526), scored prob *
 * sum_scores / sum_masks (:528-532); exact top-k (k = TOPK_CANDIDATES_TEST,
 * tf.nn.top_k sorted, ties by candidate order, :535-539); the top-k's binary
 * masks bit-packed, mask_bits [N, k, ceil(P/64)] uint64 (bit p % 64 of word
 * p / 64), classes [N, k] int64 (rows past top_count: zero masks, classes
 * -1 - t), sum_masks [N, k], scores [N, k] (:537-539).  row_off [N] device:
 * first logits row of each image; grids / strides host [L]. */
size_t d2mi_solo_select_workspace_size(int N, int T, int K, int k);
int d2mi_solo_select(const float* probs, const int32_t* live_row, const int32_t* row_off,
                     const float* logits, const float* sum_masks, const float* sum_scores,
                     const int32_t* grids, const float* strides, int L, int N, int K, int P,
                     float score_thr, float mask_thr, int k, float* top_scores,
                     int64_t* top_classes, float* top_sum_masks, int32_t* top_count,
                     uint64_t* mask_bits, void* workspace, size_t workspace_bytes, void* stream);

/* d2mi_solo_matrix_nms: matrix_nms (lib/layers/nms.py:29-83, called at
 * solo_v2.py:541-545) for N images of k binary masks at once: the
 * intersection matrix M M^T as popcounts of AND-ed mask words (exact), then
 * the IoU / class / compensation / decay arithmetic of d2mi_matrix_nms.
 * kernel 0 = gaussian, 1 = linear.  out_scores [N, k]. */
size_t d2mi_solo_matrix_nms_workspace_size(int N, int k);
int d2mi_solo_matrix_nms(const uint64_t* mask_bits, const int64_t* classes, const float* scores,
                         const float* sum_masks, int N, int k, int P, int kernel, float sigma,
                         float* out_scores, void* workspace, size_t workspace_bytes,
                         void* stream);

/* d2mi_solo_finalize: decayed Matrix-NMS scores [N, k] > update_thr in
 * candidate order, pad / clip to max_det (:547-557); the bit-packed masks
 * resized from [Hm, Wm] to the padded image [OH, OW] with TF bilinear
 * (half-pixel) and > mask_thr (:598-602) -> out_masks uint8
 * [N, max_det, OH, OW] (the reference's float 0/1 values); out_boxes
 * [N, max_det, 4] from the masks (:604-623); out_scores, out_classes int64,
 * out_valid uint8 [N, max_det]. */
size_t d2mi_solo_finalize_workspace_size(int N, int max_det, int OH);
int d2mi_solo_finalize(const float* nms_scores, const int64_t* top_classes,
                       const int32_t* top_count, const uint64_t* mask_bits, int N, int k, int Hm,
                       int Wm, float update_thr, int max_det, float mask_thr, int OH, int OW,
                       uint8_t* out_masks, float* out_boxes, float* out_scores,
                       int64_t* out_classes, uint8_t* out_valid, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------- GroupNorm
 * GroupNorm.call (lib/layers/normalization.py:235-260) on NHWC x [N,H,W,C]:
 * tf.nn.moments over (H, W, C/G) (two-pass mean / variance), then
 * y = x * inv + (beta - mean * inv), inv = rsqrt(var + eps) * gamma;
 * relu: max(y, 0) (the conv's activation after its normalizer,
 * convolutional.py:251-262); up2: y written to the 2x2 block of the nearest
 * x2 upsample (out [N,2H,2W,C], wrappers.py:104-116); accumulate: y added to
 * the output (the SOLOv2 scale-head sum, solo_v2.py:705-721).  C / G % 4 == 0,
 * C <= 1024, G <= 64, 16-B aligned; workspace from
 * d2mi_group_norm_workspace_size. */
size_t d2mi_group_norm_workspace_size(int N, int H, int W, int C, int G);
int d2mi_group_norm_nhwc(const float* x, int N, int H, int W, int C, int G, const float* gamma,
                         const float* beta, float eps, int relu, int up2, int accumulate,
                         float* y, void* workspace, size_t workspace_bytes, void* stream);
/* The same GroupNorm (+ relu) applied to up to 6 feature levels sharing the
 * layer — the SOLOv2 towers' per-level GroupNorm calls (solo_v2.py:173-183,
 * one layer per level) — in five launches for all levels.  xs[l] / ys[l]
 * [dims[3l], dims[3l+1], dims[3l+2], C]; per level identical arithmetic to
 * d2mi_group_norm_nhwc; workspace from d2mi_group_norm_levels_workspace_size. */
size_t d2mi_group_norm_levels_workspace_size(const int32_t* dims, int nlev, int C, int G);
int d2mi_group_norm_nhwc_levels(const float* const* xs, const int32_t* dims, int nlev, int C,
                                int G, const float* gamma, const float* beta, float eps, int relu,
                                float* const* ys, void* workspace, size_t workspace_bytes,
                                void* stream);

/* --------------------------------------------------------------- conv2d
 * NHWC implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32),
 * lib/layers/convolutional.py:12-23 (fix_padding: symmetric pad) and
 * :198-263 (Conv2D.call: conv + bias + activation), with the FPN top-down
 * merge fused into the epilogue (lib/modeling/necks/fpn.py:138-149):
 *   y = act(conv(x, w) + bias) + (topdown ? up2_nearest(topdown) : 0)
 *        [+ residual]
 * x [N,H,W,Cin]; w_packed [KH,KW,Cout,Cin] (d2mi_conv_pack_weights of the
 * reference's HWIO [KH,KW,Cin,Cout] variable); bias [Cout] (nullable);
 * topdown [N, ceil(OH/2), ceil(OW/2), Cout] (nullable);
 * residual [N,OH,OW,Cout] (nullable); y [N,OH,OW,Cout].
 * act: 0 none, 1 relu.  pad_beg/pad_end: explicit spatial padding
 * (fix_padding gives pad_beg = (k-1)//2, pad_end = k-1-pad_beg).
 */
int d2mi_conv_pack_weights(const float* w_hwio, int KH, int KW, int Cin, int Cout,
                           float* w_packed, void* stream);

/* d2mi_conv_pack_weights_many: n weight tensors (w_hwio[i], dims[4i..4i+3] =
 * KH, KW, Cin, Cout) packed as d2mi_conv_pack_weights does, the Cin % 64 == 0
 * ones by one launch per 32 tensors (the per-step repack of every
 * un-normalised conv after the optimizer update: FPN, RPN, ROI heads,
 * convolutional.py:198-263's weights).  Host arrays of device pointers. */
int d2mi_conv_pack_weights_many(int n, const float* const* w_hwio, const int32_t* dims,
                                float* const* w_packed, void* stream);
int d2mi_conv2d_nhwc(const float* x, const float* w_packed, const float* bias,
                     const float* topdown, const float* residual, float* y, int N, int H, int W,
                     int Cin, int Cout, int KH, int KW, int stride, int pad_beg, int pad_end,
                     int act, void* stream);
/* Extended form: flags bit0 = ReLU, bit1 = apply the ReLU after the
 * residual / top-down add (ResNet bottleneck: relu(conv3 + bias + shortcut),
 * lib/modeling/backbone/blocks.py:143-186).  With a workspace of
 * d2mi_conv2d_workspace_size() bytes, small-M shapes split K over several
 * workgroups and reduce in a fixed order (deterministic). */
size_t d2mi_conv2d_workspace_size(int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                  int stride, int pad_beg, int pad_end);
int d2mi_conv2d_nhwc_ex(const float* x, const float* w_packed, const float* bias,
                        const float* topdown, const float* residual, float* y, int N, int H,
                        int W, int Cin, int Cout, int KH, int KW, int stride, int pad_beg,
                        int pad_end, int flags, void* workspace, size_t workspace_bytes,
                        void* stream);
/* Gated form, for an input gradient (dgrad) of a ReLU output x that feeds
 * two consumers -- the next bottleneck's conv1 and its identity shortcut
 * (lib/modeling/backbone/blocks.py:143-186): writes
 *   y = gate > 0 ? conv(x, w) + bias + residual : 0
 * i.e. the conv's input gradient plus the shortcut's gradient (residual),
 * passed through the producer's ReLU backward (gate = its output), in one
 * pass.  residual / bias nullable; flags: bit2 split products, bit3 flipped
 * taps only. */
int d2mi_conv2d_nhwc_gated(const float* x, const float* w_packed, const float* bias,
                           const float* residual, const float* gate, float* y, int N, int H,
                           int W, int Cin, int Cout, int KH, int KW, int stride, int pad_beg,
                           int pad_end, int flags, void* workspace, size_t workspace_bytes,
                           void* stream);
/* Multi-level form: the same conv (shared weights) over nlev <= 6 feature
 * levels in ONE launch -- the heads the reference applies per FPN level with
 * shared variables: RetinaNet towers / predictors (retinanet.py:110-145),
 * SOLOv2 kernel / category towers (solo_v2.py:173-272).  xs[l]
 * [N_l,H_l,W_l,Cin]; dims = {N_l, H_l, W_l} per level; ys[l]
 * [N_l,OH_l,OW_l,Cout]; flags bit0 ReLU, bit2 split products.  Every level's
 * tiles share one grid: the small levels run beside the big one instead of
 * after it; when all levels together are under a round of workgroups, K is
 * split over the levels' concatenated rows (workspace of
 * d2mi_conv2d_levels_workspace_size bytes; fixed-order reduce). */
size_t d2mi_conv2d_levels_workspace_size(const int32_t* dims, int nlev, int Cin, int Cout,
                                         int KH, int KW, int stride, int pad_beg, int pad_end);
int d2mi_conv2d_nhwc_levels(const float* const* xs, const int32_t* dims, int nlev,
                            const float* w_packed, const float* bias, float* const* ys, int Cin,
                            int Cout, int KH, int KW, int stride, int pad_beg, int pad_end,
                            int flags, void* workspace, size_t workspace_bytes, void* stream);
/* flags bit2 = "split" products: the same f32 operands, each split EXACTLY
 * into three bf16 terms (x = h + m + l, truncation), multiplied with six
 * bf16 MFMA products (v_mfma_f32_32x32x16_bf16; the dropped m*l, l*m, l*l
 * terms are below f32's own rounding of the product) and accumulated in f32.
 *
 * d2mi_split_bf16x3: x [n] f32 -> out [3][n] (bf16 bit patterns of h, m, l);
 * n % 4 == 0 (the stem conv's weight planes, d2mi_stem_conv). */
int d2mi_split_bf16x3(const float* x, int64_t n, uint16_t* out, void* stream);

/* Weight gradient of the same convolution (the tf.gradients of Conv2D.call,
 * lib/layers/convolutional.py:198-263, w.r.t. its HWIO kernel):
 *   dw[kh][kw][ci][co] = sum_{n,oy,ox} x[n, oy*s-pb+kh, ox*s-pb+kw, ci] * dy[n,oy,ox,co].
 * x [N,H,W,Cin], dy [N,OH,OW,Cout] (OH/OW as the forward), dw HWIO, written;
 * dbias [Cout] (nullable) receives sum_p dy[p][co], the bias gradient.
 * Cin, Cout multiples of 4.  With d2mi_conv2d_wgrad_workspace_size() bytes the
 * pixel reduction is split over workgroups and summed in a fixed order. */
size_t d2mi_conv2d_wgrad_workspace_size(int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                        int stride, int pad_beg, int pad_end);
int d2mi_conv2d_wgrad(const float* x, const float* dy, float* dw_hwio, float* dbias, int N,
                      int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad_beg,
                      int pad_end, void* workspace, size_t workspace_bytes, void* stream);
/* flags bit2: the split-bf16 products of d2mi_conv2d_nhwc_ex (exact 3-term
 * split of x and dy, six bf16 MFMA products, f32 accumulation).  bit3:
 * accumulate -- dw_hwio (and dbias) += this call's gradient, in the reduce
 * pass (a weight shared by several calls, e.g. one head over the FPN levels);
 * the workspace must then hold the plan's slabs even for one split
 * (d2mi_conv2d_wgrad_workspace_size, or one slab when that returns 0). */
int d2mi_conv2d_wgrad_ex(const float* x, const float* dy, float* dw_hwio, float* dbias, int N,
                         int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad_beg, int pad_end, int flags, void* workspace,
                         size_t workspace_bytes, void* stream);

/* ------------------------------------------------------- FrozenBN fold
 * A frozen BatchNorm (moving statistics; lib/layers/normalization.py:15-119
 * with training=False, gamma/beta trainable above FREEZE_AT per
 * lib/modeling/backbone/resnet.py:22-46) folded into the preceding Conv2D:
 *   scale = gamma / sqrt(var + eps);  w_eff = w * scale;
 *   b_eff = bias * scale + beta - mean * scale.
 * w HWIO [KH,KW,Cin,Cout]; bias / gamma / beta nullable.  Writes w_eff (HWIO,
 * nullable), w_packed ([KH,KW,Cout,Cin] for d2mi_conv2d_nhwc, nullable) and
 * b_eff [Cout]. */
int d2mi_fold_frozen_bn(const float* w_hwio, const float* bias, const float* gamma,
                        const float* beta, const float* mean, const float* var, float eps,
                        int KH, int KW, int Cin, int Cout, float* w_eff, float* w_packed,
                        float* b_eff, void* stream);
/* Backward: from gw_eff (HWIO) and gb_eff ([Cout], nullable) writes gw, gbias,
 * ggamma, gbeta (each nullable); per-channel reductions in a fixed order. */
size_t d2mi_fold_frozen_bn_bwd_workspace_size(int Cout);
int d2mi_fold_frozen_bn_bwd(const float* gw_eff, const float* gb_eff, const float* w_hwio,
                            const float* bias, const float* gamma, const float* mean,
                            const float* var, float eps, int KH, int KW, int Cin, int Cout,
                            float* gw, float* gbias, float* ggamma, float* gbeta,
                            void* workspace, size_t workspace_bytes, void* stream);
/* Batched fold: every BN-conv of a network in one forward launch and one
 * backward pair (same arithmetic and summation order as the per-conv calls
 * above, so bit-identical results).  Replaces the per-layer
 * Conv2D -> BatchNorm(training=False) pairs of lib/modeling/backbone/resnet.py
 * (resnet_arg_scope, :22-46) for one training step.  table: DEVICE array of
 * entries sorted by fwd_begin / bwd_begin / co_begin (each ascending):
 *   fwd_begin  first forward workgroup: ceil(Cout/64)*ceil(Cin/64)*taps each;
 *   bwd_begin  first backward workgroup: ceil(Cout/64)*row_chunks each;
 *   co_begin   prefix sum of Cout;  partial_offset  floats into the backward
 *   workspace (row_chunks*Cout each).
 * Forward reads w/bias/gamma/beta/mean/var and writes w_eff/w_packed/b_eff
 * (w_eff, w_packed nullable); backward reads gw_eff/gb_eff (nullable = zero)
 * and writes gw/gbias/ggamma/gbeta (each nullable).  d2mi_fold_many_sizes
 * reports sizeof(entry) and the row-chunk count so a host can check its
 * layout. */
typedef struct d2mi_fold_entry {
  const float* w;
  const float* bias;
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* var;
  float* w_eff;
  float* w_packed;
  float* b_eff;
  const float* gw_eff;
  const float* gb_eff;
  float* gw;
  float* gbias;
  float* ggamma;
  float* gbeta;
  float eps;
  int taps, Cin, Cout;
  int fwd_begin, bwd_begin, co_begin, pad;
  long long partial_offset;
} d2mi_fold_entry;
int d2mi_fold_many_sizes(int* entry_bytes, int* row_chunks);
int d2mi_fold_frozen_bn_many(const d2mi_fold_entry* table, int num_entries, int fwd_blocks,
                             void* stream);
int d2mi_fold_frozen_bn_bwd_many(const d2mi_fold_entry* table, int num_entries, int bwd_blocks,
                                 int total_cout, float* workspace, void* stream);

/* ------------------------------------------------------- mask pasting
 * Replaces detector_postprocess (lib/modeling/postprocessing.py:9-59) for the
 * "conventional" / "fixed" SEGMENTATION_OUTPUT formats, i.e.
 * reframe_box_masks_to_image_masks (lib/structures/mask_ops.py:7-56):
 * normalise each box by the canvas (out_h, out_w), take the reverse box of the
 * unit square, tf.image.crop_and_resize the box mask onto the canvas
 * (bilinear, extrapolation 0) and threshold with tf.greater -> uint8.  Same
 * float32 sequence as the TF CPU kernels; the f32 canvas is never stored.
 * box_masks [D, mask_h, mask_w] f32 (probabilities); boxes [D, 4] f32 yxyx
 * absolute; yx_scale [D, 2] f32 (nullable): per-box (sy, sx) applied first
 * ("fixed": output_shape / image_shape, box_list_ops.scale); valid [D] u8
 * (nullable): rows with 0 are written as zeros (SparseBoxList.to_dense);
 * out [D, out_h, out_w] u8, 4-byte aligned. */
int d2mi_paste_masks(const float* box_masks, const float* boxes, const float* yx_scale,
                     const uint8_t* valid, int D, int mask_h, int mask_w, int out_h, int out_w,
                     float threshold, uint8_t* out, void* stream);

/* ------------------------------------------------ skinny 1x1 weight gradient
 * gw[Cin][Cout] = X^T G and gb[Cout] = column sums of G over P pixels, for
 * Cout <= 16 (the RPN head's objectness + anchor-delta 1x1 convs, fused:
 * lib/modeling/proposal_generator/rpn.py:83-96, whose TF gradient is
 * Conv2DBackpropFilter + BiasAddGrad).  x [P, Cin], g [P, Cout] f32
 * contiguous; gb nullable.  Fixed-order reduction (deterministic); workspace
 * from d2mi_wgrad_skinny_workspace_size. */
size_t d2mi_wgrad_skinny_workspace_size(int P, int Cin, int Cout);
int d2mi_wgrad_skinny(const float* x, const float* g, int P, int Cin, int Cout, float* gw,
                      float* gb, void* workspace, size_t workspace_bytes, void* stream);
/* d2mi_wgrad_skinny_ex: accumulate != 0 adds the result into gw / gb (old +
 * new: autograd's accumulation of a weight shared by several calls -- the RPN
 * head's fused 1x1 over the FPN levels, rpn.py:83-96). */
int d2mi_wgrad_skinny_ex(const float* x, const float* g, int P, int Cin, int Cout, float* gw,
                         float* gb, int accumulate, void* workspace, size_t workspace_bytes,
                         void* stream);
/* d2mi_wgrad_skinny_levels: the skinny wgrad of L <= 8 calls sharing one
 * weight (the RPN head's fused 1x1 over the FPN levels, rpn.py:31-96: one
 * weight applied per level, its gradient the sum over levels) in one partial
 * launch and one reduce: x[l] [P[l], Cin] (16-B aligned, Cin % 4 == 0),
 * g[l] [P[l], Cout]; each level summed exactly as one d2mi_wgrad_skinny call
 * and the levels added in array order (accumulate != 0: after the old gw /
 * gb) -- bit-identical to the per-level calls with accumulate after the
 * first.  workspace >= d2mi_wgrad_skinny_levels_workspace_size. */
size_t d2mi_wgrad_skinny_levels_workspace_size(const int* P, int L, int Cin, int Cout);
int d2mi_wgrad_skinny_levels(const float* const* x, const float* const* g, const int* P, int L,
                             int Cin, int Cout, float* gw, float* gb, int accumulate,
                             void* workspace, size_t workspace_bytes, void* stream);
/* Column sums of a row-major [rows, cols] f32 matrix (a conv's bias gradient,
 * TF BiasAddGrad, when its weight gradient runs as a library GEMM): out[cols],
 * fixed-order two-level reduction; workspace from
 * d2mi_column_sum_workspace_size. */
size_t d2mi_column_sum_workspace_size(long long rows, int cols);
int d2mi_column_sum(const float* x, long long rows, int cols, float* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/* ------------------------------------------------ IoU + Matcher
 * box_list_ops.pairwise_iou (:295-372) of gt_boxes [N,G,4] against boxes
 * ([P,4] shared by every image, or [N,P,4] with boxes_per_image = 1; yxyx
 * f32, 16-B aligned) fused with Matcher.__call__ (lib/modeling/matcher.py:
 * 8-173): matches [N,P] int64 = the first GT of maximal IoU among the
 * matchable GT (gt_flags bit0), labels [N,P] int64 from the n_intervals
 * intervals [thresholds[i], thresholds[i+1]) -> labels_of[i], low-quality
 * matches (IoU equal to that GT's best over all boxes -> 1) when
 * allow_low_quality, no matchable GT -> 0 / match 0, then -1 for background
 * boxes whose max IoU with a crowd GT (bit1) exceeds crowd_thr or with a
 * difficult GT (bit2) exceeds difficult_thr.  G <= 256; the workspace
 * (d2mi_match_workspace_size) holds the per-GT best IoU. */
size_t d2mi_match_workspace_size(int N, int G);
int d2mi_match_boxes(const float* gt_boxes, const int* gt_flags, const float* boxes,
                     int boxes_per_image, int N, int G, int P, const float* thresholds,
                     const int* labels_of, int n_intervals, int allow_low_quality,
                     float crowd_thr, float difficult_thr, long long* matches, long long* labels,
                     void* workspace, size_t workspace_bytes, void* stream);
/* d2mi_match_boxes with the GT flags as byte masks [N, G] (bool tensors as
 * they are: valid required, crowd / difficult nullable) instead of the
 * packed int32 word -- no packing passes on the host side.  The matchable GT
 * are valid && !crowd && !difficult (the reference's valid_gt_boxlist). */
int d2mi_match_boxes_ex(const float* gt_boxes, const uint8_t* valid, const uint8_t* crowd,
                        const uint8_t* difficult, const float* boxes, int boxes_per_image, int N,
                        int G, int P, const float* thresholds, const int* labels_of,
                        int n_intervals, int allow_low_quality, float crowd_thr,
                        float difficult_thr, long long* matches, long long* labels,
                        void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------ RPN losses
 * RPNOutputs.losses (rpn_outputs.py:306-401) after matching and sampling:
 * logits [N,P], deltas [N,P,4], anchors [P,4], gt_boxes [N,G,4] (yxyx),
 * matches [N,P] int64, pos / sampled [N,P] bool (uint8).  Forward writes
 * partial [N][d2mi_rpn_loss_blocks()] float2 = (sigmoid CE over sampled,
 * smooth-L1(beta) over positives of the get_deltas targets with weights[4]),
 * summed by the caller in a fixed order.  Backward: grads = device float[2]
 * (d loss_cls_sum, d loss_loc_sum) -> d_logits [N,P], d_deltas [N,P,4]. */
int d2mi_rpn_loss_blocks(void);
int d2mi_rpn_loss_fwd(const float* logits, const float* deltas, const float* anchors,
                      const float* gt_boxes, const long long* matches, const unsigned char* pos,
                      const unsigned char* sampled, int N, int P, int G, const float* weights,
                      float beta, float* partial, void* stream);
int d2mi_rpn_loss_bwd(const float* logits, const float* deltas, const float* anchors,
                      const float* gt_boxes, const long long* matches, const unsigned char* pos,
                      const unsigned char* sampled, int N, int P, int G, const float* weights,
                      float beta, const float* grads, float* d_logits, float* d_deltas,
                      void* stream);
/* d2mi_rpn_loss_bwd with the two upstream gradients as separate device
 * scalars (null: zero) and the loss normaliser folded in: the gradients used
 * are g * scale (the losses' `* normalizer * loss_weight`, rpn_outputs.py:
 * 331-342, without its multiply launches or a gradient pack). */
int d2mi_rpn_loss_bwd_ex(const float* logits, const float* deltas, const float* anchors,
                         const float* gt_boxes, const long long* matches,
                         const unsigned char* pos, const unsigned char* sampled, int N, int P,
                         int G, const float* weights, float beta, const float* g_cls,
                         const float* g_loc, float scale, float* d_logits, float* d_deltas,
                         void* stream);

/* ----------------------------------------------------- ROI-head losses
 * FastRCNNOutputs.losses (lib/modeling/roi_heads/fast_rcnn.py:269-357) on
 * dense sampled rows: logits [B, K1 = K+1], deltas [B, nreg*4] (nreg 1 =
 * class-agnostic), proposals / gt_boxes [B] yxyx float4, gt_classes int64 [B]
 * (K = background), valid uint8 [B].  stats [4] device = (loss_cls, loss_box,
 * #valid, R = max(1, #valid)): loss_cls = sum of softmax CE over valid rows /
 * R, loss_box = sum of smooth-L1(beta) of the gt-class deltas against
 * get_deltas(proposal, gt box; weights) over foreground rows / R
 * (box_regression.py:38-74, layers/loss.py).  Row terms go to the workspace
 * and are summed by one workgroup in a fixed order (deterministic).
 * _bwd: d_logits / d_deltas (every element written) for the upstream
 * gradients grads [2] device (loss_cls, loss_box). */
size_t d2mi_fast_rcnn_loss_workspace_size(int B);
int d2mi_fast_rcnn_loss_fwd(const float* logits, const float* deltas, const float* proposals,
                            const long long* gt_classes, const float* gt_boxes,
                            const unsigned char* valid, int B, int K1, int nreg,
                            const float* weights, float beta, float* stats, void* workspace,
                            size_t workspace_bytes, void* stream);
int d2mi_fast_rcnn_loss_bwd(const float* logits, const float* deltas, const float* proposals,
                            const long long* gt_classes, const float* gt_boxes,
                            const unsigned char* valid, int B, int K1, int nreg,
                            const float* weights, float beta, const float* stats,
                            const float* grads, float* d_logits, float* d_deltas, void* stream);
/* mask_rcnn_loss (lib/modeling/roi_heads/mask_head.py:17-68): logits
 * [B, P = Hm*Wm, C], target [B, P] (the rounded crop_and_resize of the GT
 * mask), classes int64 [B], fg uint8 [B]; stats [3] = (loss, #fg,
 * n = max(1, #fg * P)), loss = sum over fg rows of the sigmoid BCE of the
 * class channel (clamped to [0, C-1]; channel 0 when C == 1) / n.  _bwd
 * writes the whole d_logits for grads [1] device. */
size_t d2mi_mask_loss_workspace_size(int B);
int d2mi_mask_loss_fwd(const float* logits, const float* target, const long long* classes,
                       const unsigned char* fg, int B, int P, int C, float* stats,
                       void* workspace, size_t workspace_bytes, void* stream);
int d2mi_mask_loss_bwd(const float* logits, const float* target, const long long* classes,
                       const unsigned char* fg, int B, int P, int C, const float* stats,
                       const float* grads, float* d_logits, void* stream);

/* ------------------------------------------------ ResNet stem tail
 * relu(y + shift) -> zero pad 1 -> 3x3 stride-2 VALID max pool
 * (lib/modeling/backbone/resnet.py:73-82) on the NHWC output y [N,H,W,C] of
 * the stem conv (without its bias); out [N,(H-1)/2+1,(W-1)/2+1,C].  shift
 * [C] nullable; C % 4 == 0; 16-B aligned. */
int d2mi_stem_pool(const float* y, const float* shift, int N, int H, int W, int C, float* out,
                   void* stream);
/* The stem conv feeding it: 7x7 / stride 2, Cin 3 -> Cout 64, the symmetric
 * pad of 3 then VALID of lib/layers/convolutional.py:12-24 (fix_padding) and
 * resnet.py Stem.conv1, on the split-bf16 MFMA (f32-class).  x [N,H,W,3]
 * NHWC f32; w3 [3][64][160] bf16 planes (d2mi_split_bf16x3) of the weights
 * transposed to [Cout][K] (K = (kh * 7 + kw) * 3 + c, HWIO order) and
 * zero-padded to K = 160; y [N,(H-1)/2+1,(W-1)/2+1,64] the raw sums (no bias:
 * d2mi_stem_pool adds the folded shift).  Replaces the MIOpen conv of the
 * frozen stem. */
int d2mi_stem_conv(const float* x, const uint16_t* w3, int N, int H, int W, float* y,
                   void* stream);
/* The preprocessing ahead of it (lib/modeling/meta_arch/rcnn.py:146-157
 * preprocess_image + structures/image_list.py:89-100 with pad value 0):
 * x [N,H,W,3] NHWC f32 0-255 RGB -> out [N,OHp,OWp,3], out = (x - mean[c]) /
 * std[c] (mean / std: 3 device floats), channels reversed when flip (BGR
 * input format), zeros at rows >= H and columns >= W.  One launch; the same
 * IEEE subtract and divide per value as the unfused form. */
int d2mi_preprocess_images(const float* x, const float* mean, const float* stdv, int N, int H,
                           int W, int OHp, int OWp, int flip, float* out, void* stream);

/* ------------------------------------------------ ROI-head sampling glue
 * (lib/modeling/roi_heads/roi_heads.py:100-232 label_and_sample_proposals,
 * :35-62 select_foreground_proposals)
 * d2mi_roi_gt_classes: out [N,M] int64 = -1 where !pvalid, else the matched
 * GT class gt_cls[n][matches] (gt_cls [N,G], int64 when gt_cls_64 else
 * int32) for label 1, K (background) for label 0, the label (-1) otherwise;
 * labels / matches [N,M] int64 (d2mi_match_boxes), pvalid [N,M] bool.
 * d2mi_roi_sample_take: the sampled slots in the sampler's order (order [N,S]
 * int64, d2mi_subsample): s_boxes [N,S,4] = boxes[n][order], s_cls =
 * gt_classes[n][order], s_gidx = matches[n][order], s_gtb [N,S,4] =
 * gt_boxes[n][s_gidx]; and (F > 0) the mask branch's rows over the first F
 * slots of each image (R = N*F rows, row i = slot (i / F, i % F)): fg_all[i]
 * = valid && s_cls < K, count[0] = the number of foreground rows, and
 * m_boxes / m_cls / m_fg / m_img (the image, int32) / m_mind (s_gidx + n*G) /
 * m_gtb [R(,4)] in stable foreground-first order.  One workgroup; box arrays
 * 16-byte aligned. */
int d2mi_roi_gt_classes(const int64_t* labels, const int64_t* matches, const void* gt_cls,
                        int gt_cls_64, const uint8_t* pvalid, int N, int M, int G, int K,
                        int64_t* out, void* stream);
int d2mi_roi_sample_take(const int64_t* order, const uint8_t* valid, const float* boxes,
                         const int64_t* gt_classes, const int64_t* matches, const float* gt_boxes,
                         int N, int M, int S, int G, int F, int K, float* s_boxes, int64_t* s_cls,
                         int64_t* s_gidx, float* s_gtb, float* m_boxes, int64_t* m_cls,
                         uint8_t* m_fg, int32_t* m_img, int64_t* m_mind, float* m_gtb,
                         uint8_t* fg_all, int64_t* count, void* stream);

/* ------------------------------------------------ resampling gradients
 * d2mi_upsample2x_grad: adjoint of the FPN top-down nearest 2x upsample
 * (lib/modeling/backbone/fpn.py:138-149): gy [N,OH,OW,C] -> gtd
 * [N,ceil(OH/2),ceil(OW/2),C], each the sum of the (up to) 2x2 pixels that
 * copy it, in the order (0,0), (0,1), (1,0), (1,1).
 * d2mi_stride_scatter: input gradient of a 1x1 stride-s conv from its GEMM on
 * the strided grid: g [N,ceil(H/s),ceil(W/s),C] -> out [N,H,W,C] with zeros
 * off the grid, plus add [N,H,W,C] (nullable).  C % 4 == 0, 16-B aligned. */
int d2mi_upsample2x_grad(const float* gy, int N, int OH, int OW, int C, float* gtd, void* stream);
int d2mi_stride_scatter(const float* g, const float* add, int N, int H, int W, int C, int stride,
                        float* out, void* stream);
/* d2mi_stride_scatter_ex: the same, then + add2 (nullable), then the ReLU
 * backward of the producer (gate nullable: out = gate > 0 ? v : 0, the
 * threshold_backward(v, gate, 0) of the ReLU output `gate`).  Used when a
 * ResNet stage output feeds the next stage's strided conv1 / shortcut pair
 * AND the FPN lateral (fpn.py:121-149, resnet.py:52-253): the last of the
 * three backwards forms the whole gated gradient. */
int d2mi_stride_scatter_ex(const float* g, const float* add, const float* add2, const float* gate,
                           int N, int H, int W, int C, int stride, float* out, void* stream);

/* ------------------------------------------------------ RetinaNet losses
 * Replaces RetinaNet.losses (lib/modeling/single_stage_heads/retinanet.py:
 * 147-210) up to the loss normaliser: sigmoid_focal_loss (lib/layers/
 * loss.py:59-104, alpha / gamma, reduction "sum") over every anchor whose
 * label is not "ignore" and every class (target 1 at the matched GT's class
 * for foreground anchors), and smooth_l1_loss (loss.py:9-58, beta, "sum")
 * of the foreground anchors' deltas against get_deltas(anchor, matched GT)
 * (lib/modeling/box_regression.py:38-74, weights[4] = wy, wx, wh, ww).
 * cls[l] / box[l]: level l's head outputs [N, H_l, W_l, A*K] / [N, H_l, W_l,
 * A*4] f32 (16-byte aligned), level_anchors[l] = H_l * W_l * A; anchors [R, 4]
 * (levels concatenated, (h, w, a) order, R = sum of level_anchors); gt_boxes
 * [N, G, 4]; gt_classes [N, G] int64; matches / labels [N, R] int64 (the
 * Matcher's: labels 1 fg, 0 bg, -1 ignore).  K % 4 == 0.  fwd: partial
 * [N * d2mi_retina_loss_blocks()][2] (cls, box) per-workgroup sums, to be
 * added in a fixed order.  bwd: d_cls / d_box levels (every element written),
 * scaled by the device scalars *g_cls / *g_box (null: zero). */
int d2mi_retina_loss_blocks(void);
int d2mi_retina_loss_fwd(const float* const* cls, const float* const* box,
                         const long long* level_anchors, int L, int N, int K, int A,
                         const float* anchors, const float* gt_boxes, const long long* gt_classes,
                         int G, const long long* matches, const long long* labels, float alpha,
                         float gamma, float beta, const float* weights, float* partial,
                         void* stream);
int d2mi_retina_loss_bwd(const float* const* cls, const float* const* box, float* const* d_cls,
                         float* const* d_box, const long long* level_anchors, int L, int N, int K,
                         int A, const float* anchors, const float* gt_boxes,
                         const long long* gt_classes, int G, const long long* matches,
                         const long long* labels, float alpha, float gamma, float beta,
                         const float* weights, const float* g_cls, const float* g_box,
                         void* stream);

/* ------------------------------------------------------ Momentum-SGD step
 * Replaces the update of lib/engine/trainer.py:116-139 for every trainable
 * tensor in two launches: g' = g + wd * w (slim.l2_regularizer gradient,
 * lib/solver/regularizer.py:6-24), per-tensor tf.clip_by_norm(g', clip_norm)
 * (slim.learning.clip_gradient_norms; clip_norm <= 0 disables it), then
 * ApplyMomentum: accum = accum * momentum + g''; w -= lr * accum.
 * tensor_table / chunk_table: device arrays of the records whose sizes
 * d2mi_sgd_table_sizes reports (tensor: {float* w; const float* g (nullable:
 * zero gradient); float* accum; int64 numel; float wd; int32 first_chunk,
 * num_chunks, pad}; chunk: {int32 tensor, pad; int64 begin, end}, chunks of at
 * most chunk_elems elements, a tensor's chunks consecutive).  partial: device
 * float [num_chunks] scratch.  Per-tensor norms are fixed-order sums. */
int d2mi_sgd_table_sizes(int* tensor_bytes, int* chunk_bytes, int* chunk_elems);
int d2mi_momentum_sgd(const void* tensor_table, const void* chunk_table, int num_chunks,
                      float* partial, float clip_norm, float momentum, float lr, void* stream);
/* The same step with the learning rate read from the device float *lr_dev at
 * run time when lr_dev is non-null (lr ignored): a training step captured in
 * a hipGraph (engine/graphed.py) replays with each iteration's LR of
 * lib/solver/learning_rate.py, which the host writes to lr_dev. */
int d2mi_momentum_sgd_ex(const void* tensor_table, const void* chunk_table, int num_chunks,
                         float* partial, float clip_norm, float momentum, float lr,
                         const float* lr_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* D2MI_H */
