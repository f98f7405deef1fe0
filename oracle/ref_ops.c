/*
 * ORACLE — test infrastructure only.  A plain-C CPU restatement of the TF 1.x
 * CPU kernels and the reference glue that the detection hot path of
 * SimeonZhang/detectron2_tensorflow runs.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * TensorFlow itself (tensorflow>=1.13.1, requirements.txt:42; tf.contrib makes
 * it 1.x) is a third-party dependency absent from /root/reference and not
 * installable here, so its kernels are restated from their published source
 * (TF 1.15 core/kernels): crop_and_resize_op.cc (CropAndResize /
 * CropAndResizeGradImage CPU functors), non_max_suppression_op.cc
 * (NonMaxSuppressionV3 via DoNonMaxSuppressionOp + IOU), topk_op.cc.
 * Pinning: NMS/IoU are checked against the reference's own numpy NMS
 * (lib/structures/np_box_list_ops.py:146-217) through committed golden
 * vectors (tests/golden/make_golden.py); the CropAndResize restatement is
 * pinned by hand-computed known answers only (no reference fixture exists) —
 * see DESIGN.md "Oracle".
 *
 * Build: gcc -O2 -fPIC -shared -ffp-contract=off -fno-fast-math -fopenmp
 * (no FMA contraction: the float expressions round like TF's x86 build).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------
 * tf.image.crop_and_resize, bilinear, extrapolation_value = 0
 * (TF 1.15 crop_and_resize_op.cc, CropAndResize<CPUDevice, float>).
 * image [N,H,W,C], boxes [R,4] normalised (y1,x1,y2,x2), box_ind [R]
 * out [R,ch,cw,C].  Returns -1 if a box index is out of range (TF raises
 * InvalidArgumentError), else 0.
 * ---------------------------------------------------------------------- */
int oracle_crop_and_resize(const float* image, int N, int H, int W, int C, const float* boxes,
                           const int32_t* box_ind, int R, int ch, int cw, float* out) {
  for (int b = 0; b < R; ++b)
    if (box_ind[b] < 0 || box_ind[b] >= N) return -1;
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < R; ++b) {
    const float y1 = boxes[4 * b + 0], x1 = boxes[4 * b + 1];
    const float y2 = boxes[4 * b + 2], x2 = boxes[4 * b + 3];
    const int bi = box_ind[b];
    const float height_scale = (ch > 1) ? (y2 - y1) * (H - 1) / (ch - 1) : 0;
    const float width_scale = (cw > 1) ? (x2 - x1) * (W - 1) / (cw - 1) : 0;
    for (int y = 0; y < ch; ++y) {
      const float in_y = (ch > 1) ? y1 * (H - 1) + y * height_scale : 0.5 * (y1 + y2) * (H - 1);
      float* orow = out + ((size_t)b * ch + y) * cw * C;
      /* written as !(in range) so that a NaN coordinate (a degenerate box;
       * UB in TF: (int)floorf(NaN) indexes out of bounds) extrapolates */
      if (!(in_y >= 0 && in_y <= H - 1)) {
        memset(orow, 0, sizeof(float) * (size_t)cw * C);
        continue;
      }
      const int top_y_index = (int)floorf(in_y);
      const int bottom_y_index = (int)ceilf(in_y);
      const float y_lerp = in_y - top_y_index;
      for (int x = 0; x < cw; ++x) {
        const float in_x = (cw > 1) ? x1 * (W - 1) + x * width_scale : 0.5 * (x1 + x2) * (W - 1);
        float* o = orow + (size_t)x * C;
        if (!(in_x >= 0 && in_x <= W - 1)) {
          memset(o, 0, sizeof(float) * C);
          continue;
        }
        const int left_x_index = (int)floorf(in_x);
        const int right_x_index = (int)ceilf(in_x);
        const float x_lerp = in_x - left_x_index;
        const float* tl = image + (((size_t)bi * H + top_y_index) * W + left_x_index) * C;
        const float* tr = image + (((size_t)bi * H + top_y_index) * W + right_x_index) * C;
        const float* bl = image + (((size_t)bi * H + bottom_y_index) * W + left_x_index) * C;
        const float* br = image + (((size_t)bi * H + bottom_y_index) * W + right_x_index) * C;
        for (int d = 0; d < C; ++d) {
          const float top = tl[d] + (tr[d] - tl[d]) * x_lerp;
          const float bottom = bl[d] + (br[d] - bl[d]) * x_lerp;
          o[d] = top + (bottom - top) * y_lerp;
        }
      }
    }
  }
  return 0;
}

/* CropAndResizeGradImage (TF 1.15), accumulating into grads_image [N,H,W,C]
 * (caller zeroes it). */
int oracle_crop_and_resize_grad_image(const float* grads, const float* boxes,
                                      const int32_t* box_ind, int R, int ch, int cw, int N, int H,
                                      int W, int C, float* grads_image) {
  for (int b = 0; b < R; ++b)
    if (box_ind[b] < 0 || box_ind[b] >= N) return -1;
  for (int b = 0; b < R; ++b) {
    const float y1 = boxes[4 * b + 0], x1 = boxes[4 * b + 1];
    const float y2 = boxes[4 * b + 2], x2 = boxes[4 * b + 3];
    const int bi = box_ind[b];
    const float height_scale = (ch > 1) ? (y2 - y1) * (H - 1) / (ch - 1) : 0;
    const float width_scale = (cw > 1) ? (x2 - x1) * (W - 1) / (cw - 1) : 0;
    for (int y = 0; y < ch; ++y) {
      const float in_y = (ch > 1) ? y1 * (H - 1) + y * height_scale : 0.5 * (y1 + y2) * (H - 1);
      if (!(in_y >= 0 && in_y <= H - 1)) continue;
      const int top_y_index = (int)floorf(in_y);
      const int bottom_y_index = (int)ceilf(in_y);
      const float y_lerp = in_y - top_y_index;
      for (int x = 0; x < cw; ++x) {
        const float in_x = (cw > 1) ? x1 * (W - 1) + x * width_scale : 0.5 * (x1 + x2) * (W - 1);
        if (!(in_x >= 0 && in_x <= W - 1)) continue;
        const int left_x_index = (int)floorf(in_x);
        const int right_x_index = (int)ceilf(in_x);
        const float x_lerp = in_x - left_x_index;
        const float* g = grads + (((size_t)b * ch + y) * cw + x) * C;
        float* tl = grads_image + (((size_t)bi * H + top_y_index) * W + left_x_index) * C;
        float* tr = grads_image + (((size_t)bi * H + top_y_index) * W + right_x_index) * C;
        float* bl = grads_image + (((size_t)bi * H + bottom_y_index) * W + left_x_index) * C;
        float* br = grads_image + (((size_t)bi * H + bottom_y_index) * W + right_x_index) * C;
        for (int d = 0; d < C; ++d) {
          const float dtop = (1 - y_lerp) * g[d];
          tl[d] += (1 - x_lerp) * dtop;
          tr[d] += x_lerp * dtop;
          const float dbottom = y_lerp * g[d];
          bl[d] += (1 - x_lerp) * dbottom;
          br[d] += x_lerp * dbottom;
        }
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------
 * The reference crop_and_resize wrapper (lib/layers/functional.py:100-166)
 * on ONE level: tf.pad SYMMETRIC by 1 (materialised), boxes + 1, box
 * re-normalisation (aligned :138-152 / unaligned :153-159), then
 * tf.image.crop_and_resize.  `scale` is ROIAlign's spatial_scale
 * (roi_align.py:55), sr its sampling_ratio (crop at out*sr then
 * slim.avg_pool2d k=s=sr, roi_align.py:53-65).
 * ---------------------------------------------------------------------- */
int oracle_roi_align_level(const float* image, int N, int H, int W, int C, const float* boxes_px,
                           const int32_t* box_ind, int R, int out_h, int out_w, float scale,
                           int sr, int aligned, int pad_border, float* out) {
  const int Hp = pad_border ? H + 2 : H, Wp = pad_border ? W + 2 : W;
  float* padded = (float*)image;
  if (pad_border) {
    padded = (float*)malloc(sizeof(float) * (size_t)N * Hp * Wp * C);
    for (int n = 0; n < N; ++n)
      for (int y = 0; y < Hp; ++y) {
        const int sy = y == 0 ? 0 : (y == Hp - 1 ? H - 1 : y - 1); /* SYMMETRIC */
        for (int x = 0; x < Wp; ++x) {
          const int sx = x == 0 ? 0 : (x == Wp - 1 ? W - 1 : x - 1);
          memcpy(padded + (((size_t)n * Hp + y) * Wp + x) * C,
                 image + (((size_t)n * H + sy) * W + sx) * C, sizeof(float) * C);
        }
      }
  }
  const int ch = sr > 0 ? out_h * sr : out_h, cw = sr > 0 ? out_w * sr : out_w;
  float* nb = (float*)malloc(sizeof(float) * 4 * (size_t)(R > 0 ? R : 1));
  for (int b = 0; b < R; ++b) {
    float ymin = boxes_px[4 * b] * scale, xmin = boxes_px[4 * b + 1] * scale;
    float ymax = boxes_px[4 * b + 2] * scale, xmax = boxes_px[4 * b + 3] * scale;
    if (pad_border) {
      ymin = ymin + 1.f; xmin = xmin + 1.f; ymax = ymax + 1.f; xmax = xmax + 1.f;
    }
    if (aligned) {
      const float spacing_h = (ymax - ymin) / (float)ch;
      const float spacing_w = (xmax - xmin) / (float)cw;
      const float im0 = (float)(Hp - 1), im1 = (float)(Wp - 1);
      const float norm_ymin = (ymin + spacing_h / 2 - 0.5f) / im0;
      const float norm_xmin = (xmin + spacing_w / 2 - 0.5f) / im1;
      const float norm_h = spacing_h * (float)(ch - 1) / im0;
      const float norm_w = spacing_w * (float)(cw - 1) / im1;
      nb[4 * b] = norm_ymin;
      nb[4 * b + 1] = norm_xmin;
      nb[4 * b + 2] = norm_ymin + norm_h;
      nb[4 * b + 3] = norm_xmin + norm_w;
    } else {
      const float im0 = (float)Hp, im1 = (float)Wp;
      nb[4 * b] = ymin / im0;
      nb[4 * b + 1] = xmin / im1;
      nb[4 * b + 2] = ymax / im0;
      nb[4 * b + 3] = xmax / im1;
    }
  }
  int rc;
  if (sr > 0) {
    float* crop = (float*)malloc(sizeof(float) * (size_t)(R > 0 ? R : 1) * ch * cw * C);
    rc = oracle_crop_and_resize(padded, N, Hp, Wp, C, nb, box_ind, R, ch, cw, crop);
    const float cnt = (float)(sr * sr);
    for (int b = 0; rc == 0 && b < R; ++b)
      for (int oy = 0; oy < out_h; ++oy)
        for (int ox = 0; ox < out_w; ++ox)
          for (int d = 0; d < C; ++d) {
            float acc = 0.f;
            for (int a = 0; a < sr; ++a)
              for (int c = 0; c < sr; ++c)
                acc += crop[(((size_t)b * ch + oy * sr + a) * cw + ox * sr + c) * C + d];
            out[(((size_t)b * out_h + oy) * out_w + ox) * C + d] = acc / cnt;
          }
    free(crop);
  } else {
    rc = oracle_crop_and_resize(padded, N, Hp, Wp, C, nb, box_ind, R, ch, cw, out);
  }
  free(nb);
  if (pad_border) free(padded);
  return rc;
}

/* ------------------------------------------------------------------------
 * NonMaxSuppressionV3 (TF 1.15 non_max_suppression_op.cc DoNonMaxSuppressionOp
 * with soft_nms_sigma = 0): a max-heap of candidates with score > score_thr,
 * comparator (score, then lower box index first), each popped candidate is
 * compared against the selected boxes from newest to oldest and dropped when
 * IOU > iou_thr.  Returns the number of selected indices written to `out`.
 * ---------------------------------------------------------------------- */
static float tf_iou(const float* boxes, int i, int j) {
  const float* a = boxes + 4 * i;
  const float* b = boxes + 4 * j;
  const float ymin_i = fminf(a[0], a[2]), xmin_i = fminf(a[1], a[3]);
  const float ymax_i = fmaxf(a[0], a[2]), xmax_i = fmaxf(a[1], a[3]);
  const float ymin_j = fminf(b[0], b[2]), xmin_j = fminf(b[1], b[3]);
  const float ymax_j = fmaxf(b[0], b[2]), xmax_j = fmaxf(b[1], b[3]);
  const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
  const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
  if (area_i <= 0 || area_j <= 0) return 0.0f;
  const float intersection_ymin = fmaxf(ymin_i, ymin_j);
  const float intersection_xmin = fmaxf(xmin_i, xmin_j);
  const float intersection_ymax = fminf(ymax_i, ymax_j);
  const float intersection_xmax = fminf(xmax_i, xmax_j);
  const float intersection_area = fmaxf(intersection_ymax - intersection_ymin, 0.0f) *
                                  fmaxf(intersection_xmax - intersection_xmin, 0.0f);
  return intersection_area / (area_i + area_j - intersection_area);
}

typedef struct {
  int box_index;
  float score;
  int suppress_begin_index;
} Candidate;

/* "a ranks below b" in the priority queue (TF's cmp) */
static int cand_less(const Candidate* a, const Candidate* b) {
  return ((a->score == b->score) && (a->box_index > b->box_index)) || a->score < b->score;
}

static void heap_push(Candidate* h, int* n, Candidate c) {
  int i = (*n)++;
  h[i] = c;
  while (i > 0) {
    int p = (i - 1) / 2;
    if (cand_less(&h[p], &h[i])) {
      Candidate t = h[p]; h[p] = h[i]; h[i] = t; i = p;
    } else break;
  }
}

static Candidate heap_pop(Candidate* h, int* n) {
  Candidate top = h[0];
  h[0] = h[--(*n)];
  int i = 0;
  for (;;) {
    int l = 2 * i + 1, r = l + 1, m = i;
    if (l < *n && cand_less(&h[m], &h[l])) m = l;
    if (r < *n && cand_less(&h[m], &h[r])) m = r;
    if (m == i) break;
    Candidate t = h[m]; h[m] = h[i]; h[i] = t; i = m;
  }
  return top;
}

int oracle_nms(const float* boxes, const float* scores, int num_boxes, int max_output_size,
               float iou_threshold, float score_threshold, int32_t* selected_out) {
  Candidate* heap = (Candidate*)malloc(sizeof(Candidate) * (size_t)(num_boxes > 0 ? num_boxes : 1));
  int hn = 0;
  for (int i = 0; i < num_boxes; ++i)
    if (scores[i] > score_threshold) {
      Candidate c = {i, scores[i], 0};
      heap_push(heap, &hn, c);
    }
  int nsel = 0;
  while (nsel < max_output_size && hn > 0) {
    Candidate next = heap_pop(heap, &hn);
    const float original_score = next.score;
    int should_hard_suppress = 0;
    for (int j = nsel - 1; j >= next.suppress_begin_index; --j) {
      const float similarity = tf_iou(boxes, next.box_index, selected_out[j]);
      const float weight = similarity <= iou_threshold ? 1.0f : 0.0f;
      next.score *= weight;
      if (similarity > iou_threshold) {
        should_hard_suppress = 1;
        break;
      }
      if (next.score <= score_threshold) break;
    }
    next.suppress_begin_index = nsel;
    if (!should_hard_suppress) {
      if (next.score == original_score) {
        selected_out[nsel++] = next.box_index;
        continue;
      }
      if (next.score > score_threshold) heap_push(heap, &hn, next);
    }
  }
  free(heap);
  return nsel;
}

/* Batched form: segments [off[s], off[s+1]) of one boxes/scores array;
 * keep [S, max_out] (-1 padded), num_keep [S].  OpenMP over segments. */
void oracle_nms_batched(const float* boxes, const float* scores, const int32_t* off, int S,
                        int max_out, float iou_threshold, int32_t* keep, int32_t* num_keep) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int s = 0; s < S; ++s) {
    int32_t* k = keep + (size_t)s * max_out;
    const int n = oracle_nms(boxes + 4 * (size_t)off[s], scores + off[s], off[s + 1] - off[s],
                             max_out, iou_threshold, -INFINITY, k);
    for (int i = n; i < max_out; ++i) k[i] = -1;
    num_keep[s] = n;
  }
}

/* ------------------------------------------------------------------------
 * tf.nn.top_k(sorted=True): value desc, ties lower index first.
 * ---------------------------------------------------------------------- */
static const float* g_vals;
static int topk_cmp(const void* a, const void* b) {
  const int i = *(const int*)a, j = *(const int*)b;
  const float vi = g_vals[i], vj = g_vals[j];
  if (vi > vj) return -1;
  if (vi < vj) return 1;
  return (i < j) ? -1 : (i > j);
}

int oracle_topk(const float* values, int n, int k, float* vals_out, int32_t* idx_out) {
  if (k > n) k = n;
  int* idx = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  for (int i = 0; i < n; ++i) idx[i] = i;
  g_vals = values;
  qsort(idx, n, sizeof(int), topk_cmp);
  for (int i = 0; i < k; ++i) {
    idx_out[i] = idx[i];
    vals_out[i] = values[idx[i]];
  }
  free(idx);
  return k;
}

/* ------------------------------------------------------------------------
 * Box2BoxTransform.apply_deltas (lib/modeling/box_regression.py:76-123)
 * deltas [N, K*4], boxes [N,4] -> out [N, K*4]; float32, no contraction.
 * ---------------------------------------------------------------------- */
void oracle_apply_deltas(const float* deltas, const float* boxes, int N, int K, float wy,
                         float wx, float wh, float ww, float scale_clamp, float* out) {
#pragma omp parallel for schedule(static)
  for (int n = 0; n < N; ++n) {
    const float* b = boxes + 4 * (size_t)n;
    const float heights = b[2] - b[0];
    const float widths = b[3] - b[1];
    const float ctr_y = b[0] + 0.5f * heights;
    const float ctr_x = b[1] + 0.5f * widths;
    for (int k = 0; k < K; ++k) {
      const float* d = deltas + ((size_t)n * K + k) * 4;
      const float dy = d[0] / wy, dx = d[1] / wx;
      float dh = d[2] / wh, dw = d[3] / ww;
      dh = fminf(dh, scale_clamp);
      dw = fminf(dw, scale_clamp);
      const float pred_ctr_y = dy * heights + ctr_y;
      const float pred_ctr_x = dx * widths + ctr_x;
      const float pred_h = expf(dh) * heights;
      const float pred_w = expf(dw) * widths;
      float* o = out + ((size_t)n * K + k) * 4;
      o[0] = pred_ctr_y - 0.5f * pred_h;
      o[1] = pred_ctr_x - 0.5f * pred_w;
      o[2] = pred_ctr_y + 0.5f * pred_h;
      o[3] = pred_ctr_x + 0.5f * pred_w;
    }
  }
}
