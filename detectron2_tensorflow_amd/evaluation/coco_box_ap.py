"""COCO bbox AP, restating pycocotools COCOeval (iouType="bbox") as
lib/evaluation/coco_evaluator.py drives it: evaluateImg + accumulate +
summarize for AP@[.50:.95], AP50, AP75 and the small / medium / large area
ranges at 100 detections per image.

Per (image, category, area range): ground truth sorted non-ignored first
(ignore = crowd or area outside the range); detections sorted by score
(stable) and cut to maxDets; IoU against crowd GT is intersection / detection
area; greedy matching per IoU threshold prefers non-ignored GT and never
re-matches a non-crowd GT; unmatched detections outside the area range are
ignored.  accumulate: detections of all images merged by score (stable
mergesort), cumulative TP / FP over non-ignored ones, precision made
monotone from the right, sampled at 101 recall points (searchsorted left);
AP = mean over the defined entries.  Boxes here are yxyx absolute (this
framework's format); areas are box areas unless given.
"""
import numpy as np

IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)
AREAS = {"all": (0.0, 1e10), "small": (0.0, 32.0 ** 2), "medium": (32.0 ** 2, 96.0 ** 2),
         "large": (96.0 ** 2, 1e10)}


def _area(b):
    return np.maximum(b[:, 2] - b[:, 0], 0) * np.maximum(b[:, 3] - b[:, 1], 0)


def _iou(dt, gt, crowd):
    """maskUtils.iou on boxes: [D, G]; crowd GT use the detection area as union."""
    if len(dt) == 0 or len(gt) == 0:
        return np.zeros((len(dt), len(gt)))
    ih = np.minimum(dt[:, None, 2], gt[None, :, 2]) - np.maximum(dt[:, None, 0], gt[None, :, 0])
    iw = np.minimum(dt[:, None, 3], gt[None, :, 3]) - np.maximum(dt[:, None, 1], gt[None, :, 1])
    inter = np.maximum(ih, 0) * np.maximum(iw, 0)
    ad, ag = _area(dt)[:, None], _area(gt)[None, :]
    union = np.where(crowd[None, :], ad, ad + ag - inter)
    return np.where(union > 0, inter / np.maximum(union, 1e-12), 0.0)


class COCOBoxEvaluator:
    def __init__(self, max_dets=100):
        self.max_dets = max_dets
        self.images = []

    def add(self, gt_boxes, gt_classes, det_boxes, det_scores, det_classes, gt_crowd=None,
            gt_areas=None):
        """One image: arrays of yxyx boxes and class ids (det_scores for dets)."""
        gb = np.asarray(gt_boxes, np.float64).reshape(-1, 4)
        self.images.append({
            "gb": gb, "gc": np.asarray(gt_classes).reshape(-1),
            "crowd": (np.zeros(len(gb), bool) if gt_crowd is None
                      else np.asarray(gt_crowd, bool).reshape(-1)),
            "ga": _area(gb) if gt_areas is None else np.asarray(gt_areas, np.float64),
            "db": np.asarray(det_boxes, np.float64).reshape(-1, 4),
            "ds": np.asarray(det_scores, np.float64).reshape(-1),
            "dc": np.asarray(det_classes).reshape(-1)})

    def _eval_img(self, im, cat, rng):
        g = im["gc"] == cat
        d = im["dc"] == cat
        if not g.any() and not d.any():
            return None
        gb, crowd, ga = im["gb"][g], im["crowd"][g], im["ga"][g]
        gign = crowd | (ga < rng[0]) | (ga > rng[1])
        gord = np.argsort(gign, kind="mergesort")
        gb, crowd, gign = gb[gord], crowd[gord], gign[gord]
        db, ds = im["db"][d], im["ds"][d]
        dord = np.argsort(-ds, kind="mergesort")[: self.max_dets]
        db, ds = db[dord], ds[dord]
        ious = _iou(db, gb, crowd)
        T, D, G = len(IOU_THRS), len(db), len(gb)
        dtm = np.zeros((T, D), bool)
        dtig = np.zeros((T, D), bool)
        for ti, t in enumerate(IOU_THRS):
            gtm = np.zeros(G, bool)
            for di in range(D):
                iou, m = min(t, 1 - 1e-10), -1
                for gi in range(G):
                    if gtm[gi] and not crowd[gi]:
                        continue
                    if m > -1 and not gign[m] and gign[gi]:
                        break
                    if ious[di, gi] < iou:
                        continue
                    iou, m = ious[di, gi], gi
                if m == -1:
                    continue
                dtig[ti, di] = gign[m]
                dtm[ti, di] = True
                gtm[m] = True
        da = _area(db)
        out_rng = (da < rng[0]) | (da > rng[1])
        dtig = dtig | (~dtm & out_rng[None, :])
        return {"scores": ds, "dtm": dtm, "dtig": dtig, "npig": int((~gign).sum())}

    def _ap(self, cat_ids, rng, iou_idx=None):
        precs = []
        for cat in cat_ids:
            ev = [e for e in (self._eval_img(im, cat, rng) for im in self.images) if e is not None]
            if not ev:
                continue
            npig = sum(e["npig"] for e in ev)
            if npig == 0:
                continue
            scores = np.concatenate([e["scores"] for e in ev])
            order = np.argsort(-scores, kind="mergesort")
            dtm = np.concatenate([e["dtm"] for e in ev], axis=1)[:, order]
            dtig = np.concatenate([e["dtig"] for e in ev], axis=1)[:, order]
            tps = np.cumsum(dtm & ~dtig, axis=1).astype(np.float64)
            fps = np.cumsum(~dtm & ~dtig, axis=1).astype(np.float64)
            p = np.zeros((len(IOU_THRS), len(REC_THRS)))
            for t in range(len(IOU_THRS)):
                tp, fp = tps[t], fps[t]
                rc = tp / npig
                pr = tp / (fp + tp + np.spacing(1))
                for i in range(len(pr) - 1, 0, -1):
                    pr[i - 1] = max(pr[i - 1], pr[i])
                idx = np.searchsorted(rc, REC_THRS, side="left")
                q = np.zeros(len(REC_THRS))
                ok = idx < len(pr)
                q[ok] = pr[idx[ok]]
                p[t] = q
            precs.append(p)
        if not precs:
            return -1.0
        p = np.stack(precs)  # [K, T, R]
        if iou_idx is not None:
            p = p[:, iou_idx]
        return float(p.mean())

    def summarize(self):
        """{AP, AP50, AP75, APs, APm, APl} in percent (-1 where undefined)."""
        cats = sorted(set(np.concatenate([im["gc"] for im in self.images]).tolist())) \
            if self.images else []
        pct = lambda v: v * 100 if v >= 0 else -1.0
        return {"AP": pct(self._ap(cats, AREAS["all"])),
                "AP50": pct(self._ap(cats, AREAS["all"], 0)),
                "AP75": pct(self._ap(cats, AREAS["all"], 5)),
                "APs": pct(self._ap(cats, AREAS["small"])),
                "APm": pct(self._ap(cats, AREAS["medium"])),
                "APl": pct(self._ap(cats, AREAS["large"]))}
