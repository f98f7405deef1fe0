"""Box AP harness: the bbox COCOeval statistics of
lib/evaluation/coco_evaluator.py, restated in numpy (pycocotools is not in
the container)."""
from .coco_box_ap import COCOBoxEvaluator

__all__ = ["COCOBoxEvaluator"]
