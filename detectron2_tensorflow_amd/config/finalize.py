"""config_utils.finalize (lib/utils/config_utils.py:7-20).

The reference sets NUM_GPUS from the visible GPUs, IMS_PER_BATCH =
NUM_GPUS * IMS_PER_GPU, reads DATASETS.ROOT_DIR/category_map.json for the
class counts, freezes the config and sets the training phase.  Here the
device count comes from the torch.distributed world size (one process per
GPU), and a missing category map falls back to an explicit
``category_map`` argument (the synthetic benchmark passes COCO's 80/53).
"""
import json
import os

from ..utils.training import set_training_phase


def finalize(cfg, training=False, world_size=None, category_map=None):
    if world_size is None:
        try:
            import torch.distributed as dist
            world_size = dist.get_world_size() if dist.is_initialized() else 1
        except Exception:
            world_size = 1
    cfg.SOLVER.NUM_GPUS = int(world_size)
    cfg.SOLVER.IMS_PER_BATCH = cfg.SOLVER.NUM_GPUS * cfg.SOLVER.IMS_PER_GPU
    if category_map is None:
        path = os.path.join(cfg.DATASETS.ROOT_DIR, cfg.DATASETS.CATEGORY_MAP_NAME)
        with open(path) as fid:
            category_map = json.load(fid)
    cfg.MODEL.ROI_HEADS.NUM_CLASSES = category_map["num_thing_classes"]
    cfg.MODEL.SEM_SEG_HEAD.NUM_CLASSES = category_map["num_stuff_classes"]
    cfg.MODEL.SEM_SEG_HEAD.IGNORE_VALUE = category_map["stuff_ignore_value"]
    cfg.freeze()
    set_training_phase(training=training)
    return cfg
