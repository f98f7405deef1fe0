"""Default configuration tree.

Key names and default values follow the reference's lib/config/defaults.py
(:17-785) for every subtree the detection path reads (MODEL.* for
GeneralizedRCNN / SingleStageDetector / ResNet / FPN / RPN / ROI heads /
RetinaNet / SOLO inference, SOLVER, TRANSFORM, TEST, ...), so the reference
YAML files merge without unknown-key errors.  Subsystems this build does not
implement (SpineNet, YOLOv4, panoptic, data augmentation, TFRecord readers)
keep only the keys the shipped YAMLs set.
"""
from .config import CfgNode


def _tree():
    model = {
        "LOAD_PROPOSALS": False,
        "MASK_ON": True,
        "META_ARCHITECTURE": "GeneralizedRCNN",
        "INPUT_FORMAT": "BGR",
        "PIXEL_MEAN": [123.675, 116.280, 103.530],
        "PIXEL_STD": [1.0, 1.0, 1.0],
        "SEGMENTATION_OUTPUT": {"FORMAT": "conventional", "FIXED_RESOLUTION": 512},
        "BACKBONE": {"NAME": "ResNet", "FREEZE_AT": 2},
        "RESNETS": {
            "DEPTH": 101, "OUT_FEATURES": ["res4"], "NUM_GROUPS": 1, "NORM": "FrozenBN",
            "ACTIVATION": "mish", "WIDTH_PER_GROUP": 64, "STRIDE_IN_1X1": True,
            "RES5_DILATION": 1, "RES2_OUT_CHANNELS": 256, "STEM_OUT_CHANNELS": 64,
            "DEFORM_ON_PER_STAGE": [False, False, False, False], "DEFORM_MODULATED": False,
            "DEFORM_NUM_GROUPS": 1,
        },
        "NECK": {"NAME": "", "IN_FEATURES": [], "OUT_CHANNELS": 256, "NORM": "", "ACTIVATION": "",
                 "FUSE_TYPE": "sum", "TOP_BLOCK_TYPE": "MAXPOOL"},
        "PROPOSAL_GENERATOR": {"NAME": "RPN", "MIN_SIZE": 0},
        "ANCHOR_GENERATOR": {"NAME": "DefaultAnchorGenerator",
                             "SIZES": [[32, 64, 128, 256, 512]],
                             "ASPECT_RATIOS": [[0.5, 1.0, 2.0]], "ANGLES": [[-90, 0, 90]]},
        "RPN": {
            "HEAD_NAME": "StandardRPNHead", "IN_FEATURES": ["res4"], "BOUNDARY_THRESH": -1,
            "IOU_THRESHOLDS": [0.3, 0.7], "IOU_LABELS": [0, -1, 1], "BATCH_SIZE_PER_IMAGE": 256,
            "POSITIVE_FRACTION": 0.5, "BBOX_REG_WEIGHTS": (1.0, 1.0, 1.0, 1.0),
            "SMOOTH_L1_BETA": 0.0, "LOSS_WEIGHT": 1.0, "PRE_NMS_TOPK_TRAIN": 12000,
            "PRE_NMS_TOPK_TEST": 6000, "POST_NMS_TOPK_TRAIN": 2000, "POST_NMS_TOPK_TEST": 1000,
            "NMS_THRESH": 0.7,
        },
        "ROI_HEADS": {
            "NAME": "Res5ROIHeads", "NUM_CLASSES": 80, "IN_FEATURES": ["res4"],
            "IOU_THRESHOLDS": [0.5], "IOU_LABELS": [0, 1], "BATCH_SIZE_PER_IMAGE": 512,
            "POSITIVE_FRACTION": 0.25, "PROPOSAL_APPEND_GT": True, "SCORE_THRESH_TEST": 0.05,
            "NMS_THRESH_TEST": 0.5, "NMS_CLS_AGNOSTIC": False,
        },
        "ROI_BOX_HEAD": {
            "NAME": "", "BBOX_REG_WEIGHTS": (10.0, 10.0, 5.0, 5.0), "SMOOTH_L1_BETA": 0.0,
            "FOCAL_LOSS_ALPHA": 0.25, "FOCAL_LOSS_GAMMA": 2.0, "POOLER_RESOLUTION": 14,
            "POOLER_SAMPLING_RATIO": 0, "POOLER_TYPE": "ROIAlignV2", "NUM_FC": 0, "FC_DIM": 1024,
            "NUM_CONV": 0, "CONV_DIM": 256, "NORM": "", "CLS_AGNOSTIC_BBOX_REG": False,
        },
        "ROI_MASK_HEAD": {
            "NAME": "MaskRCNNConvUpsampleHead", "POOLER_RESOLUTION": 14,
            "POOLER_SAMPLING_RATIO": 0, "NUM_CONV": 0, "CONV_DIM": 256, "NORM": "",
            "CLS_AGNOSTIC_MASK": False, "POOLER_TYPE": "ROIAlignV2",
        },
        "SEM_SEG_HEAD": {"NAME": "SemSegFPNHead", "IN_FEATURES": ["p2", "p3", "p4", "p5"],
                         "IGNORE_VALUE": -1, "NUM_CLASSES": 54, "CONVS_DIM": 128,
                         "COMMON_STRIDE": 4, "NORM": "GN", "LOSS_WEIGHT": 1.0},
        "SINGLE_STAGE_HEAD": {"NAME": "RetinaNetHead", "NUM_CLASSES": 80,
                              "IN_FEATURES": ["p3", "p4", "p5", "p6", "p7"],
                              "IOU_THRESHOLDS": [0.4, 0.5], "IOU_LABELS": [0, -1, 1]},
        "RETINANET": {
            "NUM_CONVS": 4, "PRIOR_PROB": 0.01, "SCORE_THRESH_TEST": 0.05,
            "TOPK_CANDIDATES_TEST": 1000, "NMS_THRESH_TEST": 0.5, "NMS_CLS_AGNOSTIC": False,
            "BBOX_REG_WEIGHTS": (1.0, 1.0, 1.0, 1.0), "FOCAL_LOSS_GAMMA": 2.0,
            "FOCAL_LOSS_ALPHA": 0.25, "SMOOTH_L1_LOSS_BETA": 0.1,
        },
        "SOLO": {
            "MASK_KERNEL_NUM_CONVS": 4, "USE_DEFORM_CONV": False, "DEFORM_MODULATED": False,
            "MASK_KERNEL_NORM": "GN", "MASK_KERNEL_SIZE": 1, "MASK_KERNEL_CONVS_DIM": 512,
            "MASK_FEATURE_IN_FEATURES": ["p2", "p3", "p4", "p5"], "MASK_FEATURE_CONVS_DIM": 128,
            "MASK_FEATURE_OUT_DIMS": 256, "MASK_FEATURE_COMMON_STRIDE": 4,
            "MASK_FEATURE_NORM": "GN",
            "SCALE_RANGES": [[1, 96], [48, 192], [96, 384], [192, 768], [384, 2048]],
            "NUM_GRIDS": [40, 36, 24, 16, 12], "PRIOR_PROB": 0.01, "SIGMA": 0.2,
            "FOCAL_LOSS_GAMMA": 2.0, "FOCAL_LOSS_ALPHA": 0.25, "INS_LOSS_WEIGHT": 3.0,
            "SCORE_THRESH_TEST": 0.1, "UPDATE_SCORE_THRESH_TEST": 0.05, "MASK_THRESH_TEST": 0.5,
            "TOPK_CANDIDATES_TEST": 500, "NMS_KERNEL": "gaussian", "NMS_SIGMA": 2.0,
            "NMS_CLS_AGNOSTIC": False,
        },
    }
    weight_decay = 0.0001
    return {
        "LOGS": {"ROOT_DIR": "", "TRAIN": "train", "EVAL": "eval", "EXPORT": "export"},
        "SERVING_MODEL": {"FROZEN_GRAPH_FILE_NAME": "frozen_inference_graph.pb",
                          "INPUT_OUTPUT_TENSOR_PREFIX": "", "TYPE": "Detection",
                          "LABEL_OFFSET": 1},
        "BUILD_RECORDS": {"TYPE": "coco_pano", "ROOT_DIR": "", "TRAIN_NUM_SHARDS": 16,
                          "VAL_NUM_SHARDS": 16},
        "DATASETS": {"ROOT_DIR": "", "TRAIN": "train", "VAL": "val",
                     "CATEGORY_MAP_NAME": "category_map.json"},
        "EVAL": {"METRICS": ("coco_detection_metrics",), "NUM_EVAL": 5000,
                 "INCLUDE_METRICS_PER_CATEGORY": False, "ALL_METRICS_PER_CATEGORY": False,
                 "MAX_EXAMPLE_TO_DRAW": 100, "MIN_VISUALIZATION_SCORE_THRESH": 0.5,
                 "PASCAL_MATCHING_IOU_THRESH": 0.5, "CLASS_AGNOSTIC": False},
        "MODEL": model,
        "PRETRAINS": {"ROOT": "", "DETECTRON2": "", "ONLY_BACKBONE": False, "BACKBONE": "",
                      "WEIGHTS": "", "MMDET": "", "DARKNET": ""},
        "TRANSFORM": {"RESIZE": {"MIN_SIZE_TRAIN": (800,), "MAX_SIZE_TRAIN": 1333,
                                 "MIN_SIZE_TEST": 800, "MAX_SIZE_TEST": 1333,
                                 "USE_MINI_MASKS": True, "MINI_MASK_SIZE": 56}},
        "AUGMENT": {"HORIZONTAL_FLIP": False, "VERTICAL_FLIP": False, "ROTATE": False,
                    "ROTATE_BOTH_DIRECTION": False},
        "DATALOADER": {"NUM_READERS": 4, "READ_BLOCK_LENGTH": 1, "FILE_READ_BUFFER_SIZE": 8,
                       "SAMPLE_1_OF_N": 1, "SHUFFLE": True, "FILENAME_SHUFFLE_BUFFER_SIZE": 64,
                       "SHUFFLE_BUFFER_SIZE": 16, "NUM_PARALLEL_BATCHES": 4,
                       "NUM_PREFETCH_BATCHES": 2, "LOAD_SEMANTIC_MASKS": False},
        "SOLVER": {
            "LR_SCHEDULER_NAME": "WarmupMultiStepLR", "NUM_GPUS": 8, "IMS_PER_GPU": 2,
            "IMS_PER_BATCH": 16, "AUTO_SCALE_LR_SCHEDULE": True, "IMS_PER_BATCH_BASE": 16,
            "MAX_ITER": 40000, "SHORT_TERM_NUM_STEPS": 10000, "SHORT_TERM_SAVE_STEPS": 2000,
            "LONG_TERM_SAVE_STEPS": 10000, "BASE_LR": 0.001, "MOMENTUM": 0.9,
            "WEIGHT_DECAY": weight_decay, "WEIGHT_DECAY_NORM": 0.0, "GAMMA": 0.1,
            "STEPS": (30000,), "WARMUP_FACTOR": 1.0 / 1000, "WARMUP_ITERS": 1000,
            "WARMUP_METHOD": "linear", "CHECKPOINT_PERIOD": 5000, "BIAS_LR_FACTOR": 1.0,
            "WEIGHT_DECAY_BIAS": weight_decay, "CLIP_GRADIENTS_BY_NORM": 10.0,
        },
        "TEST": {"EXPECTED_RESULTS": [], "EVAL_PERIOD": 0, "KEYPOINT_OKS_SIGMAS": [],
                 "DETECTIONS_PER_IMAGE": 100,
                 "AUG": {"ENABLED": False,
                         "MIN_SIZES": (400, 500, 600, 700, 800, 900, 1000, 1100, 1200),
                         "MAX_SIZE": 4000, "FLIP": True},
                 "PRECISE_BN": {"ENABLED": False, "NUM_ITER": 200}},
        "OUTPUT_DIR": "./output",
        "SEED": -1,
        "CUDNN_BENCHMARK": False,
        "GLOBAL": {"HACK": 1.0},
    }


def get_cfg():
    """A fresh, mutable copy of the default configuration."""
    return CfgNode(_tree())
