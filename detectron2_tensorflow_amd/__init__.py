"""MI355X-native detection hot path of SimeonZhang/detectron2_tensorflow.

ROIAlign, batched greedy NMS, anchor/top-k/decode and the FPN convs run as
hand-written HIP kernels for gfx950 (libd2mi_hip.so, C ABI in include/d2mi.h)
behind the reference's lib/layers op signatures and its registry/config
driven GeneralizedRCNN / SingleStageDetector meta-architectures.
"""
__version__ = "0.1.0"
