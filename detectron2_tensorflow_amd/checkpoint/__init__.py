"""Weight conversion / loading: detectron2 state
dicts -> the reference's TF variable names (lib/convert_models/convert_d2.py)
-> this framework's parameters (Layer.reference_variables names)."""
from .convert_d2 import convert_weights
from .loader import load_detectron2_checkpoint, load_reference_weights, read_tensor_file

__all__ = ["convert_weights", "load_detectron2_checkpoint", "load_reference_weights",
           "read_tensor_file"]
