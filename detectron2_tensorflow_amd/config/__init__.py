from .config import CfgNode, restricted_eval
from .defaults import get_cfg
from .finalize import finalize

__all__ = ["CfgNode", "get_cfg", "finalize", "restricted_eval"]
