from .reducer import BucketedAllReduce
from .trainer import Trainer, broadcast_parameters, get_world

__all__ = ["BucketedAllReduce", "Trainer", "broadcast_parameters", "get_world"]
