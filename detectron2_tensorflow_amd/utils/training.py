"""Module-global training phase (lib/utils/tf_utils.py:5-16)."""
_TRAINING = None


def get_training_phase():
    if _TRAINING is None:
        raise ValueError("you must set training phase!")
    return _TRAINING


def set_training_phase(training: bool):
    global _TRAINING
    _TRAINING = bool(training)
