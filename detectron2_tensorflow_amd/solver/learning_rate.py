"""Piecewise-constant LR with linear warmup (lib/solver/learning_rate.py:4-39).

Evaluated on the host from the integer step (the step counter lives on the
host, so the LR never needs a device round trip)."""
import bisect


def warmup_factor_at_step(step, warmup_iters, warmup_factor):
    """learning_rate.py:28-39: linear ramp from warmup_factor to 1."""
    if step < warmup_iters:
        alpha = float(step) / float(warmup_iters)
        return warmup_factor * (1.0 - alpha) + alpha
    return 1.0


def build_learning_rate(cfg):
    """Returns lr(step).  AUTO_SCALE_LR_SCHEDULE scales the boundaries by
    IMS_PER_BATCH_BASE / IMS_PER_BATCH and the values by the inverse
    (learning_rate.py:8-16)."""
    s = cfg.SOLVER
    boundaries = [float(x) for x in s.STEPS]
    values = [s.BASE_LR * s.GAMMA ** i for i in range(len(boundaries) + 1)]
    if s.AUTO_SCALE_LR_SCHEDULE:
        factor = s.IMS_PER_BATCH / s.IMS_PER_BATCH_BASE
        boundaries = [x / factor for x in boundaries]
        values = [x * factor for x in values]

    def lr(step):
        # tf.train.piecewise_constant: values[i] for boundaries[i-1] < step <= boundaries[i]
        i = bisect.bisect_left(boundaries, float(step))
        return values[i] * warmup_factor_at_step(step, s.WARMUP_ITERS, s.WARMUP_FACTOR)

    return lr
