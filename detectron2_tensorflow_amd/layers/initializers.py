"""TF 1.x initializers used by the reference layers, as torch in-place fills.

variance_scaling(scale, mode, distribution) follows tf.variance_scaling_initializer:
n = fan_in / fan_out / their mean; 'truncated_normal' (TF's default for the
1.x variance_scaling) uses stddev = sqrt(scale / n) / 0.87962566103423978 and
re-draws beyond 2 stddev, 'untruncated_normal' / 'normal' stddev = sqrt(scale / n),
'uniform' limit = sqrt(3 * scale / n).  Fans of a conv kernel [kh, kw, in, out]
are kh*kw*in and kh*kw*out (tf's _compute_fans).
"""
import math

import torch


def _fans(shape):
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = 1
    for d in shape[:-2]:
        receptive *= d
    return shape[-2] * receptive, shape[-1] * receptive


class variance_scaling:
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal"):
        self.scale, self.mode, self.distribution = float(scale), mode, distribution

    def __call__(self, t, generator=None):
        fan_in, fan_out = _fans(tuple(t.shape))
        n = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2.0}[self.mode]
        n = max(1.0, n)
        with torch.no_grad():
            if self.distribution in ("truncated_normal",):
                std = math.sqrt(self.scale / n) / 0.87962566103423978
                t.normal_(0.0, std, generator=generator)
                bad = t.abs() > 2 * std
                while bool(bad.any()):
                    t[bad] = torch.empty(int(bad.sum()), device=t.device).normal_(0.0, std, generator=generator)
                    bad = t.abs() > 2 * std
            elif self.distribution in ("untruncated_normal", "normal"):
                t.normal_(0.0, math.sqrt(self.scale / n), generator=generator)
            elif self.distribution == "uniform":
                lim = math.sqrt(3.0 * self.scale / n)
                t.uniform_(-lim, lim, generator=generator)
            else:
                raise ValueError(f"unknown distribution {self.distribution}")
        return t


class random_normal:
    def __init__(self, stddev=1.0, mean=0.0):
        self.stddev, self.mean = float(stddev), float(mean)

    def __call__(self, t, generator=None):
        with torch.no_grad():
            return t.normal_(self.mean, self.stddev, generator=generator)


class constant:
    def __init__(self, value=0.0):
        self.value = float(value)

    def __call__(self, t, generator=None):
        with torch.no_grad():
            return t.fill_(self.value)


def zeros():
    return constant(0.0)


def ones():
    return constant(1.0)
