"""Completion checks for the gradient hand-offs between autograd nodes.

Several backwards in the training graph hand a gradient to another backward
instead of returning it (so that the receiver can add it inside its own
kernel epilogue, with no autograd add of two full maps):

* the bottleneck's residual / pair / three-consumer join hand-offs
  (layers/convolutional.py:_ConvMFMAFn, _join_backward);
* the RPN head conv <-> ROI pooler per-level hand-off (``_d2mi_grad_pair``,
  modeling/meta_arch/rcnn.py) and the box / mask pooler pair
  (ops._RoIAlignFn ``grad_share``);
* the RPN head's cross-level weight-gradient accumulator
  (modeling/proposal_generator/rpn.py:_RPNHead1x1Fn).

Each protocol assumes that every participant's backward runs in the same
backward pass.  A backward that reaches only some of them (torch.autograd.grad
or .backward on a subset of the losses, a loss that detaches one branch)
would otherwise drop the deposited gradient silently.  ``deposit`` queues an
engine callback that runs when the backward pass ends and raises if the
deposit is still there (clearing it first, so a later backward starts clean).
"""
import torch

_ENGINE = torch.autograd.Variable._execution_engine


class HandoffError(RuntimeError):
    pass


def _msg(what):
    return (f"gradient hand-off '{what}' was not completed in this backward pass: the "
            "fused training graph needs every loss that reaches the shared features in ONE "
            "backward (sum the losses, or build the model with the hand-offs disabled)")


def deposit(d, key, value, what):
    """d[key] = value, checked at the end of the current backward pass."""
    d[key] = value

    def check():
        if key in d:
            d.pop(key, None)
            raise HandoffError(_msg(what))

    _ENGINE.queue_callback(check)


def expect_complete(state, done, reset, what):
    """At the end of the current backward pass: if ``done(state)`` is false,
    ``reset(state)`` and raise (an accumulator whose last contribution never
    arrived)."""
    def check():
        if not done(state):
            reset(state)
            raise HandoffError(_msg(what))

    _ENGINE.queue_callback(check)
