"""smooth_l1_loss / sigmoid_focal_loss / dice_loss (lib/layers/loss.py:9-136)."""
import torch


def smooth_l1_loss(*, labels, predictions, beta, reduction="none"):
    n = (labels - predictions).abs()
    loss = n if beta < 1e-5 else torch.where(n < beta, 0.5 * n ** 2 / beta, n - 0.5 * beta)
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def sigmoid_focal_loss(*, predictions, targets, alpha=-1.0, gamma=2.0, reduction="none",
                       scope=None):
    """loss.py:59-101 (the reference's keyword names; scope is TF's name scope)."""
    del scope
    p = torch.sigmoid(predictions)
    ce = torch.nn.functional.binary_cross_entropy_with_logits(predictions, targets,
                                                              reduction="none")
    p_t = p * targets + (1 - p) * (1 - targets)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * targets + (1 - alpha) * (1 - targets)) * loss
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def dice_loss(*, predictions, targets, reduction="none", scope=None):
    """loss.py:104-136: per row (everything after axis 0 flattened)
    1 - 2 sum(p t) / (sum(p p) + sum(t t) + 1e-5); an empty input gives 0."""
    del scope
    if predictions.numel() == 0:
        loss = predictions.new_zeros(())
    else:
        p = predictions.reshape(predictions.shape[0], -1)
        t = targets.reshape(targets.shape[0], -1).to(p.dtype)
        a = (p * t).sum(1)
        b = (p * p).sum(1)
        c = (t * t).sum(1)
        loss = 1 - (2 * a) / (b + c + 1e-5)
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss
