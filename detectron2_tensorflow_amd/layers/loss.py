"""smooth_l1_loss / sigmoid_focal_loss (lib/layers/loss.py:9-101)."""
import torch


def smooth_l1_loss(*, labels, predictions, beta, reduction="none"):
    n = (labels - predictions).abs()
    loss = n if beta < 1e-5 else torch.where(n < beta, 0.5 * n ** 2 / beta, n - 0.5 * beta)
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def sigmoid_focal_loss(*, labels, logits, alpha=-1, gamma=2, reduction="none"):
    p = torch.sigmoid(logits)
    ce = torch.nn.functional.binary_cross_entropy_with_logits(logits, labels, reduction="none")
    p_t = p * labels + (1 - p) * (1 - labels)
    loss = ce * ((1 - p_t) ** gamma)
    if alpha >= 0:
        loss = (alpha * labels + (1 - alpha) * (1 - labels)) * loss
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss
