"""Plain-PyTorch fp64 reference implementation of the FM math (test oracle).

Mirrors the reference semantics exactly:
* score:   cc/fm_scorer_op.h:132-136
* reg:     cc/fm_scorer_op.h:138 (per occurrence)
* loss:    tffm/fm_model.py:311-333 (weighted mean; logistic = sigmoid CE on logits)
* objective = loss + reg / batch_size_cfg   (fm_model.py:345-347)
* Adagrad: TF SparseApplyAdagrad on the touched rows (acc += g^2; p -= lr g / sqrt(acc))
"""

from __future__ import annotations

import torch


def fm_scores(params: torch.Tensor, offsets: torch.Tensor, ids: torch.Tensor, vals: torch.Tensor | None):
    """params: [V, K+1] reference layout (col 0 = w). Returns (pred[B], reg_v, reg_w) in params' dtype."""
    B = offsets.numel() - 1
    nnz = ids.numel()
    ex = torch.repeat_interleave(torch.arange(B), (offsets[1:] - offsets[:-1]).long())
    x = vals.to(params.dtype) if vals is not None else torch.ones(nnz, dtype=params.dtype)
    rows = params[ids.long()]
    w, v = rows[:, 0], rows[:, 1:]
    lin = torch.zeros(B, dtype=params.dtype).index_add(0, ex, x * w)
    xv = x[:, None] * v
    s1 = torch.zeros((B, v.shape[1]), dtype=params.dtype).index_add(0, ex, xv)
    s2 = torch.zeros((B, v.shape[1]), dtype=params.dtype).index_add(0, ex, xv * xv)
    pred = lin + 0.5 * (s1 * s1 - s2).sum(1)
    return pred, (v * v).sum(), (w * w).sum()


def fm_objective(params, batch, loss_type: str, factor_lambda=0.0, bias_lambda=0.0, batch_size_cfg=None,
                 grad_scale_mult: float = 1.0):
    vals = None if batch.vals is None else batch.vals.cpu()
    pred, rv, rw = fm_scores(params, batch.offsets.cpu(), batch.ids.cpu(), vals)
    y = batch.labels.cpu().to(params.dtype)
    wt = batch.weights.cpu().to(params.dtype) if batch.weights is not None else torch.ones_like(y)
    if loss_type == "mse":
        per = wt * (pred - y) ** 2
    else:
        per = wt * torch.nn.functional.binary_cross_entropy_with_logits(pred, y, reduction="none")
    loss = per.mean()
    reg = 0.5 * factor_lambda * rv + 0.5 * bias_lambda * rw
    bcfg = batch_size_cfg or batch.B
    return (loss + reg / bcfg) * grad_scale_mult, loss, pred


def adagrad_step(params, acc, grad, lr):
    """Sparse Adagrad: only rows with a nonzero gradient row (touched rows) change."""
    touched = (grad != 0).any(dim=1)
    acc = acc.clone()
    params = params.clone()
    acc[touched] += grad[touched] ** 2
    params[touched] -= lr * grad[touched] / acc[touched].sqrt()
    return params, acc


def touched_rows(batch, V):
    t = torch.zeros(V, dtype=torch.bool)
    t[batch.ids.cpu().long()] = True
    return t


def reference_train_step(params, acc, batch, loss_type, lr, factor_lambda=0.0, bias_lambda=0.0,
                         batch_size_cfg=None):
    """One reference training step in fp64; returns (new_params, new_acc, loss)."""
    p = params.clone().requires_grad_(True)
    obj, loss, _ = fm_objective(p, batch, loss_type, factor_lambda, bias_lambda, batch_size_cfg)
    (g,) = torch.autograd.grad(obj, p)
    t = touched_rows(batch, params.shape[0])
    newp, newacc = params.clone(), acc.clone()
    newacc[t] += g[t] ** 2
    newp[t] -= lr * g[t] / newacc[t].sqrt()
    return newp, newacc, float(loss)


def ftrl_step(params, n, z, grad, touched, alpha, l1, l2, beta=0.0):
    p, n, z = params.clone(), n.clone(), z.clone()
    g = grad[touched]
    n_new = n[touched] + g * g
    sigma = (n_new.sqrt() - n[touched].sqrt()) / alpha
    z[touched] += g - sigma * p[touched]
    n[touched] = n_new
    quad = (beta + n_new.sqrt()) / alpha + 2 * l2
    zt = z[touched]
    p[touched] = torch.where(zt.abs() > l1, (torch.sign(zt) * l1 - zt) / quad, torch.zeros_like(zt))
    return p, n, z
