"""Op-level API with the reference's signatures (tffm/fm_ops.py:30-56).

* ``fm_parser(data_strings, vocab_size, hash_feature_id=False)``
    -> (labels f32[B], sizes i32[B], feature_ids i64[nnz], feature_vals f32[nnz])
* ``fm_scorer(feature_ids, feature_params, feature_vals, feature_poses, factor_lambda, bias_lambda)``
    -> (pred_score f32[B], reg_score f32[])  -- differentiable w.r.t.
    ``feature_params`` ([U, K+1], column 0 = w); the backward is the FmGrad
    equivalent (reference gradient registration: tffm/fm_ops.py:11-27).

These are convenience/parity entry points (tests, notebooks).  The training
step does not go through autograd: models/fm.py fuses loss, backward and the
optimizer into the native kernels.
"""

from __future__ import annotations

import torch

from . import kernels as K
from . import native


def fm_parser(data_strings, vocab_size: int, hash_feature_id: bool = False, threads: int = 1):
    """libsvm lines -> CSR (reference FmParser, cc/fm_parser_op.cc). Raises ValueError like the TF op."""
    if isinstance(data_strings, (str, bytes)):
        data_strings = [data_strings]
    labels, sizes, ids, vals = native.cpu().parse_lines(list(data_strings), int(vocab_size), bool(hash_feature_id),
                                                        int(threads))
    return (torch.from_numpy(labels), torch.from_numpy(sizes), torch.from_numpy(ids), torch.from_numpy(vals))


def string_to_hash_bucket(strings, num_buckets: int) -> torch.Tensor:
    """Equivalent of tf.string_to_hash_bucket (TF Hash64 % num_buckets)."""
    return torch.from_numpy(native.cpu().hash_bucket(list(strings), int(num_buckets)))


def _pack(params: torch.Tensor, K_: int):
    Kp = K.padded_k(K_, torch.float32)
    v = torch.zeros((params.shape[0], Kp), dtype=torch.float32, device=params.device)
    v[:, :K_] = params[:, 1:].to(torch.float32)
    w = params[:, 0].to(torch.float32).contiguous()
    return v, w, Kp


class _FmScorer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feature_ids, feature_params, feature_vals, feature_poses, factor_lambda, bias_lambda):
        K_ = feature_params.shape[1] - 1
        v, w, Kp = _pack(feature_params.detach(), K_)
        ids = feature_ids.to(torch.int32).contiguous()
        poses = feature_poses.to(torch.int32).contiguous()
        vals = feature_vals.to(torch.float32).contiguous()
        fo = K.fm_forward(poses, ids, vals, v, w, Kp, want_r1=True, want_reg=True)
        reg = 0.5 * factor_lambda * fo.regv + 0.5 * bias_lambda * fo.regw
        ctx.save_for_backward(ids, vals, poses, v, w, fo.r1)
        ctx.lam = (float(factor_lambda), float(bias_lambda))
        ctx.shape = feature_params.shape
        ctx.dtype = feature_params.dtype
        ctx.Kp = Kp
        return fo.pred, reg.to(feature_params.device)

    @staticmethod
    def backward(ctx, pred_grad, reg_grad):
        ids, vals, poses, v, w, r1 = ctx.saved_tensors
        lf, lb = ctx.lam
        Kp = ctx.Kp
        U, K1 = ctx.shape
        dev = ids.device
        if pred_grad is None:
            pred_grad = torch.zeros(poses.numel() - 1, dtype=torch.float32, device=dev)
        rg = 0.0 if reg_grad is None else float(reg_grad)
        ex = K.csr_rows(poses, nnz=ids.numel())
        dd = K.dedup(ids, key_bits=32, ex_of_occ=ex, vals=vals)
        n = dd.sync()
        grad_rows = torch.zeros((max(n, 1), Kp + 4), dtype=torch.float32, device=dev)
        src = torch.zeros((max(n, 1), Kp + 4), dtype=torch.float32, device=dev)
        uniq = dd.uniq[:n].to(torch.int64)
        src[:n, :Kp] = v[uniq]
        src[:n, Kp] = w[uniq]
        K.fm_backward(dd, pred_grad.to(torch.float32).contiguous(), r1, Kp, mode=K.BWD_EMIT, src_v=src[:, :Kp],
                      src_w=src[:, Kp], grad_out=grad_rows, reg_v=lf * rg, reg_w=lb * rg)
        out = torch.zeros((U, K1), dtype=torch.float32, device=dev)
        out[uniq, 0] = grad_rows[:n, Kp]
        out[uniq, 1:] = grad_rows[:n, : K1 - 1]
        return None, out.to(ctx.dtype), None, None, None, None


def fm_scorer(feature_ids, feature_params, feature_vals, feature_poses, factor_lambda=0.0, bias_lambda=0.0):
    """FM forward on locally-indexed params (reference FmScorer). Returns (pred_score, reg_score)."""
    return _FmScorer.apply(torch.as_tensor(feature_ids), feature_params, torch.as_tensor(feature_vals),
                           torch.as_tensor(feature_poses), float(factor_lambda), float(bias_lambda))
