"""Plain PyTorch fp32 restatement of ChessNet.forward -- TEST INFRASTRUCTURE ONLY.

Functional restatement of ai/model.py:51-77 (stem :58-59, ResidualBlock.forward
:19-25 over 5 blocks :61-62, policy head :64-66 with NCHW flatten, value head
:70-73) on CPU fp32, from a reference-keyed state_dict. Used as the numerics
oracle for the HIP kernels at arbitrary batch sizes (the golden fixtures pin it
to the reference module's own outputs).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

EPS = 1e-5


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def _cbr(x, sd, conv, bn, pad, relu=True):
    x = F.conv2d(x, _t(sd, conv + ".weight"), _t(sd, conv + ".bias"), padding=pad)
    x = F.batch_norm(x, _t(sd, bn + ".running_mean"), _t(sd, bn + ".running_var"), _t(sd, bn + ".weight"),
                     _t(sd, bn + ".bias"), training=False, eps=EPS)
    return F.relu(x) if relu else x


@torch.no_grad()
def forward(sd, planes):
    """planes: [B,12,8,8] float32 -> (policy [B,4096], value [B,1])."""
    x = planes if isinstance(planes, torch.Tensor) else torch.from_numpy(np.asarray(planes, dtype=np.float32))
    x = _cbr(x, sd, "conv1", "bn1", 1)
    x = _cbr(x, sd, "conv2", "bn2", 1)
    for i in range(5):
        p = f"res_blocks.{i}"
        r = x
        y = _cbr(x, sd, p + ".conv1", p + ".bn1", 1)
        y = _cbr(y, sd, p + ".conv2", p + ".bn2", 1, relu=False)
        y += r
        x = F.relu(y)
    pol = _cbr(x, sd, "policy_conv", "policy_bn", 0)
    pol = F.linear(torch.flatten(pol, 1), _t(sd, "policy_fc.weight"), _t(sd, "policy_fc.bias"))
    val = _cbr(x, sd, "value_conv", "value_bn", 0)
    val = val.view(val.size(0), -1)
    val = F.relu(F.linear(val, _t(sd, "value_fc1.weight"), _t(sd, "value_fc1.bias")))
    val = torch.tanh(F.linear(val, _t(sd, "value_fc2.weight"), _t(sd, "value_fc2.bias")))
    return pol, val


def make_eval_fn(sd):
    sdt = {k: _t(sd, k) for k in sd}

    def ev(planes):
        p, v = forward(sdt, planes)
        return p.numpy(), v.numpy().reshape(-1)
    return ev


def torch_softmax(logits):
    return torch.softmax(torch.from_numpy(np.asarray(logits, dtype=np.float32)), dim=0).numpy()


# ---------------------------------------------------------------- training --
def forward_train(params, planes):
    """Training-mode ChessNet.forward (ai/model.py:51-77, BatchNorm on batch
    statistics) over a dict of leaf tensors keyed like the reference's
    state_dict, in their dtype (float64 for the update-step oracle)."""
    def cbr(h, conv, bn, pad, relu=True):
        h = F.conv2d(h, params[conv + ".weight"], params[conv + ".bias"], padding=pad)
        h = F.batch_norm(h, None, None, params[bn + ".weight"], params[bn + ".bias"], training=True, eps=EPS)
        return F.relu(h) if relu else h
    x = cbr(planes, "conv1", "bn1", 1)
    x = cbr(x, "conv2", "bn2", 1)
    for i in range(5):
        p = f"res_blocks.{i}"
        y = cbr(cbr(x, p + ".conv1", p + ".bn1", 1), p + ".conv2", p + ".bn2", 1, relu=False)
        x = F.relu(y + x)
    pol = F.linear(torch.flatten(cbr(x, "policy_conv", "policy_bn", 0), 1), params["policy_fc.weight"],
                   params["policy_fc.bias"])
    val = torch.flatten(cbr(x, "value_conv", "value_bn", 0), 1)
    val = torch.tanh(F.linear(F.relu(F.linear(val, params["value_fc1.weight"], params["value_fc1.bias"])),
                              params["value_fc2.weight"], params["value_fc2.bias"]))
    return pol, val


def reference_epoch(sd, batches, lr, accumulate_steps, entropy_coef, clip=1.0, dtype=torch.float64, trace=None):
    """scripts/train.py _train_one_epoch (:126-196) restated on the CPU in
    `dtype`: per batch the loss of :169-176 (cross entropy + MSE - coef *
    entropy), NaN/Inf skip (:178-180), loss / accumulate_steps backward, and
    every accumulate_steps batches (or at the last) clip_grad_norm(1.0) + Adam
    step (GradScaler's scale / unscale is the identity in exact arithmetic).
    batches: list of (planes [B,12,8,8], moves [B], outcomes [B]).
    Returns (parameters after the epoch, per-batch losses, gradients of the
    first optimizer step after clipping). `trace` (a dict) also receives every
    step's clipped gradients ("grads") and the parameters after the first step
    ("after1")."""
    params = {k: torch.tensor(np.asarray(v), dtype=dtype).requires_grad_(True) for k, v in sd.items()
              if not (k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"))}
    opt = torch.optim.Adam(list(params.values()), lr=lr)
    opt.zero_grad()
    losses, first_grads = [], None
    n = len(batches)
    for i, (x, mv, oc) in enumerate(batches):
        pol, val = forward_train(params, torch.as_tensor(x, dtype=dtype))
        mv = torch.as_tensor(mv, dtype=torch.int64)
        oc = torch.as_tensor(oc, dtype=dtype)
        lp = F.cross_entropy(pol, mv)
        lv = F.mse_loss(val.squeeze(), oc)
        probs = F.softmax(pol, dim=1)
        ent = -(probs * F.log_softmax(pol, dim=1)).sum(dim=1).mean()
        loss = lp + lv - entropy_coef * ent
        if torch.isnan(loss) or torch.isinf(loss):
            continue
        (loss / accumulate_steps).backward()
        losses.append(float(loss))
        if (i + 1) % accumulate_steps == 0 or i == n - 1:
            torch.nn.utils.clip_grad_norm_(list(params.values()), max_norm=clip)
            if first_grads is None:
                first_grads = {k: p.grad.detach().clone() for k, p in params.items()}
            if trace is not None:
                trace.setdefault("grads", []).append({k: p.grad.detach().clone() for k, p in params.items()})
            opt.step()
            opt.zero_grad()
            if trace is not None and "after1" not in trace:
                trace["after1"] = {k: p.detach().clone() for k, p in params.items()}
    return {k: p.detach() for k, p in params.items()}, losses, first_grads
