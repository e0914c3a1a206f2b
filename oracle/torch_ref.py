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
