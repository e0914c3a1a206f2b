"""Autograd ops of the update step on the HIP training kernels (csrc/kv_train.hip,
include/kv.h "train" section).

The reference trains ChessNet under torch.cuda.amp.autocast
(scripts/train.py:161-184): the tower's 3x3 convolutions (ai/model.py:34-40,
:8-25) run on fp16 operands with fp32 accumulation and fp16 outputs, and its
BatchNorms in training mode. `tower_forward` restates the tower's training
forward (conv1 -> bn1 -> relu -> conv2 -> bn2 -> relu -> 5 residual blocks)
on those kernels with NHWC fp16 activations [boards, 64 squares, C]:

  * Conv3x3: forward = kv_tr_conv3x3_f16; backward = the same kernel on dy
    with the flipped weight image (data gradient) + kv_tr_conv3x3_wgrad_f16
    (weight gradient, rounded to fp16 as the autocast conv's is) and the
    channel sums of dy (bias gradient);
  * BNAct: training BatchNorm (batch statistics) + optional residual add +
    ReLU, in the reference's rounding order; backward in one reduction and
    one elementwise kernel. Running statistics are updated as
    nn.BatchNorm2d does (momentum, unbiased variance);
  * fusions across the two (FUSE, on by default): the BatchNorm backward
    also sums its dx per channel -- the producing conv's bias gradient, so
    dy is not read a second time -- and hands it to that conv through a
    shared dict; a residual block's second BatchNorm hands the residual
    branch's gradient to the block's first conv, whose data-gradient kernel
    adds it in its epilogue, rounded as autograd's fp16 accumulation of the
    two would be (the same bits, one fewer pass over the activations);
  * Head1x1: the heads' policy / value 1x1 convolutions over the tower output.

Only the fp16 autocast path runs here; an fp32 (autocast off) update uses the
PyTorch-ROCm ops (model.ChessNet._train_forward).
"""
from __future__ import annotations

import torch

from . import _lib

STEM_CI = 64  # encode_board's 12 planes padded to the weight-gradient kernel's 64-channel tile
FUSE = True   # the BatchNorm -> conv backward fusions (module docstring); False: separate passes

_ws = {}


def _workspace(device, nbytes: int) -> torch.Tensor:
    """A cached device byte buffer of at least nbytes (one per device; every op
    runs on the current stream in order, so one buffer serves them all)."""
    key = device.index if device.index is not None else 0
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def planes_to_nhwc(planes: torch.Tensor, cpad: int = STEM_CI) -> torch.Tensor:
    """encode_board planes fp32 [n,12,8,8] -> NHWC fp16 [n,64,cpad] (zero channels >= 12)."""
    planes = planes.to(torch.float32).contiguous()
    n = planes.shape[0]
    out = torch.empty((n, 64, cpad), dtype=torch.float16, device=planes.device)
    _lib.check(_lib.lib().kv_tr_planes_to_nhwc(planes.data_ptr(), n, cpad, out.data_ptr(), _stream(planes)),
               "kv_tr_planes_to_nhwc")
    return out


def conv_weight_images(weight: torch.Tensor, ci: int, flipped: bool):
    """fp32 [co, ci_real, 3, 3] -> fp16 [co, 9, ci] (and the flipped [ci, 9, co] image)."""
    w = weight.detach().to(torch.float32).contiguous()
    co, ci_real = w.shape[0], w.shape[1]
    wf = torch.empty((co, 9, ci), dtype=torch.float16, device=w.device)
    wt = torch.empty((ci, 9, co), dtype=torch.float16, device=w.device) if flipped else None
    _lib.check(_lib.lib().kv_tr_conv_weights_f16(w.data_ptr(), co, ci_real, ci, wf.data_ptr(), _ptr(wt), _stream(w)),
               "kv_tr_conv_weights_f16")
    return wf, wt


def conv3x3_f16(x: torch.Tensor, wf: torch.Tensor, bias32, add=None) -> torch.Tensor:
    """Raw kernel call: x fp16 [n,64,ci], wf fp16 [co,9,ci] -> fp16 [n,64,co] (+ fp16 `add`, fused)."""
    n, _, ci = x.shape
    co = wf.shape[0]
    y = torch.empty((n, 64, co), dtype=torch.float16, device=x.device)
    if add is not None:
        assert add.dtype == torch.float16 and add.shape == y.shape and add.is_contiguous()
    _lib.check(_lib.lib().kv_tr_conv3x3_add_f16(x.data_ptr(), n, ci, wf.data_ptr(), _ptr(bias32), co, _ptr(add),
                                                y.data_ptr(), _stream(x)), "kv_tr_conv3x3_f16")
    return y


def conv3x3_wgrad_f16(dy: torch.Tensor, x: torch.Tensor, ci_real: int) -> torch.Tensor:
    """dw fp32 [co, ci_real, 3, 3] (fp16-rounded values) of y = conv3x3(x, w)."""
    n, _, co = dy.shape
    ci = x.shape[2]
    L = _lib.lib()
    nbytes = L.kv_tr_wgrad_workspace(n, ci, co, None)
    ws = _workspace(dy.device, nbytes)
    dw = torch.empty((co, ci_real, 3, 3), dtype=torch.float32, device=dy.device)
    _lib.check(L.kv_tr_conv3x3_wgrad_f16(dy.data_ptr(), x.data_ptr(), n, ci, ci_real, co, dw.data_ptr(),
                                         ws.data_ptr(), ws.numel(), _stream(dy)), "kv_tr_conv3x3_wgrad_f16")
    return dw


def channel_sum_f16(t: torch.Tensor) -> torch.Tensor:
    rows, C = t.shape[0] * t.shape[1], t.shape[2]
    L = _lib.lib()
    ws = _workspace(t.device, L.kv_tr_bn_workspace(rows, C))
    out = torch.empty(C, dtype=torch.float32, device=t.device)
    _lib.check(L.kv_tr_channel_sum_f16(t.data_ptr(), rows, C, out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(t)),
               "kv_tr_channel_sum_f16")
    return out


class Conv3x3(torch.autograd.Function):
    """y fp16 [n,64,co] = conv3x3(x fp16 [n,64,ci], weight fp32 [co,ci_real,3,3]) + bias, as an
    autocast fp16 convolution (weight and bias rounded to fp16, fp32 accumulation).
    bias_link: dict the consuming BNAct's backward leaves the bias gradient in ("db");
    dx_link: dict a residual BNAct's backward leaves x's other gradient in ("dres"), added to dx here."""

    @staticmethod
    def forward(ctx, x, weight, bias, need_dx: bool, bias_link=None, dx_link=None):
        x = x.contiguous()
        ci = x.shape[2]
        wf, wt = conv_weight_images(weight, ci, need_dx)
        b32 = bias.detach().to(torch.float16).to(torch.float32).contiguous() if bias is not None else None
        y = conv3x3_f16(x, wf, b32)
        ctx.save_for_backward(x, wt)
        ctx.need_dx = need_dx
        ctx.ci_real = weight.shape[1]
        ctx.has_bias = bias is not None
        ctx.links = (bias_link, dx_link)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        bias_link, dx_link = ctx.links
        dy = dy.to(torch.float16).contiguous()
        dres = dx_link.pop("dres", None) if dx_link is not None else None
        dx = None
        if ctx.need_dx and ctx.needs_input_grad[0]:
            dx = conv3x3_f16(dy, wt, None, dres)
        elif dres is not None and ctx.needs_input_grad[0]:
            dx = dres
        dw = conv3x3_wgrad_f16(dy, x, ctx.ci_real) if ctx.needs_input_grad[1] else None
        db = bias_link.pop("db", None) if bias_link is not None else None
        if db is None and ctx.has_bias and ctx.needs_input_grad[2]:
            db = channel_sum_f16(dy)
        if db is not None:
            db = db.to(torch.float16).to(torch.float32)
        return dx, dw, db, None, None, None


class BNAct(torch.autograd.Function):
    """Training BatchNorm over boards x squares of fp16 x [n,64,C] (+ fp16 residual) (+ ReLU) -> fp16.
    `stats` (a list) receives (mean, biased var) for the running-statistics update.
    bias_link: the producing Conv3x3's dict -- the backward leaves the channel sums of dx there ("db");
    res_link: the dict of the Conv3x3 that consumes `res` -- the backward leaves res's gradient there
    ("dres") for that conv's data-gradient kernel to add, and returns none of its own."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, relu: bool, eps: float, stats: list, bias_link=None, res_link=None):
        x = x.contiguous()
        n, _, C = x.shape
        rows = n * 64
        L = _lib.lib()
        st = _stream(x)
        ws = _workspace(x.device, L.kv_tr_bn_workspace(rows, C))
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        var = torch.empty_like(mean)
        invstd = torch.empty_like(mean)
        _lib.check(L.kv_tr_bn_stats_f16(x.data_ptr(), rows, C, float(eps), mean.data_ptr(), var.data_ptr(),
                                        invstd.data_ptr(), ws.data_ptr(), ws.numel(), st), "kv_tr_bn_stats_f16")
        g32 = gamma.detach().to(torch.float32).contiguous()
        b32 = beta.detach().to(torch.float32).contiguous()
        r = res.contiguous() if res is not None else None
        y = torch.empty_like(x)
        _lib.check(L.kv_tr_bn_apply_f16(x.data_ptr(), rows, C, mean.data_ptr(), invstd.data_ptr(), g32.data_ptr(),
                                        b32.data_ptr(), _ptr(r), int(relu), y.data_ptr(), st), "kv_tr_bn_apply_f16")
        stats.append((mean, var))
        ctx.save_for_backward(x, y, mean, invstd, g32)
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.links = (bias_link, res_link)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd, g32 = ctx.saved_tensors
        dy = dy.to(torch.float16).contiguous()
        n, _, C = x.shape
        rows = n * 64
        L = _lib.lib()
        ws = _workspace(x.device, L.kv_tr_bn_workspace(rows, C))
        dx = torch.empty_like(x)
        bias_link, res_link = ctx.links
        dres = torch.empty_like(x) if ctx.has_res else None
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
        dbeta = torch.empty_like(dgamma)
        dxsum = torch.empty_like(dgamma) if bias_link is not None else None
        _lib.check(L.kv_tr_bn_backward_f16(x.data_ptr(), dy.data_ptr(), y.data_ptr(), rows, C, int(ctx.relu),
                                           mean.data_ptr(), invstd.data_ptr(), g32.data_ptr(), dgamma.data_ptr(),
                                           dbeta.data_ptr(), dx.data_ptr(), _ptr(dres), _ptr(dxsum), ws.data_ptr(),
                                           ws.numel(), _stream(x)), "kv_tr_bn_backward_f16")
        if dxsum is not None:
            bias_link["db"] = dxsum
        if dres is not None and res_link is not None:
            res_link["dres"] = dres
            dres = None
        return dx, dgamma, dbeta, dres, None, None, None, None, None


class Head1x1(torch.autograd.Function):
    """The heads' 1x1 convolutions (policy 512 -> 2, value 512 -> 1; ai/model.py:42-49) as autocast
    fp16 ops over the tower output h fp16 [n,64,512] -> fp16 [n,64,4] (columns 0-1 policy, 2 value)."""

    @staticmethod
    def forward(ctx, h, wp, bp, wv, bv):
        h = h.contiguous()
        n = h.shape[0]
        w16 = torch.cat([wp.detach().reshape(2, 512), wv.detach().reshape(1, 512)]).to(torch.float16).contiguous()
        b32 = torch.cat([bp.detach(), bv.detach()]).to(torch.float16).to(torch.float32).contiguous()
        out = torch.empty((n, 64, 4), dtype=torch.float16, device=h.device)
        _lib.check(_lib.lib().kv_tr_head1x1_f16(h.data_ptr(), n * 64, w16.data_ptr(), b32.data_ptr(), out.data_ptr(),
                                                _stream(h)), "kv_tr_head1x1_f16")
        ctx.save_for_backward(h, w16)
        return out

    @staticmethod
    def backward(ctx, dout):
        h, w16 = ctx.saved_tensors
        dout = dout.to(torch.float16).contiguous()
        n = h.shape[0]
        L = _lib.lib()
        ws = _workspace(h.device, L.kv_tr_head1x1_workspace(n * 64))
        dh = torch.empty_like(h)
        dw = torch.empty((3, 512), dtype=torch.float32, device=h.device)
        db = torch.empty(3, dtype=torch.float32, device=h.device)
        _lib.check(L.kv_tr_head1x1_backward_f16(h.data_ptr(), dout.data_ptr(), n * 64, w16.data_ptr(), dh.data_ptr(),
                                                dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(), _stream(h)),
                   "kv_tr_head1x1_backward_f16")
        return dh, dw[:2].reshape(2, 512, 1, 1), db[:2].clone(), dw[2:].reshape(1, 512, 1, 1), db[2:].clone()


def update_running_stats(bn: torch.nn.BatchNorm2d, mean: torch.Tensor, var: torch.Tensor, count: int):
    """nn.BatchNorm2d's running-statistics update from a training batch of `count` values per channel."""
    if not bn.track_running_stats:
        return
    with torch.no_grad():
        bn.num_batches_tracked.add_(1)
        mom = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
        bn.running_mean.mul_(1 - mom).add_(mean, alpha=mom)
        bn.running_var.mul_(1 - mom).add_(var * (count / max(count - 1, 1)), alpha=mom)


def conv_bn_act(x, conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, res=None, need_dx: bool = True,
                dx_link=None, res_link=None):
    """relu(bn(conv(x)) [+ res]) on the HIP kernels (training mode). dx_link / res_link: the
    residual-gradient hand-over (BNAct, Conv3x3)."""
    bias_link = {} if FUSE else None
    y = Conv3x3.apply(x, conv.weight, conv.bias, need_dx, bias_link, dx_link)
    stats = []
    out = BNAct.apply(y, bn.weight, bn.bias, res, True, bn.eps, stats, bias_link, res_link)
    update_running_stats(bn, stats[0][0], stats[0][1], y.shape[0] * 64)
    return out


def tower_forward(net, planes: torch.Tensor) -> torch.Tensor:
    """ChessNet's tower in training mode (ai/model.py:58-62) under autocast fp16:
    planes fp32 [n,12,8,8] -> NHWC fp16 [n,64,512] (the input of both heads)."""
    x = planes_to_nhwc(planes)
    h = conv_bn_act(x, net.conv1, net.bn1, need_dx=False)
    h = conv_bn_act(h, net.conv2, net.bn2)
    for blk in net.res_blocks:
        link = {} if FUSE else None  # bn2's residual gradient -> conv1's data gradient (both take h)
        a = conv_bn_act(h, blk.conv1, blk.bn1, dx_link=link)
        h = conv_bn_act(a, blk.conv2, blk.bn2, res=h, res_link=link)
    return h
