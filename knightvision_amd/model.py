"""ChessNet: drop-in for ai/model.py ChessNet (same parameter names, shapes and
state_dict keys, ai/model.py:31-49), whose forward runs on the hand-written
HIP kernels of libkv.so (knightvision_amd/csrc/kv_nn.hip).

forward(x[N,12,8,8]) -> (policy logits [N,4096], value [N,1]). In eval mode
(the self-play path always calls model.eval(), self_play.py:77, :108) the
forward is the HIP tower with BN folded; in train mode under autocast fp16 on a
GPU (the reference's update step, train.py:161-184) the tower runs on the HIP
training kernels (train_ops.py: fp16 implicit-GEMM convolutions, training
BatchNorm) with the heads as PyTorch ops; otherwise (fp32, CPU) it is
PyTorch autograd over the same parameters. The module keeps torch Parameters so checkpoints
load and save exactly like the reference's; the kernels read a BN-folded packed
copy that is rebuilt whenever a parameter or BN statistic changes.
"""
from __future__ import annotations

import os

import ctypes as C

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .weights import pack_weights, state_dict_to_numpy


# KV_PREC_* / KV_ALGO_* (include/kv.h). fp32 + auto: the conv path is chosen per weight load by the
# library's calibration against an fp64 forward (KVNet.calibration()); f64w: the fp64 Winograd domain.
PRECISIONS = {"fp32": 0, "f64w": 4, "i8x5": 5, "i8r4": 6}  # 3 (f16x3) retired in round 6
ALGOS = {"auto": 0, "direct": 1, "winograd88": 4, "winograd88i8": 5, "winograd88i8v": 6,
         "winograd88i8r3": 7}  # 3 (winograd48, F(4x8)) retired in round 6


def batch_norm_rows(bn: nn.BatchNorm2d, x, n_real=None, explicit: bool = False):
    """Training-mode BatchNorm2d whose batch statistics (and running-statistics
    update) cover only the first n_real rows -- the rows after them are padding
    that gives the update step a bucketed batch shape (knightvision_amd.train);
    those rows are normalised with the real rows' statistics and carry no loss.
    n_real None / = batch: the module itself, unless `explicit` (the same
    arithmetic as elementwise torch ops: MIOpen compiles a BatchNorm kernel for
    every new batch shape, tens of seconds on a fresh machine)."""
    if not explicit and (n_real is None or n_real >= x.shape[0]) or not bn.training:
        return bn(x)
    if n_real is None:
        n_real = x.shape[0]
    acc = torch.float32 if x.dtype in (torch.float16, torch.bfloat16) else x.dtype  # statistics at >= fp32
    xr = x[:n_real].to(acc)
    mean = xr.mean(dim=(0, 2, 3))
    var = xr.var(dim=(0, 2, 3), unbiased=False)
    if bn.track_running_stats:
        with torch.no_grad():
            cnt = xr.numel() // xr.shape[1]
            bn.num_batches_tracked.add_(1)
            mom = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
            bn.running_mean.mul_(1 - mom).add_(mom * mean)
            bn.running_var.mul_(1 - mom).add_(mom * var * (cnt / max(cnt - 1, 1)))
    inv = torch.rsqrt(var + bn.eps)
    y = (x.to(acc) - mean[None, :, None, None]) * (inv * bn.weight.to(acc))[None, :, None, None] \
        + bn.bias.to(acc)[None, :, None, None]
    return y.to(x.dtype)


# MIOpen runs these 8x8 convolutions well up to ~1024 images per call and
# several times slower above (measured per update step: 21 ms at 1024, 272 ms at
# 4096): convolution is per image, so training-mode calls are split into chunks
# of CONV_CHUNK images (BatchNorm still sees the whole batch).
CONV_CHUNK = int(os.getenv("KV_TRAIN_CONV_CHUNK", "1024"))


# Update step under autocast fp16 on a GPU: "hip" = the tower on the HIP
# training kernels (train_ops), "miopen" = PyTorch-ROCm's MIOpen convolutions.
TRAIN_BACKEND = os.getenv("KV_TRAIN_BACKEND", "hip")


def _autocast_on() -> bool:
    try:
        return torch.is_autocast_enabled("cuda")
    except TypeError:  # older signature
        return torch.is_autocast_enabled()


def conv_chunked(conv: nn.Conv2d, x):
    if CONV_CHUNK <= 0 or x.shape[0] <= CONV_CHUNK or not x.is_cuda:
        return conv(x)
    return torch.cat([conv(c) for c in x.split(CONV_CHUNK)])


class ResidualBlock(nn.Module):
    """One residual block (ai/model.py:8-25). Its own forward is the training
    path only; evaluation runs the whole tower in libkv.so."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(channels)
        self.conv2 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn2 = nn.BatchNorm2d(channels)

    def forward(self, x, n_real=None):
        y = batch_norm_rows(self.bn1, conv_chunked(self.conv1, x), n_real)
        y = batch_norm_rows(self.bn2, conv_chunked(self.conv2, F.relu(y)), n_real)
        return F.relu(y + x)


class KVNet:
    """Owner of one kv_net (device weights + workspace) on one GPU."""

    def __init__(self, device_index: int, packed: np.ndarray, precision: str = "fp32", algo: str = "auto"):
        L = _lib.lib()
        if packed.size != L.kv_net_packed_size():
            raise _lib.KVError(f"packed weights have {packed.size} floats, library expects {L.kv_net_packed_size()}")
        self.device_index = device_index
        h = C.c_void_p()
        _lib.check(L.kv_net_create(device_index, C.byref(h)), "kv_net_create")
        self.h = h
        _lib.check(L.kv_net_set_precision(self.h, PRECISIONS[precision]), "kv_net_set_precision")
        _lib.check(L.kv_net_set_algo(self.h, ALGOS[algo]), "kv_net_set_algo")
        p = np.ascontiguousarray(packed, dtype=np.float32)
        _lib.check(L.kv_net_load(self.h, p.ctypes.data_as(C.POINTER(C.c_float)), p.size), "kv_net_load")

    def calibration(self) -> dict:
        """The conv paths this net runs (> 16 / <= 16 boards) and, for fp32 + auto, the load-time
        calibration's measured errors against the fp64 forward (kv_net_calibration)."""
        c = _lib.Calib()
        _lib.check(_lib.lib().kv_net_calibration(self.h, C.byref(c)), "kv_net_calibration")
        return _lib.calib_dict(c)

    def forward_planes(self, x: torch.Tensor):
        """x: CUDA fp32 [B,12,8,8] -> (policy [B,4096], value [B,1])."""
        B = x.shape[0]
        x = x.contiguous()
        pol = torch.empty((B, 4096), dtype=torch.float32, device=x.device)
        val = torch.empty((B, 1), dtype=torch.float32, device=x.device)
        st = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(_lib.lib().kv_net_forward(self.h, x.data_ptr(), B, pol.data_ptr(), val.data_ptr(), st),
                   "kv_net_forward")
        return pol, val

    def forward_boards(self, boards: torch.Tensor):
        """boards: CUDA int8 [B,64] piece codes -> (policy [B,4096], value [B,1])."""
        B = boards.shape[0]
        boards = boards.contiguous()
        pol = torch.empty((B, 4096), dtype=torch.float32, device=boards.device)
        val = torch.empty((B, 1), dtype=torch.float32, device=boards.device)
        st = torch.cuda.current_stream(boards.device).cuda_stream
        _lib.check(_lib.lib().kv_net_forward_boards(self.h, boards.data_ptr(), B, pol.data_ptr(), val.data_ptr(), st),
                   "kv_net_forward_boards")
        return pol, val

    def forward_boards_legal(self, boards: torch.Tensor, moves: torch.Tensor, n_moves: torch.Tensor):
        """boards int8 [B,64], moves uint16-as-int16 [B,maxm] (from | to << 6), n_moves int32 [B], all CUDA ->
        (legal logits [B,maxm], value [B,1]): only the listed moves' logits (kv_net_forward_boards_legal)."""
        B, maxm = moves.shape
        boards, moves, n_moves = boards.contiguous(), moves.contiguous(), n_moves.contiguous()
        out = torch.zeros((B, maxm), dtype=torch.float32, device=boards.device)
        val = torch.empty((B, 1), dtype=torch.float32, device=boards.device)
        st = torch.cuda.current_stream(boards.device).cuda_stream
        _lib.check(_lib.lib().kv_net_forward_boards_legal(self.h, boards.data_ptr(), B, moves.data_ptr(),
                                                          n_moves.data_ptr(), maxm, out.data_ptr(), val.data_ptr(),
                                                          st), "kv_net_forward_boards_legal")
        return out, val

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().kv_net_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ChessNet(nn.Module):
    """ai/model.py:27-77 ChessNet with the HIP forward."""

    def __init__(self, verbose: bool = False, precision: str = "fp32", algo: str = "auto"):
        super().__init__()
        self.verbose = verbose
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {list(PRECISIONS)}")
        if algo not in ALGOS:
            raise ValueError(f"algo must be one of {list(ALGOS)}")
        self.precision = precision
        self.algo = algo
        self.conv1 = nn.Conv2d(12, 256, kernel_size=3, padding=1)
        self.bn1 = nn.BatchNorm2d(256)
        self.conv2 = nn.Conv2d(256, 512, kernel_size=3, padding=1)
        self.bn2 = nn.BatchNorm2d(512)
        self.res_blocks = nn.ModuleList([ResidualBlock(512) for _ in range(5)])
        self.policy_conv = nn.Conv2d(512, 2, kernel_size=1)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_fc = nn.Linear(2 * 8 * 8, 4096)
        self.value_conv = nn.Conv2d(512, 1, kernel_size=1)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(1 * 8 * 8, 512)
        self.value_fc2 = nn.Linear(512, 1)
        self._kv = None
        self._kv_key = None

    # -- packed device weights ------------------------------------------------
    def _version_key(self, device_index):
        return (device_index, self.precision, self.algo) + tuple(t._version for t in self.state_dict().values())

    def packed_weights(self) -> np.ndarray:
        return pack_weights(state_dict_to_numpy(self.state_dict()))[0]

    def kv_net(self, device_index: int) -> KVNet:
        key = self._version_key(device_index)
        if self._kv is None or self._kv_key != key:
            if self._kv is not None:
                self._kv.close()
            self._kv = KVNet(device_index, self.packed_weights(), self.precision, self.algo)
            self._kv_key = key
        return self._kv

    supports_row_padding = True  # training forward takes n_real (knightvision_amd.train bucketing)

    def _train_forward(self, x, n_real=None):
        """Training mode (ai/model.py:51-77 with batch-statistics BatchNorm):
        PyTorch-ROCm autograd over the same parameters, for train.py's update
        step (knightvision_amd.train). Evaluation never comes here. n_real:
        rows after the first n_real are padding (batch_norm_rows)."""
        p = next(self.parameters())
        x = x.to(device=p.device, dtype=p.dtype)
        bn = batch_norm_rows
        cv = conv_chunked
        h = F.relu(bn(self.bn1, cv(self.conv1, x), n_real))
        h = F.relu(bn(self.bn2, cv(self.conv2, h), n_real))
        for blk in self.res_blocks:
            h = blk(h, n_real)
        pol = self.policy_fc(torch.flatten(F.relu(bn(self.policy_bn, cv(self.policy_conv, h), n_real)), 1))
        v = torch.flatten(F.relu(bn(self.value_bn, cv(self.value_conv, h), n_real)), 1)
        val = torch.tanh(self.value_fc2(F.relu(self.value_fc1(v))))
        return pol, val

    def _train_forward_hip(self, x, n_real=None):
        """Training mode under autocast fp16 on CUDA: the tower on the HIP
        training kernels (knightvision_amd/train_ops.py, csrc/kv_train.hip),
        NHWC fp16; the heads' 1x1 convs on HIP kernels too (train_ops.Head1x1),
        their BatchNorms and FCs as PyTorch ops, in ai/model.py:64-73's order
        with the NCHW flatten (index c*64 + square). Rows after n_real (padding) are
        dropped before the tower and returned as zeros."""
        from . import train_ops
        n = x.shape[0]
        xr = x[:n_real] if n_real is not None else x
        h = train_ops.tower_forward(self, xr)  # [m, 64, 512] fp16
        m = h.shape[0]

        def bn(mod, t):  # no MIOpen BatchNorm: it compiles a kernel per new batch shape
            return batch_norm_rows(mod, t, explicit=True)
        hv = train_ops.Head1x1.apply(h, self.policy_conv.weight, self.policy_conv.bias, self.value_conv.weight,
                                     self.value_conv.bias)  # [m, 64, 4] fp16: policy 0-1, value 2
        pc = hv[..., 0:2].permute(0, 2, 1).reshape(m, 2, 8, 8)
        pol = self.policy_fc(torch.flatten(F.relu(bn(self.policy_bn, pc)), 1))
        vc = hv[..., 2:3].permute(0, 2, 1).reshape(m, 1, 8, 8)
        v = torch.flatten(F.relu(bn(self.value_bn, vc)), 1)
        val = torch.tanh(self.value_fc2(F.relu(self.value_fc1(v))))
        if m < n:
            pol = torch.cat([pol, pol.new_zeros((n - m,) + tuple(pol.shape[1:]))])
            val = torch.cat([val, val.new_zeros((n - m,) + tuple(val.shape[1:]))])
        return pol, val

    def forward(self, x, n_real=None):
        if self.training:
            if not isinstance(x, torch.Tensor):
                x = torch.as_tensor(np.asarray(x))
            if x.is_cuda and TRAIN_BACKEND == "hip" and _autocast_on():
                return self._train_forward_hip(x, n_real)
            return self._train_forward(x, n_real)
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(np.asarray(x))
        dev = x.device if x.is_cuda else torch.device("cuda", torch.cuda.current_device())
        x = x.to(device=dev, dtype=torch.float32)
        if self.verbose:
            print("📥 Forward input shape:", x.shape)
        with torch.no_grad():
            pol, val = self.kv_net(dev.index if dev.index is not None else 0).forward_planes(x)
        if self.verbose:
            print("📤 Policy output shape:", pol.shape)
            print("📤 Value output shape:", val.shape)
        return pol, val

    def __getstate__(self):
        d = self.__dict__.copy()
        d["_kv"] = None
        d["_kv_key"] = None
        return d
