"""HIP training kernels (csrc/kv_train.hip via knightvision_amd/train_ops.py)
against plain PyTorch fp32 restatements of the same autocast-fp16 ops
(scripts/train.py:161-184 trains ai/model.py's ChessNet under
torch.cuda.amp.autocast):

* conv forward / data gradient / weight gradient: fp16 operands, fp32
  accumulation, fp16 results -> within fp16 rounding of the fp32 result of
  the fp16-rounded operands (|err| <= 2^-10 |ref| + 2^-14 max|ref|);
* BatchNorm (+residual)(+ReLU) forward and backward: the same ops in fp32 on
  the fp16 inputs, fp16 rounding of the results;
* the whole tower + heads under autocast against the MIOpen path
  (KV_TRAIN_BACKEND=miopen: torch's fp16 convolutions) -- two fp16
  computations of the same network: logits and gradients agree to the
  accumulated fp16 rounding.
The update step itself (loss, accumulation, clip, GradScaler, Adam) through
this path is pinned against the float64 restatement in test_train_gpu.py."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from knightvision_amd import train_ops as TO

pytestmark = pytest.mark.gpu


def _nchw(t):  # [n,64,C] -> [n,C,8,8]
    return t.permute(0, 2, 1).reshape(t.shape[0], t.shape[2], 8, 8)


def _nhwc(t):  # [n,C,8,8] -> [n,64,C]
    return t.reshape(t.shape[0], t.shape[1], 64).permute(0, 2, 1).contiguous()


def _close16(y, ref, what, mag=None):
    """|y - ref| within fp16 rounding: 2^-10 of the magnitude (|ref|, or `mag` where an intermediate
    rounded at a larger magnitude, e.g. BN output before a residual add) + 2^-14 max |ref|"""
    y, ref = y.float().cpu(), ref.float().cpu()
    tol = (ref.abs() if mag is None else mag) * 2.0 ** -10 + float(ref.abs().max()) * 2.0 ** -14
    bad = (y - ref).abs() > tol
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} of {bad.numel()} outside fp16 rounding, max |err| " \
                                f"{float((y - ref).abs().max()):.3e} (max |ref| {float(ref.abs().max()):.3e})"


@pytest.mark.parametrize("n,ci_real,ci,co", [(5, 12, 64, 256), (9, 256, 256, 512), (37, 512, 512, 512),
                                             (4, 512, 512, 256)])
def test_conv_forward_and_grads(n, ci_real, ci, co):
    g = torch.Generator().manual_seed(n * 1000 + co)
    x = torch.zeros(n, 64, ci, dtype=torch.float16)
    x[..., :ci_real] = (torch.randn(n, 64, ci_real, generator=g)).half()
    w = torch.randn(co, ci_real, 3, 3, generator=g) / (3.0 * ci_real ** 0.5)
    b = torch.randn(co, generator=g) * 0.1
    dy = (torch.randn(n, 64, co, generator=g)).half()
    xc, wc, bc, dyc = x.cuda(), w.cuda(), b.cuda(), dy.cuda()

    wf, wt = TO.conv_weight_images(wc, ci, True)
    y = TO.conv3x3_f16(xc, wf, bc.half().float())
    w16 = w.half().float()
    x32 = _nchw(x[..., :ci_real].float())
    ref = F.conv2d(x32, w16, b.half().float(), padding=1)
    _close16(y, _nhwc(ref), "forward")

    if ci % 128 == 0:  # the stem's input (the planes) takes no gradient
        dx = TO.conv3x3_f16(dyc, wt, None)
        ref_dx = torch.nn.grad.conv2d_input(x32.shape, w16, _nchw(dy.float()), padding=1)
        _close16(dx[..., :ci_real], _nhwc(ref_dx), "data gradient")

    dw = TO.conv3x3_wgrad_f16(dyc, xc, ci_real)
    ref_dw = torch.nn.grad.conv2d_weight(x32, w.shape, _nchw(dy.float()), padding=1)
    assert torch.equal(dw.cpu(), dw.cpu().half().float()), "weight gradient not fp16-rounded"
    _close16(dw, ref_dw, "weight gradient")

    db = TO.channel_sum_f16(dyc)
    assert torch.allclose(db.cpu(), dy.float().sum(dim=(0, 1)), rtol=1e-5, atol=1e-3)

    # the fused addend (a residual block's data gradient + the residual branch's): autograd's fp16 add, bit for bit
    add = torch.randn(y.shape, generator=g).half().cuda()
    ya = TO.conv3x3_f16(xc, wf, bc.half().float(), add)
    assert torch.equal(ya, (y.float() + add.float()).half())


def test_wgrad_is_deterministic():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 64, 512, generator=g).half().cuda()
    dy = torch.randn(64, 64, 512, generator=g).half().cuda()
    a = TO.conv3x3_wgrad_f16(dy, x, 512)
    b = TO.conv3x3_wgrad_f16(dy, x, 512)
    assert torch.equal(a, b)


@pytest.mark.parametrize("res,C", [(False, 256), (True, 512), (True, 192)])  # 192: C/8 does not divide 256
def test_bn_act_forward_backward(res, C):
    g = torch.Generator().manual_seed(C + res)
    n = 7
    x = (torch.randn(n, 64, C, generator=g) * 2 + 0.5).half()
    r = torch.randn(n, 64, C, generator=g).half() if res else None
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(n, 64, C, generator=g).half()
    eps = 1e-5
    # kernels
    xc = x.cuda().requires_grad_(True)
    rc = r.cuda().requires_grad_(True) if res else None
    gc = gamma.cuda().requires_grad_(True)
    bc = beta.cuda().requires_grad_(True)
    stats = []
    y = TO.BNAct.apply(xc, gc, bc, rc, True, eps, stats)
    y.backward(dy.cuda())
    # fp32 restatement on the fp16 values, rounded where the autocast ops round
    xf = x.float().requires_grad_(True)
    rf = r.float() if res else None
    gf, bf = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    mean = xf.mean(dim=(0, 1))
    var = xf.var(dim=(0, 1), unbiased=False)
    yb = (xf - mean) * torch.rsqrt(var + eps) * gf + bf
    assert torch.allclose(stats[0][0].cpu(), mean.detach(), rtol=1e-5, atol=1e-6)
    assert torch.allclose(stats[0][1].cpu(), var.detach(), rtol=1e-5, atol=1e-6)
    y16 = yb.detach().half().float()
    mag = None
    if res:
        # two fp16 roundings (the BN output, then the sum), each may land one ulp off when the fp32 values
        # differ in their last bits
        mag = 2 * (y16.abs() + rf.abs())
        y16 = (y16 + rf).half().float()
    yref = torch.relu(y16)
    _close16(y, yref, "BN forward", mag)
    # backward: the ReLU mask of the kernel's own output, then the BN gradient in fp32
    mask = (y.detach().float().cpu() > 0).float()
    gmask = dy.float() * mask
    yb.backward(gmask)
    _close16(xc.grad, xf.grad, "BN data gradient")
    assert torch.allclose(gc.grad.cpu(), gf.grad, rtol=1e-4, atol=1e-3)
    assert torch.allclose(bc.grad.cpu(), bf.grad, rtol=1e-4, atol=1e-3)
    if res:
        assert torch.equal(rc.grad.cpu().float(), gmask.half().float())


def test_tower_matches_miopen_autocast():
    """HIP and MIOpen autocast runs of the same training forward/backward (loss
    scaled by 65536 as GradScaler starts, so fp16 gradients do not underflow),
    each against the fp32 (no autocast) gradients: the HIP path must be as close
    to fp32 as torch's own fp16 path is (within 1.5x + 1e-3 per tensor)."""
    from knightvision_amd import model as KM
    from knightvision_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(42, "bn")
    g = torch.Generator().manual_seed(11)
    codes = torch.randint(0, 13, (48, 64), generator=g)
    planes = F.one_hot(codes, 13)[..., 1:].permute(0, 2, 1).reshape(-1, 12, 8, 8).float().cuda()
    moves = torch.randint(0, 4096, (48,), generator=g).cuda()
    scale = 65536.0
    runs = {}
    for name, backend, amp in (("hip", "hip", True), ("miopen", "miopen", True), ("fp32", "miopen", False)):
        KM.TRAIN_BACKEND = backend
        try:
            m = KM.ChessNet()
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
            m.cuda().train()
            with torch.autocast("cuda", enabled=amp):
                pol, val = m(planes)
            loss = F.cross_entropy(pol.float(), moves) + (val.float() ** 2).mean()
            (loss * scale).backward()
            grads = {k: p.grad.detach().double() / scale for k, p in m.named_parameters()}
            bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
            runs[name] = (pol.detach().float(), val.detach().float(), float(loss), grads, bufs)
        finally:
            KM.TRAIN_BACKEND = "hip"
    ph, vh, lh, gh, bh = runs["hip"]
    pm, vm, lm, gm, bm = runs["miopen"]
    p32, v32, l32, g32, _ = runs["fp32"]
    perr = float((ph - p32).abs().max() / p32.abs().max())
    perr_m = float((pm - p32).abs().max() / p32.abs().max())
    print(f"policy vs fp32: HIP {perr:.2e}, MIOpen fp16 {perr_m:.2e}; loss {lh:.6f} / {lm:.6f} / {l32:.6f}")
    assert perr < 1.5 * perr_m + 1e-3 and abs(lh - l32) < 1e-2 * abs(l32)
    assert float((vh - v32).abs().max()) < 1.5 * float((vm - v32).abs().max()) + 1e-3
    worst = []
    for k in g32:
        if k.endswith(".bias") and "conv" in k:
            continue  # conv biases ahead of BatchNorm: exact gradient 0, rounding noise on every side
        ref = g32[k]
        eh = float((gh[k] - ref).norm() / ref.norm().clamp_min(1e-30))
        em = float((gm[k] - ref).norm() / ref.norm().clamp_min(1e-30))
        worst.append((eh, em, k))
    worst.sort(reverse=True)
    print("gradients vs fp32 (HIP, MIOpen fp16): " + ", ".join(f"{k} {a:.1e}/{b:.1e}" for a, b, k in worst))
    mean_h = sum(a for a, _, _ in worst) / len(worst)
    mean_m = sum(b for _, b, _ in worst) / len(worst)
    print(f"mean per-tensor relative error vs fp32: HIP {mean_h:.2e}, MIOpen fp16 {mean_m:.2e}")
    assert mean_h < 1.25 * mean_m + 1e-3
    for a, b, k in worst:
        assert a < 2.5 * b + 2e-3, (k, a, b)
    # running statistics follow nn.BatchNorm2d's update
    for k in bm:
        if bm[k].dtype.is_floating_point:
            assert torch.allclose(bh[k], bm[k], rtol=2e-2, atol=2e-3), k
        else:
            assert torch.equal(bh[k], bm[k]), k


def test_fused_backward_is_the_unfused_one():
    """train_ops.FUSE: the BatchNorm backward's dx channel sums (conv bias gradients) and the residual
    gradient added inside the data-gradient kernel give the same gradients as the separate passes:
    every weight / BatchNorm gradient bit for bit, the conv biases to their summation noise (the channel
    sums add the same fp16 values in another order)."""
    from knightvision_amd import model as KM
    from knightvision_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(7, "bn")
    g = torch.Generator().manual_seed(5)
    codes = torch.randint(0, 13, (40, 64), generator=g)
    planes = F.one_hot(codes, 13)[..., 1:].permute(0, 2, 1).reshape(-1, 12, 8, 8).float().cuda()
    moves = torch.randint(0, 4096, (40,), generator=g).cuda()
    grads = {}
    for fuse in (False, True):
        TO.FUSE = fuse
        try:
            m = KM.ChessNet()
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
            m.cuda().train()
            with torch.autocast("cuda"):
                pol, val = m(planes)
            loss = F.cross_entropy(pol.float(), moves) + (val.float() ** 2).mean()
            (loss * 65536.0).backward()
            grads[fuse] = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        finally:
            TO.FUSE = True
    for k, a in grads[False].items():
        b = grads[True][k]
        if k.endswith(".bias") and "conv" in k:
            # exact value 0 (BatchNorm removes the bias): both sides are the cancellation noise of the same
            # fp16 dx values summed in another order, ~2^-12 of the largest here
            assert torch.allclose(a, b, rtol=0.0, atol=float(a.abs().max()) * 2.0 ** -8), k
        else:
            assert torch.equal(a, b), k


def test_head1x1_forward_backward():
    g = torch.Generator().manual_seed(5)
    n = 6
    h = torch.randn(n, 64, 512, generator=g).half()
    wp, bp = torch.randn(2, 512, 1, 1, generator=g) / 20, torch.randn(2, generator=g) * 0.1
    wv, bv = torch.randn(1, 512, 1, 1, generator=g) / 20, torch.randn(1, generator=g) * 0.1
    dout = torch.randn(n, 64, 4, generator=g).half()
    dout[..., 3] = 0
    params = [t.cuda().requires_grad_(True) for t in (wp, bp, wv, bv)]
    hc = h.cuda().requires_grad_(True)
    out = TO.Head1x1.apply(hc, *params)
    out.backward(dout.cuda())
    w16 = torch.cat([wp.reshape(2, 512), wv.reshape(1, 512)]).half().float()
    b16 = torch.cat([bp, bv]).half().float()
    ref = h.float() @ w16.t() + b16
    _close16(out[..., :3], ref, "head 1x1 forward")
    d = dout[..., :3].float()
    _close16(hc.grad, d @ w16, "head 1x1 data gradient")
    dw = torch.einsum("nsj,nsc->jc", d, h.float())
    _close16(torch.cat([params[0].grad.reshape(2, 512), params[2].grad.reshape(1, 512)]), dw, "head 1x1 weight grad")
    db = d.sum(dim=(0, 1))
    assert torch.allclose(torch.cat([params[1].grad, params[3].grad]).cpu(), db.half().float(), rtol=1e-3, atol=1e-3)


def test_training_trajectory_matches_miopen():
    """30 update steps (autocast fp16, GradScaler, accumulation 2, clip 1.0, Adam; train.py:126-196) on the
    same engine-played records with the HIP training kernels and with torch's MIOpen path: the loss
    trajectories agree to fp16-rounding drift and both fall (the HIP step trains the network as the
    reference's does)."""
    from knightvision_amd import model as KM
    from knightvision_amd import train as T
    from knightvision_amd.engine import SelfPlayEngine
    from knightvision_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(42, "init")
    with SelfPlayEngine(sd, slots=64, n_games=64, seed=42, max_moves=60, batch=16) as eng:
        eng.run()
        recs, games = eng.records(), eng.games()
    codes, moves, rew = T.records_to_tensors(recs, games, "cuda")
    curves = {}
    for backend in ("hip", "miopen"):
        KM.TRAIN_BACKEND = backend
        try:
            m = KM.ChessNet()
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
            m.cuda().train()
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)
            scaler = T.make_scaler("cuda")
            gen = torch.Generator().manual_seed(5)
            losses = []
            for _ in range(15):  # 15 epochs of 4 batches of 256, accumulation 2: 30 optimizer steps
                st = T.train_one_epoch(m, T.batches(codes[:1024], moves[:1024], rew[:1024], 256, True, gen), opt,
                                       scaler, accumulate_steps=2)
                losses.append(st["loss"] / st["batches"])
            curves[backend] = np.array(losses)
        finally:
            KM.TRAIN_BACKEND = "hip"
    h, mi = curves["hip"], curves["miopen"]
    print("loss per epoch  HIP:", np.round(h, 4).tolist())
    print("loss per epoch MIOp:", np.round(mi, 4).tolist())
    assert h[-1] < 0.8 * h[0] and mi[-1] < 0.8 * mi[0], "the loss did not fall"
    assert np.abs(h - mi).max() <= 0.03 * np.abs(mi).max(), "HIP and MIOpen loss trajectories diverge"
