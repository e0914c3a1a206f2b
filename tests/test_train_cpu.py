"""CPU tests of the learn-loop update step (knightvision_amd.train / learn):
the data bridge against encode_board, the per-batch loss and the epoch loop
against a plain restatement of scripts/train.py _train_one_epoch (:126-196),
ChessNet's training-mode forward against a functional restatement of
ai/model.py:51-77, and the world-size-2 gloo paths (DDP gradient averaging,
the end-of-iteration all-gather + re-shard)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from knightvision_amd import train as T


class TinyNet(nn.Module):
    """Same output contract as ChessNet (policy [B,4096], value [B,1]); small
    enough for fast CPU tests of the update-step logic."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(12, 4, 3, padding=1)
        self.bn = nn.BatchNorm2d(4)
        self.pol = nn.Linear(256, 4096)
        self.val = nn.Linear(256, 1)

    def forward(self, x):
        h = torch.flatten(F.relu(self.bn(self.conv(x))), 1)
        return self.pol(h), torch.tanh(self.val(h))


def _data(n, seed):
    g = np.random.default_rng(seed)
    codes = torch.from_numpy((g.integers(0, 13, size=(n, 64)) * (g.random((n, 64)) < 0.4)).astype(np.int8))
    moves = torch.from_numpy(g.integers(0, 4096, size=n).astype(np.int64))
    rew = torch.from_numpy(g.choice([-1.0, 0.2, 1.0], size=n).astype(np.float32))
    return codes, moves, rew


def test_codes_to_planes_matches_encode_board():
    from knightvision_amd.ai import codes_to_planes
    codes, _, _ = _data(50, 0)
    got = T.codes_to_planes_t(codes).numpy()
    assert np.array_equal(got, codes_to_planes(codes.numpy().astype(np.int64)))


def _ref_loss(pol, val, moves, outcomes, coef):
    # scripts/train.py:169-176, restated
    lp = F.cross_entropy(pol.float(), moves)
    lv = F.mse_loss(val.squeeze().float(), outcomes)
    probs = F.softmax(pol.float(), dim=1)
    ent = -(probs * F.log_softmax(pol.float(), dim=1)).sum(dim=1).mean()
    return lp + lv - coef * ent


def test_batch_loss_matches_reference_formula():
    torch.manual_seed(0)
    m = TinyNet()
    codes, moves, rew = _data(32, 1)
    b = T.Batch(T.codes_to_planes_t(codes), moves, rew)
    loss = T.batch_loss(m, b, 0.01)[0]
    pol, val = m(b.boards)
    assert torch.allclose(loss, _ref_loss(pol, val, moves, rew, 0.01), rtol=1e-6, atol=1e-6)


def _ref_epoch(model, data, opt, accum, coef):
    # scripts/train.py:138-192 without the logging (GradScaler disabled on CPU)
    opt.zero_grad()
    n = len(data)
    for i, b in enumerate(data):
        pol, val = model(b.boards)
        loss = _ref_loss(pol, val, b.moves, b.outcomes, coef)
        if torch.isnan(loss) or torch.isinf(loss):
            continue
        (loss / accum).backward()
        if ((i + 1) % accum == 0) or (i == n - 1):
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
            opt.step()
            opt.zero_grad()


@pytest.mark.parametrize("accum", [1, 2, 3])
def test_train_one_epoch_matches_reference_loop(accum):
    torch.manual_seed(1)
    a = TinyNet()
    b = TinyNet()
    b.load_state_dict(a.state_dict())
    codes, moves, rew = _data(70, 2)
    data = list(T.batches(codes, moves, rew, 16, shuffle=False))
    oa = torch.optim.Adam(a.parameters(), lr=1e-3)
    ob = torch.optim.Adam(b.parameters(), lr=1e-3)
    st = T.train_one_epoch(a, data, oa, T.make_scaler("cpu"), accumulate_steps=accum, entropy_coef=0.01)
    _ref_epoch(b, data, ob, accum, 0.01)
    assert st["batches"] == 5 and st["optimizer_steps"] == -(-5 // accum)
    for (k, x), y in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.equal(x, y), k


def test_chessnet_train_forward_matches_functional_restatement():
    from knightvision_amd.model import ChessNet
    torch.manual_seed(3)
    m = ChessNet().train()
    codes, _, _ = _data(6, 4)
    x = T.codes_to_planes_t(codes)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    pol, val = m(x)

    def cbr(h, c, bn, relu=True):  # conv + batch-statistics BN (+ ReLU), ai/model.py:58-73
        h = F.conv2d(h, sd[c + ".weight"], sd[c + ".bias"], padding=sd[c + ".weight"].shape[-1] // 2)
        h = F.batch_norm(h, sd[bn + ".running_mean"].clone(), sd[bn + ".running_var"].clone(),
                         sd[bn + ".weight"], sd[bn + ".bias"], training=True, momentum=0.1, eps=1e-5)
        return F.relu(h) if relu else h
    h = cbr(cbr(x, "conv1", "bn1"), "conv2", "bn2")
    for i in range(5):
        p = f"res_blocks.{i}"
        h = F.relu(cbr(cbr(h, p + ".conv1", p + ".bn1"), p + ".conv2", p + ".bn2", relu=False) + h)
    rp = F.linear(torch.flatten(cbr(h, "policy_conv", "policy_bn"), 1), sd["policy_fc.weight"], sd["policy_fc.bias"])
    v = torch.flatten(cbr(h, "value_conv", "value_bn"), 1)
    rv = torch.tanh(F.linear(F.relu(F.linear(v, sd["value_fc1.weight"], sd["value_fc1.bias"])),
                             sd["value_fc2.weight"], sd["value_fc2.bias"]))
    assert torch.allclose(pol, rp, atol=1e-5) and torch.allclose(val, rv, atol=1e-6)
    # the running statistics moved (training mode), so the eval-mode pack must be rebuilt
    assert not torch.equal(m.state_dict()["bn1.running_mean"], sd["bn1.running_mean"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(5)
    m = TinyNet()
    ddp = T.wrap_ddp(m, "cpu")
    codes, moves, rew = _data(64, 6)
    mine = [T.Batch(T.codes_to_planes_t(codes[i:i + 8][rank::2]), moves[i:i + 8][rank::2],
                    rew[i:i + 8][rank::2]) for i in range(0, 64, 8)]
    opt = torch.optim.SGD(m.parameters(), lr=0.1)  # SGD: Adam would amplify the pure-noise conv-bias gradient
    T.train_one_epoch(ddp, mine, opt, T.make_scaler("cpu"), accumulate_steps=2, entropy_coef=0.01)
    # end-of-iteration exchange: all-gather + global decisive filter + round-robin re-shard
    c2, m2, r2 = _data(5 + 3 * rank, 10 + rank)
    from knightvision_amd.distributed import gather_rows
    union = [gather_rows(x, dst=None) for x in (c2, m2, r2)]
    q.put((rank, {k: v.numpy().copy() for k, v in m.state_dict().items()}, [u.numpy().copy() for u in union]))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_world2_matches_gradient_average():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: each global batch of 8 split into the two ranks' halves; DDP averages the
    # two halves' gradients (BatchNorm statistics stay per half, as in each DDP replica)
    torch.manual_seed(5)
    m = TinyNet()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    codes, moves, rew = _data(64, 6)
    opt.zero_grad()
    for j, i in enumerate(range(0, 64, 8)):
        for r in range(2):
            b = T.Batch(T.codes_to_planes_t(codes[i:i + 8][r::2]), moves[i:i + 8][r::2], rew[i:i + 8][r::2])
            (T.batch_loss(m, b, 0.01)[0] / 2 / 2).backward()
        if (j + 1) % 2 == 0 or j == 7:
            torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=1.0)
            opt.step()
            opt.zero_grad()
    for rank, sd, _ in res:
        for k, v in m.state_dict().items():
            if "running" in k or "num_batches" in k:
                continue  # buffers follow rank 0's replica (DDP broadcast_buffers)
            assert torch.allclose(torch.from_numpy(sd[k]), v, atol=2e-6), (rank, k)
    # the gathered union is the same on both ranks, in rank order
    want = [torch.cat([_data(5, 10)[t], _data(8, 11)[t]]) for t in range(3)]
    for _, _, union in res:
        for u, w in zip(union, want):
            assert torch.equal(torch.from_numpy(u), w)


def test_row_bucketing_is_the_unpadded_update():
    """batch_loss with the batch padded to a row bucket (the GPU path, which keeps
    MIOpen's convolution shapes fixed): the padding rows are excluded from every
    BatchNorm statistic and from the loss, so loss, gradients and BN running
    statistics equal the unpadded batch's."""
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()}
    codes, moves, rew = _data(5, 3)
    # float64: the update is the same function of the real rows; in fp32 the
    # BatchNorm backward's cancellations turn kernel-order noise into ~1e-3
    b = T.Batch(T.codes_to_planes_t(codes).double(), moves, rew)
    outs = []
    for bucket in (0, 8):
        torch.manual_seed(0)
        m = ChessNet()
        m.load_state_dict(sd)
        m = m.double()
        m.train()
        loss = T.batch_loss(m, b, amp=False, bucket=bucket)[0]
        loss.backward()
        grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        stats = {k: v.detach().clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
        outs.append((float(loss), grads, stats))
    (l0, g0, s0), (l1, g1, s1) = outs
    assert abs(l0 - l1) < 1e-9 * max(1.0, abs(l0))
    for k in g0:
        assert torch.allclose(g0[k], g1[k], rtol=1e-9, atol=1e-12), k
    for k in s0:
        assert torch.allclose(s0[k].double(), s1[k].double(), rtol=1e-9, atol=1e-12), k



def _spawn(target, world=2, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=timeout) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _loop_batch_worker(rank, world, port, q):
    """The learn loop's update path on one rank: the round-robin shard of the
    filtered union (learn.extend_dataset) trained with learn.rank_batch_size."""
    import torch.distributed as dist
    from knightvision_amd import learn as L
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(5)
    m = TinyNet()
    ddp = T.wrap_ddp(m, "cpu")
    codes, moves, rew = _data(64, 6)
    shard = (codes[rank::world], moves[rank::world], rew[rank::world])
    bs = L.rank_batch_size(8, world)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    ep = T.train_one_epoch(ddp, T.batches(*shard, bs, False, total=32), opt, T.make_scaler("cpu"),
                           accumulate_steps=2, entropy_coef=0.01)
    q.put((rank, bs, ep, {k: v.numpy().copy() for k, v in m.state_dict().items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_learn_loop_world2_keeps_the_reference_global_batch():
    """with W ranks each micro-batch is W x (batch_size // W) rows --
    the reference's DataParallel batch (utils/model_utils.py:26-28) -- so an
    epoch of 64 samples at batch 8, accumulation 2 takes 4 optimizer steps on
    every rank, and the update equals one process averaging the two ranks'
    halves of each global batch."""
    res = _spawn(_loop_batch_worker)
    for rank, bs, ep, _ in res:
        assert bs == 4
        assert ep["batches"] == 8 and ep["optimizer_steps"] == 4 and ep["samples"] == 32
    torch.manual_seed(5)
    m = TinyNet()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    codes, moves, rew = _data(64, 6)
    halves = [tuple(x[r::2] for x in (codes, moves, rew)) for r in range(2)]
    opt.zero_grad()
    for j in range(8):
        for r in range(2):
            c, mv, rw = (x[4 * j:4 * j + 4] for x in halves[r])
            (T.batch_loss(m, T.Batch(T.codes_to_planes_t(c), mv, rw), 0.01)[0] / 2 / 2).backward()
        if (j + 1) % 2 == 0:
            torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=1.0)
            opt.step()
            opt.zero_grad()
    for rank, _, _, sd in res:
        for k, v in m.state_dict().items():
            if "running" in k or "num_batches" in k:
                continue
            assert torch.allclose(torch.from_numpy(sd[k]), v, atol=2e-6), (rank, k)


def _nan_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(5)
    m = TinyNet()
    ddp = T.wrap_ddp(m, "cpu")
    codes, moves, rew = _data(32, 7 + rank)
    batches = [T.Batch(T.codes_to_planes_t(codes[i:i + 8]), moves[i:i + 8], rew[i:i + 8].clone())
               for i in range(0, 32, 8)]
    if rank == 1:
        batches[1].outcomes[0] = float("nan")  # one rank's loss of batch 1 is NaN
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    ep = T.train_one_epoch(ddp, batches, opt, T.make_scaler("cpu"), accumulate_steps=1, entropy_coef=0.01)
    q.put((rank, ep, {k: v.numpy().copy() for k, v in m.state_dict().items() if "running" not in k}))
    dist.barrier()
    dist.destroy_process_group()


def test_nan_batch_is_skipped_on_every_rank():
    """a non-finite loss on one rank skips that batch on all ranks
    (MIN all-reduce of the finiteness flag), so DDP's gradient all-reduces
    stay paired and the replicas stay identical."""
    res = _spawn(_nan_worker)
    for rank, ep, _ in res:
        assert ep["skipped"] == 1 and ep["optimizer_steps"] == 3, (rank, ep)
    (_, _, a), (_, _, b) = res
    for k in a:
        if "num_batches" in k:
            continue
        assert np.allclose(a[k], b[k], atol=1e-6), k


def test_explicit_batch_norm_matches_module():
    """The HIP update step computes the heads' BatchNorms with elementwise ops
    (model.batch_norm_rows(explicit=True): MIOpen compiles a BatchNorm kernel for
    every new batch shape); outputs, gradients and running statistics equal
    nn.BatchNorm2d's training mode."""
    from knightvision_amd.model import batch_norm_rows
    torch.manual_seed(3)
    for C in (1, 2):
        a, b = torch.nn.BatchNorm2d(C), torch.nn.BatchNorm2d(C)
        with torch.no_grad():
            a.weight.uniform_(0.5, 1.5)
            a.bias.normal_()
        b.load_state_dict(a.state_dict())
        x = (torch.randn(37, C, 8, 8) * 3 + 1).requires_grad_(True)
        x2 = x.detach().clone().requires_grad_(True)
        y1, y2 = a(x), batch_norm_rows(b, x2, explicit=True)
        g = torch.randn_like(y1)
        y1.backward(g)
        y2.backward(g)
        assert torch.allclose(y1, y2, atol=2e-6)
        assert torch.allclose(x.grad, x2.grad, atol=2e-6)
        assert torch.allclose(a.weight.grad, b.weight.grad, atol=1e-4)
        assert torch.allclose(a.running_mean, b.running_mean) and torch.allclose(a.running_var, b.running_var)
        assert int(a.num_batches_tracked) == int(b.num_batches_tracked) == 1


def _val_worker(rank, world, port, q):
    """learn.split_train_val / evaluate_sharded on two gloo ranks."""
    import torch.distributed as dist
    from knightvision_amd import learn as L
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(5)
    m = TinyNet()
    data = _data(57, 3)
    tr, va = L.split_train_val(57, torch.Generator().manual_seed(0))
    loss = L.evaluate_sharded(m, data, va, 8, torch.device("cpu"))
    q.put((rank, tr.tolist(), va.tolist(), loss))
    dist.barrier()
    dist.destroy_process_group()


def test_validation_split_and_sharded_evaluate_world2():
    """The learn loop's random_split (learn.py:162-165: int(0.9 n) train samples) is the same on every
    rank, and the validation loss of the ranks' round-robin shards (sums all-reduced) equals train.evaluate
    over the whole validation subset on one process (train.py:109-124)."""
    from knightvision_amd import learn as L
    res = _spawn(_val_worker)
    (r0, tr0, va0, l0), (r1, tr1, va1, l1) = res
    assert tr0 == tr1 and va0 == va1 and len(tr0) == int(0.9 * 57) and len(va0) == 57 - int(0.9 * 57)
    assert sorted(tr0 + va0) == list(range(57))
    torch.manual_seed(5)
    m = TinyNet()
    data = _data(57, 3)
    va = torch.tensor(va0)
    want = T.evaluate(m, list(T.batches(*(x[va] for x in data), 8, False)))
    assert abs(l0 - want) < 1e-5 * abs(want) and l0 == l1


def test_train_with_validation_steps_the_reference_lr_schedulers():
    """train.py train_with_validation builds CosineAnnealingWarmRestarts(T_0=10), ReduceLROnPlateau
    and StepLR(10, 0.1) per call (:293-307) and steps the cosine schedule with epoch + 1, then StepLR, after
    each epoch's validation (:421-423); a second call restarts the cosine schedule from the initial LR. With
    lr 1e-3 the LR after epochs 1, 2, 3 is 1e-3 (1 + cos(k pi / 10)) / 2."""
    import math
    from knightvision_amd import learn as L
    torch.manual_seed(5)
    m = TinyNet()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    data = _data(40, 11)
    want = [1e-3 * (1 + math.cos(k * math.pi / L.COSINE_T0)) / 2 for k in (1, 2, 3)]
    for call in range(2):
        tv = L.train_with_validation(m, m, opt, data, 3, 8, 2, torch.Generator().manual_seed(call),
                                     torch.Generator().manual_seed(0), torch.device("cpu"))
        assert tv["epochs_run"] == 3
        assert np.allclose(tv["lr_per_epoch"], want, rtol=1e-12, atol=0), (call, tv["lr_per_epoch"])


def test_lr_schedulers_match_the_reference_over_a_step_boundary():
    """Epochs 1..12 of one call: the cosine restart at T_0 and StepLR's x gamma at epoch 10 compose in the
    reference's order (cos.step(epoch + 1) then step.step()); the plateau scheduler is fed a falling loss."""
    from knightvision_amd import learn as L
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-3)
    cos, plateau, step = L.make_lr_schedulers(opt)
    # the same schedulers, built directly as train.py:293-307 builds them
    p2 = torch.nn.Parameter(torch.zeros(1))
    opt2 = torch.optim.Adam([p2], lr=1e-3)
    c2 = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(opt2, T_0=10, T_mult=1)
    r2 = torch.optim.lr_scheduler.ReduceLROnPlateau(opt2, mode="min", factor=0.1, patience=5)
    s2 = torch.optim.lr_scheduler.StepLR(opt2, step_size=10, gamma=0.1)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for epoch in range(12):
            for o, (c, r, s) in ((opt, (cos, plateau, step)), (opt2, (c2, r2, s2))):
                r.step(1.0 / (epoch + 1))
                c.step(epoch + 1)
                s.step()
            assert opt.param_groups[0]["lr"] == opt2.param_groups[0]["lr"], epoch
    assert opt.param_groups[0]["lr"] != 1e-3
