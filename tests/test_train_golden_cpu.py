"""The update step (scripts/train.py _train_one_epoch :126-196) pinned by the
REFERENCE's own output: tests/golden/train_epoch.npz was written by running the
reference function itself on the CPU (tests/golden/make_train_golden.py: the
reference ChessNet, synthetic "bn" weights, Adam 1e-3, accumulation 2, entropy
coefficient 0.01, 4 batches of 16; fp32 -- autocast is inactive on a CPU).

* oracle/torch_ref.reference_epoch (the float64 restatement the GPU update-step
  test compares against) reproduces the reference's output;
* knightvision_amd.train.train_one_epoch on knightvision_amd.model.ChessNet
  (fp32, CPU) does too -- the product's update logic against the reference's.

Bounds (fp32 vs fp64 rounding): the epoch loss within 1e-5 relative; the first
optimizer step's clipped gradients within 1e-4 of each tensor's norm; its
parameter changes within 0.05 lr wherever the gradient is not negligible
(|g| > 1e-3 of the tensor's largest sampled |g|; at most 1 % of those may
differ -- Adam's first step is ~lr * sign(g)). Adam's first step also turns the
rounding noise of near-zero gradients (and of the conv biases ahead of a
BatchNorm, whose exact gradient is 0: skipped) into +-lr moves, so the second
step's gradients move by up to 0.6 % between fp32 and fp64 (measured): bound
2e-2 of the norm there."""
import os

import numpy as np
import pytest
import torch

from knightvision_amd import train as T
from knightvision_amd.ai import codes_to_planes
from knightvision_amd.weights import synthetic_state_dict


@pytest.fixture(scope="module")
def gold(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "train_epoch.npz")))


def batches_of(g):
    nb, bs = int(g["meta"][0]), int(g["meta"][1])
    planes = codes_to_planes(g["codes"])
    return [(planes[i:i + bs], g["moves"][i:i + bs], g["rewards"][i:i + bs]) for i in range(0, nb * bs, bs)]


def check_against_reference(g, grads, delta1, loss_total, what, grad_tol=(1e-4, 2e-2), flip_frac=0.01,
                            loss_rtol=1e-5):
    """grads: per optimizer step {name: clipped gradient}; delta1: {name: parameter change of step 1}."""
    names = g["param_names"].tolist()
    lr = float(g["meta"][4])
    gmax = max(float(g[f"grad0.norm.{k}"][0]) for k in names)
    assert abs(loss_total - g["losses"][0]) <= loss_rtol * abs(g["losses"][0]), (what, loss_total, g["losses"][0])
    worst = [0.0, 0.0]
    flips = checked = 0
    for k in names:
        if float(g[f"grad0.norm.{k}"][0]) < 1e-6 * gmax:  # a conv bias ahead of BatchNorm: exact gradient 0
            continue
        idx = g[f"idx.{k}"]
        for s, gs in enumerate(grads):
            got = np.asarray(gs[k], dtype=np.float64).reshape(-1)[idx]
            worst[s] = max(worst[s], float(np.abs(got - g[f"grad{s}.at.{k}"]).max()) / float(g[f"grad{s}.norm.{k}"][0]))
        gref = np.abs(g[f"grad0.at.{k}"])
        sel = gref > 1e-3 * gref.max()
        d = np.asarray(delta1[k], dtype=np.float64).reshape(-1)[idx]
        flips += int(((np.abs(d - g[f"delta1.at.{k}"]) > 0.05 * lr) & sel).sum())
        checked += int(sel.sum())
    print(f"{what}: loss {loss_total:.6f} (reference {g['losses'][0]:.6f}); clipped gradients, worst sampled error "
          f"/ tensor norm: step 1 {worst[0]:.2e}, step 2 {worst[1]:.2e}; first-step parameter changes off by > "
          f"0.05 lr: {flips}/{checked}")
    assert worst[0] <= grad_tol[0] and worst[1] <= grad_tol[1], (what, worst)
    assert flips <= flip_frac * checked, what


def test_float64_restatement_matches_reference_epoch(gold):
    from oracle import torch_ref
    sd = synthetic_state_dict(42, "bn")
    _, _, accum, coef, lr = gold["meta"]
    tr = {}
    _, losses, _ = torch_ref.reference_epoch(sd, batches_of(gold), lr, int(accum), coef, trace=tr)
    grads = [{k: v.numpy() for k, v in gs.items()} for gs in tr["grads"]]
    delta1 = {k: (v - torch.tensor(np.asarray(sd[k]), dtype=torch.float64)).numpy() for k, v in tr["after1"].items()}
    check_against_reference(gold, grads, delta1, float(sum(losses)), "float64 restatement")


def test_train_one_epoch_matches_reference_epoch(gold):
    from knightvision_amd.model import ChessNet
    sd = synthetic_state_dict(42, "bn")
    _, _, accum, coef, lr = gold["meta"]
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=float(lr))
    grads, after1 = [], {}
    inner = opt.step

    def step(*a, **kw):
        grads.append({k: p.grad.detach().double().numpy().copy() for k, p in m.named_parameters()})
        r = inner(*a, **kw)
        if not after1:
            after1.update({k: p.detach().double().numpy().copy() for k, p in m.named_parameters()})
        return r
    opt.step = step
    batches = [T.Batch(torch.from_numpy(x), torch.from_numpy(mv), torch.from_numpy(oc)) for x, mv, oc in
               batches_of(gold)]
    st = T.train_one_epoch(m, batches, opt, T.make_scaler("cpu"), accumulate_steps=int(accum),
                           entropy_coef=float(coef), amp=False)
    assert st["optimizer_steps"] == 2 and len(grads) == 2
    delta1 = {k: v - np.asarray(sd[k], dtype=np.float64) for k, v in after1.items()}
    check_against_reference(gold, grads, delta1, st["loss"], "train.train_one_epoch (CPU fp32)")
    after = m.state_dict()
    for k in gold["buffer_names"].tolist():  # BatchNorm running statistics after the epoch
        got = after[k].double().reshape(-1).numpy()[gold[f"idx.{k}"]]
        assert np.allclose(got, gold[f"buf.at.{k}"], rtol=1e-3, atol=1e-6), k
