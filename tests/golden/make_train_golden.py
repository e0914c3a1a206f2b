"""Generate tests/golden/train_epoch.npz by running the REFERENCE's own update
step, scripts/train.py `_train_one_epoch` (:126-196), on the CPU.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_golden.py [/root/reference]

scripts/train.py cannot be imported (module-level tensorflow / google.colab
imports, Drive paths, a dataset read and sys.exit: SURVEY.md 8c), so the one
function is taken from its syntax tree and executed by itself, with its
module globals supplied: torch (with torch.cuda.memory_allocated answering 0
-- the function logs GPU memory every 5 batches and there is no GPU here), F,
a pass-through tqdm and a silent print. Nothing of the reference is copied
into the repo: the fixture is data (inputs and the function's outputs).

Model: the reference ChessNet (ai/model.py, imported as make_golden.py does)
with the synthetic "bn" weights; optimizer Adam(lr 1e-3); GradScaler() as
train_with_validation builds it (on a CPU-only host it disables itself and
is the identity, as under exact arithmetic); ENTROPY_COEF 0.01,
accumulate_steps 2; 4 batches of 16 samples (board codes from the golden
move-generation positions, seeded move targets and rewards). The function
runs under torch.cuda.amp.autocast(), which is inactive on the CPU: this is
the reference's fp32 update step.

Recorded (per parameter tensor, 32 seeded sample positions each):
  * the clipped gradient at each optimizer step (captured at optimizer.step,
    after the reference's clip_grad_norm_), full norm + sampled entries;
  * the parameter change of the first optimizer step and over the epoch
    (sampled entries; + sum for the epoch);
  * BatchNorm running statistics after the epoch (sampled entries);
  * total_loss, the last batch's loss_policy / loss_value (the returns).
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

N_BATCHES, BS, ACCUM, COEF, LR = 4, 16, 2, 0.01, 1e-3
N_SAMPLE = 32


def reference_function(ref, name):
    """The reference's top-level function `name` from scripts/train.py, compiled by itself."""
    path = os.path.join(ref, "scripts", "train.py")
    tree = ast.parse(open(path).read(), filename=path)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name]
    assert len(fn) == 1, name
    mod = ast.Module(body=fn, type_ignores=[])
    return compile(mod, path, "exec")


def sample_index(shape, seed):
    n = int(np.prod(shape))
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=min(N_SAMPLE, n), replace=False))


def fixture_inputs():
    """Board codes [64, 64] int8, move targets [64] int64, rewards [64] float32 (4 batches of 16)."""
    g = np.load(os.path.join(HERE, "movegen.npz"))
    rng = np.random.default_rng(20250717)
    pick = rng.choice(g["states"].shape[0], size=N_BATCHES * BS, replace=False)
    codes = np.ascontiguousarray(g["states"][pick, :64]).astype(np.int8)
    moves = rng.integers(0, 4096, N_BATCHES * BS).astype(np.int64)
    rewards = rng.choice(np.array([1.0, -1.0, 0.2], dtype=np.float32), N_BATCHES * BS)
    return codes, moves, rewards


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import torch
    import torch.nn.functional as F
    from make_golden import PIECES, import_reference
    from knightvision_amd.weights import synthetic_state_dict
    _, _, ref_model, ref_ai = import_reference(ref)
    torch.manual_seed(0)
    torch.set_num_threads(8)

    codes, moves, rewards = fixture_inputs()
    planes = np.stack([ref_ai.encode_board([[PIECES[int(c)] for c in row] for row in cd.reshape(8, 8)])
                       for cd in codes]).astype(np.float32)
    batches = [(torch.from_numpy(planes[i:i + BS]), torch.from_numpy(moves[i:i + BS]),
                torch.from_numpy(rewards[i:i + BS])) for i in range(0, N_BATCHES * BS, BS)]

    sd = synthetic_state_dict(42, "bn")
    model = ref_model.ChessNet()
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    model.train()
    names = [k for k, _ in model.named_parameters()]
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=LR)
    grads = []
    inner_step = opt.step

    after1 = {}

    def step(*a, **kw):  # the gradients the reference steps with (after its clip_grad_norm_)
        grads.append({k: p.grad.detach().clone() for k, p in model.named_parameters()})
        r = inner_step(*a, **kw)
        if len(grads) == 1:  # the parameters after the first optimizer step
            after1.update({k: p.detach().clone() for k, p in model.named_parameters()})
        return r
    opt.step = step

    class _Cuda(types.SimpleNamespace):
        pass
    torch_ns = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch) if not k.startswith("__")})
    torch_ns.cuda = _Cuda(amp=torch.cuda.amp, memory_allocated=lambda *a, **k: 0)
    glb = {"torch": torch_ns, "F": F, "tqdm": lambda it, **kw: it, "print": lambda *a, **k: None}
    exec(reference_function(ref, "_train_one_epoch"), glb)
    writer = types.SimpleNamespace(add_scalar=lambda *a, **k: None)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        scaler = torch.cuda.amp.GradScaler()  # train.py:272
        out = glb["_train_one_epoch"](model, batches, opt, 0, "cpu", writer, scaler, 0.0, COEF,
                                      accumulate_steps=ACCUM)
    total_loss, loss_policy, loss_value = float(out[0]), float(out[1]), float(out[2])
    assert len(grads) == N_BATCHES // ACCUM
    after = model.state_dict()

    rec = {"codes": codes, "moves": moves, "rewards": rewards,
           "meta": np.array([N_BATCHES, BS, ACCUM, COEF, LR]),
           "losses": np.array([total_loss, loss_policy, loss_value]),
           "param_names": np.array(names), "buffer_names": np.array(
               [k for k in after if k.endswith("running_mean") or k.endswith("running_var")])}
    for j, k in enumerate(names):
        idx = sample_index(before[k].shape, 1000 + j)
        rec[f"idx.{k}"] = idx
        for s, gs in enumerate(grads):
            g = gs[k].double().reshape(-1)
            rec[f"grad{s}.norm.{k}"] = np.array([float(g.norm())])
            rec[f"grad{s}.at.{k}"] = g[idx].numpy()
        rec[f"delta1.at.{k}"] = (after1[k].double() - before[k].double()).reshape(-1)[idx].numpy()
        d = (after[k].double() - before[k].double()).reshape(-1)
        rec[f"delta.at.{k}"] = d[idx].numpy()
        rec[f"delta.sum.{k}"] = np.array([float(d.sum())])
    for j, k in enumerate(rec["buffer_names"].tolist()):
        idx = sample_index(after[k].shape, 5000 + j)
        rec[f"idx.{k}"] = idx
        rec[f"buf.at.{k}"] = after[k].double().reshape(-1)[idx].numpy()
    out_path = os.path.join(HERE, "train_epoch.npz")
    np.savez_compressed(out_path, **rec)
    print(f"wrote {out_path}: total_loss {total_loss:.6f}, {len(names)} parameter tensors, "
          f"{len(grads)} optimizer steps")


if __name__ == "__main__":
    main()
