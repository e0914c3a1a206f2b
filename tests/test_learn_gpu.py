"""The learn loop on one GPU (knightvision_amd.learn): self-play on the HIP
engine -> records -> update step (PyTorch-ROCm autograd) -> self-play with the
updated weights; after training, the eval-mode HIP forward of the trained
module (BN folded from the updated running statistics) must match the torch
fp32 restatement of ai/model.py within the logit tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_learn_loop_two_iterations():
    from knightvision_amd.learn import reinforcement_loop
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict, state_dict_to_numpy
    from oracle import torch_ref
    torch.manual_seed(0)
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
    before = {k: v.clone() for k, v in m.state_dict().items()}
    stats = reinforcement_loop(m, iterations=2, games_per_iter=8, device="cuda:0", epochs=1, batch_size=64,
                               max_moves=24, slots=8, log=None)
    assert stats[0]["records"] > 0 and stats[0]["games"] == 8
    assert stats[1]["optimizer_steps"] > 0 and np.isfinite(stats[1]["train_loss"])
    after = m.state_dict()
    assert any(not torch.equal(before[k].cpu(), after[k].cpu()) for k in before if "weight" in k)
    # trained weights + updated BN statistics through the HIP eval forward
    m.eval()
    g = np.random.default_rng(1)
    codes = (g.integers(0, 13, size=(24, 64)) * (g.random((24, 64)) < 0.4))
    from knightvision_amd.ai import codes_to_planes
    planes = codes_to_planes(codes)
    p, v = m(torch.from_numpy(planes).cuda())
    sd = state_dict_to_numpy(m.state_dict())
    rp, rv = torch_ref.forward({k: torch.from_numpy(x) for k, x in sd.items()}, planes)
    assert np.abs(p.cpu().numpy() - rp.numpy()).max() <= 1e-4
    assert np.abs(v.cpu().numpy() - rv.numpy()).max() <= 1e-5


def test_selfplay_shard_lazy_equals_faithful(monkeypatch):
    """KV_SELFPLAY_EVAL=lazy (the compact schedule: only the consumed network rows) plays the learn
    loop's self-play shard record for record like the default faithful schedule."""
    from knightvision_amd.learn import selfplay_shard
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "peaked").items()})
    out = {}
    for mode in ("faithful", "lazy"):
        monkeypatch.setenv("KV_SELFPLAY_EVAL", mode)
        out[mode] = selfplay_shard(m, 48, 0, "cuda:0", max_moves=40, slots=24)
    (ra, ga), (rb, gb) = out["faithful"], out["lazy"]
    assert len(ra) > 0 and np.array_equal(ra, rb) and np.array_equal(ga, gb)


def test_learn_loop_with_jsonl_dataset_and_validation(tmp_path):
    """learn.py's loop with its JSONL training data (ChessPGNDataset, learn.py:162): the self-play records
    extend it, every iteration trains on a 90/10 random split with a validation loss (train.py:293-420's
    train_with_validation: plateau scheduler, early stopping)."""
    import json
    from knightvision_amd.learn import reinforcement_loop
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    sans = ["a3", "a4", "b3", "b4", "c3", "c4", "d3", "d4", "e3", "e4", "f3", "f4", "g3", "g4", "h3", "h4",
            "Na3", "Nc3", "Nf3", "Nh3"]
    path = tmp_path / "games.jsonl"
    with open(path, "w") as f:
        for k in range(3):
            for i, san in enumerate(sans):
                f.write(json.dumps({"fen": start, "move": san, "result": ["1-0", "0-1", "1/2-1/2"][(i + k) % 3]}) + "\n")
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
    stats = reinforcement_loop(m, iterations=2, games_per_iter=8, device="cuda:0", epochs=2, batch_size=16,
                               max_moves=24, slots=8, games_path=str(path), max_samples=60, log=None)
    s0, s1 = stats
    assert s0["train_split"] == 54 and s0["val_split"] == 6 and s0["epochs_run"] == 2
    assert np.isfinite(s0["val_loss"]) and np.isfinite(s1["val_loss"]) and s0["optimizer_steps"] > 0
    assert s1["train_split"] + s1["val_split"] == s0["records"] and s0["records"] > 60  # extended by self-play
