"""weights.py's synthetic weight sets (CPU): the "stress" set is the "bn" set
with data-calibrated BatchNorm statistics and scaled heads, deterministic and
returned as fresh copies; the reference ChessNet's golden outputs for it
(tests/golden/nn.npz) match the functional fp32 restatement."""
import os

import numpy as np
import torch

from knightvision_amd.weights import STRESS_LOGIT_STD, _stress_calibration_codes, synthetic_state_dict


def test_stress_is_bn_with_calibrated_statistics():
    bn, st = synthetic_state_dict(42, "bn"), synthetic_state_dict(42, "stress")
    assert list(bn) == list(st)
    for k in bn:
        if k.endswith(("running_mean", "running_var")) or k in ("policy_fc.weight", "value_fc2.weight"):
            continue
        assert np.array_equal(bn[k], st[k]), k
    # conv1's BN statistics are the batch statistics of conv1's output on the calibration boards
    from knightvision_amd.ai import codes_to_planes
    x = torch.from_numpy(codes_to_planes(_stress_calibration_codes(42)).astype(np.float64))
    z = torch.nn.functional.conv2d(x, torch.from_numpy(st["conv1.weight"].astype(np.float64)),
                                   torch.from_numpy(st["conv1.bias"].astype(np.float64)), padding=1)
    assert np.allclose(z.mean(dim=(0, 2, 3)).numpy(), st["bn1.running_mean"], rtol=1e-5, atol=1e-6)
    assert np.allclose(z.var(dim=(0, 2, 3), unbiased=False).numpy(), st["bn1.running_var"], rtol=1e-5)
    # policy_fc.weight scaled so that W f has standard deviation STRESS_LOGIT_STD on those boards (the bias,
    # unscaled, moves the logits' std by ~1 %)
    from oracle import torch_ref
    p, _ = torch_ref.forward({k: torch.from_numpy(np.asarray(v, dtype=np.float64)) for k, v in st.items()}, x)
    assert abs(float(p.std()) / STRESS_LOGIT_STD - 1) < 0.03


def test_stress_copies_are_independent():
    a = synthetic_state_dict(42, "stress")
    a["policy_fc.weight"][:] = 0
    b = synthetic_state_dict(42, "stress")
    assert np.abs(b["policy_fc.weight"]).max() > 0


def test_stress_golden_matches_restatement(golden_dir):
    from oracle import torch_ref
    g = np.load(os.path.join(golden_dir, "nn.npz"))
    p, v = torch_ref.forward(synthetic_state_dict(42, "stress"), g["planes"])
    # the reference module's fp32 outputs vs the functional restatement's (both CPU fp32)
    assert np.abs(p.numpy() - g["policy_stress"]).max() < 1e-4
    assert np.abs(v.numpy().reshape(-1) - g["value_stress"].reshape(-1)).max() < 1e-5
