"""Which stage of the fp32 tower on int8 digits sets its error on learn-loop weights:
run the learn loop (MCTS, 64 sims, 256 games per iteration) on the GPU until the load-time calibration
moves self-play off `winograd88_i8f32`, then (a) the library's calibration errors of the candidates on those
weights and (b) host emulation (tools/wino_precision_emulate.py) of the F(8x8) tower with each stage in
fp32 or fp64 on seeded boards, against the float64 forward. Planning tool: nothing in the product depends
on it.

    python tools/r05_learn_stage_emulate.py [max_iterations] [n_boards]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    max_it = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    from knightvision_amd.learn import reinforcement_loop
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict
    torch.cuda.set_device(0)
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
    stats = reinforcement_loop(m, max_it, 256, "cuda:0", max_moves=80, sims=64, log=None)
    paths = [st.get("nn_path") for st in stats]
    print(json.dumps({"nn_path_per_iteration": paths}), flush=True)
    m.eval()
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()
          if v.dtype.is_floating_point}
    cal = m.kv_net(0).calibration()
    print(json.dumps({"calibration_final_weights": {k: cal[k] for k in ("path_large", "err_logit", "err_value")}}),
          flush=True)
    import wino_precision_emulate as W
    from knightvision_amd.ai import codes_to_planes
    from oracle import torch_ref
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 13, size=(nb, 64)) * (rng.random((nb, 64)) < 0.4)
    planes = codes_to_planes(codes)
    p64, v64 = torch_ref.forward({k: torch.from_numpy(v) for k, v in sd.items()},
                                 torch.from_numpy(planes.astype(np.float64)))
    p64, v64 = p64.numpy(), v64.numpy().reshape(-1)
    p32, v32 = torch_ref.forward({k: torch.from_numpy(v.astype(np.float32)) for k, v in sd.items()},
                                 torch.from_numpy(planes.astype(np.float32)))
    print(f"reference fp32 forward (torch CPU)            dlogit {np.abs(p32.numpy() - p64).max():.3e} "
          f"dvalue {np.abs(v32.numpy().reshape(-1) - v64).max():.3e}", flush=True)
    T88 = W.toom_cook(W.P88, 8)
    F32, D = np.float32, np.float64
    cases = [("fp32 MFMA tower (V, U, M, out fp32; fp32 GEMM)", F32, F32, F32, True),
             ("~ int8-digit fp32 tower (V f32, U f64, GEMM f64, M+out f32)", F32, D, F32, False),
             ("  + output transform and M in fp64", F32, D, D, False),
             ("  + input transform and V in fp64 (M+out f32)", D, D, F32, False),
             ("all fp64 (the fp64 domain)", D, D, D, False)]
    for name, vp, gp, op, seq in cases:
        p, v = W.fwd(sd, planes, 8, T88, vp, gp, op, seq)
        print(f"{name:62s} dlogit {np.abs(p - p64).max():.3e} dvalue {np.abs(v - v64).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
