"""numpy restatement of the F(8x8) input transform for the GPU tests (test infrastructure): B10^T of the
points 0, +-2/5, +-4/5, +-5/4, +-2 and infinity (csrc/kv_wino88d.h w88d_bt, derived exactly by
tools/wino_emulate.toom_cook_exact), applied in fp64 to the zero-padded 10x10 plane of each (board, channel)."""
import os
import sys
from fractions import Fraction as Fr

import numpy as np

P88 = [Fr(0), Fr(2, 5), Fr(-2, 5), Fr(4, 5), Fr(-4, 5), Fr(5, 4), Fr(-5, 4), Fr(2), Fr(-2)]


def bt88():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from wino_emulate import toom_cook
    return toom_cook(P88, 8)[2]


def input_transform_f64(Y):
    """Y [boards][64][C] (pixel = row * 8 + col) -> V [100][boards][C], V = B^T d B of the padded plane d."""
    B, _, C = Y.shape
    d = np.zeros((B, 10, 10, C))
    d[:, 1:9, 1:9] = Y.reshape(B, 8, 8, C)
    BT = bt88()
    V = np.einsum("ai,bijc,dj->adbc", BT, d, BT)  # [10][10][boards][C]
    return V.reshape(100, B, C)
