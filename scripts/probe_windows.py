"""How many distinct conv2 / conv3 receptive-field windows does a bench-like rollout hold?

CPU probe on the C oracle (N mediumhard envs x 256 random-action steps): conv3 output (i, j)
of a frame depends only on the 5x5 tile-class window at (i, j) (translation invariance),
conv2 output (py, px) on the 3x3 window at (py, px).  Prints distinct frames / windows per
random 131072-frame minibatch and over the whole rollout (diagnostic only)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402

N, T, MB = int(os.environ.get("N", 4096)), 256, 131072
rng = np.random.default_rng(1)
acts = rng.integers(0, 3, size=(T, N))
codes, *_ = oracle.batch_rollout(777 + np.arange(N), acts)
frames = codes[:T].reshape(-1, 7, 7).astype(np.int64)
B = frames.shape[0]


def keys(fr, k, npos):
    out = np.zeros((fr.shape[0], npos, npos), dtype=np.int64)
    for a in range(k):
        for b in range(k):
            out = out * 5 + fr[:, a:a + npos, b:b + npos]
    return out


k3 = keys(frames, 5, 3).reshape(B, 9)
k2 = keys(frames, 3, 5).reshape(B, 25)
k3p = k3 * 9 + np.arange(9)  # (position, window) pairs: fc1's weights are per position
print(f"frames {B}")
for m in range(3):
    idx = rng.permutation(B)[:MB]
    uf = np.unique(frames[idx].reshape(MB, 49), axis=0).shape[0]
    u3 = np.unique(k3[idx]).shape[0]
    u3p = np.unique(k3p[idx]).shape[0]
    u2 = np.unique(k2[idx]).shape[0]
    print(f"mb {m}: distinct frames {uf} ({uf / MB:.3f}); conv3 windows {u3} ({u3 / (9 * MB):.4f} of 9*MB), "
          f"(p3, window) {u3p} ({u3p / (9 * uf):.3f} of 9*distinct); conv2 windows {u2}")
print("whole rollout: distinct frames", np.unique(frames.reshape(B, 49), axis=0).shape[0],
      "conv3 windows", np.unique(k3).shape[0], "conv2 windows", np.unique(k2).shape[0])
