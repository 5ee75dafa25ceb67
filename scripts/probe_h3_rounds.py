"""Probe: time per round of blocks of the h3 NT GEMM (fc1 forward shape, both towers) at row counts whose A panel
fits L2 (few blocks) up to the update's shape: if the per-round time stays flat, global-load latency is not what
sets the k loop's pace.   python scripts/probe_h3_rounds.py [cfg ...]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat

TILES = {0: (256, 128), 1: (128, 192), 2: (128, 128), 3: (128, 256), 4: (256, 128), 6: (128, 192), 14: (256, 128), 10: (256, 128), 11: (128, 192), 12: (128, 128),
         20: (256, 128), 21: (128, 192), 22: (256, 128), 23: (128, 256), 24: (128, 128), 25: (128, 192),
         30: (256, 128), 31: (128, 192), 32: (256, 128), 33: (128, 256), 34: (128, 128), 35: (128, 192),
         13: (128, 256)}


def timeit(fn, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    cfgs = [int(c) for c in sys.argv[1:]] or [0, 3]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    W = torch.randn(2, 512, 576, device=dev, generator=g) / 24
    amW = nat.h3_amax(W)
    Hp = nat.h3_split(W, amW)
    b = torch.zeros(2, 512, device=dev)
    for U in (256, 2048, 8192, 32768, 111000):
        a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
        am = nat.h3_amax(a3)
        for cfg in cfgs:
            BM, BN = TILES[cfg]
            blocks = math.ceil(U / BM) * (512 // BN) * 2
            us = min(timeit(lambda: nat.h3_gemm_nt(a3, am, Hp, amW, bias=b, cfg=cfg)) for _ in range(3))
            rounds = math.ceil(blocks / 256)
            print(f"U {U:6d} cfg {cfg:2d} blocks {blocks:5d} rounds {rounds:3d}  {us:8.1f} us  {us / rounds:6.2f} us/round",
                  flush=True)


if __name__ == "__main__":
    main()
