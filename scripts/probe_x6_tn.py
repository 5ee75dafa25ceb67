"""A/B of the x6 TN (weight-gradient) GEMM variants at fc1's update shape, one process, interleaved
rounds, median per (cfg, splits); error vs float64 relative to the result's norm on a cancelling
gradient.  python scripts/probe_x6_tn.py [U] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import _native as nat


def ev_time(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 116192
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    combos = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("COMBOS", "0:32,20:32,30:32,30:16").split(",")]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    a3 = torch.relu(torch.randn(2, U, 576, device=dev, generator=g))
    sgn = torch.where(torch.rand(2, U, 1, device=dev, generator=g) < 0.5005, 1.0, -1.0)
    dz = sgn * torch.rand(2, U, 512, device=dev, generator=g) * (torch.rand(2, U, 512, device=dev, generator=g) > 0.5)
    W64 = torch.bmm(dz.double().transpose(1, 2), a3.double())
    rel = lambda W: float((W.double() - W64).norm() / W64.norm())  # noqa: E731
    print(f"hipBLASLt fp32 rel err {rel(torch.bmm(dz.transpose(1, 2), a3)):.3e}", flush=True)
    dzp, a3p = nat.x6_split(dz), nat.x6_split(a3)  # planes operands for the cfg >= 30 kernels
    ops = lambda c: (dzp, a3p) if c >= 30 else (dz, a3)  # noqa: E731
    ok = {}
    for c, s in combos:
        try:
            W = nat.x6_gemm_tn(*ops(c), splits=s, cfg=c)
            ok[(c, s)] = (rel(W), bool(torch.equal(W, nat.x6_gemm_tn(*ops(c), splits=s, cfg=c))))
        except nat.MerlinNativeError as ex:
            print(c, s, ex)
    times = {k: [] for k in ok}
    for _ in range(rounds):
        for c, s in ok:
            times[(c, s)].append(ev_time(lambda: nat.x6_gemm_tn(*ops(c), splits=s, cfg=c)))
    ex = 6 * 2 * 2 * U * 512 * 576
    for k in ok:
        med = statistics.median(times[k])
        print(f"cfg {k[0]:2d} splits {k[1]:2d}: median {med:8.1f} us  min {min(times[k]):8.1f}  "
              f"{ex / med / 1e6:7.1f} TF executed ({ex / med / 1e6 / 2500:.3f} of 2.5 PF)  rel err {ok[k][0]:.3e} "
              f"reproducible {ok[k][1]}", flush=True)


if __name__ == "__main__":
    main()
