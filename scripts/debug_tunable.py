"""Debug: are the shipped TunableOp solutions dispatched inside merlin.gemm_tuning.tuned()?  Prints
the loaded results count and the kernel names torch.profiler records for a tuned-shape bmm with
dispatch on / off, on the main thread and inside an autograd backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def kernels(fn):
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as p:
        fn()
        torch.cuda.synchronize()
    return sorted({e.name[:60] for e in p.events() if e.device_type == torch.autograd.DeviceType.CUDA})


def main():
    import torch.cuda.tunable as tunable

    from merlin import gemm_tuning

    dev = torch.device("cuda", 0)
    print("enable ->", gemm_tuning.enable(), "rows", gemm_tuning._state["rows"][:3], flush=True)
    print("results loaded:", len(tunable.get_results()), "filename", tunable.get_filename(), flush=True)
    n = gemm_tuning._state["rows"][5]
    dz = torch.randn(2, n, 512, device=dev)
    W = torch.randn(2, 512, 576, device=dev)
    def on():
        with gemm_tuning.tuned():
            torch.bmm(dz, W)
    print("on (first):", kernels(on), flush=True)
    print("off:", kernels(lambda: torch.bmm(dz, W)), flush=True)
    print("on:", kernels(on), flush=True)
    W2 = torch.randn(2, 576, 512, device=dev)
    a3 = torch.randn(2, n, 576, device=dev)
    print("wgrad-like on:", kernels(lambda: [gemm_tuning.tuned().__enter__(), torch.bmm(a3[:, :n // 32 * 32].reshape(2 * 32, n // 32, 576).transpose(1, 2), dz[:, :n // 32 * 32].reshape(64, n // 32, 512)), torch.cuda.tunable.enable(False)]), flush=True)

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            with gemm_tuning.tuned():
                torch.bmm(dz, W)
            return g

    x = torch.randn(4, device=dev, requires_grad=True)
    print("in backward:", kernels(lambda: F.apply(x).sum().backward()), flush=True)
    print("results after:", len(tunable.get_results()), flush=True)


if __name__ == "__main__":
    main()
