"""Offline GEMM tuning for merlin/gemm_tuning.py (run on an MI355X; writes a TunableOp CSV).

    python scripts/tune_gemms.py --lo 98304 --hi 131072 [--out gpurun_out/gemm_gfx950.csv]

For every fc1 row count npad in [lo, hi] that is a multiple of ROW_BUCKET, runs the update's fc1
GEMMs once with TunableOp tuning on -- the forward with its bias+ReLU epilogue per tower
(actor_critic.bias_relu_bmm), the input gradient (bmm) and the 32-chunk split-K weight gradient
(_splitk_bmm_tn) -- plus the rollout's fixed-shape conv3 / fc1 GEMMs at --envs envs.  An existing
--out file is read first and rewritten with old + new results at exit, so ranges can be tuned in
several runs.  Copy the result to ppo-2dgrid_amd/merlin/tuning/gemm_gfx950.csv."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lo", type=int, default=98304)
    ap.add_argument("--hi", type=int, default=131072)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out",
                                                  "gemm_gfx950.csv"))
    ap.add_argument("--inp", default=None, help="results to start from (default: --out if it exists)")
    ap.add_argument("--ms", type=int, default=10, help="max tuning ms per solution")
    ap.add_argument("--windows", action="store_true", help="also the window GEMMs, --wlo..--whi windows")
    ap.add_argument("--wlo", type=int, default=4096)
    ap.add_argument("--whi", type=int, default=9984)
    ap.add_argument("--no-rows", action="store_true", help="skip the fc1 row counts")
    args = ap.parse_args()
    from merlin.actor_critic import _splitk_bmm_tn, bias_relu_bmm
    from merlin.gemm_tuning import ROW_BUCKET

    import torch.cuda.tunable as tunable

    dev = torch.device("cuda", 0)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_max_tuning_duration(args.ms)
    tunable.set_max_tuning_iterations(20)
    tunable.set_filename(args.out)
    inp = args.inp or args.out
    if os.path.exists(inp):
        print("read", inp, tunable.read_file(inp), flush=True)
    K, H = 576, 512
    W = torch.randn(2, H, K, device=dev) * 0.05
    b = torch.randn(2, H, device=dev)
    t0 = time.time()
    n = args.envs
    A3 = torch.randn(2, n * 9, 576, device=dev)
    W3t = torch.randn(2, 576, 64, device=dev)
    torch.bmm(A3, W3t)
    torch.bmm(torch.randn(2, n, 576, device=dev), W.transpose(1, 2))
    torch.cuda.synchronize()
    print(f"rollout shapes ({n} envs) tuned, {time.time() - t0:.0f} s", flush=True)
    if args.windows:
        from merlin.gemm_tuning import WINDOW_BUCKET

        W3r = torch.randn(2, 64, 576, device=dev)
        for nw in range(args.wlo, args.whi + 1, WINDOW_BUCKET):  # merlin/windows.py _TunedBmm shapes
            a2w = torch.randn(2, nw, 64, device=dev)
            dQ = torch.randn(2, nw, 576, device=dev)
            torch.bmm(a2w, W3r)
            torch.bmm(dQ, W3r.transpose(1, 2))
            torch.bmm(a2w.transpose(1, 2), dQ)
        torch.cuda.synchronize()
        print(f"window GEMMs tuned, {time.time() - t0:.0f} s", flush=True)
    lo = (args.lo + ROW_BUCKET - 1) // ROW_BUCKET * ROW_BUCKET
    for npad in ([] if args.no_rows else range(lo, args.hi + 1, ROW_BUCKET)):
        a3 = torch.randn(2, npad, K, device=dev)
        dz = torch.randn(2, npad, H, device=dev)
        bias_relu_bmm(a3, W.transpose(1, 2), b)
        torch.bmm(dz, W)
        _splitk_bmm_tn(a3, dz, 32)
        torch.cuda.synchronize()
        del a3, dz
        print(f"rows {npad} tuned, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
