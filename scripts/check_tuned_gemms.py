"""Check the shipped TunableOp solutions (merlin/gemm_tuning.py) against PyTorch's default GEMMs on
the same operands: every fc1 shape in the file (forward with epilogue, input gradient, split-K
weight gradient) and the rollout shapes, eager and inside a captured HIP graph."""
import os
import re
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    import torch.cuda.tunable as tunable

    from merlin import gemm_tuning
    from merlin.actor_critic import _splitk_bmm_tn, bias_relu_bmm

    dev = torch.device("cuda", 0)
    rows = sorted({int(m.group(1)) for m in re.finditer(r"nn_576_(\d+)_512_B_2", open(gemm_tuning.TUNED_FILE).read())})
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    W = torch.randn(2, 512, 576, device=dev, generator=g) * 0.05
    b = torch.randn(2, 512, device=dev, generator=g)
    n = 4096
    A3 = torch.randn(2, n * 9, 576, device=dev, generator=g)
    W3t = torch.randn(2, 64, 576, device=dev, generator=g).transpose(1, 2).contiguous()
    a3r = torch.randn(2, n, 576, device=dev, generator=g)
    W4t = W.transpose(1, 2)

    def run_all(npad_list):
        out = [torch.bmm(A3, W3t), torch.bmm(a3r, W4t)]
        for npad in npad_list:
            gg = torch.Generator(device=dev)
            gg.manual_seed(npad)
            a3 = torch.randn(2, npad, 576, device=dev, generator=gg)
            dz = torch.randn(2, npad, 512, device=dev, generator=gg)
            out += [bias_relu_bmm(a3, W.transpose(1, 2), b), torch.bmm(dz, W), _splitk_bmm_tn(a3, dz, 32)]
        return out

    ref = run_all(rows)
    assert gemm_tuning.enable(), "tuned file not loaded"
    with gemm_tuning.tuned():
        print("tunable enabled:", tunable.is_enabled(), "tuning:", tunable.tuning_is_enabled(), flush=True)
        got = run_all(rows)
    assert not tunable.is_enabled()
    bad = 0
    for i, (x, y) in enumerate(zip(got, ref)):
        r = rel(x, y)
        ok = torch.isfinite(x).all().item() and r < 1e-5
        bad += not ok
        print(f"op {i}: rel {r:.2e} finite {torch.isfinite(x).all().item()}", flush=True)
    # the rollout shapes inside a captured graph
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            torch.bmm(A3, W3t)
    torch.cuda.current_stream(dev).wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr), gemm_tuning.tuned():
        o1 = torch.bmm(A3, W3t)
        o2 = torch.bmm(a3r, W4t)
    gr.replay()
    torch.cuda.synchronize()
    for x, y in ((o1, ref[0]), (o2, ref[1])):
        r = rel(x, y)
        print(f"graph: rel {r:.2e} finite {torch.isfinite(x).all().item()}", flush=True)
        bad += not (torch.isfinite(x).all().item() and r < 1e-5)
    print("BAD" if bad else "OK", bad, flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
