"""Debug: which pre-tuned GEMM produces non-finite values in the bench workload?  Wraps
merlin.gemm_tuning.tuned() so that every GEMM issued inside it is re-run outside TunableOp on the
same operands and compared (non-finite outputs or a large relative difference are reported with
the op, shapes and strides); runs the bench's PPO loop for --iters iterations."""
import argparse
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd"))

_orig_bmm = torch.bmm
_active = {"on": False}
_bad = []


def checked_bmm(a, b, *args, **kw):
    out = _orig_bmm(a, b, *args, **kw)
    if _active["on"] and not torch.cuda.is_current_stream_capturing():
        import torch.cuda.tunable as tunable

        tunable.enable(False)
        ref = _orig_bmm(a, b)
        tunable.enable(True)
        o = out if out is not None else kw.get("out")
        fin = bool(torch.isfinite(o).all())
        rel = float((o - ref).norm() / ref.norm().clamp_min(1e-30)) if fin else float("inf")
        if not fin or rel > 1e-4:
            _bad.append((tuple(a.shape), a.stride(), tuple(b.shape), b.stride(), fin, rel))
            print("BAD bmm", _bad[-1], flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--graph", action="store_true", help="capture the rollout as in the bench")
    ap.add_argument("--nocheck", action="store_true", help="do not re-run the tuned GEMMs")
    args = ap.parse_args()
    from merlin import MerlinVecEnv, gemm_tuning
    from merlin.ppo import PPO

    orig_tuned = gemm_tuning.tuned

    @contextlib.contextmanager
    def tuned(which=""):
        with orig_tuned(which):
            _active["on"] = gemm_tuning._state["on"]
            try:
                yield
            finally:
                _active["on"] = False

    gemm_tuning.tuned = tuned
    if not args.nocheck:
        torch.bmm = checked_bmm
    dev = torch.device("cuda", 0)
    N, T = 4096, 256
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    agent = PPO(env, batch_size=N * T, minibatch_size=N * T // 8, ent_coef=0.05, device=dev, rollout_graph=args.graph)
    for it in range(args.iters):
        try:
            lv = agent.collect_rollouts()
        except Exception as e:  # noqa: BLE001
            fin = [bool(torch.isfinite(p).all()) for p in agent.ac.parameters()]
            lp = agent.buf.logprobs
            print(f"iter {it}: rollout failed: {e}; params finite {all(fin)}; logprobs finite "
                  f"{bool(torch.isfinite(lp).all())}; first bad step "
                  f"{int((~torch.isfinite(lp)).any(1).nonzero()[0]) if not torch.isfinite(lp).all() else -1}", flush=True)
            break
        stats = agent.update(lv)
        fin = all(bool(torch.isfinite(p).all()) for p in agent.ac.parameters())
        print(f"iter {it}: params finite {fin} windows {agent.last_num_windows} bad {len(_bad)} {stats}", flush=True)
        if not fin:
            break


if __name__ == "__main__":
    main()
