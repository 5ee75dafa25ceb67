"""Debug: bench-shaped training iterations with fc1 on the h3 GEMMs; after every update check the parameters; on the
first non-finite one, replay that update from its saved state with a per-optimizer-step check (fast step) and print
the step, the GEMM operand scales and where the first non-finite values appear.
    python scripts/debug_h3_iter.py [iters] [num_envs] [k_steps]"""
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo-2dgrid_amd"))
import torch

from merlin import MerlinVecEnv
from merlin import fast_step as fs
from merlin.ppo import PPO


def finite(agent):
    return [k for k, p in agent.ac.named_parameters() if not torch.isfinite(p).all()]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for kv in os.environ.get("FS", "").split(","):  # fast_step switches, e.g. FS=WGRAD_SIDE=0,AMAX_FUSED=0
        if kv:
            k, v = kv.split("=")
            setattr(fs, k, bool(int(v)))
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    dev = torch.device("cuda", 0)
    env = MerlinVecEnv(N, "mediumhard", seed=777, device=dev)
    torch.manual_seed(777)
    B = N * T
    agent = PPO(env, batch_size=B, minibatch_size=B // 8, update_epochs=10, ent_coef=0.05, device=dev)
    agent.ac.fc1_impl = os.environ.get("FC1", agent.ac.fc1_impl)
    check_all = os.environ.get("CHECK_ALL") == "1"
    for it in range(iters):
        lv = agent.collect_rollouts()
        if check_all and it == iters - 1:
            bad = ["forced"]
            sd = copy.deepcopy(agent.ac.state_dict())
            opt = copy.deepcopy(agent.optimizer.state_dict())
            rng = torch.cuda.get_rng_state(dev)
        else:
            bad = None
        if bad is None:
            sd = copy.deepcopy(agent.ac.state_dict())
            opt = copy.deepcopy(agent.optimizer.state_dict())
            rng = torch.cuda.get_rng_state(dev)
            stats = agent.update(lv)
            torch.cuda.synchronize()
            bad = finite(agent)
            print(it, {k: round(v, 6) for k, v in stats.items()}, "non-finite:", bad, flush=True)
            if not bad:
                continue
        # replay with a check after every optimizer step
        agent.ac.load_state_dict(sd)
        agent.optimizer.load_state_dict(opt)
        torch.cuda.set_rng_state(rng, dev)
        orig = fs.WindowStep.step
        count = [0]

        def step(self, plan, mb, mb_idx, actions, logp_old, adv, ret, totals):
            orig(self, plan, mb, mb_idx, actions, logp_old, adv, ret, totals)
            torch.cuda.synchronize()
            st = self.stage
            o = st.offs["W4p"]
            nW = st.DG[o:st.offs["W4pT"]].numel()
            seen = st.flat_grad.index_select(0, st.fwd_map[o:o + nW])
            if not torch.equal(seen, st.DG[o:o + nW]):
                print(f"  step {count[0]}: the backward graph copied a dW4p other than the side stream's final one "
                      f"(max diff {float((seen - st.DG[o:o + nW]).abs().max()):.3e})", flush=True)
            am = self.amax_act.view(torch.float32).tolist()
            g = self.stage.grads
            gbad = [i for i, x in enumerate(g) if not torch.isfinite(x).all()]
            fbad = not torch.isfinite(self.flat).all()
            if gbad or fbad or count[0] % 10 == 0:
                print(f"  step {count[0]} amax act {am} amaxW {self.stage.amaxW.view(torch.float32).tolist()} "
                      f"non-finite stage grads {gbad} flat grad bad {fbad} U {int(mb.groups.numel())}", flush=True)
            if gbad or fbad:
                raise SystemExit(1)
            count[0] += 1

        fs.WindowStep.step = step
        agent.update(lv)
        print("replay finished without non-finite gradients; params:", finite(agent))
        return


if __name__ == "__main__":
    main()
