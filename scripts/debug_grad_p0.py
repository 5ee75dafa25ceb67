"""Diagnostic (round 6): which weights does the benched update's first step differentiate at?  Loads the fixture's
starting weights into an agent, then compares the first-step gradient of (a) the benched path and (b) the plain
frame path (F.conv2d towers, no windows / grouping) with the fixture's reference gradient.
    python scripts/debug_grad_p0.py"""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "ppo-2dgrid_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np
import torch


def run(fast: bool, load=True):
    from merlin import MerlinVecEnv
    from merlin.ppo import PPO
    from test_gpu_obs_gae import pack

    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(REPO, "tests", "golden", "update_grad_ref.npz"))
    B, MB, EP = (int(x) for x in g["cfg"])
    env = MerlinVecEnv(1, "mediumhard", seed=1, device=dev)
    perms = torch.from_numpy(g["perms"])
    torch.manual_seed(0)
    kw = {} if fast else dict(conv1_from_codes=False, dedup=False, windows=False)
    agent = PPO(env, lr=3e-4, gamma=0.99, lam=0.95, clip_eps=0.2, update_epochs=EP, batch_size=B, minibatch_size=MB,
                vf_coef=0.5, ent_coef=0.05, device=dev, perm_fn=lambda n, e: perms[e], **kw)
    named = list(agent.ac.named_parameters())
    before = [p.detach().clone() for _, p in named]
    with torch.no_grad():
        for i, (_, p) in enumerate(named):
            if load is True or (load and any(named[i][0].startswith(pre) for pre in load)):
                p.copy_(torch.from_numpy(g[f"p0_{i}"]).to(dev))
    flat = getattr(agent, "_flat_params", None)
    if flat is not None:
        cat = torch.cat([p.detach().reshape(-1) for _, p in named])
        print("flat buffer == parameters:", torch.equal(flat, cat), "wstep before update:", agent._wstep is not None)
    print("init differs from the fixture by", max((b.cpu() - torch.from_numpy(g[f"p0_{i}"])).abs().max().item()
                                                    for i, b in enumerate(before)))
    buf = agent.buf
    buf.codes[:B, 0] = torch.from_numpy(pack(g["codes"])).to(dev)
    for dst, key, dt in ((buf.actions, "actions", torch.int64), (buf.logprobs, "logp", torch.float32),
                         (buf.values, "values", torch.float32), (buf.rewards, "rewards", torch.float32),
                         (buf.dones, "dones", torch.float32)):
        dst[:, 0] = torch.from_numpy(g[key]).to(device=dev, dtype=dt)
    rec = {}
    adv_orig = agent._advantages

    def adv_wrap(rewards, values, dones, last_value, *a, **k):
        _, ret = adv_orig(rewards, values, dones, last_value, *a, **k)
        ret.copy_(torch.from_numpy(g["returns"]).to(dev).view_as(ret))
        return torch.from_numpy(g["adv_norm"]).to(dev).view_as(ret), ret

    agent._advantages = adv_wrap
    opt_step = agent._clip_adam.step if agent._clip_adam is not None else None

    def grab():
        if "g" not in rec:
            rec["g"] = [p.grad.detach().clone() for _, p in named]
            rec["p"] = [p.detach().clone() for _, p in named]

    if opt_step is not None:
        def step_wrap():
            grab()
            return opt_step()
        agent._clip_adam.step = step_wrap
    else:
        o = agent.optimizer.step

        def ostep(*a, **k):
            grab()
            return o(*a, **k)
        agent.optimizer.step = ostep
    agent.update(float(g["last_value"]))
    pdiff = max((p.cpu() - torch.from_numpy(g[f"p0_{i}"])).abs().max().item() for i, p in enumerate(rec["p"]))
    print(("fast" if fast else "frame"), "path, loaded" if load else "path, own init", ": params at the first step vs "
          "fixture p0:", pdiff)
    for i, (n, _) in enumerate(named[:4] + named[6:7] + named[12:13]):
        j = [m for m, _ in named].index(n)
        gr = torch.from_numpy(g[f"grad{j}"]).double()
        print(f"   {n:36s} vs reference {((rec['g'][j].double().cpu() - gr).norm() / gr.norm()).item():.2e}")
    return rec["g"]


if __name__ == "__main__":
    rel = lambda x, y: max(((u - v).norm() / v.norm()).item() for u, v in zip(x, y))  # noqa: E731
    b = run(True, load=False)
    d = run(False, load=False)
    for sub_ in (("actor.2",), ("actor.0",), ("actor_extractor",), ("critic",)):
        a = run(True, load=sub_)
        c = run(False, load=sub_)
        print(sub_, "fast: loaded vs own", rel(a, b), "| frame: loaded vs own", rel(c, d), "| fast vs frame", rel(a, c))
