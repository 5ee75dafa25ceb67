"""GPU: the ppo_train.py drop-in CLI end to end (tiny budget) and the batched evaluation
against a serial single-env loop (the reference's evaluate_policy structure)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _load_cli():
    import importlib.util

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd", "ppo_train.py")
    spec = importlib.util.spec_from_file_location("ppo_train", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_cli_vectorised_run_writes_reference_layout(tmp_path, monkeypatch, device):
    mod = _load_cli()
    monkeypatch.chdir(tmp_path)
    args = mod.parse_args(["--device", "cuda", "--difficulty", "mediumhard", "--seed", "777", "--num_envs", "128",
                           "--k_steps", "16", "--minibatch_size", "512", "--update_epochs", "2",
                           "--total_steps", "4096", "--save_interval", "2048", "--group_timestamp", "T"])
    agent = mod.train_minigrid(args)
    d = tmp_path / "checkpoints" / "MERLIN-MediumHard-v0_16x16_mediumhard_T" / "seed_777"
    names = sorted(os.listdir(d))
    assert "best_model.pth" in names and "ppo_model_final.pth" in names and "ppo_model_4k.pth" in names
    sd = torch.load(d / "ppo_model_final.pth", weights_only=True)
    assert set(sd) == set(agent.ac.state_dict())
    assert (tmp_path / "tb_logs").exists()


def test_cli_cfg1_single_env_reference_run(tmp_path):
    """BASELINE cfg 1, the reference's own CPU-runnable plumbing config, end to end as a user runs it:
    `ppo_train.py --num_envs 1 --difficulty mediumhard --seed 777 --total_steps 10000` (the loop of
    ppo/ppo_train.py:112-196: 5 iterations of a 2048-step single-env rollout, 10 epochs x 8 minibatches
    of 256, a 3-episode deterministic eval per iteration, best / milestone / final checkpoints)."""
    import json
    import subprocess
    import sys

    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd",
                          "ppo_train.py")
    r = subprocess.run([sys.executable, script, "--difficulty", "mediumhard", "--seed", "777", "--total_steps",
                        "10000", "--num_envs", "1", "--device", "cuda", "--group_timestamp", "CFG1"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("[")]
    assert len([ln for ln in lines if "R:" in ln]) == 5, r.stdout[-2000:]  # 5 x 2048 >= 10000
    assert lines[-1].startswith("[  10240]")
    d = tmp_path / "checkpoints" / "MERLIN-MediumHard-v0_16x16_mediumhard_CFG1" / "seed_777"
    names = set(os.listdir(d))
    assert {"best_model.pth", "ppo_model_10k.pth", "ppo_model_final.pth"} <= names
    sd = torch.load(d / "ppo_model_final.pth", weights_only=True)
    assert "actor_extractor.network.0.weight" in sd and "critic.2.bias" in sd
    tb = tmp_path / "tb_logs" / "MERLIN-MediumHard-v0_16x16_mediumhard_CFG1" / "seed_777"
    if (tb / "scalars.jsonl").exists():  # no tensorboard in the image: the JSONL stand-in
        tags = {json.loads(ln)["tag"] for ln in open(tb / "scalars.jsonl")}
        assert {"reward/avg_eval_reward", "loss/policy_loss", "diagnostics/gradnorm"} <= tags


def test_batched_eval_matches_serial_single_env(device):
    from merlin import MerlinEnv
    from merlin.actor_critic import CNNActorCritic
    from merlin.evaluation import evaluate_policy

    torch.manual_seed(3)
    ac = CNNActorCritic((56, 56, 3), 3).to(device)
    rewards, steps = evaluate_policy(ac, "mediumhard", episodes=3, seed=1776, device=device, max_steps=60)
    env = MerlinEnv("mediumhard", device=device, max_steps=60)
    for ep in range(3):
        obs, _ = env.reset(seed=1776 + ep)
        total, n, done = 0.0, 0, False
        while not done:
            with torch.no_grad():
                a, _, _ = ac.act(torch.from_numpy(obs.astype(np.float32)).to(device)[None], deterministic=True)
            obs, r, te, tr, _ = env.step(int(a.item()))
            total += r
            n += 1
            done = te or tr
        assert n == steps[ep]
        assert abs(total - rewards[ep]) < 1e-6


def test_cli_single_env_seed_reproducible(tmp_path, monkeypatch, device):
    """--seed reproduces a single-env (num_envs 1) run: the env is reset with seed + rank once
    (create_env ignores its seed, like the reference's, so ppo_train sets it), and two runs with
    the same seed give the same maps, episodes and weights; another seed gives other maps."""
    mod = _load_cli()
    monkeypatch.chdir(tmp_path)

    def run(seed, ts):
        args = mod.parse_args(["--device", "cuda", "--difficulty", "mediumhard", "--seed", str(seed), "--num_envs",
                               "1", "--batch_size", "128", "--minibatch_size", "64", "--update_epochs", "1",
                               "--total_steps", "256", "--eval_episodes", "1", "--group_timestamp", ts])
        agent = mod.train_minigrid(args)
        return (agent.buf.codes.cpu().clone(), agent.vec.get_state()["rng"],
                {k: v.cpu().clone() for k, v in agent.ac.state_dict().items()})

    c1, r1, s1 = run(777, "A")
    c2, r2, s2 = run(777, "B")
    c3, r3, _ = run(778, "C")
    assert torch.equal(c1, c2) and (r1 == r2).all()
    assert all(torch.equal(s1[k], s2[k]) for k in s1)
    assert not (r1 == r3).all()


def test_fomaml_cli_smoke(tmp_path, monkeypatch, capsys, device):
    """fomaml_train.py (drop-in for the reference's fomaml/fomaml_train.py:37-178) end to end at a tiny budget:
    ten meta-iterations of 4 tasks; the reference's output files (best_model.pth :128-132, fomaml_iter_<k>.pth and
    training_curves.png :138-157) and its per-10-iteration log fields (:136)."""
    import importlib.util
    import re

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ppo-2dgrid_amd",
                        "fomaml_train.py")
    spec = importlib.util.spec_from_file_location("fomaml_train", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.chdir(tmp_path)
    args = mod.parse_args(["--device", "cuda", "--difficulty", "mediumhard", "--seed", "7", "--iterations", "10",
                           "--tasks_per_batch", "4", "--k_steps", "32", "--save_every", "5"])
    fomaml = mod.train_fomaml(args)
    out = capsys.readouterr().out
    runs = os.listdir(tmp_path / "checkpoints")
    assert len(runs) == 1 and runs[0].startswith("MERLIN-MediumHard-v0_16x16_mediumhard_FOMAML_")
    d = tmp_path / "checkpoints" / runs[0] / "seed_7"
    names = sorted(os.listdir(d))
    assert names == ["best_model.pth", "fomaml_iter_10.pth", "fomaml_iter_5.pth", "training_curves.png"]
    assert (d / "training_curves.png").read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    for name in ("best_model.pth", "fomaml_iter_10.pth"):
        sd = torch.load(d / name, weights_only=True)
        assert set(sd) == set(fomaml.meta_policy.state_dict())
        assert all(torch.isfinite(v).all() for v in sd.values())
    line = [ln for ln in out.splitlines() if ln.startswith("Iter ")]
    assert len(line) == 1
    assert re.fullmatch(r"Iter\s+10 \| R: -?[\d.]+ \| L: -?[\d.]+ \| pi: -?[\d.]+ \| V: -?[\d.]+ \| Ent: -?[\d.]+ \| "
                        r"KL: -?[\d.]+ \| Steps: [\d.]+ \| Best: -?[\d.]+ \| T: [\d.]+m", line[0]), line[0]
    assert "[*] New Best Model Saved (Rew: " in out and "[*] Saved training curves to: " in out
