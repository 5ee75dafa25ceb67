"""CPU: the PyTorch actor-critic matches the reference model (cnn_ref.npz, captured
from src/actor_critic.py under torch.manual_seed(0)): same init RNG consumption,
same state_dict keys/shapes, same act/evaluate outputs (fp32 tolerance 1e-5)."""
import numpy as np
import torch


def _frames(codes, atlas):
    import oracle as O

    return torch.from_numpy(O.render(codes, atlas).astype(np.float32))


def test_state_dict_and_init_match_reference(golden):
    from merlin.actor_critic import CNNActorCritic

    g = golden("cnn_ref")
    torch.manual_seed(int(g["seed"]))
    ac = CNNActorCritic((56, 56, 3), 3)
    sd = ac.state_dict()
    assert list(sd.keys()) == [str(k) for k in g["keys"]]
    for (k, t), (s, a, first) in zip(sd.items(), g["sums"]):
        t = t.double()
        # orthogonal_ init = CPU QR; a different host LAPACK may move the last bits
        assert abs(t.sum().item() - s) <= 1e-5 * max(1.0, a), k
        assert abs(t.abs().sum().item() - a) <= 1e-6 * max(1.0, a), k
        assert abs(t.reshape(-1)[0].item() - first) <= 1e-6, k


def test_forward_matches_reference(golden):
    from merlin.actor_critic import CNNActorCritic

    g = golden("cnn_ref")
    torch.manual_seed(int(g["seed"]))
    ac = CNNActorCritic((56, 56, 3), 3)
    obs = _frames(g["codes"], golden("atlas")["atlas"])
    acts = torch.from_numpy(g["actions"])
    with torch.no_grad():
        a, lp, v = ac.act(obs, deterministic=True)
        lp2, ent, v2 = ac.evaluate(obs, acts)
        # the pre-scaled NCHW path used with the HIP expansion gives the same numbers
        lp3, ent3, v3 = ac.evaluate(obs.permute(0, 3, 1, 2).contiguous() * (1.0 / 255.0), acts, prescaled=True)
    assert (a.numpy() == g["act_action"]).all()
    for mine, ref in ((lp, "act_logp"), (v, "act_value"), (lp2, "ev_logp"), (ent, "ev_entropy"), (v2, "ev_value")):
        np.testing.assert_allclose(mine.numpy(), g[ref], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lp3.numpy(), g["ev_logp"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ent3.numpy(), g["ev_entropy"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v3.numpy(), g["ev_value"], rtol=1e-5, atol=1e-5)


def test_reference_checkpoint_keys_load():
    from merlin.actor_critic import CNNActorCritic

    a = CNNActorCritic((56, 56, 3), 3)
    b = CNNActorCritic((56, 56, 3), 3)
    b.load_state_dict(a.state_dict())  # strict: same key set


def test_mlp_variant_shapes():
    from merlin.actor_critic import MLPActorCritic

    m = MLPActorCritic(147, 3)
    x = torch.randn(5, 147)
    a, lp, v = m.act(x)
    assert a.shape == (5,) and lp.shape == (5,) and v.shape == (5,)
    lp2, ent, v2 = m.evaluate(x, a)
    assert torch.allclose(lp, lp2) and (ent > 0).all()
