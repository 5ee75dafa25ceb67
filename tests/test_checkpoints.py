"""CPU: checkpoint interop (merlin/checkpoints.py).  The legacy layout of the reference's older
checkpoints (one shared conv stack under feature_extractor.conv.*) is copied into both towers as
src/sweep_checkpoints.py:31-47 does; current checkpoints round-trip through torch.save /
torch.load(weights_only=True) with the reference's keys."""
import torch


def _legacy_from(model):
    sd = model.state_dict()
    out = {}
    for k, v in sd.items():
        if k.startswith("actor_extractor.network"):
            out[k.replace("actor_extractor.network", "feature_extractor.conv")] = v.clone()
        elif not k.startswith("critic_extractor"):
            out[k] = v.clone()
    return out


def test_legacy_state_dict_maps_into_both_towers(tmp_path):
    from merlin.actor_critic import CNNActorCritic
    from merlin.checkpoints import is_legacy, load_policy, remap_legacy_state_dict

    torch.manual_seed(3)
    src = CNNActorCritic((56, 56, 3), 3)
    legacy = _legacy_from(src)
    assert is_legacy(legacy)
    mapped = remap_legacy_state_dict(legacy)
    for k, v in src.state_dict().items():
        if k.startswith("critic_extractor"):  # the shared stack lands in the critic tower too
            assert torch.equal(mapped[k], src.state_dict()[k.replace("critic_", "actor_")])
        else:
            assert torch.equal(mapped[k], v)
    path = tmp_path / "legacy.pth"
    torch.save(legacy, path)
    pol = load_policy(str(path), device="cpu")
    assert not pol.training
    for k, v in pol.state_dict().items():
        assert torch.equal(v, mapped[k])


def test_current_checkpoint_round_trip(tmp_path):
    from merlin.actor_critic import CNNActorCritic
    from merlin.checkpoints import is_legacy, load_policy

    torch.manual_seed(4)
    src = CNNActorCritic((56, 56, 3), 3)
    path = tmp_path / "ppo_model_final.pth"
    torch.save(src.state_dict(), path)
    sd = torch.load(path, weights_only=True)
    assert not is_legacy(sd)
    pol = load_policy(str(path), device="cpu")
    for (k, a), (k2, b) in zip(src.state_dict().items(), pol.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
