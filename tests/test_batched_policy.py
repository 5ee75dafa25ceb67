"""CPU: merlin.batched_policy (per-task stacked weights, used by FOMAML) equals running
each task's CNNActorCritic separately -- outputs and per-task gradients."""
import torch


def test_stacked_forward_and_grads_match_individual_models():
    from merlin import batched_policy as bp
    from merlin.actor_critic import CNNActorCritic

    torch.manual_seed(0)
    models = [CNNActorCritic((56, 56, 3), 3) for _ in range(3)]
    names = [n for n, _ in models[0].named_parameters()]
    params = {n: torch.stack([dict(m.named_parameters())[n].detach() for m in models]).requires_grad_(True)
              for n in names}
    frames = torch.rand(3, 5, 3, 56, 56)
    acts = torch.randint(0, 3, (3, 5))
    lp, ent, v = bp.evaluate(params, frames, acts)
    (lp.sum() + 0.3 * ent.sum() + (v ** 2).sum()).backward()
    for g, m in enumerate(models):
        lp_r, ent_r, v_r = m.evaluate(frames[g], acts[g], prescaled=True)
        torch.testing.assert_close(lp[g], lp_r, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(ent[g], ent_r, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(v[g], v_r, rtol=1e-5, atol=1e-6)
        (lp_r.sum() + 0.3 * ent_r.sum() + (v_r ** 2).sum()).backward()
        for n, p in m.named_parameters():
            torch.testing.assert_close(params[n].grad[g], p.grad, rtol=1e-4, atol=1e-6)


def test_stack_params_copies_and_act_shapes():
    from merlin import batched_policy as bp
    from merlin.actor_critic import CNNActorCritic

    m = CNNActorCritic((56, 56, 3), 3)
    st = bp.stack_params(m, 4)
    assert all(v.shape[0] == 4 and v.requires_grad and v.is_leaf for v in st.values())
    a, lp, v = bp.act(st, torch.rand(4, 2, 3, 56, 56), deterministic=True)
    assert a.shape == (4, 2) and lp.shape == (4, 2) and v.shape == (4, 2)
