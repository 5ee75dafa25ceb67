"""CNNActorCritic with one weight set per group (task), on the tile-code path, batched over groups.

FOMAML (src/fomaml.py:158-223) adapts its own copy of the policy per task.  The per-task copies live as
stacked tensors [G, *shape] under CNNActorCritic's parameter names (merlin.batched_policy.stack_params),
and every tower of every task is one "tower" of the code path's kernels: tower 2g is task g's actor
extractor, 2g + 1 its critic extractor.  Group g's frames (codes rows g*F .. g*F + F - 1) run through

  conv1 + conv2   per-tower tables (CNNActorCritic.conv2_tables' construction, 2G towers) and grouped
                  table lookups (merlin_tower_conv2_lut_fwd_grouped: each frame only through its own
                  task's two towers); backward: the grouped fixed-point histogram
                  (merlin_tower_conv2_lut_bwd_grouped) and autograd through the tables
  conv3           im2col (merlin_tower_conv3_im2col_fwd, 2G towers) + one batched GEMM over the 2G towers
  fc1, heads      batched GEMMs over the towers / tasks

-- the same function as src/actor_critic.py:9-64 for each task's weights, fp32 sums regrouped, with
every task's gradient from one autograd pass (tasks share no parameters).  No frame is ever expanded:
the reference's RGB frames are 7x7 blits of 5 atlas tiles (merlin/actor_critic.py)."""
from __future__ import annotations

import torch

from . import _native as nat
from .actor_critic import _Conv2Tables, _entropy, _lut2_gather_matrix

TOWERS = ("actor_extractor", "critic_extractor")
_STATE = {}


def _consts(device):
    c = _STATE.get(device)
    if c is None:
        a = torch.from_numpy(nat.tile_atlas()).permute(0, 3, 1, 2).float() / 255.0
        G, part = _lut2_gather_matrix()
        c = _STATE[device] = (a.contiguous().to(device), G.to(device), part.to(device))
    return c


def _towers(params, key):
    """[2G, *shape]: group g's actor tower at 2g, critic tower at 2g + 1."""
    a, c = params[f"{TOWERS[0]}.{key}"], params[f"{TOWERS[1]}.{key}"]
    return torch.stack([a, c], 1).reshape(-1, *a.shape[1:])


def conv2_tables(params):
    """T2 [2G, 2720, 64] and b2 [2G, 64] of every tower of every group (differentiable)."""
    W1 = _towers(params, "network.0.weight")
    dev = W1.device
    atlas, Gm, part = _consts(dev)
    T = W1.shape[0]
    P = torch.einsum("tocakbl,zcekfl->toabzef", W1.view(T, 32, 3, 2, 4, 2, 4), atlas.view(5, 3, 2, 4, 2, 4))
    T2 = _Conv2Tables.apply(P.reshape(T, 32, 80), _towers(params, "network.0.bias"), _towers(params, "network.2.weight"),
                            Gm, part)
    return T2, _towers(params, "network.2.bias")


class _GroupedConv2LutTower(torch.autograd.Function):
    """A3 [2G, F*9, 576] = im2col(relu(conv2(relu(conv1)) + b2)) of each group's F frames with its own
    two towers; backward dT2 [2G, 2720, 64] by the grouped histogram, db2 = tap (0, 0)'s rows."""

    @staticmethod
    def forward(ctx, T2, b2, codes, F):
        b2c = b2.detach().contiguous()
        Z2 = nat.conv2_lut_fwd_grouped(codes, T2.detach().contiguous(), F)
        ctx.save_for_backward(Z2, b2c, codes)
        return nat.conv3_im2col_fwd(Z2, b2c)

    @staticmethod
    def backward(ctx, dA3):
        Z2, b2, codes = ctx.saved_tensors
        dZ2c, absmax = nat.conv3_col2im_bwd_chunked(dA3.contiguous(), Z2, b2)
        dT = nat.conv2_lut_bwd_grouped(codes, dZ2c, absmax)
        return dT, dT[:, 0:20:4, :].sum(1), None, None


def forward(params, codes, F):
    """(logits [G, F, A], value [G, F]) of the groups' frames codes int32 [G*F, 8] (group g's rows
    contiguous) with each group's own weights params[name] [G, *shape]."""
    T2, b2 = conv2_tables(params)
    T = T2.shape[0]
    A3 = _GroupedConv2LutTower.apply(T2.contiguous(), b2, codes.contiguous(), F)  # [2G, F*9, 576]
    W3t = _towers(params, "network.4.weight").permute(0, 3, 4, 2, 1).reshape(T, 576, 64)
    b3 = _towers(params, "network.4.bias").unsqueeze(1)
    a3 = torch.relu(torch.baddbmm(b3, A3, W3t)).view(T, F, 576)  # rows (p3, co)
    return _heads(params, a3, T)


def _heads(params, a3, T):
    W4 = torch.stack([params["actor.0.weight"], params["critic.0.weight"]], 1)  # [G, 2, H, 576] (co, p3)
    H = W4.shape[2]
    W4p = W4.reshape(T, H, 64, 9).transpose(2, 3).reshape(T, H, 576)  # (p3, co)
    b4 = torch.stack([params["actor.0.bias"], params["critic.0.bias"]], 1).reshape(T, 1, H)
    h = torch.relu(torch.baddbmm(b4, a3, W4p.transpose(1, 2))).view(T // 2, 2, a3.shape[1], H)
    logits = torch.baddbmm(params["actor.2.bias"].unsqueeze(1), h[:, 0], params["actor.2.weight"].transpose(1, 2))
    value = torch.baddbmm(params["critic.2.bias"].unsqueeze(1), h[:, 1], params["critic.2.weight"].transpose(1, 2))
    return logits, value.squeeze(-1)


def evaluate(params, codes, F, actions):
    """CNNActorCritic.evaluate per group: (logp, entropy, value), each [G, F]; actions [G, F]."""
    logits, value = forward(params, codes, F)
    logp_all = logits.log_softmax(-1)
    probs = logp_all.exp()
    logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
    return logp, _entropy(logp_all, probs), value


@torch.no_grad()
def pack(params):
    """The weights of the acting path for a whole rollout (fixed while acting): every tower's conv2
    table, conv3 / fc1 in GEMM layout, the heads."""
    T2, b2 = conv2_tables(params)
    T = T2.shape[0]
    W4 = torch.stack([params["actor.0.weight"], params["critic.0.weight"]], 1)
    H = W4.shape[2]
    return {"T2": T2.contiguous(), "b2": b2.contiguous(),
            "W3t": _towers(params, "network.4.weight").permute(0, 3, 4, 2, 1).reshape(T, 576, 64).contiguous(),
            "b3": _towers(params, "network.4.bias").unsqueeze(1).contiguous(),
            "W4t": W4.reshape(T, H, 64, 9).transpose(2, 3).reshape(T, H, 576).transpose(1, 2).contiguous(),
            "b4": torch.stack([params["actor.0.bias"], params["critic.0.bias"]], 1).reshape(T, 1, H).contiguous(),
            "Wa": params["actor.2.weight"].transpose(1, 2).contiguous(), "ba": params["actor.2.bias"].unsqueeze(1),
            "Wc": params["critic.2.weight"].transpose(1, 2).contiguous(), "bc": params["critic.2.bias"].unsqueeze(1),
            # merlin_group_act's layouts: fc1 rows with (p3, co) columns, the heads' weight rows and biases per task
            "W4p": W4.reshape(T, H, 64, 9).transpose(2, 3).reshape(T, H, 576).contiguous(),
            "Wa_r": params["actor.2.weight"].contiguous(), "ba_r": params["actor.2.bias"].contiguous(),
            "Wc_r": params["critic.2.weight"].contiguous(), "bc_r": params["critic.2.bias"].contiguous()}


@torch.no_grad()
def pack_into(dst, params):
    """Refresh a pack's tensors in place (a captured rollout graph reads them by address)."""
    for k, v in pack(params).items():
        dst[k].copy_(v)


@torch.no_grad()
def act_packed(pk, codes, deterministic=False, out=None):
    """CNNActorCritic.act for one frame per group, codes int32 [G, 8] (frame g with group g's weights):
    (action int64 [G], logp [G], value [G]).  The draw is the Gumbel-max form of Categorical(logits)
    .sample() on torch's generator (capturable in a HIP graph: every replay draws afresh)."""
    T = pk["T2"].shape[0]
    G = T // 2
    Z2 = nat.conv2_lut_fwd_grouped(codes, pk["T2"], 1)
    A3 = nat.conv3_im2col_fwd(Z2, pk["b2"])  # [2G, 9, 576]
    a3 = torch.relu_(torch.baddbmm(pk["b3"], A3, pk["W3t"])).view(T, 1, 576)
    h = torch.relu_(torch.baddbmm(pk["b4"], a3, pk["W4t"])).view(G, 2, 1, -1)
    logits = torch.baddbmm(pk["ba"], h[:, 0], pk["Wa"]).squeeze(1)  # [G, A]
    value = torch.baddbmm(pk["bc"], h[:, 1], pk["Wc"]).view(G)
    logp_all = logits.log_softmax(-1)
    if deterministic:
        a = logits.argmax(-1)
    else:
        u = torch.rand(logits.shape, device=logits.device).clamp_(min=1e-12)
        a = (logp_all - torch.log(-torch.log(u))).argmax(-1)
    lp = logp_all.gather(-1, a.unsqueeze(-1)).squeeze(-1)
    if out is not None:
        out[0].copy_(a)
        out[1].copy_(lp)
        out[2].copy_(value)
        return out
    return a, lp, value


def act_parts(pk, codes, part=None, a3_ws=None):
    """The acting step of every group's frame codes int32 [G, 8] with its own weights in one library call
    (merlin_group_act: conv tables + conv3 per (task, tower), fc1 + the heads' dot products per 64-column chunk):
    head partials f32[2, 8, G, 4] with the head biases folded into chunk 0, for merlin_env_act_step (draw + env step
    in one launch, zero biases) or act_draw.  The logits / value are the sums over the 8 chunks."""
    return nat.group_act(codes, pk["T2"], pk["b2"], pk["W3t"], pk["b3"], pk["W4p"], pk["b4"], pk["Wa_r"], pk["ba_r"],
                         pk["Wc_r"], pk["bc_r"], a3_ws=a3_ws, part=part)
