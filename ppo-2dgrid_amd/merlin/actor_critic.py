"""Actor-critic networks: the model-side drop-in surface (src/actor_critic.py).

Frozen contract with the reference:
  * ``CNNActorCritic(obs_shape=(H, W, C), act_dim, hidden_dim=512)`` with separate
    actor / critic towers conv(C->32,k8,s4) -> conv(32->64,k4,s2) -> conv(64->64,k3,s1)
    -> flatten -> Linear(hidden) -> ReLU -> Linear(act_dim | 1); state_dict keys
    ``{actor,critic}_extractor.network.{0,2,4}.*`` and ``{actor,critic}.{0,2}.*``,
    so reference ``.pth`` checkpoints load unchanged (actor_critic.py:6-41);
  * modules are created and initialised in the reference's order, so the same
    torch seed gives the same weights (layer_init, utils_rl.py:6-9);
  * ``act(obs, deterministic) -> (action, logp, value)`` and
    ``evaluate(obs, actions) -> (logp, entropy, value)`` (actor_critic.py:48-64),
    obs as float [B, H, W, C] in 0..255 (permuted like ``_format_obs``) or [B, C, H, W].

MERLIN-AMD addition: ``prescaled=True`` tells the towers that the input is already
divided by 255 (the HIP observation expansion folds the /255 of
CNNFeatureExtractor.forward, actor_critic.py:20-21, into its store), so the rollout
and update never materialise an extra scaled copy of the observation batch.
The categorical head is computed directly with log_softmax instead of building a
torch.distributions.Categorical per call (same formulas: log-prob of the
normalised logits, entropy = -sum p*log p).

``act_codes`` / ``evaluate_codes`` take the packed 7x7 tile codes of the GPU envs
instead of frames.  Every frame is a blit of 5 atlas tiles, so each tower's first
Conv2d(3,32,k8,s4) equals bias + a sum of 4 entries of a [32][4 slots][20] table P
(W1 contracted with the /255-scaled atlas); P is formed here with an einsum (autograd
turns dP into dW1) and the lookups / their transposed histogram run in the HIP library
(merlin_conv1_lut_fwd/bwd, csrc/merlin_conv1.hip).  Same function, fp32 sums in a
different order; conv2..heads are the reference modules unchanged.

``evaluate_windows`` (the update's path) evaluates conv2 and conv3 once per distinct
receptive-field window of the rollout (merlin/windows.py, csrc/merlin_window.hip) and fc1 +
the heads once per distinct frame of the minibatch.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .utils.utils_rl import layer_init

# (out_channels, kernel, stride) of the three convs -- actor_critic.py:9-14
_CONV_SPEC = ((32, 8, 4), (64, 4, 2), (64, 3, 1))
# the rollout's all-windows conv3 table on the f16 two-plane GEMM (False: hipBLASLt's fp32 bmm; 0.8 ms less per
# rollout, scripts/probe_rollout.py); the rollout's fc1 on it too (False: the x6 kernel), with a3's scale reduced by
# k_codes_conv3 as it writes a3: 31.9 vs 33.4 ms per rollout (before the scale reduction skipped its redundant
# same-address atomics, 39.0 vs 34.7: one atomic per block of a 8,192-block grid serialised)
QALL_H3 = True
ROLLOUT_FC1_H3 = True


class CNNFeatureExtractor(nn.Module):
    def __init__(self, channels, height, width):
        super().__init__()
        layers = []
        cin = channels
        for cout, k, s in _CONV_SPEC:
            layers += [layer_init(nn.Conv2d(cin, cout, kernel_size=k, stride=s)), nn.ReLU()]
            cin = cout
        layers.append(nn.Flatten())
        self.network = nn.Sequential(*layers)
        with torch.no_grad():
            self.output_dim = self.network(torch.zeros(1, channels, height, width)).shape[1]

    def forward(self, x, prescaled: bool = False):
        return self.network(x if prescaled else x / 255.0)


def _head(in_dim: int, hidden: int, out_dim: int, out_std: float, act=nn.ReLU) -> nn.Sequential:
    return nn.Sequential(layer_init(nn.Linear(in_dim, hidden)), act(),
                         layer_init(nn.Linear(hidden, out_dim), std=out_std))


def _categorical(logits: torch.Tensor):
    """(normalised log-probs, probs) of Categorical(logits=...)."""
    logp = logits - logits.logsumexp(dim=-1, keepdim=True)
    return logp, F.softmax(logp, dim=-1)


def _sample_or_argmax(logits: torch.Tensor, logp_all: torch.Tensor, probs: torch.Tensor, deterministic: bool):
    if deterministic:
        return torch.argmax(logits, dim=1)
    # one Categorical(probs) sample per row by exponential races, argmax_i p_i / E_i with
    # E_i ~ Exp(1): the form torch.multinomial uses for a single sample, without its host-side
    # validity check, so the rollout can be captured as a HIP graph (merlin/ppo.py)
    return (probs / torch.empty_like(probs).exponential_()).argmax(dim=-1)


def _entropy(logp_all: torch.Tensor, probs: torch.Tensor) -> torch.Tensor:
    lp = torch.clamp(logp_all, min=torch.finfo(logp_all.dtype).min)
    return -(lp * probs).sum(-1)


class _Conv1FromCodes(torch.autograd.Function):
    """relu(conv1) of both towers from tile codes (HIP lookup / histogram kernels)."""

    @staticmethod
    def forward(ctx, tables, bias, codes, index):
        from . import _native as nat

        a1 = nat.conv1_lut_fwd(codes, index, tables.detach().contiguous(), bias.detach().contiguous())
        ctx.save_for_backward(a1, codes, index if index is not None else codes.new_empty(0))
        ctx.has_index = index is not None
        return a1

    @staticmethod
    def backward(ctx, grad):
        from . import _native as nat

        a1, codes, index = ctx.saved_tensors
        dt, db = nat.conv1_lut_bwd(codes, index if ctx.has_index else None, a1, grad.contiguous())
        return dt, db, None, None


class _Conv2Im2colFromCodes(torch.autograd.Function):
    """A2 = im2col(relu(conv1(frames))) of both towers, straight from tile codes."""

    @staticmethod
    def forward(ctx, tables, bias, codes, index):
        from . import _native as nat

        t, b = tables.detach().contiguous(), bias.detach().contiguous()
        A2 = nat.conv2_im2col_fwd(codes, index, t, b)
        ctx.save_for_backward(t, b, codes, index if index is not None else codes.new_empty(0))
        ctx.has_index = index is not None
        return A2

    @staticmethod
    def backward(ctx, dA2):
        from . import _native as nat

        t, b, codes, index = ctx.saved_tensors
        dt, db = nat.conv2_im2col_bwd(codes, index if ctx.has_index else None, t, b, dA2.contiguous())
        return dt, db, None, None


class _Conv3Im2col(torch.autograd.Function):
    """A3 = im2col(relu(Z2 + b2)) of both towers (conv2's bias + ReLU fused)."""

    @staticmethod
    def forward(ctx, Z2, b2):
        from . import _native as nat

        Z2, b2 = Z2.contiguous(), b2.detach().contiguous()
        ctx.save_for_backward(Z2, b2)
        return nat.conv3_im2col_fwd(Z2, b2)

    @staticmethod
    def backward(ctx, dA3):
        from . import _native as nat

        Z2, b2 = ctx.saved_tensors
        dZ2 = nat.conv3_col2im_bwd(dA3.contiguous(), Z2, b2)
        return dZ2, dZ2.sum(dim=1)


class _Conv2LutTower(torch.autograd.Function):
    """A3 = im2col(relu(conv2(relu(conv1(frame))) + b2)) of both towers from tile codes, with
    conv1 + conv2 as lookups in the tables T (csrc/merlin_conv2lut.hip); backward returns
    dT (a histogram of dZ2 over the rows each position read) and db2."""

    @staticmethod
    def forward(ctx, T2, b2, codes, index):
        from . import _native as nat

        b2c = b2.detach().contiguous()
        if index is not None:  # the minibatch's code rows, gathered once (32 B per frame)
            codes = codes.index_select(0, index)
        Z2 = nat.conv2_lut_fwd(codes, None, T2.detach().contiguous())
        ctx.save_for_backward(Z2, b2c, codes)
        return nat.conv3_im2col_fwd(Z2, b2c)

    @staticmethod
    def backward(ctx, dA3):
        from . import _native as nat

        Z2, b2, codes = ctx.saved_tensors
        dZ2c, absmax = nat.conv3_col2im_bwd_chunked(dA3.contiguous(), Z2, b2)
        dT = nat.conv2_lut_bwd(codes, dZ2c, absmax)
        # every output position reads exactly one row of tap (0, 0) (rows 0, 4, .., 16)
        return dT, dT[:, 0:20:4, :].sum(1), None, None


def _gemm_span(name, T, M, N, K):
    """HIP-event span of a hipBLASLt GEMM batch (T GEMMs of M x N x K) for bench.py's FLOP roofline."""
    from ._native import KernelTimer

    return KernelTimer.span(name, 0, 2 * T * M * N * K)


def bias_relu_bmm(X, W, b):
    """relu(X[t] @ W[t] + b[t]) for every tower t (X [T, M, K], W [T, K, N], b [T, N]): one GEMM per
    tower with the bias and ReLU in hipBLASLt's epilogue (torch._addmm_activation), bit-identical to
    the GEMM followed by merlin_tower_bias_relu, without its extra pass over the [T, M, N] output
    (scripts/probe_gemm3.py: fc1 at the bench size 1247 -> 1135 us; used for fc1, N = 512)."""
    T, M, _ = X.shape
    out = X.new_empty((T, M, W.shape[2]))
    for t in range(T):
        torch._addmm_activation(b[t], X[t], W[t], out=out[t])
    return out


def _splitk_bmm_tn(X, dY, chunks, min_chunk=1024, name="gemm_wgrad", out=None):
    """X^T @ dY for X [T, M, K], dY [T, M, N] with the long M reduction split into `chunks`
    batched GEMMs plus a sum: hipBLASLt runs the plain tall-skinny product at about half the
    FP32 rate on these shapes (scripts/probe_gemm2.py), the split form at ~105-125 TFLOP/s."""
    T, M, K = X.shape
    N = dY.shape[2]
    c = M // chunks
    if chunks <= 1 or c < min_chunk:
        with _gemm_span(name, T, K, N, M):
            return torch.bmm(X.transpose(1, 2), dY) if out is None else torch.bmm(X.transpose(1, 2), dY, out=out)
    # per tower the first c*chunks rows are a view [chunks, c, K] (merging the tower and chunk
    # dims would copy both operands whenever M % chunks != 0: 2 x 0.1 ms per call at the bench size)
    part = X.new_empty((T, chunks, K, N))
    with _gemm_span(name, T, K, N, c * chunks):
        for t in range(T):
            torch.bmm(X[t, : c * chunks].view(chunks, c, K).transpose(1, 2), dY[t, : c * chunks].view(chunks, c, N),
                      out=part[t])
    if c * chunks < M:
        tail = torch.bmm(X[:, c * chunks:].transpose(1, 2), dY[:, c * chunks:])
        return part.sum(1) + tail if out is None else torch.add(part.sum(1), tail, out=out)
    return part.sum(1) if out is None else torch.sum(part, 1, out=out)


class _BiasReluBmm(torch.autograd.Function):
    """relu(X @ W + b) over both towers (X [T, M, K], W [T, K, N], b [T, 1, N]): a plain bmm and
    the in-place bias + ReLU epilogue (merlin_tower_bias_relu); backward: the ReLU mask and the
    bias gradient in one HIP pass (merlin_tower_relu_bwd), the input gradient as a bmm and the
    weight gradient as the split-K product."""

    @staticmethod
    def forward(ctx, X, W, b, chunks):
        from . import _native as nat

        Y = nat.bias_relu_(torch.bmm(X, W), b.detach().reshape(b.shape[0], -1).contiguous())
        ctx.save_for_backward(X, W, Y)
        ctx.chunks = chunks
        return Y

    @staticmethod
    def backward(ctx, dY):
        from . import _native as nat

        X, W, Y = ctx.saved_tensors
        dZ, db = nat.relu_bwd(Y, dY.contiguous())
        dX = torch.bmm(dZ, W.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        dW = _splitk_bmm_tn(X, dZ, ctx.chunks)
        return dX, dW, db.unsqueeze(1), None


class _TowerHead(torch.autograd.Function):
    """fc1 -> ReLU -> heads of both towers (actor_critic.py:30-41) on a3 [2, n, 576] (rows
    (p3, co), W4's columns permuted to match, W4p [2, H, 576]): one bmm + the bias/ReLU
    epilogue, then the two small heads.  Backward: the heads' backward, fc1's ReLU mask, fc1's
    bias gradient and the heads' weight gradients in one HIP pass over h
    (merlin_tower_head_bwd), then fc1's input gradient (bmm) and weight gradient (split-K)."""

    @staticmethod
    def forward(ctx, a3, W4p, b4, Wa, ba, Wc, bc):
        from . import _native as nat

        T, n, K = a3.shape
        # (the forward keeps hipBLASLt's own pick: the searched solution measured faster alone
        # but slower in the update, rocprofv3 profiles/r02_tuning_ab.md)
        with _gemm_span("gemm_fc1_fwd", T, n, W4p.shape[1], K):
            h = bias_relu_bmm(a3, W4p.transpose(1, 2), b4.detach().contiguous())
        logits = torch.mm(h[0], Wa.t()) if ba is None else torch.addmm(ba, h[0], Wa.t())
        value = (torch.mm(h[1], Wc.t()) if bc is None else torch.addmm(bc, h[1], Wc.t())).squeeze(-1)
        ctx.save_for_backward(a3, W4p, h, Wa, Wc)
        ctx.head_bias = (ba is not None, bc is not None)
        return logits, value

    @staticmethod
    def backward(ctx, dlogits, dvalue):
        from . import _native as nat
        from .gemm_tuning import tuned

        a3, W4p, h, Wa, Wc = ctx.saved_tensors
        n = h.shape[1]
        dlogits = h.new_zeros(n, Wa.shape[0]) if dlogits is None else dlogits.contiguous()
        dvalue = h.new_zeros(n) if dvalue is None else dvalue.contiguous()
        dz, db4, dWa, dWc = nat.head_bwd(h, dlogits, dvalue, Wa.detach().contiguous(), Wc.detach().contiguous())
        da3 = None
        if ctx.needs_input_grad[0]:
            with _gemm_span("gemm_fc1_dgrad", dz.shape[0], n, W4p.shape[2], dz.shape[2]), tuned("dgrad"):
                da3 = torch.bmm(dz, W4p)
        # (the split-K wgrad keeps hipBLASLt's pick: the searched solutions were faster in the
        # tuning loop, slower inside the update)
        dW4p = _splitk_bmm_tn(a3, dz, 32).transpose(1, 2)
        dba = dlogits.sum(0) if ctx.head_bias[0] else None
        dbc = dvalue.sum(0, keepdim=True) if ctx.head_bias[1] else None
        return da3, dW4p, db4, dWa, dba, dWc.view_as(Wc), dbc


def _lut2_h1_index():
    """Per conv1-position parity type (yp, xp), in table order ee, eo, oe, oo: the flat
    indices (slot*20 + 4*class + 2*qy + qx) into P[t][co] of the 4 slot terms of every tile
    combination v (tiles (ar, ac), ar <= yp, ac <= xp, row-major, class digits base 5)."""
    out = []
    for yp, xp in ((0, 0), (0, 1), (1, 0), (1, 1)):
        tiles = [(ar, ac) for ar in range(yp + 1) for ac in range(xp + 1)]
        V = 5 ** len(tiles)
        idx = torch.empty((V, 4), dtype=torch.long)
        for v in range(V):
            digits = [(v // 5 ** (len(tiles) - 1 - i)) % 5 for i in range(len(tiles))]
            for dy in range(2):
                for dx in range(2):
                    tile = tiles.index(((yp + dy) >> 1, (xp + dx) >> 1))
                    qy, qx = (yp + dy) & 1, (xp + dx) & 1
                    idx[v, 2 * dy + dx] = (2 * dy + dx) * 20 + 4 * digits[tile] + 2 * qy + qx
        out.append(((yp, xp), idx))
    return out


_LUT2_H1 = _lut2_h1_index()


def _lut2_gather_matrix():
    """(G f32 [680, 80], part int64 [680]): the 680 tile combinations of the four parity types
    in table order (row 4*v + j of T2), G[v][k] = how often P's flat entry k enters combination
    v's conv1 sum (Pf[:, :, idx].sum(-1) == Pf @ G.T), part[v] = its parity type."""
    G = torch.cat([torch.zeros(idx.shape[0], 80).scatter_add_(1, idx, torch.ones(idx.shape, dtype=torch.float32))
                   for _, idx in _LUT2_H1])
    part = torch.cat([torch.full((idx.shape[0],), p, dtype=torch.int64) for p, (_, idx) in enumerate(_LUT2_H1)])
    return G, part


class _Conv2Tables(torch.autograd.Function):
    """T2 [2, 2720, 64] from P [2, 32, 80], b1 [2, 32], W2 [2, 64, 32, 4, 4] in a handful of
    kernels, forward and backward written out (the autograd graph of the per-parity-type
    formulation, CNNActorCritic._conv2_tables_autograd, ran ~25 forward and ~90 backward kernels
    per optimizer step, four of them sort-based index_put backwards):
      HT   = relu(G @ P[t]^T + b1[t])                 [2, 680, 32]  conv1 of every combination
      X    = HT @ Wall[t]                             [2, 680, 1024] all four tap-parity blocks
      T2   = X[:, v, part(v)]                         the block of each combination's own type
    Wall[t][ci][(yp, xp, a, b, co)] = W2[t][co][ci][2a + yp][2b + xp]; X computes the three other
    blocks too (89 MFLOP per call, negligible) so one bmm replaces eight."""

    @staticmethod
    def forward(ctx, P, b1, W2, G, part):
        T = P.shape[0]  # 2 towers (or 2 per group: merlin/grouped_policy.py)
        HT = torch.matmul(G, P.transpose(1, 2))
        HT = torch.relu_(HT.add_(b1.unsqueeze(1)))
        Wall = W2.reshape(T, 64, 32, 2, 2, 2, 2).permute(0, 2, 4, 6, 3, 5, 1).reshape(T, 32, 1024)
        X = torch.bmm(HT, Wall).view(T, -1, 4, 256)
        ar = torch.arange(part.numel(), device=part.device)
        ctx.save_for_backward(HT, Wall, G, part, ar)
        return X[:, ar, part].reshape(T, -1, 64)

    @staticmethod
    def backward(ctx, dT2):
        HT, Wall, G, part, ar = ctx.saved_tensors
        V = part.numel()
        T = HT.shape[0]
        dX = dT2.new_zeros((T, V, 4, 256))
        dX[:, ar, part] = dT2.reshape(T, V, 256)
        dX = dX.view(T, V, 1024)
        dWall = torch.bmm(HT.transpose(1, 2), dX)
        dW2 = dWall.view(T, 32, 2, 2, 2, 2, 64).permute(0, 6, 1, 4, 2, 5, 3).reshape(T, 64, 32, 4, 4)
        dH = torch.bmm(dX, Wall.transpose(1, 2)).mul_(HT > 0)
        return torch.matmul(dH.transpose(1, 2), G), dH.sum(1), dW2, None, None


class CNNActorCritic(nn.Module):
    def __init__(self, obs_shape, act_dim, hidden_dim=512):
        super().__init__()
        h, w, c = obs_shape
        self.actor_extractor = CNNFeatureExtractor(c, h, w)
        self.critic_extractor = CNNFeatureExtractor(c, h, w)
        self.actor = _head(self.actor_extractor.output_dim, hidden_dim, act_dim, 0.01)
        self.critic = _head(self.critic_extractor.output_dim, hidden_dim, 1, 1.0)
        self._atlas = None  # f32 [5, 3, 8, 8] / 255 on the model's device (codes path only)
        self._lut2_idx = None
        self._lut2_gather = None
        self._all_rows = None  # int32 [458752, 16] table rows of every observable window (acting path)
        # "lut2": conv1+conv2 as table lookups, conv3/fc as hipBLASLt GEMMs (default)
        # "gemm": conv1 lookups, conv2/conv3/fc as GEMMs | "lut_nchw": conv1 lookups + MIOpen convs
        self.codes_impl = "lut2"
        # fc1 of the update (heads_windows): "h3" = fp32-class products on the f16 matrix cores in two-plane
        # form, three products each, error below hipBLASLt's fp32 GEMM (csrc/merlin_h3.hip); "x6" = exact fp32
        # products on the bf16 matrix cores in three-plane form, six products (csrc/merlin_gemm.hip);
        # "hipblaslt" = torch's fp32 GEMMs
        self.fc1_impl = "h3"

    # -- tile-code path (GPU envs) --------------------------------------------------
    def _atlas_on(self, device):
        if self._atlas is None or self._atlas.device != device:
            from . import _native as nat

            a = torch.from_numpy(nat.tile_atlas()).permute(0, 3, 1, 2).float() / 255.0
            self._atlas = a.contiguous().to(device)
        return self._atlas

    def conv1_tables(self):
        """P[t][co][slot][bin] (t: actor, critic; slot = 2*dy + dx; bin = 4*class + 2*qy + qx)."""
        c1a, c1c = self.actor_extractor.network[0], self.critic_extractor.network[0]
        return self.conv1_tables_from(torch.stack([c1a.weight, c1c.weight])), torch.stack([c1a.bias, c1c.bias])

    def conv1_tables_from(self, W1):
        """conv1_tables of the stacked conv1 weights W1 [2, 32, 3, 8, 8]."""
        W = W1.view(2, 32, 3, 2, 4, 2, 4)  # t o c dy ky dx kx
        A = self._atlas_on(W1.device).to(W1.dtype).view(5, 3, 2, 4, 2, 4)  # cls c qy ky qx kx
        P = torch.einsum("tocakbl,zcekfl->toabzef", W, A)
        return P.reshape(2, 32, 4, 20)

    def conv2_tables(self):
        """T2[t][row][co] (t: actor, critic; 2720 rows, csrc/merlin_conv2lut.hip layout):
        W2[:, :, ky, kx] applied to relu(conv1) of each tile combination (_Conv2Tables: autograd
        maps dT2 to the conv1 and conv2 weight gradients)."""
        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        return self.conv2_tables_from(torch.stack([ea[0].weight, ec[0].weight]), torch.stack([ea[0].bias, ec[0].bias]),
                                      torch.stack([ea[2].weight, ec[2].weight]))

    def stage_consts(self, device):
        """(atlas f32[5, 3, 8, 8] / 255, idx int16[680, 4], koff int16[81], kv int16[2720]) for the HIP table
        kernels (merlin_stage_tables_fwd / _bwd): each combination's four conv1-table entries, in table order,
        and per entry k the combinations reading it (CSR, (v, e) order)."""
        if getattr(self, "_stage_consts", None) is None or self._stage_consts[0].device != device:
            idx = torch.cat([i for _, i in _LUT2_H1])  # [680, 4] int64
            flat = idx.reshape(-1)
            order = torch.sort(flat, stable=True).indices  # (v, e) positions grouped by entry, (v, e) order
            kv = (order // 4).to(torch.int16)
            koff = torch.zeros(81, dtype=torch.int64)
            koff[1:] = torch.cumsum(torch.bincount(flat, minlength=80), 0)
            self._stage_consts = (self._atlas_on(device).contiguous(), idx.to(torch.int16).to(device),
                                  koff.to(torch.int16).to(device), kv.to(device))
        return self._stage_consts

    def conv2_tables_from(self, W1, b1, W2):
        """conv2_tables of the stacked weights W1 [2, 32, 3, 8, 8], b1 [2, 32], W2 [2, 64, 32, 4, 4]."""
        P = self.conv1_tables_from(W1)
        if self._lut2_gather is None or self._lut2_gather[0].device != P.device or self._lut2_gather[0].dtype != P.dtype:
            G, part = _lut2_gather_matrix()
            self._lut2_gather = (G.to(device=P.device, dtype=P.dtype), part.to(P.device))
        return _Conv2Tables.apply(P.reshape(2, 32, 80), b1, W2, *self._lut2_gather)

    def _conv2_tables_autograd(self):
        """conv2_tables as plain differentiable torch ops, one bmm per parity type (the
        definition _Conv2Tables is tested against)."""
        P, b1 = self.conv1_tables()
        Pf = P.reshape(2, 32, 80)
        if self._lut2_idx is None or self._lut2_idx[0][1].device != Pf.device:
            self._lut2_idx = [(k, idx.to(Pf.device)) for k, idx in _LUT2_H1]
        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        W2 = torch.stack([ea[2].weight, ec[2].weight])  # [2, co 64, ci 32, ky 4, kx 4]
        parts = []
        for (yp, xp), idx in self._lut2_idx:
            H = torch.relu(b1.unsqueeze(-1) + Pf[:, :, idx].sum(-1))  # [2, 32, V]
            Wsel = W2[:, :, :, yp::2, xp::2].permute(0, 2, 3, 4, 1).reshape(2, 32, 256)  # ci, (a, b), co
            parts.append(torch.bmm(H.transpose(1, 2), Wsel).reshape(2, -1, 64))  # rows 4*v + j
        return torch.cat(parts, 1)

    def _forward_codes_lut2(self, codes, index=None):
        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        n = index.numel() if index is not None else codes.shape[0]
        A3 = _Conv2LutTower.apply(self.conv2_tables(), torch.stack([ea[2].bias, ec[2].bias]), codes, index)
        return self._tower_tail(A3, n)

    def _tower_tail(self, A3, n):
        """conv3 (GEMM on the im2col rows A3 [2, n*9, 576]) -> fc1 -> heads."""
        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        W3t = torch.stack([ea[4].weight, ec[4].weight]).permute(0, 3, 4, 2, 1).reshape(2, 576, 64)
        b3 = torch.stack([ea[4].bias, ec[4].bias]).unsqueeze(1)
        a3 = _BiasReluBmm.apply(A3, W3t, b3, 64).view(2, n, 576)  # rows (p3, co)
        return self._tower_head(a3, n)

    def _tower_head(self, a3, n, head_bias: bool = True):
        """fc1 (W4's columns permuted to the (p3, co) order of a3 [2, n, 576]) -> ReLU -> heads."""
        fa, fc = self.actor[0], self.critic[0]
        W4 = torch.stack([fa.weight, fc.weight])  # [2, hidden, 576] in (co, p3) order
        W4p = W4.view(2, W4.shape[1], 64, 9).transpose(2, 3).reshape(2, W4.shape[1], 576)
        ba, bc = (self.actor[2].bias, self.critic[2].bias) if head_bias else (None, None)
        return _TowerHead.apply(a3, W4p, torch.stack([fa.bias, fc.bias]), self.actor[2].weight, ba,
                                self.critic[2].weight, bc)

    def _forward_codes(self, codes, index=None):
        """Both towers from tile codes as GEMMs (csrc/merlin_tower.hip for the data movement):
        A2 = im2col(relu(conv1)) -> Z2 = A2 @ W2t -> A3 = im2col(relu(Z2 + b2)) ->
        relu(A3 @ W3t + b3) -> fc1 (columns permuted to the (position, channel) row order)
        -> heads.  The GEMMs are batched over the two towers (hipBLASLt fp32)."""
        if self.codes_impl == "lut2":
            return self._forward_codes_lut2(codes, index)
        if self.codes_impl == "lut_nchw":
            return self._forward_codes_nchw(codes, index)
        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        n = index.numel() if index is not None else codes.shape[0]
        tables, b1 = self.conv1_tables()
        A2 = _Conv2Im2colFromCodes.apply(tables, b1, codes, index)  # [2, n*25, 512]
        W2t = torch.stack([ea[2].weight, ec[2].weight]).permute(0, 3, 4, 2, 1).reshape(2, 512, 64)
        Z2 = torch.bmm(A2, W2t)  # [2, n*25, 64]
        A3 = _Conv3Im2col.apply(Z2, torch.stack([ea[2].bias, ec[2].bias]))  # [2, n*9, 576]
        return self._tower_tail(A3, n)

    def _forward_codes_nchw(self, codes, index=None):
        tables, bias = self.conv1_tables()
        a1 = _Conv1FromCodes.apply(tables, bias, codes, index)
        fa = self.actor_extractor.network[2:](a1[0])
        fc = self.critic_extractor.network[2:](a1[1])
        return self.actor(fa), self.critic(fc).squeeze(-1)

    def _all_window_rows(self, device):
        """int32 [458,752, 16]: the conv2 table rows of every 3x3 tile window an observation can hold, in the acting
        table's compact key order (merlin/windows.py compact_window_keys, window_rows), built once per device."""
        if self._all_rows is None or self._all_rows.device != device:
            from . import _native as nat
            from .windows import compact_window_keys, window_rows

            keys = compact_window_keys(device)
            assert keys.numel() == nat.ALL_WINDOWS
            self._all_rows = window_rows(keys).contiguous()
        return self._all_rows

    # below this many frames per rollout the acting path looks conv2 up per frame instead of building
    # the all-windows table (Qall: 2.1 GB and ~68 GFLOP per rollout, whatever the rollout's size)
    ALL_WINDOWS_MIN_FRAMES = 1 << 18
    ALL_WINDOWS_HEADROOM = 5 << 29  # 2.5 GiB: the all-windows tables plus their GEMM's planes

    def rollout_pack(self, frames: int | None = None, all_windows: bool | None = None, steps: int | None = None):
        """The weights of the acting path in the layouts its kernels and GEMMs read, built once
        per rollout (the weights do not change while acting).

        Large rollouts (frames >= ALL_WINDOWS_MIN_FRAMES, or frames not given): conv2 (from the
        conv1+conv2 tables) and conv3's per-tap products for every 3x3 tile window an observation can hold, Qall
        [2, 458752, 576] (2.1 GB + 0.23 GB of conv2 rows while it is built: conv2 + ReLU of the 458,752 windows of
        merlin/windows.py compact_window_keys and one [458752, 64] x [64, 576] GEMM per tower, ~1 ms per rollout);
        each step then sums 81 table rows per frame.  Small rollouts, or when the device has less than ~12 GB free:
        the conv2 table T2 (2,720 rows) and conv3's weights, and each step looks conv2 up per frame
        position and runs conv3 as a GEMM over the im2col rows (merlin_tower_conv2_lut_fwd +
        conv3_im2col_fwd, a few MB).  Both: fc1 with columns permuted to (p3, co), biases stacked.
        all_windows: the layout decided by the caller (PPO decides once, before its rollout is captured: the
        free-memory reading changes between the eager rollout and the capture); None = decide here.
        steps: the act_codes_packed steps the pack serves (0 .. steps - 1): each gets its own operand-scale row, all
        zeroed here at once (None: one row, zeroed before every step)."""
        from . import _native as nat

        ea, ec = self.actor_extractor.network, self.critic_extractor.network
        fa, fc = self.actor[0], self.critic[0]
        W4 = torch.stack([fa.weight, fc.weight])
        H = W4.shape[1]
        T2 = self.conv2_tables().contiguous()
        W3r = torch.stack([ea[4].weight, ec[4].weight]).permute(0, 2, 3, 4, 1).reshape(2, 64, 576)
        W4p = W4.view(2, H, 64, 9).transpose(2, 3).reshape(2, H, 576)
        pack = {
            "b3": torch.stack([ea[4].bias, ec[4].bias]).contiguous(),
            "b4": torch.stack([fa.bias, fc.bias]).contiguous(),
        }
        if all_windows is None:
            all_windows = self._use_all_windows(frames, T2.device)
        if all_windows:
            # relu(conv2) of every observable window [2, 458752, 64] (bias and ReLU in the lookup kernel)
            a2 = nat.window_lut(self._all_window_rows(T2.device), T2,
                                bias=torch.stack([ea[2].bias, ec[2].bias]).contiguous())
            if self.fc1_impl in ("x6", "h3") and QALL_H3:
                # the table GEMM [5^9, 64] x [64, 576] per tower on the f16 two-plane kernels (hipBLASLt's fp32
                # GEMM took ~3.6 ms per rollout; the error bound is the same, tests/test_gpu_h3.py)
                W3t = W3r.transpose(1, 2).contiguous()  # [2, 576, 64]: the NT kernel's B rows
                am = nat.h3_amax(W3t)
                pack["Qall"] = nat.h3_gemm_nt(a2, nat.h3_amax(a2), nat.h3_split(W3t, am), am,
                                              cfg=nat.H3_NT_CFG["qall"], name="gemm_rollout_qall")
            else:
                pack["Qall"] = torch.bmm(a2, W3r)  # [2, windows, (ky, kx, co)]
        else:
            pack["T2"] = T2
            pack["b2"] = torch.stack([ea[2].bias, ec[2].bias]).contiguous()
            # im2col rows of A3 are (ky, kx, ci): conv3 weights as [2, 576, 64] in that order
            pack["W3t"] = torch.stack([ea[4].weight, ec[4].weight]).permute(0, 3, 4, 2, 1).reshape(2, 576, 64).contiguous()
        if self.fc1_impl == "h3" and ROLLOUT_FC1_H3:  # fc1 of every step on merlin_h3.hip, either conv3 layout
            amW = nat.h3_amax(W4p.contiguous())
            pack["W4h"] = (nat.h3_split(W4p.contiguous(), amW), amW)
            # per step: max |a3| per tower, one row per step of the rollout when the caller says how many (all zeroed
            # here by one kernel: this is built inside the captured rollout graph, where a memset would replay
            # wrong), else one row zeroed before each step's conv3
            pack["am3"] = nat.h3_zero(torch.empty((max(1, int(steps or 1)), 2), dtype=torch.int32, device=W4p.device))
        elif self.fc1_impl in ("x6", "h3"):  # fc1 of every step on the bf16 MFMA, exact fp32 products (merlin_gemm2.hip)
            pack["W4pp"] = nat.x6_split(W4p.contiguous())
        else:
            pack["W4t"] = W4p.transpose(1, 2).contiguous()
        return pack

    def _use_all_windows(self, frames, device) -> bool:
        """The acting layout from the rollout's frame count and the device's total memory only (not the memory
        free at the time: the same seed must act through the same layout whatever else is allocated, and every
        DP rank decides alike); PPO records the choice (PPO.rollout_all_windows, the bench line's
        rollout_acting)."""
        if frames is not None and frames < self.ALL_WINDOWS_MIN_FRAMES:
            return False
        try:
            free, total = torch.cuda.mem_get_info(device)
        except Exception:
            return True
        if total < (64 << 30):
            return False
        # the all-windows layout allocates its tables once per rollout (Qall [2, 458752, 576] fp32, 2.1 GB, plus
        # relu(conv2) of every window, 0.23 GB): check the headroom once, here, before any capture -- running out
        # inside the captured rollout would fail there, and switching layouts by free memory would make the acting
        # draws depend on what else the device holds
        need = self.ALL_WINDOWS_HEADROOM
        if free + torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device) < need:
            from ._native import MerlinNativeError

            raise MerlinNativeError(
                f"the all-windows acting layout needs ~{need / 2**30:.1f} GiB of free device memory "
                f"({free / 2**30:.1f} GiB free); free memory or set CNNActorCritic.ALL_WINDOWS_MIN_FRAMES above the "
                f"rollout's frame count for the per-frame layout")
        return True

    @torch.no_grad()
    def heads_partials_ok(self, pack) -> bool:
        """The acting GEMM can leave the heads' partial dot products (h3 fc1 with the heads epilogue), so the draw
        can run elsewhere (act_draw, or fused into the env step: MerlinVecEnv.act_step_into)."""
        from . import _native as nat

        return ("W4h" in pack and nat.H3_HEADS_EPILOGUE and self.actor[2].weight.shape[0] <= 4 and
                nat.lib().merlin_h3_heads_parts(pack["W4h"][0].shape[1], nat.H3_NT_CFG["rollout"]) > 0)

    def act_codes_packed(self, codes, pack, deterministic=False, seed=0, epoch=None, step=0, out=None, env_offset=0,
                         partials=False):
        """act_codes with the layouts of rollout_pack(): conv1+conv2+conv3 from the all-windows
        table (merlin_tower_codes_conv3: 81 table rows per frame and tower), fc1 as a plain bmm,
        then fc1's bias/ReLU, the heads, the log-probs and the categorical draw in one HIP pass
        (merlin_act_heads; draws keyed by (seed, epoch[0], step, env_offset + env)).
        out = (action, logp, value) tensors to write in place.  partials=True: return the heads' partial dot
        products f32[2, P, n, 4] instead of drawing (heads_partials_ok packs only)."""
        from . import _native as nat
        from .gemm_tuning import tuned

        n = codes.shape[0]
        am3 = pack.get("am3")
        if am3 is not None:
            if am3.shape[0] > step:  # this step's own row, zeroed with the others when the pack was built
                am3 = am3[step]
            else:
                am3 = nat.h3_zero(am3[0])  # a kernel: this runs inside the captured rollout graph
        if "Qall" in pack:
            a3 = nat.codes_conv3(codes, pack["Qall"], pack["b3"], amax=am3).view(2, n, 576)
        else:  # per-frame conv2 lookups + conv3 GEMM (small rollouts, rollout_pack)
            A3 = nat.conv3_im2col_fwd(nat.conv2_lut_fwd(codes, None, pack["T2"]), pack["b2"])
            a3 = nat.bias_relu_(torch.bmm(A3, pack["W3t"]), pack["b3"]).view(2, n, 576)
            if am3 is not None:  # fc1 on h3: the operand scale of this step's a3 (zeroed by a kernel inside)
                am3 = nat.h3_amax(a3, out=am3)
        if self.heads_partials_ok(pack):
            # fc1 + bias + ReLU + both heads in the GEMM's epilogue (h never written), then the draw from the sums
            P4, amW = pack["W4h"]
            part = nat.h3_gemm_nt_heads(a3, am3, P4, amW, pack["b4"], self.actor[2].weight, self.critic[2].weight,
                                        cfg=nat.H3_NT_CFG["rollout"], name="gemm_rollout_fc1", partials_only=True)
            if partials:  # the caller draws (merlin_env_act_step: the draw fused into the env step)
                return part
            return nat.act_draw(part, self.actor[2].bias, self.critic[2].bias, deterministic, seed=seed, epoch=epoch,
                                step=step, out=out, env_offset=env_offset)
        assert not partials, "head partials need the h3 acting GEMM with the heads epilogue (heads_partials_ok)"
        if "W4h" in pack:
            P4, amW = pack["W4h"]
            z = nat.h3_gemm_nt(a3, am3, P4, amW, cfg=nat.H3_NT_CFG["rollout"], name="gemm_rollout_fc1")
        elif "W4pp" in pack:
            z = nat.x6_gemm_nt(a3, pack["W4pp"], cfg=nat.X6_NT_CFG["rollout"], name="gemm_rollout_fc1")
        else:
            with tuned("rollout"):
                z = torch.bmm(a3, pack["W4t"])
        return nat.act_heads(z, pack["b4"], self.actor[2].weight, self.actor[2].bias, self.critic[2].weight,
                             self.critic[2].bias, deterministic, seed=seed, epoch=epoch, step=step, out=out,
                             env_offset=env_offset)

    def act_codes(self, codes, deterministic=False, index=None):
        logits, value = self._forward_codes(codes, index)
        logp_all, probs = _categorical(logits)
        action = _sample_or_argmax(logits, logp_all, probs, deterministic)
        return action, logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1), value

    def evaluate_codes(self, codes, actions, index=None, groups=None):
        """groups = (rep_idx, inv) (merlin.dedup.FrameGroups.minibatch): the towers run on the
        distinct frames rep_idx only and sample k takes row inv[k] (same values and gradients)."""
        if groups is not None:
            rep_idx, inv = groups
            logits, value = self._forward_codes(codes, rep_idx)
            # index_select: its backward is one index_add (advanced indexing's is a sort)
            logits, value = logits.index_select(0, inv), value.index_select(0, inv)
        else:
            logits, value = self._forward_codes(codes, index)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), value

    def heads_windows(self, plan, mb, head_bias: bool = True):
        """(logits [U, act_dim], value [U]) of the minibatch's distinct frames mb.groups through
        the receptive-field windows (merlin/windows.py): conv2 / conv3 once per distinct window of
        the rollout, fc1 and the heads once per distinct frame.  head_bias=False leaves the heads'
        biases out (merlin.ppo's fused loss adds them and returns their gradients)."""
        from .gemm_tuning import padded_rows
        from .windows import tower_conv3, window_tower_head_x6

        if self.fc1_impl in ("x6", "h3"):
            return window_tower_head_x6(self, plan, mb, head_bias)
        n = int(mb.groups.numel())
        npad = padded_rows(n)  # fc1's rows on a tuned GEMM shape (merlin/gemm_tuning.py); zero rows past n
        logits, value = self._tower_head(tower_conv3(self, plan, mb, npad).view(2, npad, 576), npad, head_bias)
        return (logits[:n], value[:n]) if npad != n else (logits, value)

    def evaluate_windows(self, plan, mb, actions):
        """evaluate_codes for one minibatch of the update through heads_windows; sample k takes
        frame row mb.inv[k]."""
        logits, value = self.heads_windows(plan, mb)
        logits, value = logits.index_select(0, mb.inv), value.index_select(0, mb.inv)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), value

    def _format_obs(self, x):
        # NHWC observations (the gym frame layout) -> NCHW for the convs
        if x.ndim == 4 and x.shape[-1] == 3:
            return x.permute(0, 3, 1, 2).float()
        return x.float()

    def _forward(self, obs, prescaled: bool):
        obs = self._format_obs(obs)
        logits = self.actor(self.actor_extractor(obs, prescaled=prescaled))
        value = self.critic(self.critic_extractor(obs, prescaled=prescaled)).squeeze(-1)
        return logits, value

    def act(self, obs, deterministic=False, prescaled: bool = False):
        logits, value = self._forward(obs, prescaled)
        logp_all, probs = _categorical(logits)
        action = _sample_or_argmax(logits, logp_all, probs, deterministic)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, value

    def evaluate(self, obs, actions, prescaled: bool = False):
        logits, value = self._forward(obs, prescaled)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), value


class MLPActorCritic(nn.Module):
    """Flat-observation variant (actor_critic.py:66-99), used when scenario.yaml sets flatten."""

    def __init__(self, obs_dim, act_dim, hidden_dim=64):
        super().__init__()
        self.actor = nn.Sequential(layer_init(nn.Linear(obs_dim, hidden_dim)), nn.Tanh(),
                                   layer_init(nn.Linear(hidden_dim, hidden_dim)), nn.Tanh(),
                                   layer_init(nn.Linear(hidden_dim, act_dim), std=0.01))
        self.critic = nn.Sequential(layer_init(nn.Linear(obs_dim, hidden_dim)), nn.Tanh(),
                                    layer_init(nn.Linear(hidden_dim, hidden_dim)), nn.Tanh(),
                                    layer_init(nn.Linear(hidden_dim, 1), std=1.0))

    def act(self, obs, deterministic=False, prescaled: bool = False):
        logits = self.actor(obs)
        logp_all, probs = _categorical(logits)
        action = _sample_or_argmax(logits, logp_all, probs, deterministic)
        logp = logp_all.gather(-1, action.unsqueeze(-1)).squeeze(-1)
        return action, logp, self.critic(obs).squeeze(-1)

    def evaluate(self, obs, actions, prescaled: bool = False):
        logits = self.actor(obs)
        logp_all, probs = _categorical(logits)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        return logp, _entropy(logp_all, probs), self.critic(obs).squeeze(-1)
