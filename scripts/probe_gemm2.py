"""Time the tower GEMMs at the bench's distinct-frame count (U ~ 80k per minibatch) and
alternative formulations of the weight gradients (diagnostic)."""
import torch

dev = torch.device("cuda:0")
U = 80000
f = lambda *s: torch.randn(*s, device=dev)  # noqa: E731
A3, W3t, dZ3 = f(2, U * 9, 576), f(2, 576, 64), f(2, U * 9, 64)
a3, W4, dh = f(2, U, 576), f(2, 512, 576), f(2, U, 512)
b3 = f(2, 1, 64)


def t(name, fn, gmac, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name:50s} {ms:7.3f} ms  {2 * gmac / ms / 1e3:6.1f} TFLOP/s", flush=True)


g3 = 2 * U * 9 * 576 * 64 / 1e9
g4 = 2 * U * 576 * 512 / 1e9
t("conv3 fwd baddbmm", lambda: torch.baddbmm(b3, A3, W3t), g3)
t("conv3 dgrad dZ3 @ W3t^T", lambda: torch.bmm(dZ3, W3t.transpose(1, 2)), g3)
t("conv3 wgrad A3^T @ dZ3", lambda: torch.bmm(A3.transpose(1, 2), dZ3), g3)
t("conv3 wgrad (dZ3^T @ A3)^T", lambda: torch.bmm(dZ3.transpose(1, 2), A3), g3)
t("conv3 wgrad per-tower mm", lambda: [torch.mm(A3[i].t(), dZ3[i]) for i in range(2)], g3)
for S in (8, 32, 64):
    def sk(S=S):
        K = U * 9 // S
        return torch.bmm(A3[:, :K * S].reshape(2 * S, K, 576).transpose(1, 2), dZ3[:, :K * S].reshape(2 * S, K, 64)).view(2, S, 576, 64).sum(1)
    t(f"conv3 wgrad split-K {S}", sk, g3)
t("fc1 fwd a3 @ W4^T", lambda: torch.bmm(a3, W4.transpose(1, 2)), g4)
t("fc1 dgrad dh @ W4", lambda: torch.bmm(dh, W4), g4)
t("fc1 wgrad dh^T @ a3", lambda: torch.bmm(dh.transpose(1, 2), a3), g4)
t("fc1 wgrad (a3^T @ dh)^T", lambda: torch.bmm(a3.transpose(1, 2), dh), g4)
for S in (8, 32):
    def sk4(S=S):
        K = U // S
        return torch.bmm(dh[:, :K * S].reshape(2 * S, K, 512).transpose(1, 2), a3[:, :K * S].reshape(2 * S, K, 576)).view(2, S, 512, 576).sum(1)
    t(f"fc1 wgrad split-K {S}", sk4, g4)
