"""dlogits of confident rows in fp32: (A) reference autograd (model log_softmax + cross_entropy),
(B) single log_softmax + NLL autograd, (C) manual exp(logp) - onehot, (D) softmax - onehot, vs fp64."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
N, C = 32, 10
logits64 = torch.randn(N, C, dtype=torch.float64) * 8
logits64[:, 3] += 20  # confident rows
y = torch.full((N,), 3, dtype=torch.long)
y[::4] = 5
ref = None
for name in ["A", "B", "C", "D"]:
    out = {}
    for dt in (torch.float32, torch.float64):
        z = logits64.to(dt).clone().requires_grad_(True)
        if name == "A":
            F.cross_entropy(torch.log_softmax(z, 1), y).backward(); d = z.grad
        elif name == "B":
            F.nll_loss(torch.log_softmax(z, 1), y).backward(); d = z.grad
        elif name == "C":
            lp = torch.log_softmax(z.detach(), 1); d = (lp.exp() - F.one_hot(y, C).to(dt)) / N
        else:
            d = (torch.softmax(z.detach(), 1) - F.one_hot(y, C).to(dt)) / N
        out[dt] = d.double()
    err = (out[torch.float32] - out[torch.float64]).abs()
    rel_y = (err / out[torch.float64].abs().clamp_min(1e-30))[torch.arange(N), y]
    print(f"{name}: max abs err {err.max().item():.2e}  true-class rel err: max {rel_y.max().item():.2e} median {rel_y.median().item():.2e}  "
          f"true-class grad min |.| {out[torch.float64][torch.arange(N), y].abs().min().item():.2e}")
