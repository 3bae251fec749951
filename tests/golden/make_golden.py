"""Generate the golden fixtures of the FaceVAE path FROM THE REFERENCE ITSELF.

Run in the build container only (it needs /root/reference, which does not exist on the
GPU box):

    python tests/golden/make_golden.py

It imports the reference classes (`modules.py`, `models.py`, `losses.py`) read-only,
builds the FaceVAE composition of SURVEY.md §0 out of them, runs reference training steps
(the Logger.step sequence, logger.py:150-164, with torch.optim.Adam as logger.py:60) and
stores inputs + outputs as plain tensors (torch.save of dicts of tensors; loaded with
weights_only=True).  No reference source enters the repo; only data.

`losses.py` has a top-level `import torchvision` (losses.py:4) that is absent here; an
empty placeholder module is registered under that name so the file imports.  Only
KLDivergenceLoss / ReconLoss are instantiated (nothing of torchvision is touched).

Fixtures written next to this script:
  toy_step.pt    toy config (64², B=4): init state, x, eps, step-1 outputs/grads/state,
                 step-3 losses/state.
  blocks.pt      per-block cases (ConvBlock2D CNA/NAC/leaky, DownBlock2D, UpBlock2D,
                 ResBlock2D; fwd output, input grad, param grads, updated buffers).
  full256.pt     full config (256², B=2): per-key checksums of the seed-0 init, losses of
                 two steps and strided samples of the reconstruction.
"""
import os
import sys
import types

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    sys.path.insert(0, REF)
    if "torchvision" not in sys.modules:
        sys.modules["torchvision"] = types.ModuleType("torchvision")  # inert placeholder
    import modules, models, losses  # noqa: E402  (reference, read-only)
    return modules, models, losses


class RefFaceVAE(torch.nn.Module):
    """SURVEY.md §0 composition built from reference classes only."""

    def __init__(self, models, cfg):
        super().__init__()
        self.latent = cfg["latent"]
        # AFE 2-D trunk: C*D = 2*latent so mid_conv emits [mu | logstd]; no 3-D ResBlocks.
        self.afe = models.AFE(use_weight_norm=False, down_seq=list(cfg["down_seq"]), n_res=0,
                              C=2 * cfg["latent"], D=1)
        self.generator = models.Generator(use_weight_norm=True, n_res=cfg["n_res"],
                                          up_seq=list(cfg["up_seq"]), D=1, C=cfg["latent"])

    def forward(self, x, eps):
        a = self.afe
        h = a.mid_conv(a.down(a.in_conv(x)))
        mu, logstd = h[:, :self.latent], h[:, self.latent:]
        z = mu + torch.exp(logstd) * eps                      # models.py:561 with eps input
        g = self.generator
        f = g.mid_conv(g.in_conv(z))                           # occlusion == 1
        f = g.up(g.res(f))
        y = torch.sigmoid(g.out_conv(f))
        return y, mu, logstd, z


TOY = dict(H=64, B=4, down_seq=(16, 32), latent=16, n_res=1, up_seq=(32, 16))
FULL = dict(H=256, B=2, down_seq=(64, 128, 256), latent=256, n_res=6, up_seq=(256, 128, 64))


def inputs(cfg):
    H, B, L = cfg["H"], cfg["B"], cfg["latent"]
    x = torch.rand(B, 3, H, H, generator=torch.Generator().manual_seed(1234))
    lat = H >> (len(cfg["down_seq"]) - 1)
    eps = torch.randn(B, L, lat, lat, generator=torch.Generator().manual_seed(1235))
    return x, eps


def run_steps(models, losses, cfg, nsteps, w_R=1.0, w_K=1.0, lr=5e-5):
    torch.manual_seed(0)
    net = RefFaceVAE(models, cfg)
    init = {k: v.detach().clone() for k, v in net.state_dict().items()}
    opt = torch.optim.Adam(net.parameters(), lr=lr, betas=(0.5, 0.999))
    kl, rec = losses.KLDivergenceLoss(), losses.ReconLoss()
    x, eps = inputs(cfg)
    hist = []
    for step in range(nsteps):
        opt.zero_grad()
        y, mu, logstd, z = net(x, eps)
        R = rec((x, y))
        K = kl((mu, logstd))
        loss = w_R * R + w_K * K
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
        opt.step()
        hist.append(dict(y=y.detach().clone(), mu=mu.detach().clone(), logstd=logstd.detach().clone(),
                         R=R.detach().clone(), K=K.detach().clone(), loss=loss.detach().clone(),
                         grads=grads,
                         state={k: v.detach().clone() for k, v in net.state_dict().items()}))
    return init, x, eps, hist


def make_toy(models, losses):
    init, x, eps, hist = run_steps(models, losses, TOY, 3)
    h1, h3 = hist[0], hist[2]
    out = dict(cfg=torch.tensor([TOY["H"], TOY["B"], TOY["latent"], TOY["n_res"]]),
               init=init, x=x, eps=eps,
               step1=dict(y=h1["y"], mu=h1["mu"], logstd=h1["logstd"], R=h1["R"], K=h1["K"],
                          loss=h1["loss"], grads=h1["grads"], state=h1["state"]),
               step3=dict(R=torch.stack([h["R"] for h in hist]), K=torch.stack([h["K"] for h in hist]),
                          y=h3["y"], state=h3["state"]))
    torch.save(out, os.path.join(HERE, "toy_step.pt"))


def make_full(models, losses):
    init, x, eps, hist = run_steps(models, losses, FULL, 2)
    sums = {k: torch.tensor([v.double().sum().item(), v.double().abs().sum().item()], dtype=torch.float64)
            for k, v in init.items()}
    y1 = hist[0]["y"]
    out = dict(init_checksums=sums,
               R=torch.stack([h["R"] for h in hist]), K=torch.stack([h["K"] for h in hist]),
               loss=torch.stack([h["loss"] for h in hist]),
               y1_samples=y1[:, :, ::17, ::13].clone(),
               y1_mean=y1.double().mean(), mu1_mean=hist[0]["mu"].double().mean(),
               logstd1_mean=hist[0]["logstd"].double().mean())
    torch.save(out, os.path.join(HERE, "full256.pt"))


def make_blocks(modules):
    """Per-block fwd+bwd cases on small shapes (reference modules, training mode)."""
    cases = {}

    def run(name, ctor, x_shape, seed):
        torch.manual_seed(seed)
        m = ctor()
        g = torch.Generator().manual_seed(seed + 1)
        x = torch.randn(*x_shape, generator=g).requires_grad_(True)
        init = {k: v.detach().clone() for k, v in m.state_dict().items()}
        y = m(x)
        gy = torch.randn(y.shape, generator=g)
        (y * gy).sum().backward()
        cases[name] = dict(init=init, x=x.detach().clone(), y=y.detach().clone(), gy=gy,
                           gx=x.grad.detach().clone(),
                           grads={n: p.grad.detach().clone() for n, p in m.named_parameters()},
                           state={k: v.detach().clone() for k, v in m.state_dict().items()})

    run("cna_relu", lambda: modules.ConvBlock2D("CNA", 16, 32, 3, 1, 1, False), (2, 16, 12, 10), 10)
    run("cna_leaky_sn", lambda: modules.ConvBlock2D("CNA", 32, 32, 3, 1, 1, True,
                                                    nonlinearity_type="leakyrelu"), (2, 32, 8, 8), 11)
    run("cna_7x7", lambda: modules.ConvBlock2D("CNA", 3, 16, 7, 1, 3, False), (2, 3, 16, 16), 12)
    run("down", lambda: modules.DownBlock2D(16, 32, False), (2, 16, 16, 16), 13)
    run("up_sn", lambda: modules.UpBlock2D(32, 16, True), (2, 32, 8, 8), 14)
    run("res_sn", lambda: modules.ResBlock2D(32, True), (2, 32, 8, 8), 15)
    run("same", lambda: modules.SameBlock2D(32, 64, False), (2, 32, 8, 8), 16)
    torch.save(cases, os.path.join(HERE, "blocks.pt"))


def main():
    modules, models, losses = import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    make_toy(models, losses)
    make_blocks(modules)
    make_full(models, losses)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".pt"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
