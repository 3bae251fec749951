"""TEST INFRASTRUCTURE ONLY — fp32 NCHW torch-CPU restatement of the reference FaceVAE step.

This is the parity oracle (and the `cpu_baseline` leg of bench.py).  It restates, with
plain functional torch-CPU ops, the composition SURVEY.md §0 defines out of reference
classes:

    AFE 2-D trunk  (models.py:922-945: in_conv 932, down 933, mid_conv 934)
    latent split + reparameterisation (flatten_vae_nl convention, models.py:559-561)
    Generator 2-D trunk (models.py:1085-1111: in_conv 1095, mid_conv 1096, res 1097,
                         up 1098, out_conv 1099, sigmoid 1110)
    losses: ReconLoss = MSE (losses.py:396-403), KLDivergenceLoss (losses.py:385-393)
    optimiser: Adam(lr, betas=(0.5, 0.999)) (logger.py:60), one step per batch
               (logger.py:150-164)

Every tensor is addressed by the reference's own state-dict key (e.g.
`generator.res.0.layers.1.layers.2.weight_orig`), so the same dict loads into the
product modules and into the reference classes.

Pinned by tests/golden/*.pt (generated from the reference classes by
tests/golden/make_golden.py) — see tests/test_oracle_golden.py.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

BN_EPS = 1e-5       # nn.SyncBatchNorm default (modules.py:19)
BN_MOMENTUM = 0.1
SN_EPS = 1e-12      # torch/nn/utils/spectral_norm.py default
LEAKY_SLOPE = 0.2   # modules.py:29


@dataclass
class OracleConfig:
    """Shapes of the FaceVAE composition (SURVEY.md §0 / §8 header)."""
    H: int = 256
    down_seq: Tuple[int, ...] = (64, 128, 256)
    latent: int = 256
    n_res: int = 6
    up_seq: Tuple[int, ...] = (256, 128, 64)
    w_R: float = 1.0
    w_K: float = 1.0
    lr: float = 5e-5
    betas: Tuple[float, float] = (0.5, 0.999)
    adam_eps: float = 1e-8

    @staticmethod
    def toy() -> "OracleConfig":
        return OracleConfig(H=64, down_seq=(16, 32), latent=16, n_res=1, up_seq=(32, 16))


# ----------------------------------------------------------------------------------------
# layer inventory (mirrors the reference constructors; used to walk the state dict)
# ----------------------------------------------------------------------------------------

@dataclass
class ConvSpec:
    prefix: str          # state-dict prefix of the nn.Conv2d
    cin: int
    cout: int
    k: int
    sn: bool             # spectral_norm applied (modules.py:14,32)
    block: str = "plain"  # "cna" (BN on output, index 1) | "nac" (BN on input, index 0) | "plain"


def conv_specs(cfg: OracleConfig) -> List[ConvSpec]:
    """All convs of the composition in reference construction order."""
    s: List[ConvSpec] = []
    d = cfg.down_seq
    s.append(ConvSpec("afe.in_conv.layers.0", 3, d[0], 7, False, "cna"))                 # models.py:932
    for i in range(len(d) - 1):                                                     # models.py:933
        s.append(ConvSpec(f"afe.down.{i}.layers.0.layers.0", d[i], d[i + 1], 3, False, "cna"))
    s.append(ConvSpec("afe.mid_conv", d[-1], 2 * cfg.latent, 1, False))            # models.py:934
    u = cfg.up_seq
    s.append(ConvSpec("generator.in_conv.layers.0", cfg.latent, u[0], 3, True, "cna"))    # models.py:1095
    s.append(ConvSpec("generator.mid_conv", u[0], u[0], 1, False))                 # models.py:1096
    for i in range(cfg.n_res):                                                      # models.py:1097
        for j in range(2):
            s.append(ConvSpec(f"generator.res.{i}.layers.{j}.layers.2", u[0], u[0], 3, True, "nac"))
    for i in range(len(u) - 1):                                                     # models.py:1098
        s.append(ConvSpec(f"generator.up.{i}.layers.1.layers.0", u[i], u[i + 1], 3, True, "cna"))
    s.append(ConvSpec("generator.out_conv", u[-1], 3, 7, False))                   # models.py:1099
    return s


def bn_prefix(spec: ConvSpec):
    """State-dict prefix + channels of the BatchNorm paired with a conv (None if plain conv)."""
    p = spec.prefix
    if spec.block == "nac":                           # N at index 0, normalises the input
        return p[: -len(".layers.2")] + ".layers.0", spec.cin
    if spec.block == "cna":                           # N at index 1, normalises the output
        return p[: -len(".layers.0")] + ".layers.1", spec.cout
    return None


def init_state(cfg: OracleConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Restates the reference constructors' default init, in construction order:
    nn.Conv2d.reset_parameters (kaiming_uniform_(a=sqrt 5), bias U(±1/sqrt fan_in)),
    then spectral_norm's u/v draws (torch/nn/utils/spectral_norm.py:163-169), BN ones/zeros."""
    torch.manual_seed(seed)
    sd: Dict[str, torch.Tensor] = {}
    for s in conv_specs(cfg):
        w = torch.empty(s.cout, s.cin, s.k, s.k)
        b = torch.empty(s.cout)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(s.cin * s.k * s.k)
        torch.nn.init.uniform_(b, -bound, bound)
        sd[s.prefix + ".bias"] = b
        if s.sn:
            sd[s.prefix + ".weight_orig"] = w
            sd[s.prefix + ".weight_u"] = F.normalize(torch.empty(s.cout).normal_(0, 1), dim=0, eps=SN_EPS)
            sd[s.prefix + ".weight_v"] = F.normalize(torch.empty(s.cin * s.k * s.k).normal_(0, 1),
                                                     dim=0, eps=SN_EPS)
        else:
            sd[s.prefix + ".weight"] = w
        bn = bn_prefix(s)
        if bn is not None:
            p, c = bn
            sd[p + ".weight"] = torch.ones(c)
            sd[p + ".bias"] = torch.zeros(c)
            sd[p + ".running_mean"] = torch.zeros(c)
            sd[p + ".running_var"] = torch.ones(c)
            sd[p + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return sd


# ----------------------------------------------------------------------------------------
# primitives
# ----------------------------------------------------------------------------------------

def _conv_weight(sd: Dict[str, torch.Tensor], prefix: str, training: bool) -> torch.Tensor:
    """Effective conv weight; spectral norm as torch/nn/utils/spectral_norm.py:62-113."""
    if prefix + ".weight_orig" not in sd:
        return sd[prefix + ".weight"]
    w = sd[prefix + ".weight_orig"]
    u, v = sd[prefix + ".weight_u"], sd[prefix + ".weight_v"]
    wm = w.reshape(w.shape[0], -1)
    if training:  # one power iteration, u/v updated in place (no grad)
        with torch.no_grad():
            v.copy_(F.normalize(torch.mv(wm.t(), u), dim=0, eps=SN_EPS))
            u.copy_(F.normalize(torch.mv(wm, v), dim=0, eps=SN_EPS))
        u, v = u.clone(), v.clone()
    sigma = torch.dot(u, torch.mv(wm, v))
    return w / sigma


def conv(sd, prefix, x, training):
    """nn.Conv2d / nn.Conv3d (modules.py:15, 32), stride 1, 'same' padding."""
    w = _conv_weight(sd, prefix, training)
    if w.dim() == 5:
        return F.conv3d(x, w, sd[prefix + ".bias"], 1, w.shape[-1] // 2)
    return F.conv2d(x, w, sd[prefix + ".bias"], 1, w.shape[-1] // 2)


def batchnorm(sd, prefix, x, training):
    """nn.SyncBatchNorm single-process path == F.batch_norm (torch/nn/modules/batchnorm.py:790-826)."""
    if training:
        sd[prefix + ".num_batches_tracked"].add_(1)
    return F.batch_norm(x, sd[prefix + ".running_mean"], sd[prefix + ".running_var"],
                        sd[prefix + ".weight"], sd[prefix + ".bias"], training, BN_MOMENTUM, BN_EPS)


def act(x, kind):
    return F.relu(x) if kind == "relu" else F.leaky_relu(x, LEAKY_SLOPE)


def conv_block(sd, prefix, x, pattern, training, nonlin="relu"):
    """_ConvBlock (modules.py:8-42): layers applied in `pattern` order, indices = positions."""
    for i, c in enumerate(pattern):
        p = f"{prefix}.layers.{i}"
        if c == "C":
            x = conv(sd, p, x, training)
        elif c == "N":
            x = batchnorm(sd, p, x, training)
        else:
            x = act(x, nonlin)
    return x


# ----------------------------------------------------------------------------------------
# forward
# ----------------------------------------------------------------------------------------

def encode(sd, x, cfg, training=True):
    """AFE 2-D trunk (models.py:932-934)."""
    h = conv_block(sd, "afe.in_conv", x, "CNA", training)
    for i in range(len(cfg.down_seq) - 1):               # DownBlock2D: CNA then AvgPool2d(2)
        h = conv_block(sd, f"afe.down.{i}.layers.0", h, "CNA", training)
        h = F.avg_pool2d(h, 2)
    return conv(sd, "afe.mid_conv", h, training)


def res_block_3d(sd, prefix, x, training=True):
    """ResBlock3D (modules.py:133-135 -> _ResBlock 116-126): x + NAC(NAC(x)), each NAC a
    ConvBlock3D (modules.py:52-56) = SyncBatchNorm (5-D input) -> ReLU -> Conv3d 3x3x3."""
    t = conv_block(sd, f"{prefix}.layers.0", x, "NAC", training)
    t = conv_block(sd, f"{prefix}.layers.1", t, "NAC", training)
    return x + t


def encode_afe(sd, x, down_seq, C, D, n_res, training=True, prefix="afe"):
    """The whole AFE (models.py:936-945): the 2-D trunk, x.view(N, C, D, H, W) (941-942), then
    n_res ResBlock3D (943)."""
    h = conv_block(sd, f"{prefix}.in_conv", x, "CNA", training)
    for i in range(len(down_seq) - 1):
        h = conv_block(sd, f"{prefix}.down.{i}.layers.0", h, "CNA", training)
        h = F.avg_pool2d(h, 2)
    h = conv(sd, f"{prefix}.mid_conv", h, training)
    N, _, H, W = h.shape
    h = h.view(N, C, D, H, W)
    for i in range(n_res):
        h = res_block_3d(sd, f"{prefix}.res.{i}", h, training)
    return h


def reparameterise(h, eps, latent):
    """Latent split + reparam: flatten_vae_nl convention (models.py:559-561), eps as input."""
    mu, logstd = h[:, :latent], h[:, latent:]
    return mu, logstd, mu + torch.exp(logstd) * eps


def decode(sd, z, cfg, training=True):
    """Generator 2-D trunk with grid_sample / occlusion as identity (models.py:1095-1110)."""
    g = conv_block(sd, "generator.in_conv", z, "CNA", training, "leakyrelu")
    g = conv(sd, "generator.mid_conv", g, training)
    for i in range(cfg.n_res):                            # ResBlock2D: x + NAC(NAC(x))
        t = conv_block(sd, f"generator.res.{i}.layers.0", g, "NAC", training)
        t = conv_block(sd, f"generator.res.{i}.layers.1", t, "NAC", training)
        g = g + t
    for i in range(len(cfg.up_seq) - 1):                  # UpBlock2D: nearest x2 then CNA
        g = F.interpolate(g, scale_factor=2, mode="nearest")
        g = conv_block(sd, f"generator.up.{i}.layers.1", g, "CNA", training)
    return torch.sigmoid(conv(sd, "generator.out_conv", g, training))


# ----------------------------------------------------------------------------------------
# warp path
# ----------------------------------------------------------------------------------------

def coordinate_grid_3d(d, h, w):
    """make_coordinate_grid_3d (utils.py:91-103) without the .cuda(): [D, H, W, (x, y, z)]."""
    z = 2 * (torch.arange(d) / (d - 1)) - 1
    x = 2 * (torch.arange(h) / (h - 1)) - 1
    y = 2 * (torch.arange(w) / (w - 1)) - 1
    zz, xx, yy = z.view(-1, 1, 1).repeat(1, h, w), x.view(1, -1, 1).repeat(d, 1, w), y.view(1, 1, -1).repeat(d, h, 1)
    return torch.cat([yy.unsqueeze(3), xx.unsqueeze(3), zz.unsqueeze(3)], 3)


def sparse_motions(fs, kp_s, kp_d, Rs, Rd):
    """create_sparse_motions (utils.py:139-152)."""
    N, _, D, H, W = fs.shape
    K = kp_s.shape[1]
    ident = coordinate_grid_3d(D, H, W).view(1, 1, D, H, W, 3).repeat(N, 1, 1, 1, 1, 1)
    cg = ident.repeat(1, K, 1, 1, 1, 1) - kp_d.view(N, K, 1, 1, 1, 3)
    jac = torch.matmul(Rs, torch.inverse(Rd)).view(N, 1, 1, 1, 1, 3, 3)
    cg = torch.matmul(jac, cg.unsqueeze(-1)).squeeze(-1) + kp_s.view(N, K, 1, 1, 1, 3)
    return torch.cat([ident, cg], dim=1)


def heatmap_representations(fs, kp_s, kp_d, var=0.01):
    """create_heatmap_representations (utils.py:130-137, kp2gaussian_3d 123-129)."""
    N, _, D, H, W = fs.shape
    grid = coordinate_grid_3d(D, H, W).view(1, 1, D, H, W, 3)

    def gauss(kp):
        return torch.exp(-0.5 * ((grid - kp.view(N, -1, 1, 1, 1, 3)) ** 2).sum(-1) / var)
    hm = gauss(kp_d) - gauss(kp_s)
    return torch.cat([torch.zeros(N, 1, D, H, W), hm], dim=1).unsqueeze(2)


def deformed_source(fs, sm):
    """create_deformed_source_image (utils.py:155-179)."""
    N, _, D, H, W = fs.shape
    K1 = sm.shape[1]
    rep = fs.unsqueeze(1).repeat(1, K1, 1, 1, 1, 1).view(N * K1, -1, D, H, W)
    out = F.grid_sample(rep, sm.view(N * K1, D, H, W, -1), align_corners=True)
    return out.view(N, K1, -1, D, H, W)


def motion_mask(logits, sm):
    """MFE.forward tail (models.py:1076-1078) -> (deformation, mask)."""
    mask = F.softmax(logits, dim=1).unsqueeze(-1)
    return (sm * mask).sum(dim=1), mask


def generator_warp(sd, fs, deformation, occlusion, n_res, n_up, training=True, prefix="generator"):
    """Generator.forward (models.py:1101-1111) with the warp and the occlusion."""
    N, _, D, H, W = fs.shape
    g = F.grid_sample(fs, deformation, align_corners=True).view(N, -1, H, W)
    g = conv_block(sd, f"{prefix}.in_conv", g, "CNA", training, "leakyrelu")
    g = conv(sd, f"{prefix}.mid_conv", g, training) * occlusion
    for i in range(n_res):
        t = conv_block(sd, f"{prefix}.res.{i}.layers.0", g, "NAC", training)
        g = g + conv_block(sd, f"{prefix}.res.{i}.layers.1", t, "NAC", training)
    for i in range(n_up):
        g = F.interpolate(g, scale_factor=2, mode="nearest")
        g = conv_block(sd, f"{prefix}.up.{i}.layers.1", g, "CNA", training)
    return torch.sigmoid(conv(sd, f"{prefix}.out_conv", g, training))


# ----------------------------------------------------------------------------------------
# perceptual loss
# ----------------------------------------------------------------------------------------

VGG19_MAP = {1: "relu_1_1", 3: "relu_1_2", 6: "relu_2_1", 8: "relu_2_2", 11: "relu_3_1", 13: "relu_3_2",
             15: "relu_3_3", 17: "relu_3_4", 20: "relu_4_1", 22: "relu_4_2", 24: "relu_4_3", 26: "relu_4_4",
             29: "relu_5_1"}                                    # losses.py:60-74
VGG16_MAP = {1: "relu_1_1", 3: "relu_1_2", 6: "relu_2_1", 8: "relu_2_2", 11: "relu_3_1", 13: "relu_3_2",
             15: "relu_3_3", 18: "relu_4_1", 20: "relu_4_2", 22: "relu_4_3", 25: "relu_5_1"}   # losses.py:106-118
PERCEPTUAL_WEIGHTS = {"relu_1_1": 0.03125, "relu_2_1": 0.0625, "relu_3_1": 0.125, "relu_4_1": 0.25,
                      "relu_5_1": 1.0}                          # losses.py:124


def vgg_features(sd, x, mapping, layers):
    """_PerceptualNetwork.forward (losses.py:42-49) over a torchvision `features` stack given
    as {"features.{i}.weight/bias"}: conv 3x3 pad 1 at i, ReLU at i+1, MaxPool2d(2, 2) where no
    conv sits.  Stops after the last requested layer (later layers cannot change outputs)."""
    want = {i for i, n in mapping.items() if n in layers}
    out, i = {}, 0
    while i <= max(want):
        if f"features.{i}.weight" in sd:
            x = F.conv2d(x, sd[f"features.{i}.weight"], sd[f"features.{i}.bias"], 1, 1)
        elif f"features.{i - 1}.weight" in sd:
            x = F.relu(x)
        else:
            x = F.max_pool2d(x, 2, 2)
        if mapping.get(i) in layers:
            out[mapping[i]] = x
        i += 1
    return out


def imagenet_norm(x):
    """apply_imagenet_normalization (utils.py:182-186)."""
    return (x - x.new_tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) / x.new_tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def vggface_norm(x):
    """apply_vggface_normalization (utils.py:189-193)."""
    return (x * 255 - x.new_tensor([129.186279296875, 104.76238250732422, 93.59396362304688]).view(1, 3, 1, 1))


def perceptual_loss(inp, target, w19, w16, layers_weight=None, n_scale=3):
    """PerceptualLoss.forward (losses.py:131-151), including the multi-scale loop's reuse of the
    leaked `layer` / `weight` (the last layers_weight item) at every scale (:145-150)."""
    layers_weight = layers_weight or PERCEPTUAL_WEIGHTS
    loss = F.l1_loss(inp, target)
    fi = vgg_features(w16, vggface_norm(inp), VGG16_MAP, layers_weight)
    ft = vgg_features(w16, vggface_norm(target), VGG16_MAP, layers_weight)
    inp, target = imagenet_norm(inp), imagenet_norm(target)
    gi = vgg_features(w19, inp, VGG19_MAP, layers_weight)
    gt = vgg_features(w19, target, VGG19_MAP, layers_weight)
    for layer, weight in layers_weight.items():
        loss = loss + weight * F.l1_loss(fi[layer], ft[layer].detach()) / 255
        loss = loss + weight * F.l1_loss(gi[layer], gt[layer].detach())
    for _ in range(n_scale):
        inp = F.interpolate(inp, mode="bilinear", scale_factor=0.5, align_corners=False, recompute_scale_factor=True)
        target = F.interpolate(target, mode="bilinear", scale_factor=0.5, align_corners=False,
                               recompute_scale_factor=True)
        gi = vgg_features(w19, inp, VGG19_MAP, layers_weight)
        gt = vgg_features(w19, target, VGG19_MAP, layers_weight)
        loss = loss + weight * F.l1_loss(gi[layer], gt[layer].detach())
    return loss


def kl_loss(mu, logstd):
    """KLDivergenceLoss (losses.py:392)."""
    return torch.mean(-0.5 - logstd + 0.5 * mu ** 2 + 0.5 * torch.exp(2 * logstd), dim=-1).mean()


def recon_loss(target, pred):
    """ReconLoss = nn.MSELoss()(target, pred) (losses.py:399-402)."""
    return F.mse_loss(target, pred)


def forward(sd, x, eps, cfg: OracleConfig, training=True):
    h = encode(sd, x, cfg, training)
    mu, logstd, z = reparameterise(h, eps, cfg.latent)
    y = decode(sd, z, cfg, training)
    R = recon_loss(x, y)
    K = kl_loss(mu, logstd)
    loss = cfg.w_R * R + cfg.w_K * K                      # loss = sum(losses) (logger.py:160)
    return {"y": y, "mu": mu, "logstd": logstd, "z": z, "R": R, "K": K, "loss": loss}


# ----------------------------------------------------------------------------------------
# state + optimiser
# ----------------------------------------------------------------------------------------

def is_param(key: str) -> bool:
    return not any(key.endswith(s) for s in
                   (".running_mean", ".running_var", ".num_batches_tracked", ".weight_u", ".weight_v"))


def prepare_state(state_dict: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    sd = {k: v.detach().clone().float() if v.is_floating_point() else v.detach().clone()
          for k, v in state_dict.items()}
    for k, v in sd.items():
        if is_param(k):
            v.requires_grad_(True)
    return sd


def adam_init(sd):
    return {k: {"step": 0, "exp_avg": torch.zeros_like(v), "exp_avg_sq": torch.zeros_like(v)}
            for k, v in sd.items() if is_param(k)}


@torch.no_grad()
def adam_update(sd, opt, cfg: OracleConfig):
    """torch.optim.Adam single-tensor math (lr, betas, eps; no weight decay) — logger.py:60."""
    b1, b2 = cfg.betas
    for k, st in opt.items():
        p = sd[k]
        g = p.grad
        st["step"] += 1
        st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** st["step"]
        bc2 = 1 - b2 ** st["step"]
        denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(cfg.adam_eps)
        p.addcdiv_(st["exp_avg"], denom, value=-cfg.lr / bc1)


def train_step(sd, opt, x, eps, cfg: OracleConfig):
    """One Logger.step iteration (logger.py:150-164): zero_grad, fwd, loss.backward, Adam."""
    for k in opt:
        sd[k].grad = None
    out = forward(sd, x, eps, cfg, training=True)
    out["loss"].backward()
    grads = {k: sd[k].grad.detach().clone() for k in opt}
    adam_update(sd, opt, cfg)
    return out, grads


def flops_per_image(cfg: OracleConfig) -> Tuple[float, float]:
    """Algorithmic conv FLOPs per image (reference formulation), (forward, train step)."""
    H = cfg.H
    fwd = 0.0
    first = 0.0
    res = H
    spatial = {}
    d = cfg.down_seq
    spatial["afe.in_conv.layers.0"] = H
    for i in range(len(d) - 1):
        spatial[f"afe.down.{i}.layers.0.layers.0"] = H >> i
    lat = H >> (len(d) - 1)
    spatial["afe.mid_conv"] = lat
    spatial["generator.in_conv.layers.0"] = lat
    spatial["generator.mid_conv"] = lat
    for i in range(cfg.n_res):
        for j in range(2):
            spatial[f"generator.res.{i}.layers.{j}.layers.2"] = lat
    for i in range(len(cfg.up_seq) - 1):
        spatial[f"generator.up.{i}.layers.1.layers.0"] = lat << (i + 1)
    spatial["generator.out_conv"] = lat << (len(cfg.up_seq) - 1)
    for s in conv_specs(cfg):
        r = spatial[s.prefix]
        f = 2.0 * r * r * s.cout * s.cin * s.k * s.k
        fwd += f
        if s.prefix == "afe.in_conv.layers.0":
            first = f
    del res
    return fwd, 3 * fwd - first


# ----------------------------------------------------------------------------------------
# ConvTranspose2dELR (models_utils.py:404-516) -- SURVEY.md §8a-a15 (off the FaceVAE graph)
# ----------------------------------------------------------------------------------------

def convt_elr_gain(inch, kernel_size, stride, norm, act_slope=None):
    """weightgain of models_utils.py:420-433 (act: None, ReLU (slope 0) or LeakyReLU)."""
    if act_slope is None:
        actgain = 1.0
    elif act_slope == 0.0:
        actgain = math.sqrt(2.0)                                    # calculate_gain("relu")
    else:
        actgain = math.sqrt(2.0 / (1 + act_slope ** 2))             # calculate_gain("leaky_relu", slope)
    fan_in = inch * (kernel_size ** 2 / (stride ** 2))
    initgain = stride if norm == "demod" else 1.0 / math.sqrt(fan_in)
    return actgain * initgain


def convt_elr(x, weight, bias, stride, padding, norm, gain, act_slope=None):
    """getweight (models_utils.py:454-472) + forward without modulation (:480-514):
    F.normalize over dims [0, 2, 3] when demod, times gain; conv_transpose2d; + bias (tied
    [outch] or untied [outch, H, W]); optional ReLU / LeakyReLU."""
    w = F.normalize(weight, dim=[0, 2, 3]) if norm == "demod" else weight
    out = F.conv_transpose2d(x, w * gain, None, stride=stride, padding=padding)
    out = out + (bias[None, :, None, None] if bias.dim() == 1 else bias[None])
    if act_slope is not None:
        out = F.leaky_relu(out, act_slope) if act_slope > 0 else F.relu(out)
    return out


def convt_elr_mod(x, wstyle, weight, bias, aff_w, aff_b, aff_gain, stride, padding, norm, gain, act_slope=None):
    """ConvTranspose2dELR.forward with the per-sample affine modulation (models_utils.py:484-505):
    s = LinearELR(w) * 0.1 + 1 (addmm with alpha = weightgain, :197-198), weight * s over the input
    channels, F.normalize over dims [1, 3, 4] when demod, times gain, grouped conv_transpose2d."""
    b = x.shape[0]
    aff = torch.addmm(aff_b[None], wstyle, aff_w.t(), alpha=aff_gain)
    w = weight[None] * (aff[:, :, None, None, None] * 0.1 + 1.)
    if norm == "demod":
        w = F.normalize(w, dim=[1, 3, 4])
    w = w * gain
    inch, outch, k = weight.shape[0], weight.shape[1], weight.shape[2]
    out = F.conv_transpose2d(x.reshape(1, b * inch, x.shape[2], x.shape[3]), w.reshape(b * inch, outch, k, k), None,
                             stride=stride, padding=padding, groups=b)
    out = out.view(b, outch, out.shape[2], out.shape[3])
    out = out + (bias[None, :, None, None] if bias.dim() == 1 else bias[None])
    if act_slope is not None:
        out = F.leaky_relu(out, act_slope) if act_slope > 0 else F.relu(out)
    return out
