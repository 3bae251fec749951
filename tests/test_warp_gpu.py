"""GPU parity of the warp path: the grid_sample kernels against torch's
F.grid_sample on the CPU (same operands), the MFE motion assembly and the warped Generator
against fixtures generated from the reference (tests/golden/warp.pt).

Tolerances: fp32 1e-5 (kernels; grid_sample's input gradient sums each cell's buckets in voxel
order, bit-reproducible: test_grid_sample3d_input_gradient_is_deterministic), Generator fp32 mode 1e-4 (the north_star 1e-3 bar with
margin); bf16 storage of the sampled volume: 4e-3 rel-L2 / 1.6e-2 max-abs of max|ref|."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import warp  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CL3 = torch.channels_last_3d


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def maxd(a, b):
    return (a.detach().double().cpu() - b.detach().double().cpu()).abs().max().item()


def load(k):
    return torch.load(os.path.join(GOLD, "warp.pt"), weights_only=True)[k]


@pytest.mark.parametrize("N,C,Di,Hi,Wi,Do,Ho,Wo,group,dtype", [
    (2, 32, 4, 8, 16, 4, 8, 16, 1, torch.float32),
    (2, 32, 4, 8, 16, 3, 5, 7, 1, torch.bfloat16),
    (2, 4, 4, 8, 8, 4, 8, 8, 6, torch.float32),      # deformed source: one input per 6 grids
    (1, 24, 3, 5, 6, 2, 4, 9, 1, torch.float32),     # channel count off the power-of-two lanes
    (1, 6, 3, 5, 6, 4, 3, 5, 1, torch.bfloat16),     # C % 8 != 0: one channel per lane
    (3, 8, 2, 3, 4, 5, 6, 7, 2, torch.bfloat16),     # group > 1 on the 8-channel rows
])
def test_grid_sample3d_vs_torch(N, C, Di, Hi, Wi, Do, Ho, Wo, group, dtype):
    g = torch.Generator().manual_seed(9)
    inp = torch.randn(N, C, Di, Hi, Wi, generator=g)
    grid = (torch.rand(N * group, Do, Ho, Wo, 3, generator=g) - 0.5) * 2.4    # some samples outside
    gout = torch.randn(N * group, C, Do, Ho, Wo, generator=g)
    xi = inp.cuda().to(dtype).contiguous(memory_format=CL3).requires_grad_(True)
    gr = grid.cuda().requires_grad_(True)
    out = warp.GridSample3dFn.apply(xi, gr, group, dtype)
    out.backward(gout.cuda().to(dtype))
    torch.cuda.synchronize()
    ir = inp.to(dtype).float().requires_grad_(True)
    grr = grid.clone().requires_grad_(True)
    rep = ir.unsqueeze(1).expand(N, group, C, Di, Hi, Wi).reshape(N * group, C, Di, Hi, Wi)
    ref = F.grid_sample(rep, grr, align_corners=True)
    ref.backward(gout.to(dtype).float())
    if dtype == torch.float32:
        assert rel(out, ref) < 1e-5 and rel(xi.grad, ir.grad) < 1e-5 and rel(gr.grad, grr.grad) < 1e-5
    else:
        assert rel(out.float(), ref) < 4e-3 and maxd(out.float(), ref) <= 1.6e-2 * ref.abs().max().item()
        assert rel(xi.grad.float(), ir.grad) < 4e-3 and rel(gr.grad, grr.grad) < 1e-4


def test_motion_assembly_matches_reference():
    m = load("motion")
    ins = [m[k].cuda().requires_grad_(True) for k in ("fs", "kp_s", "kp_d", "Rs", "Rd")]
    fs = ins[0]
    sm = warp.create_sparse_motions(fs, *ins[1:])
    hm = warp.create_heatmap_representations(fs, ins[1], ins[2])
    ds = warp.create_deformed_source_image(fs, sm)
    assert rel(sm, m["sm"]) < 1e-5 and rel(hm, m["hm"]) < 1e-5 and rel(ds, m["ds"]) < 1e-5
    ((sm * m["g_sm"].cuda()).sum() + (hm * m["g_hm"].cuda()).sum() + (ds * m["g_ds"].cuda()).sum()).backward()
    torch.cuda.synchronize()
    for n, t in zip(("fs", "kp_s", "kp_d", "Rs", "Rd"), ins):
        assert rel(t.grad, m["grads"][n]) < 1e-4, n


def test_motion_mask_matches_reference():
    m = load("mask")
    lt, st = m["logits"].cuda().requires_grad_(True), m["sm"].cuda().requires_grad_(True)
    d, mask = warp.deformation_from_mask(lt, st)
    assert rel(d, m["deformation"]) < 1e-5 and rel(mask, m["mask"]) < 1e-5
    ((d * m["g_def"].cuda()).sum() + (mask * m["g_mask"].cuda()).sum()).backward()
    torch.cuda.synchronize()
    assert rel(lt.grad, m["d_logits"]) < 1e-5 and rel(st.grad, m["d_sm"]) < 1e-5


def _generator(mode):
    gd = load("generator")
    gen = fv.Generator(True, n_res=1, up_seq=[32, 16], D=2, C=16)
    gen.load_state_dict(gd["init"])
    gen = gen.cuda().train().set_compute_dtype(mode)
    ins = [gd[k].cuda().requires_grad_(True) for k in ("fs", "deformation", "occlusion")]
    y = gen(*ins)
    (y * gd["g"].cuda()).sum().backward()
    torch.cuda.synchronize()
    return gd, gen, ins, y


def test_generator_warp_fp32_matches_reference():
    gd, gen, ins, y = _generator(torch.float32)
    assert rel(y, gd["out"]) < 1e-4
    for n, t in zip(("d_fs", "d_deformation", "d_occlusion"), ins):
        assert rel(t.grad, gd[n]) < 1e-4, n
    for k, p in gen.named_parameters():
        if k == "in_conv.layers.0.bias" or k.endswith("layers.0.layers.2.bias") or k == "up.0.layers.1.layers.0.bias":
            continue
        assert rel(p.grad, gd["grads"][k]) < 1e-3, k


def test_generator_warp_bf16_vs_reference():
    gd, gen, ins, y = _generator(torch.bfloat16)
    e = {"out": rel(y, gd["out"])}
    e.update({n: rel(t.grad, gd[n]) for n, t in zip(("d_fs", "d_deformation", "d_occlusion"), ins)})
    print("\nwarped Generator bf16 vs reference: " + " ".join(f"{k} {v:.2e}" for k, v in e.items()))
    # the parity gate is fp32 mode (above); in bf16 every activation and gradient of this narrow
    # (16-32 channel, 512-pixel BN) trunk is stored in bf16, and the input gradients pass back
    # through 6 convs and 4 BN layers (measured: image 1.8e-3, input gradients 0.09-0.13)
    assert e["out"] < 2e-2 and max(e["d_fs"], e["d_occlusion"], e["d_deformation"]) < 2.5e-1


def test_reference_size_afe_to_warped_generator_vs_oracle():
    """The reference's full-size decoder input path (trainer.py:268, 296-297 without the keypoint
    nets): fs = AFE()(x) [1, 32, 16, 64, 64] with its ResBlock3D trunk, then
    Generator()(fs, deformation, occlusion) at 256x256 in fp32 parity mode, against the CPU
    oracle on the same weights run in float64.  Forward: 1e-3 (north_star).  Weight gradients:
    at this depth the reference's own fp32 arithmetic (the oracle in float32) is already up to
    ~1e-2 away from float64 (BatchNorm-backward cancellation, compounding through 18 BN layers),
    so each parameter's error is gated at 2x the fp32 reference's own error + 1e-4: the product
    is as accurate as the reference computed in fp32."""
    from oracle import facevae_cpu as O
    torch.manual_seed(3)
    afe, gen = fv.AFE(), fv.Generator()
    base = {**{f"afe.{k}": v for k, v in afe.state_dict().items()},
            **{f"generator.{k}": v for k, v in gen.state_dict().items()}}
    g = torch.Generator().manual_seed(4)
    x = torch.rand(1, 3, 256, 256, generator=g)
    ident = warp.make_coordinate_grid_3d((16, 64, 64))[None]
    deform = ident + 0.05 * torch.randn(1, 16, 64, 64, 3, generator=g)
    occ = torch.sigmoid(torch.randn(1, 1, 64, 64, generator=g))
    gy = torch.randn(1, 3, 256, 256, generator=g)
    afe = afe.cuda().train().set_compute_dtype(torch.float32)
    gen = gen.cuda().train().set_compute_dtype(torch.float32)
    fs = afe(x.cuda())
    y = gen(fs, deform.cuda(), occ.cuda())
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    ref = {}
    for dt in (torch.float64, torch.float32):
        sd = O.prepare_state(base)
        sd = {k: (v.detach().to(dt).requires_grad_(v.requires_grad) if v.is_floating_point() else v.clone())
              for k, v in sd.items()}
        fso = O.encode_afe(sd, x.to(dt), [64, 128, 256], 32, 16, 6, True)
        yo = O.generator_warp(sd, fso, deform.to(dt), occ.to(dt), n_res=6, n_up=2, training=True)
        (yo * gy.to(dt)).sum().backward()
        ref[dt] = (fso.detach(), yo.detach(), {k: v.grad for k, v in sd.items() if v.grad is not None})
    f64, f32 = ref[torch.float64], ref[torch.float32]
    fwd = {"fs": rel(fs, f64[0]), "image": rel(y, f64[1])}
    prm = {**{f"generator.{k}": p for k, p in gen.named_parameters()}, **{f"afe.{k}": p for k, p in afe.named_parameters()}}
    worst = []
    for k, p in prm.items():
        if k.endswith("bias"):
            continue
        e_prod, e_ref = rel(p.grad, f64[2][k]), rel(f32[2][k], f64[2][k])
        worst.append((e_prod / (2 * e_ref + 1e-4), k, e_prod, e_ref))
    worst.sort(reverse=True)
    print("\nfull-size AFE -> warped Generator, fp32 vs float64 oracle: "
          + " ".join(f"{k} {v:.2e}" for k, v in fwd.items()) + " | weight grads (product, fp32 reference): "
          + " ".join(f"{k} {a:.1e}/{b:.1e}" for _, k, a, b in worst[:4]))
    assert max(fwd.values()) < 1e-3, fwd
    assert worst[0][0] < 1.0, worst[:4]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_grid_sample3d_warp_shape_vs_torch(dtype):
    """The §8(f) warp at its real volume (C = 32, 16 x 64 x 64, two images) with the fbench
    deformation (identity + 0.05 N(0, 1)): every input cell's gradient gathered from its buckets."""
    g = torch.Generator().manual_seed(11)
    N, C, D, H, W = 2, 32, 16, 64, 64
    inp = torch.randn(N, C, D, H, W, generator=g)
    grid = warp.make_coordinate_grid_3d((D, H, W))[None] + 0.05 * torch.randn(N, D, H, W, 3, generator=g)
    gout = torch.randn(N, C, D, H, W, generator=g)
    xi = inp.cuda().to(dtype).contiguous(memory_format=CL3).requires_grad_(True)
    out = warp.GridSample3dFn.apply(xi, grid.cuda(), 1, dtype)
    out.backward(gout.cuda().to(dtype))
    torch.cuda.synchronize()
    ir = inp.to(dtype).float().requires_grad_(True)
    ref = F.grid_sample(ir, grid, align_corners=True)
    ref.backward(gout.to(dtype).float())
    if dtype == torch.float32:
        assert rel(out, ref) < 1e-5 and rel(xi.grad, ir.grad) < 1e-5
    else:
        for a, b in ((out, ref), (xi.grad, ir.grad)):
            assert rel(a.float(), b) < 4e-3 and maxd(a.float(), b) <= 1.6e-2 * b.abs().max().item()


@pytest.mark.parametrize("collapse", [False, True])
def test_grid_sample3d_input_gradient_is_deterministic(collapse):
    """The bucketed gather's buckets are sorted by voxel index (warp.hip gs_bucket_sort), so the
    input gradient is bit-identical run to run; `collapse` squeezes every sample into two corner
    cells (buckets of 17..2048 voxels: the workgroup bitonic sort of gs_bucket_sort_coop) --
    still vs F.grid_sample."""
    g = torch.Generator().manual_seed(11)
    N, C, Di, Hi, Wi, Do, Ho, Wo = 2, 32, 4, 8, 16, 8, 16, 16
    inp = torch.randn(N, C, Di, Hi, Wi, generator=g)
    grid = (torch.rand(N, Do, Ho, Wo, 3, generator=g) - 0.5) * 2.2
    if collapse:
        grid = grid * 0.01 - 0.99
    gout = torch.randn(N, C, Do, Ho, Wo, generator=g)
    grads = []
    for _ in range(3):
        xi = inp.cuda().contiguous(memory_format=CL3).requires_grad_(True)
        out = warp.GridSample3dFn.apply(xi, grid.cuda(), 1, torch.float32)
        out.backward(gout.cuda())
        torch.cuda.synchronize()
        grads.append(xi.grad.cpu())
    assert all(torch.equal(grads[0], t) for t in grads[1:])
    ir = inp.clone().requires_grad_(True)
    F.grid_sample(ir, grid, align_corners=True).backward(gout)
    assert rel(grads[0], ir.grad) < 1e-5


@pytest.mark.parametrize("mode", ["constant", "half"])
def test_grid_sample3d_input_gradient_degenerate_grid(mode):
    """A degenerate motion grid: every voxel ("constant") or the front half of the volume
    ("half") samples one point, so one bucket per image holds 32-64 K voxels (more than
    GS_MID: gs_bucket_sort_coop's stable compaction, not one lane's sort).  Bit-identical run to
    run, within 1e-4 of a float64 F.grid_sample (65 K-term sums per cell), and bounded in time:
    the warm backward finishes in well under a second (one lane sorting the bucket took
    seconds)."""
    g = torch.Generator().manual_seed(5)
    N, C, Di, Hi, Wi, Do, Ho, Wo = 2, 32, 8, 16, 16, 16, 64, 64
    inp = torch.randn(N, C, Di, Hi, Wi, generator=g)
    grid = (torch.rand(N, Do, Ho, Wo, 3, generator=g) - 0.5) * 2.0
    pt = torch.tensor([0.1, -0.2, 0.3])
    if mode == "constant":
        grid[:] = pt
    else:
        grid[:, : Do // 2] = pt
    gout = torch.randn(N, C, Do, Ho, Wo, generator=g)
    gd, god = grid.cuda(), gout.cuda()
    grads, times = [], []
    for _ in range(3):
        xi = inp.cuda().contiguous(memory_format=CL3).requires_grad_(True)
        out = warp.GridSample3dFn.apply(xi, gd, 1, torch.float32)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        out.backward(god)
        t1.record()
        torch.cuda.synchronize()
        times.append(t0.elapsed_time(t1))
        grads.append(xi.grad.cpu())
    print(f"\ndegenerate grid ({mode}): backward {min(times[1:]):.2f} ms")
    assert all(torch.equal(grads[0], t) for t in grads[1:])
    ir = inp.double().requires_grad_(True)
    F.grid_sample(ir, grid.double(), align_corners=True).backward(gout.double())
    assert rel(grads[0], ir.grad) < 1e-4
    assert min(times[1:]) < 500.0, times
