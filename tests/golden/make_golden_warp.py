"""Generate the golden fixtures of the warp path FROM THE REFERENCE ITSELF.

Run in the build container only (it needs /root/reference):

    python tests/golden/make_golden_warp.py

The reference's coordinate grids hard-code `.cuda()` (utils.py:81-82, 93-95, 134); this
container has no GPU, so for the duration of this script torch.Tensor.cuda is the identity
(the arithmetic is unchanged: CPU fp32).  Stores plain tensors in tests/golden/warp.pt:

  motion     create_sparse_motions / create_heatmap_representations /
             create_deformed_source_image (utils.py:130-179) on fs [2, 4, 4, 8, 8], K = 5
             keypoints, head rotations Rs / Rd; outputs and the gradients of sum(out * g)
             w.r.t. every input.
  mask       the MFE tail (models.py:1076-1078): softmax of mask logits [2, 6, 4, 8, 8] and
             the deformation sum; outputs and input gradients.
  generator  models.Generator(use_weight_norm=True, n_res=1, up_seq=[32, 16], D=2, C=16) in
             training mode on fs [2, 16, 2, 16, 16] with a deformation [2, 2, 16, 16, 3] (partly
             outside [-1, 1]) and occlusion [2, 1, 16, 16]: output and the gradients of
             sum(out * g) w.r.t. fs, deformation, occlusion and every parameter.
"""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402


def rot(g, n):
    a = torch.rand(n, 3, generator=g) - 0.5
    sys.path.insert(0, "/root/reference")
    import utils  # noqa: E402  (reference)
    return utils.rotation_matrix_y(a[:, 1]) @ utils.rotation_matrix_x(a[:, 0]) @ utils.rotation_matrix_z(a[:, 2])


def main():
    torch.Tensor.cuda = lambda self, *a, **k: self       # reference grids call .cuda()
    _, models, _ = import_reference()
    import utils  # noqa: E402  (reference)
    g = torch.Generator().manual_seed(31)
    out = {}

    N, K, C, D, H, W = 2, 5, 4, 4, 8, 8
    fs = torch.randn(N, C, D, H, W, generator=g)
    kp_s = (torch.rand(N, K, 3, generator=g) - 0.5) * 1.6
    kp_d = (torch.rand(N, K, 3, generator=g) - 0.5) * 1.6
    Rs, Rd = rot(g, N), rot(g, N)
    ins = [t.clone().requires_grad_(True) for t in (fs, kp_s, kp_d, Rs, Rd)]
    sm = utils.create_sparse_motions(*ins)
    hm = utils.create_heatmap_representations(ins[0], ins[1], ins[2])
    ds = utils.create_deformed_source_image(ins[0], sm)
    g_sm = torch.randn(sm.shape, generator=g)
    g_hm = torch.randn(hm.shape, generator=g)
    g_ds = torch.randn(ds.shape, generator=g)
    ((sm * g_sm).sum() + (hm * g_hm).sum() + (ds * g_ds).sum()).backward()
    out["motion"] = dict(fs=fs, kp_s=kp_s, kp_d=kp_d, Rs=Rs, Rd=Rd, sm=sm.detach(), hm=hm.detach(), ds=ds.detach(),
                         g_sm=g_sm, g_hm=g_hm, g_ds=g_ds,
                         grads={n: t.grad.clone() for n, t in zip(("fs", "kp_s", "kp_d", "Rs", "Rd"), ins)})

    logits = torch.randn(N, K + 1, D, H, W, generator=g)
    smot = torch.randn(N, K + 1, D, H, W, 3, generator=g)
    lt, st = logits.clone().requires_grad_(True), smot.clone().requires_grad_(True)
    mask = F.softmax(lt, dim=1).unsqueeze(-1)                   # models.py:1076
    deformation = (st * mask).sum(dim=1)                        # models.py:1078
    g_def = torch.randn(deformation.shape, generator=g)
    g_mask = torch.randn(mask.shape, generator=g)
    ((deformation * g_def).sum() + (mask * g_mask).sum()).backward()
    out["mask"] = dict(logits=logits, sm=smot, deformation=deformation.detach(), mask=mask.detach(), g_def=g_def,
                       g_mask=g_mask, d_logits=lt.grad.clone(), d_sm=st.grad.clone())

    torch.manual_seed(41)
    gen = models.Generator(use_weight_norm=True, n_res=1, up_seq=[32, 16], D=2, C=16).train()
    init = {k: v.detach().clone() for k, v in gen.state_dict().items()}
    fs = torch.randn(2, 16, 2, 16, 16, generator=g)
    deform = (torch.rand(2, 2, 16, 16, 3, generator=g) - 0.5) * 2.3
    occ = torch.sigmoid(torch.randn(2, 1, 16, 16, generator=g))
    ins = [t.clone().requires_grad_(True) for t in (fs, deform, occ)]
    y = gen(*ins)
    gy = torch.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    out["generator"] = dict(seed=torch.tensor(41), init=init, fs=fs, deformation=deform, occlusion=occ, out=y.detach(),
                            g=gy, d_fs=ins[0].grad.clone(), d_deformation=ins[1].grad.clone(),
                            d_occlusion=ins[2].grad.clone(),
                            grads={k: p.grad.clone() for k, p in gen.named_parameters()})
    path = os.path.join(HERE, "warp.pt")
    torch.save(out, path)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
