"""Warp path of the Generator and the MFE motion assembly over libfacevae's
warp.hip kernels.  No CPU fallback: every compute call goes through `_lib.call`.

Reference functions mirrored (file:line in Luh1124/face-vae), same names and argument
meaning, device-agnostic (the reference hard-codes .cuda(), utils.py:81-82, 93-95):
  make_coordinate_grid_3d             utils.py:91-103
  create_heatmap_representations      utils.py:130-137 (kp2gaussian_3d 123-129, variance 0.01)
  create_sparse_motions               utils.py:139-152
  create_deformed_source_image        utils.py:155-179
  deformation_from_mask               MFE.forward models.py:1076-1078 (softmax over K+1, sum)
  grid_sample_3d                      F.grid_sample(..., align_corners=True) for 5-D inputs
                                      (models.py:1103, utils.py:175): trilinear, zeros padding
  occlusion_multiply                  fs * occlusion (models.py:1106)
The 5-D feature volumes are NDHWC (torch.channels_last_3d); motion fields / grids stay fp32
[N, ..., 3] as the reference's.  grid_sample's input gradient is a bucketed gather (output
voxels counting-sorted by base input cell, each bucket then ordered by voxel index, each input
cell summing its <= 8 neighbouring buckets): no float atomics and a fixed summation order, so
it is bit-reproducible (torch's own GPU kernel uses float atomics).
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import ops
from ._lib import call, ptr, stream

CL3 = torch.channels_last_3d
F32 = torch.float32


def _cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("facevae_amd ops run on the GPU only (HIP); got a CPU tensor")


def _f32(t):
    return t.detach().float().contiguous() if t is not None else None


def make_coordinate_grid_3d(spatial_size, device=None):
    """[D, H, W, 3] grid of (x over W, y over H, z over D) in [-1, 1] (utils.py:91-103)."""
    d, h, w = spatial_size
    z = 2 * (torch.arange(d, device=device) / (d - 1)) - 1
    x = 2 * (torch.arange(h, device=device) / (h - 1)) - 1
    y = 2 * (torch.arange(w, device=device) / (w - 1)) - 1
    zz = z.view(-1, 1, 1).repeat(1, h, w)
    xx = x.view(1, -1, 1).repeat(d, 1, w)
    yy = y.view(1, 1, -1).repeat(d, h, 1)
    return torch.cat([yy.unsqueeze(3), xx.unsqueeze(3), zz.unsqueeze(3)], 3)


# ----------------------------------------------------------------------------------------
# grid sampling
# ----------------------------------------------------------------------------------------

class GridSample3dFn(torch.autograd.Function):
    """out[b] = grid_sample(inp[b // group], grid[b]) (trilinear, zeros, align_corners=True)."""

    @staticmethod
    def forward(ctx, inp, grid, group, dtype):
        _cuda(inp, grid)
        Bi, C, Di, Hi, Wi = inp.shape
        B, Do, Ho, Wo, three = grid.shape
        if three != 3 or B != Bi * group:
            raise RuntimeError(f"grid_sample_3d: grid {tuple(grid.shape)} does not match input {tuple(inp.shape)}")
        xb = inp.to(dtype).contiguous(memory_format=CL3)
        g32 = _f32(grid)
        out = torch.empty((B, C, Do, Ho, Wo), dtype=dtype, device=inp.device, memory_format=CL3)
        call("fv_grid_sample3d_fwd", L.dtype_code(dtype), ptr(xb), ptr(g32), B, Di, Hi, Wi, Do, Ho, Wo, C, group,
             ptr(out), stream())
        ctx.save_for_backward(xb, g32)
        ctx.group, ctx.dtype, ctx.in_dtype = group, dtype, inp.dtype
        return out

    @staticmethod
    def backward(ctx, gout):
        xb, g32 = ctx.saved_tensors
        Bi, C, Di, Hi, Wi = xb.shape
        B, Do, Ho, Wo, _ = g32.shape
        go = gout.to(ctx.dtype).contiguous(memory_format=CL3)
        gin = ggrid = None
        if ctx.needs_input_grad[0]:
            # input gradient by bucketed gather (no float atomics, no fp32 staging buffer); an fp32
            # input sampled in bf16 gets its gradient summed and stored in fp32
            gd = F32 if ctx.in_dtype == F32 else ctx.dtype
            gsrc = go if gd == ctx.dtype else go.to(gd)
            nws = L.query("fv_grid_sample3d_bwd_input_ws_bytes", B, Di, Hi, Wi, Do, Ho, Wo, ctx.group)
            ws = ops._empty(nws, torch.uint8, xb.device)
            gin = torch.empty((Bi, C, Di, Hi, Wi), dtype=gd, device=xb.device, memory_format=CL3)
            call("fv_grid_sample3d_bwd_input", L.dtype_code(gd), ptr(g32), ptr(gsrc), B, Di, Hi, Wi, Do, Ho, Wo,
                 C, ctx.group, ptr(gin), ptr(ws), stream())
            gin = gin.to(ctx.in_dtype)
        if ctx.needs_input_grad[1]:
            ggrid = torch.empty_like(g32)
            call("fv_grid_sample3d_bwd", L.dtype_code(ctx.dtype), ptr(xb), ptr(g32), ptr(go), B, Di, Hi, Wi, Do, Ho,
                 Wo, C, ctx.group, None, ptr(ggrid), stream())
        return gin, ggrid, None, None


def grid_sample_3d(inp, grid, dtype=None):
    """F.grid_sample(inp, grid, align_corners=True) for inp [N, C, D, H, W], grid [N, Do, Ho, Wo, 3]."""
    dtype = dtype or (inp.dtype if inp.dtype in (F32, torch.bfloat16) else F32)
    return GridSample3dFn.apply(inp, grid, 1, dtype)


class OcclusionFn(torch.autograd.Function):
    """fs [N, C, H, W] (NHWC) * occlusion [N, 1, H, W] (models.py:1106)."""

    @staticmethod
    def forward(ctx, fs, occ, dtype):
        _cuda(fs, occ)
        fb, C = ops.to_nhwc(fs, dtype)
        N, Cv, H, W = fs.shape
        if C != Cv or tuple(occ.shape) != (N, 1, H, W):
            raise RuntimeError("occlusion: fs [N, C, H, W] (C a power of two >= 8) and occlusion [N, 1, H, W]")
        o32 = _f32(occ)
        y = torch.empty_like(fb)
        call("fv_occlusion_fwd", L.dtype_code(dtype), ptr(fb), ptr(o32), N * H * W, C, ptr(y), stream())
        ctx.save_for_backward(fb, o32)
        ctx.dtype = dtype
        return y

    @staticmethod
    def backward(ctx, g):
        fb, o32 = ctx.saved_tensors
        N, C, H, W = fb.shape
        gb = ops.grad_in(g, ctx.dtype)
        dx = torch.empty_like(fb) if ctx.needs_input_grad[0] else None
        docc = torch.empty((N, 1, H, W), dtype=F32, device=fb.device) if ctx.needs_input_grad[1] else None
        call("fv_occlusion_bwd", L.dtype_code(ctx.dtype), ptr(gb), ptr(fb), ptr(o32), N * H * W, C, ptr(dx), ptr(docc),
             stream())
        return dx, docc, None


def occlusion_multiply(fs, occlusion, mode):
    return OcclusionFn.apply(fs, occlusion, ops.storage(mode))


# ----------------------------------------------------------------------------------------
# MFE motion assembly
# ----------------------------------------------------------------------------------------

class SparseMotionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kp_s, kp_d, J, D, H, W):
        _cuda(kp_s, kp_d, J)
        N, K, _ = kp_s.shape
        ks, kd, j = _f32(kp_s), _f32(kp_d), _f32(J)
        out = torch.empty((N, K + 1, D, H, W, 3), dtype=F32, device=kp_s.device)
        call("fv_sparse_motion_fwd", ptr(ks), ptr(kd), ptr(j), N, K, D, H, W, ptr(out), stream())
        ctx.save_for_backward(kd, j)
        ctx.dims = (D, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        kd, j = ctx.saved_tensors
        N, K, _ = kd.shape
        D, H, W = ctx.dims
        sums = torch.empty((N, K, 12), dtype=F32, device=kd.device)
        call("fv_sparse_motion_bwd", ptr(_f32(g)), ptr(kd), N, K, D, H, W, ptr(sums), stream())
        sg = sums[..., :3]                       # sum_v g          [N, K, 3]
        sgc = sums[..., 3:].view(N, K, 3, 3)     # sum_v g c^T      [N, K, 3, 3]
        dkp_s = sg
        dkp_d = -torch.einsum("nji,nkj->nki", j, sg)      # -J^T sum_v g
        dJ = sgc.sum(1)
        return dkp_s, dkp_d, dJ, None, None, None


def create_sparse_motions(fs, kp_s, kp_d, Rs, Rd):
    """[N, K+1, D, H, W, 3] (utils.py:139-152); J = Rs inv(Rd) is formed here (3x3 per sample)."""
    N, _, D, H, W = fs.shape
    J = torch.matmul(Rs, torch.inverse(Rd))
    return SparseMotionFn.apply(kp_s, kp_d, J, D, H, W)


class HeatmapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kp_s, kp_d, D, H, W, var):
        _cuda(kp_s, kp_d)
        N, K, _ = kp_s.shape
        ks, kd = _f32(kp_s), _f32(kp_d)
        out = torch.empty((N, K + 1, D, H, W), dtype=F32, device=kp_s.device)
        call("fv_heatmap_fwd", ptr(ks), ptr(kd), N, K, D, H, W, float(var), ptr(out), stream())
        ctx.save_for_backward(ks, kd)
        ctx.dims = (D, H, W, var)
        return out

    @staticmethod
    def backward(ctx, g):
        ks, kd = ctx.saved_tensors
        N, K, _ = ks.shape
        D, H, W, var = ctx.dims
        dks, dkd = torch.empty_like(ks), torch.empty_like(kd)
        call("fv_heatmap_bwd", ptr(_f32(g)), ptr(ks), ptr(kd), N, K, D, H, W, float(var), ptr(dks), ptr(dkd),
             stream())
        return dks, dkd, None, None, None, None


def create_heatmap_representations(fs, kp_s, kp_d, kp_variance=0.01):
    """[N, K+1, 1, D, H, W]: zeros, then gauss(kp_d) - gauss(kp_s) (utils.py:130-137)."""
    N, _, D, H, W = fs.shape
    return HeatmapFn.apply(kp_s, kp_d, D, H, W, kp_variance).unsqueeze(2)


def create_deformed_source_image(fs, sparse_motions, dtype=None):
    """[N, K+1, C, D, H, W]: fs sampled at each of the K+1 motions (utils.py:155-179), without
    materialising the (K+1)-fold repeat of fs (the kernel maps output batch b to input b // (K+1))."""
    N, C, D, H, W = fs.shape
    K1 = sparse_motions.shape[1]
    dtype = dtype or (fs.dtype if fs.dtype in (F32, torch.bfloat16) else F32)
    grid = sparse_motions.reshape(N * K1, D, H, W, 3)
    out = GridSample3dFn.apply(fs, grid, K1, dtype)          # [N*K1, C, D, H, W] NDHWC
    return out.view(N, K1, C, D, H, W)


class MotionMaskFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, sm):
        _cuda(logits, sm)
        N, K1, D, H, W = logits.shape
        V = D * H * W
        lg, s = _f32(logits), _f32(sm)
        prob = torch.empty((N, K1, D, H, W), dtype=F32, device=logits.device)
        deform = torch.empty((N, D, H, W, 3), dtype=F32, device=logits.device)
        call("fv_motion_mask_fwd", ptr(lg), ptr(s), N, K1, V, ptr(prob), ptr(deform), stream())
        ctx.save_for_backward(prob, s)
        return deform, prob

    @staticmethod
    def backward(ctx, gdef, gprob):
        prob, s = ctx.saved_tensors
        N, K1, D, H, W = prob.shape
        gd = _f32(gdef) if gdef is not None else torch.zeros((N, D, H, W, 3), dtype=F32, device=prob.device)
        gp = _f32(gprob)
        dl = torch.empty_like(prob) if ctx.needs_input_grad[0] else None
        ds = torch.empty_like(s) if ctx.needs_input_grad[1] else None
        call("fv_motion_mask_bwd", ptr(prob), ptr(s), ptr(gd), ptr(gp), N, K1, D * H * W, ptr(dl), ptr(ds), stream())
        return dl, ds


def deformation_from_mask(mask_logits, sparse_motion):
    """MFE.forward tail (models.py:1076-1078): mask = softmax(mask_logits, dim=1).unsqueeze(-1),
    deformation = (sparse_motion * mask).sum(dim=1).  -> (deformation [N, D, H, W, 3], mask
    [N, K+1, D, H, W, 1])."""
    deform, prob = MotionMaskFn.apply(mask_logits, sparse_motion)
    return deform, prob.unsqueeze(-1)
