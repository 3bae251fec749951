"""ctypes binding of libfacevae.so (the C-ABI declared in include/facevae.h).

The library is built in-tree (face-vae_amd/csrc/build.py -> face-vae_amd/libfacevae.so).
There is no fallback: if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_long, c_size_t, c_void_p

import torch  # noqa: F401  (must be imported first: the HIP runtime is shared with torch)

_HERE = os.path.dirname(os.path.realpath(__file__))
# FV_LIB_PATH: another build of the library (A/B of two builds on one box, tools/gpu.sh ab)
LIB_PATH = os.environ.get("FV_LIB_PATH") or os.path.join(_HERE, "libfacevae.so")

FV_F32, FV_BF16, FV_F64 = 0, 1, 2
FV_E_BADARG, FV_E_UNSUPPORTED, FV_E_COMM = 1001, 1002, 1003
ADAM_CHUNK = 4096
ABI_VERSION = 2


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", c_int), ("n", c_int), ("h", c_int), ("w", c_int),
        ("cin", c_int), ("cin_valid", c_int), ("cout", c_int), ("ldy", c_int),
        ("ksize", c_int), ("upsample", c_int), ("pro_act", c_int), ("pro_slope", c_float),
        ("epi_sigmoid", c_int), ("out_nchw_f32", c_int),
    ]


class Conv3dDesc(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("n", c_int), ("d", c_int), ("h", c_int), ("w", c_int),
                ("cin", c_int), ("cout", c_int)]


class StoreReduce(ctypes.Structure):
    _fields_ = [("mode", c_int), ("records", c_void_p), ("bn_input", c_void_p), ("mean", c_void_p),
                ("invstd", c_void_p), ("gamma", c_void_p), ("beta", c_void_p), ("slope", c_float)]


class SnLayer(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("u", c_void_p), ("v", c_void_p), ("sigma", c_void_p), ("usnap", c_void_p),
                ("vsnap", c_void_p), ("rows", c_int), ("cols", c_int)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p),
                ("exp_avg_sq", c_void_p), ("numel", c_long)]


P = c_void_p
D = POINTER(ConvDesc)
D3 = POINTER(Conv3dDesc)
# name -> (restype, argtypes)
_SIGS = {
    "fv_abi_version": (c_int, []),
    "fv_last_error": (ctypes.c_char_p, []),
    "fv_conv_wk_elems": (c_size_t, [D]),
    "fv_conv_wt_elems": (c_size_t, [D]),
    "fv_conv2d_stats_blocks": (c_int, [D]),
    "fv_conv2d_stats_block_pixels": (c_int, [D]),
    "fv_conv_weight_prep": (c_int, [D, P, P, P, P, P]),
    "fv_conv2d_fwd": (c_int, [D, P, P, P, P, P, P, P, P, P]),
    "fv_conv2d_bwd_data": (c_int, [D, P, c_int, P, P, P]),
    "fv_conv2d_dgrad_lowres": (c_int, [D]),
    "fv_conv2d_wgrad_nsplit": (c_int, [D]),
    "fv_conv2d_wgrad_slab_elems": (c_size_t, [D]),
    "fv_conv2d_wgrad_bias_slab_elems": (c_size_t, [D]),
    "fv_conv2d_bwd_weight": (c_int, [D, P, P, P, P, c_int, P, P, P]),
    "fv_conv2d_wgrad_reduce": (c_int, [D, P, P, P, P, P]),
    "fv_conv2d_sr_records": (c_int, [D, c_int, POINTER(c_int)]),
    "fv_conv2d_fwd_sr": (c_int, [D, P, P, P, P, P, P, P]),
    "fv_conv2d_bwd_data_sr": (c_int, [D, P, c_int, P, P, P, P]),
    "fv_bn_bwd_from_records": (c_int, [P, c_int, c_int, c_long, c_int, c_long, P, P, P, P, P, P]),
    "fv_convt_supported": (c_int, [D]),
    "fv_convt_weight_prep": (c_int, [D, P, c_int, c_float, P, P, P, P]),
    "fv_convt_wgrad_reduce": (c_int, [D, P, P, P, c_int, c_float, P, P, P, P]),
    "fv_convt_eff_weight": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "fv_convt_weight_grad": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "fv_convt_direct_fwd": (c_int, [c_int, P, c_int, c_int, c_int, c_int, c_int, P, P, c_int, c_int, c_int, c_int,
                                    c_int, P, P]),
    "fv_convt_direct_dgrad": (c_int, [c_int, P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int,
                                      c_int, P, P]),
    "fv_convt_direct_wgrad": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, P, P, P]),
    "fv_chan_scale_fwd": (c_int, [c_int, P, c_int, c_long, c_int, c_int, P, P, P, P]),
    "fv_chan_scale_bwd": (c_int, [c_int, P, P, c_int, c_long, c_int, c_int, P, P, P, P, P]),
    "fv_fp8_ws_bytes": (c_size_t, []),
    "fv_quantize_fp8": (c_int, [c_int, P, c_long, P, P, P, P]),
    "fv_conv2d_fp8_supported": (c_int, [D]),
    "fv_conv_fp8_wk_bytes": (c_size_t, [D]),
    "fv_conv_fp8_wt_bytes": (c_size_t, [D]),
    "fv_conv_weight_prep_fp8": (c_int, [D, P, P, P, P, P, P, P]),
    "fv_conv2d_fwd_fp8": (c_int, [D, P, P, P, P, P, P, P, P, P]),
    "fv_conv2d_bwd_data_fp8": (c_int, [D, P, P, P, P, P, P]),
    "fv_fp8_site_bytes": (c_size_t, []),
    "fv_quantize_fp8_site": (c_int, [c_int, P, c_long, P, P, c_int, P, P]),
    "fv_conv2d_fwd_fp8_site": (c_int, [D, P, P, P, P, P, P, P, P, P]),
    "fv_conv2d_fwd_fp8_site_sr": (c_int, [D, P, P, P, P, P, P, P, P, P]),
    "fv_conv2d_bwd_data_fp8_site": (c_int, [D, P, P, P, P, P, P]),
    "fv_fp8_set_deferred_roll": (c_int, [c_int]),
    "fv_fp8_amax": (c_int, [c_int, P, c_long, P, P, P]),
    "fv_fp8_site_seed": (c_int, [P, P, P]),
    "fv_fp8_sites_inflight": (c_int, [c_int, P, P, P]),
    "fv_fp8_sites_roll": (c_int, [c_int, P, P, P]),
    "fv_conv2d_wgrad_fp8_supported": (c_int, [D]),
    "fv_conv2d_bwd_weight_fp8": (c_int, [D, P, P, P, P, P, P, P]),
    "fv_conv2d_wgrad_fp8_reduce": (c_int, [D, P, P, P, P, P]),
    "fv_conv2d_fp8_stats_blocks": (c_int, [D]),
    "fv_conv2d_fp8_stats_block_pixels": (c_int, [D]),
    "fv_fp8_mfma_probe": (c_int, [P, P, P, P]),
    "fv_tr8_probe": (c_int, [P, P, P]),
    "fv_conv3d_wk_bytes": (c_size_t, [D3]),
    "fv_conv3d_weight_prep": (c_int, [D3, P, P, P, P]),
    "fv_conv3d_weight_prep_multi": (c_int, [D3, c_int, P, P, P, P]),
    "fv_conv3d_stats_blocks": (c_int, [D3]),
    "fv_conv3d_stats_block_pixels": (c_int, [D3]),
    "fv_conv3d_fwd": (c_int, [D3, P, P, P, P, P, P, P]),
    "fv_conv3d_bwd_data": (c_int, [D3, P, P, P, P]),
    "fv_conv3d_wgrad_ws_bytes": (c_size_t, [D3]),
    "fv_conv3d_bwd_weight": (c_int, [D3, P, P, P, P, P, P]),
    "fv_depth_split": (c_int, [c_int, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "fv_grid_sample3d_fwd": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                     P, P]),
    "fv_grid_sample3d_bwd": (c_int, [c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_int, P, P, P]),
    "fv_grid_sample3d_bwd_input_ws_bytes": (c_size_t, [c_int] * 8),
    "fv_grid_sample3d_bwd_input": (c_int, [c_int, P, P] + [c_int] * 9 + [P, P, P]),
    "fv_f32_to": (c_int, [c_int, P, P, c_long, P]),
    "fv_occlusion_fwd": (c_int, [c_int, P, P, c_long, c_int, P, P]),
    "fv_occlusion_bwd": (c_int, [c_int, P, P, P, c_long, c_int, P, P, P]),
    "fv_sparse_motion_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "fv_sparse_motion_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "fv_heatmap_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_float, P, P]),
    "fv_heatmap_bwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "fv_motion_mask_fwd": (c_int, [P, P, c_int, c_int, c_long, P, P, P]),
    "fv_motion_mask_bwd": (c_int, [P, P, P, P, c_int, c_int, c_long, P, P, P]),
    "fv_relu_bwd": (c_int, [c_int, P, P, c_long, P, P]),
    "fv_maxpool2_fwd": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_maxpool2_bwd": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_avgpool2_bwd": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_l1t_ws_bytes": (c_size_t, []),
    "fv_l1t_fwd": (c_int, [c_int, P, P, c_long, P, P, P]),
    "fv_l1t_bwd": (c_int, [c_int, P, P, c_long, P, c_float, P, P]),
    "fv_spectral_norm_ws_bytes": (c_size_t, [c_int, c_int]),
    "fv_spectral_norm_fwd": (c_int, [P, c_int, c_int, P, P, P, c_int, P, P]),
    "fv_spectral_norm_bwd": (c_int, [P, P, c_int, c_int, P, P, P, P, P, P]),
    "fv_spectral_norm_batch_ws_floats": (c_size_t, [P, c_int]),
    "fv_spectral_norm_batch_table_bytes": (c_size_t, [c_int]),
    "fv_spectral_norm_batch_build": (c_int, [P, c_int, P, P, P]),
    "fv_spectral_norm_fwd_batch": (c_int, [P, c_int, P, c_int, P]),
    "fv_bn_ws_bytes": (c_size_t, [c_int]),
    "fv_bn_stats_from_partials": (c_int, [P, c_int, c_int, c_long, c_int, P, P, P]),
    "fv_bn_stats_tensor": (c_int, [c_int, P, c_long, c_int, c_int, P, P, P]),
    "fv_bn_finalize": (c_int, [P, c_int, P, P, c_float, c_float, c_int, P, P, P, P, P, P, P, P]),
    "fv_bn_stats_finalize_partials": (c_int, [P, c_int, c_int, c_long, c_int, P, P, c_float, c_float, P, P, P, P, P,
                                              P, P, P, P]),
    "fv_bn_stats_finalize_tensor": (c_int, [c_int, P, c_long, c_int, c_int, P, P, c_float, c_float, P, P, P, P, P, P,
                                            P, P, P]),
    "fv_bn_act_bwd_reduce_finalize": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, c_float,
                                              c_int, c_long, P, P, P, P, P]),
    "fv_bn_act_fwd": (c_int, [c_int, P, c_int, c_int, c_int, c_int, c_int, P, P, c_float, c_int, P, P]),
    "fv_bn_act_bwd_reduce": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, c_float,
                                     c_int, P, P, P]),
    "fv_bn_bwd_finalize": (c_int, [P, c_int, c_long, P, P, P, P]),
    "fv_bn_bwd_finalize_dev": (c_int, [P, c_int, P, P, P, P, P]),
    "fv_bn_act_bwd_apply": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, c_float,
                                    c_int, P, P, P, P]),
    "fv_bn_act_fwd_q8": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P, c_float, P, P, P, P]),
    "fv_bn_act_bwd_apply_q8": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, P, P, P, P, c_float, P, P, P, P,
                                       P, P]),
    "fv_nchw_to_nhwc": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_nhwc_to_nchw": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_cast": (c_int, [c_int, P, c_int, P, c_long, P]),
    "fv_upsample2x_bwd": (c_int, [c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_sigmoid_bwd_to_nhwc": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, P, P]),
    "fv_loss_ws_bytes": (c_size_t, []),
    "fv_reparam_fwd": (c_int, [c_int, P, P, c_int, c_int, c_int, P, P, P, P]),
    "fv_reparam_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "fv_reparam_kl_fwd": (c_int, [c_int, P, P, c_int, c_int, c_int, P, P, P, P, P, P]),
    "fv_reparam_bwd": (c_int, [c_int, P, P, c_int, c_int, c_int, P, P, P, P, P]),
    "fv_reparam_kl_bwd": (c_int, [c_int, P, P, c_int, c_int, c_int, P, P, P, P, P, P]),
    "fv_reparam_tiled": (c_int, [c_int, c_int]),
    "fv_kl_fwd": (c_int, [c_int, P, P, c_long, P, P, P]),
    "fv_kl_bwd": (c_int, [c_int, P, P, c_long, P, P, P, P]),
    "fv_mse_fwd": (c_int, [P, P, c_long, P, P, P]),
    "fv_mse_bwd": (c_int, [P, P, c_long, P, P, P, P]),
    "fv_l1_fwd": (c_int, [P, P, c_long, P, P, P]),
    "fv_l1_bwd": (c_int, [P, P, c_long, P, P, P, P]),
    "fv_adam_step": (c_int, [P, P, c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                             c_long, P]),
    "fv_adam_step_dev": (c_int, [P, P, c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 P, P, P]),
    "fv_copy_h2d_async": (c_int, [P, P, c_size_t, P]),
    "fv_conv_weight_prep_batchable": (c_int, [D]),
    "fv_spectral_norm_bwd_multi": (c_int, [c_int, P, P, P]),
    "fv_conv_weight_prep_multi": (c_int, [c_int, P, P, P, P, P, P]),
    "fv_conv_weight_prep_fp8_multi": (c_int, [c_int, P, P, P, P, P, P, P, P]),
    "fv_comm_unique_id": (c_int, [P]),
    "fv_comm_init": (c_int, [P, c_int, c_int, c_int, POINTER(c_void_p)]),
    "fv_comm_allreduce": (c_int, [c_void_p, P, c_size_t, c_int, c_int, P]),
    "fv_comm_allgather": (c_int, [c_void_p, P, P, c_size_t, c_int, P]),
    "fv_comm_broadcast": (c_int, [c_void_p, P, c_size_t, c_int, c_int, P]),
    "fv_comm_destroy": (c_int, [c_void_p]),
    "fv_comm_async_error": (c_int, [c_void_p, POINTER(c_int)]),
    "fv_comm_count": (c_int, [c_void_p, POINTER(c_int)]),
    "fv_comm_abort": (c_int, [c_void_p]),
}

_lib = None


class SnBwdLayer(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("g", c_void_p), ("u", c_void_p), ("v", c_void_p), ("sigma", c_void_p),
                ("rows", c_int), ("cols", c_int)]


class FaceVAELibError(RuntimeError):
    pass


def exported_symbols():
    return list(_SIGS)


def load():
    """Load libfacevae.so (idempotent).  Raises if it is missing — there is no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python face-vae_amd/csrc/build.py` "
                          "(or __graft_entry__.build()); the FaceVAE path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if os.environ.get("FV_LIB_PATH"):   # an A/B build of an older tree lacks newer entries
                continue
            raise
        f.restype = res
        f.argtypes = args
    if lib.fv_abi_version() != ABI_VERSION:
        raise ImportError("libfacevae ABI mismatch")
    _lib = lib
    return lib


_SYNC_CALLS = os.environ.get("FV_SYNC_CALLS", "0") == "1"   # debugging: a fault names its entry


def call(name, *args):
    """Call an fv_* entry; raise FaceVAELibError with fv_last_error() on failure."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        msg = lib.fv_last_error().decode(errors="replace")
        raise FaceVAELibError(f"{name} failed ({st}): {msg}")
    if _SYNC_CALLS:
        import torch
        try:
            torch.cuda.synchronize()
        except Exception as e:
            raise FaceVAELibError(f"{name}: device error after this call: {e}") from e
    return st


def query(name, *args):
    return getattr(load(), name)(*args)


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return FV_F32
    if dt == torch.bfloat16:
        return FV_BF16
    if dt == torch.float64:
        return FV_F64
    raise TypeError(f"unsupported dtype {dt}")


class _Staging:
    """Host -> device copies of the descriptor tables the batched launches read (spectral-norm
    layers, Adam tensors).  Eager: a fresh pinned buffer per copy, copied with torch's
    non_blocking copy (torch's pinned allocator keeps it until the copy has run).  Under HIP-
    graph capture (graph.StepGraph): persistent pinned buffers, one per copy in issue order,
    reserved from the sizes recorded during the last eager step before the capture, with their
    device tables allocated before the capture and written once when it ends (end()); both live
    as long as the graph."""

    def __init__(self):
        self.mode = "eager"          # "eager" | "record" | "capture"
        self.sizes = []
        self.bufs = []
        self.i = 0
        self.devs = []               # the captured tables' device buffers (allocated before the capture)
        self.deferred = []           # (device table, pinned buffer, bytes) filled at capture end
        self.keep = []               # the captured tables, alive as long as the graph

    def begin_record(self):
        self.mode, self.sizes = "record", []

    def begin_capture(self):
        if self.mode != "record":
            raise RuntimeError("staging: capture without a recorded eager step")
        self.bufs = [torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True) for n in self.sizes]
        # the device tables are allocated HERE, before the capture, from the ordinary pool: a
        # table allocated inside the capture may reuse the block of a tensor the step freed
        # earlier, which every replay overwrites before the table's reader runs (the copy node
        # of the old scheme re-wrote the table after it; a copy done once at capture end does not)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.devs = [torch.empty(max(n, 1), dtype=torch.uint8, device=dev) for n in self.sizes]
        self.mode, self.i = "capture", 0
        return self.bufs

    def end(self):
        """End of a capture: the tables are constant for every replay (their bytes were frozen at
        capture), so they are copied into their pre-allocated device buffers ONCE here instead of
        by a memcpy node in every replay (3 dependent ~5 us copy kernels per replayed step)."""
        if self.mode == "capture" and self.deferred:
            for dev, hb, n in self.deferred:
                dev.copy_(hb[:n])
            torch.cuda.synchronize()
            self.keep = self.deferred
        self.deferred = []
        self.mode = "eager"


staging = _Staging()


def h2d_table(data: bytes, device):
    """-> (device uint8 tensor holding `data`, host buffer to keep alive until consumed)."""
    n = len(data)
    if staging.mode == "capture":
        if staging.i >= len(staging.bufs) or staging.bufs[staging.i].numel() < n:
            raise RuntimeError("staging: the captured step issues other table copies than the recorded one")
        hb = staging.bufs[staging.i]
        dev = staging.devs[staging.i]
        staging.i += 1
        want = torch.device(device)
        if want.type != "cuda" or (want.index is not None and want.index != dev.device.index):
            raise RuntimeError("staging: the captured table's device differs from the current device")
        hb[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        # filled once by end(); referenced as long as the graph (staging.keep -> StepGraph)
        staging.deferred.append((dev, hb, n))
        return dev[:n], hb
    if staging.mode == "record":
        staging.sizes.append(n)
    hb = torch.frombuffer(bytearray(data), dtype=torch.uint8).pin_memory()
    return hb.to(device, non_blocking=True), hb
