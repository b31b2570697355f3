"""ctypes binding of libdmc.so (include/dmc.h) plus thin torch-tensor wrappers.

This module is the only place that talks to the native library. It fails loudly: importing it on a
machine where libdmc.so is missing raises, and there is no Python/PyTorch fallback for any kernel.
Every wrapper launches on torch's current HIP stream and never synchronises.
"""
import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must be loaded first so libdmc binds to torch's libamdhip64.so.7)

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DMC_LIB", _PKG / "libdmc.so"))

DMC_F32, DMC_BF16 = 0, 1
MODE_NORMAL, MODE_UPSAMPLE, MODE_DILATE = 0, 1, 2
PRO_NONE, PRO_AFFINE_SILU, PRO_SILU, PRO_AFFINE, PRO_GN_SILU = 0, 1, 2, 3, 4
LOSS = {"l1": 0, "l2": 1, "huber": 2}
PACK_FWD, PACK_DGRAD, PACK_UPDGRAD = 0, 1, 2

_c_int, _c_p, _c_f, _c_u32, _c_long, _c_size = (ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_uint32,
                                                ctypes.c_long, ctypes.c_size_t)


ACT_NONE, ACT_GELU, ACT_GELU_DROP, ACT_DGELU = 0, 1, 2, 3   # include/dmc.h DMC_ACT_*
FUSED_GN_STATS = 1   # dmc_conv2d_fused_epilogue bits


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", _c_int), ("N", _c_int), ("H", _c_int), ("W", _c_int),
        ("C1", _c_int), ("C2", _c_int), ("ld1", _c_int), ("ld2", _c_int), ("Kc", _c_int),
        ("OH", _c_int), ("OW", _c_int), ("Cout", _c_int), ("ntaps", _c_int), ("mode", _c_int), ("stride", _c_int),
        ("tap_dy", _c_int * 16), ("tap_dx", _c_int * 16),
        ("prologue", _c_int), ("pro_scale", _c_p), ("pro_shift", _c_p), ("ld_pro", _c_int),
        ("drop_seed", _c_u32), ("drop_thresh", _c_u32), ("drop_scale", _c_f), ("drop_ld", _c_int),
        ("drop_seed_base", _c_p),
        ("bias", _c_p), ("addvec", _c_p), ("ld_add", _c_int), ("resid", _c_p), ("ld_res", _c_int),
        ("silu_pre", _c_p), ("ld_silu", _c_int), ("Csplit", _c_int), ("ldy1", _c_int), ("ldy2", _c_int),
        ("out_f32", _c_int), ("out_nchw", _c_int), ("act", _c_int), ("y_pre", _c_p), ("ld_pre", _c_int),
        ("gn_part", _c_p), ("wg_bias", _c_p), ("pro_groups", _c_int), ("pro_eps", _c_f),
    ]


class WgradJob(ctypes.Structure):
    """include/dmc.h dmc_wgrad_job"""
    _fields_ = [("slab", ctypes.c_void_p), ("bslab", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("dbias", ctypes.c_void_p), ("splits", ctypes.c_int), ("KK", ctypes.c_int), ("Cpad", ctypes.c_int),
                ("Cout", ctypes.c_int), ("Ctot", ctypes.c_int), ("ntaps", ctypes.c_int), ("Kc", ctypes.c_int),
                ("scale", ctypes.c_float), ("layout", ctypes.c_int)]


class ColsumJob(ctypes.Structure):
    """include/dmc.h dmc_colsum_job"""
    _fields_ = [("in_", ctypes.c_void_p), ("R", ctypes.c_int), ("C", ctypes.c_int), ("ld", ctypes.c_long),
                ("stride", ctypes.c_int), ("out0", ctypes.c_void_p), ("out1", ctypes.c_void_p),
                ("scale", ctypes.c_float)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", _c_p), ("dst", _c_p), ("dtype", _c_int), ("mode", _c_int), ("Cout", _c_int), ("Cin", _c_int),
                ("kh", _c_int), ("kw", _c_int), ("Kc", _c_int), ("koff", _c_int)]


class TensorRef(ctypes.Structure):
    _fields_ = [("a", _c_p), ("b", _c_p), ("n", _c_long)]


def _load():
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"libdmc.so not found at {LIB_PATH}. Build it with `python -m diffusion_models_collection_amd.build` "
            "(there is no fallback: the diffusion hot path runs only on the gfx950 HIP kernels).")
    lib = ctypes.CDLL(str(LIB_PATH))
    sig = {
        "dmc_version": (_c_int, []),
        "dmc_set_option": (_c_int, [ctypes.c_char_p, _c_long]),
        "dmc_get_option": (_c_long, [ctypes.c_char_p]),
        "dmc_reset_options": (None, [_c_int]),
        "dmc_last_error": (ctypes.c_char_p, []),
        "dmc_conv2d_workspace": (_c_size, [ctypes.POINTER(ConvDesc)]),
        "dmc_conv_halo_prologue": (_c_int, [ctypes.POINTER(ConvDesc)]),
        "dmc_conv2d_fused_epilogue": (_c_int, [ctypes.POINTER(ConvDesc), ctypes.c_size_t]),
        "dmc_conv2d": (_c_int, [ctypes.POINTER(ConvDesc), _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_size, _c_p]),
        "dmc_conv2d_wgrad_workspace": (_c_size, [ctypes.POINTER(ConvDesc)]),
        "dmc_conv2d_wgrad": (_c_int, [ctypes.POINTER(ConvDesc), _c_p, _c_int, _c_p, _c_p, _c_p, _c_p, _c_f, _c_p]),
        "dmc_conv2d_wgrad_partial": (_c_int, [ctypes.POINTER(ConvDesc), _c_p, _c_int, _c_p, _c_p, _c_p, _c_p, _c_f,
                                              ctypes.POINTER(WgradJob), _c_p]),
        "dmc_wgrad_reduce_batch": (_c_int, [ctypes.POINTER(WgradJob), _c_int, _c_p]),
        "dmc_pack_weight": (_c_int, [_c_int, _c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p]),
        "dmc_pack_tiles": (_c_int, [ctypes.POINTER(PackJob), _c_int, _c_p, _c_int]),
        "dmc_pack_weights": (_c_int, [_c_p, _c_p, _c_int, _c_p]),
        "dmc_gn_workspace": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
        "dmc_gn_stats": (_c_int, [_c_int, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_f,
                                  _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
        "dmc_gn_finalize": (_c_int, [_c_p, _c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_f, _c_p, _c_p, _c_p, _c_p,
                                     _c_p, _c_p]),
        "dmc_gn_stats_apply_ok": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int]),
        "dmc_gn_stats_apply": (_c_int, [_c_int, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                        _c_f, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_u32, _c_p, _c_u32, _c_f, _c_p,
                                        _c_int, _c_p]),
        "dmc_gn_apply": (_c_int, [_c_int, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p,
                                  _c_int, _c_u32, _c_p, _c_u32, _c_f, _c_p, _c_int, _c_p]),
        "dmc_gn_silu_bwd": (_c_int, [_c_int, _c_p, _c_int, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int,
                                     _c_int, _c_int, _c_p, _c_p, _c_p, _c_int, _c_u32, _c_p, _c_u32, _c_f, _c_p, _c_p,
                                     _c_int, _c_int, _c_int, _c_int, _c_p, _c_p, _c_p, _c_int, _c_p, _c_p, _c_p,
                                     _c_p]),
        "dmc_gn_silu_bwd_deferred": (_c_int, [_c_int, _c_p, _c_int, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int,
                                              _c_int, _c_int, _c_int, _c_p, _c_p, _c_p, _c_int, _c_u32, _c_p, _c_u32,
                                              _c_f, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p, _c_p,
                                              _c_int, _c_p, _c_p, _c_p, _c_p, _c_p, ctypes.POINTER(ctypes.c_int),
                                              _c_p, _c_int, _c_p]),
        "dmc_colsum_batch": (_c_int, [ctypes.POINTER(ColsumJob), _c_int, _c_p]),
        "dmc_channel_sum_workspace": (_c_size, [_c_int, _c_int, _c_int]),
        "dmc_channel_sum": (_c_int, [_c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_p, _c_int, _c_p, _c_f, _c_p,
                                     _c_p]),
        "dmc_attn_fwd": (_c_int, [_c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_int, _c_p, _c_u32,
                                  _c_p, _c_u32, _c_f, _c_p]),
        "dmc_attn_workspace": (_c_size, [_c_int, _c_int, _c_int]),
        "dmc_attn_bwd": (_c_int, [_c_int, _c_p, _c_int, _c_p, _c_p, _c_int, _c_p, _c_int, _c_int, _c_int, _c_int,
                                  _c_p, _c_int, _c_p, _c_u32, _c_p, _c_u32, _c_f, _c_p]),
        "dmc_time_embed": (_c_int, [_c_p, _c_int, _c_int, _c_p, _c_p]),
        "dmc_embed_fwd": (_c_int, [_c_p, _c_int, _c_int, _c_p, _c_int, _c_p, _c_p]),
        "dmc_embed_bwd": (_c_int, [_c_p, _c_int, _c_int, _c_p, _c_int, _c_p, _c_p]),
        "dmc_pack_input": (_c_int, [_c_int, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_p,
                                    _c_int, _c_p]),
        "dmc_q_sample": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_p, _c_p]),
        "dmc_loss_fwd": (_c_int, [_c_int, _c_p, _c_p, _c_long, _c_p, _c_p, _c_p]),
        "dmc_loss_bwd": (_c_int, [_c_int, _c_p, _c_p, _c_long, _c_p, _c_p, _c_p]),
        "dmc_ddim_step": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_f, _c_int, _c_p, _c_p,
                                   _c_p]),
        "dmc_ddpm_step": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_int,
                                   _c_p, _c_p, _c_p]),
        "dmc_cfg_x0": (_c_int, [_c_p, _c_p, _c_p, _c_f, _c_p, _c_p, _c_p, _c_int, _c_int, _c_int, _c_f, _c_p, _c_p,
                                _c_p]),
        "dmc_ema_update": (_c_int, [_c_p, _c_int, _c_f, _c_p]),
        "dmc_clip_grad_norm": (_c_int, [_c_p, _c_int, _c_f, _c_p, _c_p, _c_p]),
        "dmc_grad_norm_flat": (_c_int, [_c_p, _c_long, _c_f, _c_p, _c_p, _c_p, _c_p]),
        "dmc_adamw_flat": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_long, _c_p] + [_c_f] * 9 + [_c_p]),
        "dmc_adamw_flat_dev": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_long, _c_p, _c_p, _c_p]),
        "dmc_silu_fwd": (_c_int, [_c_p, _c_p, _c_long, _c_p]),
        "dmc_upsample2x_nhwc": (_c_int, [_c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_int, _c_p]),
        "dmc_unpack_output": (_c_int, [_c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p]),
        "dmc_add": (_c_int, [_c_int, _c_p, _c_p, _c_long, _c_p]),
        "dmc_ln_mod_fwd": (_c_int, [_c_int, _c_p, _c_p, _c_int, _c_p, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_f,
                                    _c_u32, _c_p, _c_u32, _c_f, _c_p, _c_p, _c_int, _c_p, _c_p, _c_p]),
        "dmc_ln_mod_bwd": (_c_int, [_c_int, _c_p, _c_int, _c_p, _c_p, _c_p, _c_p, _c_int, _c_int, _c_int, _c_int, _c_p,
                                    _c_p, _c_p, _c_p, _c_p]),
        "dmc_dit_rowsum_workspace": (_c_size, [_c_int, _c_int, _c_int]),
        "dmc_gate_bwd": (_c_int, [_c_int, _c_p, _c_p, _c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_u32, _c_p, _c_u32,
                                  _c_f, _c_p, _c_int, _c_p, _c_p, _c_p]),
        "dmc_gelu_fwd": (_c_int, [_c_int, _c_p, _c_long, _c_int, _c_int, _c_u32, _c_p, _c_u32, _c_f, _c_p, _c_p]),
        "dmc_gelu_bwd": (_c_int, [_c_int, _c_p, _c_p, _c_long, _c_int, _c_int, _c_u32, _c_p, _c_u32, _c_f, _c_p, _c_p]),
        "dmc_timestep_embedding": (_c_int, [_c_p, _c_int, _c_int, _c_f, _c_p, _c_p]),
        "dmc_unpatchify": (_c_int, [_c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p]),
        "dmc_patchify_grad": (_c_int, [_c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_int, _c_p]),
        "dmc_add_bcast": (_c_int, [_c_p, _c_p, _c_long, _c_long, _c_p]),
        "dmc_batch_sum": (_c_int, [_c_p, _c_long, _c_long, _c_p, _c_p]),
        "dmc_patch_dgrad": (_c_int, [_c_p, _c_int, _c_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_p, _c_p]),
        "dmc_load_batch": (_c_int, [_c_p, _c_long, _c_int, _c_int, _c_int, _c_p, _c_int, _c_p, _c_u32, _c_u32, _c_long,
                                    ctypes.POINTER(_c_f), ctypes.POINTER(_c_f), _c_p, _c_p, _c_p, _c_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib, list(sig)


LIB, EXPORTS = _load()


class DMCError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != 0:
        raise DMCError(f"{what} failed ({rc}): {LIB.dmc_last_error().decode()}")


def set_option(name: str, value) -> None:
    """Launch-plan A/B switch (include/dmc.h dmc_set_option), e.g. set_option("DMC_NO_HALO", 1)."""
    check(LIB.dmc_set_option(name.encode(), int(value)), "set_option")


def get_option(name: str) -> int:
    return LIB.dmc_get_option(name.encode())


def reset_options(from_env: bool = False) -> None:
    LIB.dmc_reset_options(1 if from_env else 0)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream():
    """Raw hipStream_t of torch's current stream on the current device (the direct C accessors: the
    torch.cuda.current_stream() object path costs several microseconds per kernel launch)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DMC_F32
    if dt == torch.bfloat16:
        return DMC_BF16
    raise DMCError(f"unsupported storage dtype {dt}")


def kc_for(cin: int, dt: torch.dtype) -> int:
    """Packed K per tap: channel count rounded up to the kernel stage depth (32 fp32 / 64 bf16)."""
    bk = 32 if dt == torch.float32 else 64
    return (cin + bk - 1) // bk * bk


def chunk_for(dt: torch.dtype) -> int:
    return 4 if dt == torch.float32 else 8
