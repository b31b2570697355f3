"""UNet epsilon-predictor with the reference's API and parameter layout, executed by gfx950 HIP kernels.

Drop-in for models/unet.py of sunyzhi55/Diffusion_Models_Collection:
  * same class names (TimeEmbedding :12, ResidualBlock :28, AttentionBlock :75, Downsample :102,
    Upsample :112, UNet :123), same constructor signatures (:139-151) and the same nn.Module tree, so the
    parameter initialisation (under the same torch seed) and every state_dict key/shape are identical and
    checkpoints interchange both ways;
  * UNet.forward(x[B,C,H,W] f32, t[B] i64, y[B] i64 | None) -> eps[B,C_out,H,W] f32 (:243-292).

The nn.Modules here are parameter containers: their arithmetic is never run through PyTorch ops. The
whole network (forward and backward) is executed by `_unet_exec.UNetExecutor`, which drives the HIP
kernels of libdmc.so over NHWC activations (bf16 or fp32 storage, fp32 accumulation). Calling a
sub-module's forward directly raises.

Extra (optional) constructor argument: compute_dtype = "fp32" | "bf16" (default: env DMC_COMPUTE_DTYPE or
"fp32"). fp32 reproduces the reference within fp32 tolerance; bf16 is the mixed-precision perf mode
(bf16 activations/weights on the MFMA path, fp32 master weights, statistics and accumulation).
"""
import math
import os
from typing import Tuple

import torch
import torch.nn as nn


class _KernelOnly:
    def forward(self, *args, **kwargs):
        raise RuntimeError(f"{type(self).__name__} is executed by the UNet HIP executor; call UNet.forward")


class TimeEmbedding(_KernelOnly, nn.Module):
    """Sinusoidal time embedding (models/unet.py:12-25); computed by dmc_time_embed."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class ResidualBlock(_KernelOnly, nn.Module):
    """GN-SiLU-Conv3x3 (+time/label embedding) -> GN-SiLU-Dropout-Conv3x3 + shortcut (models/unet.py:28-72)."""

    def __init__(self, in_channels, out_channels, time_emb_dim, num_classes=None, dropout=0.1):
        super().__init__()
        self.num_classes = num_classes
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.dropout_p = dropout
        self.conv1 = nn.Sequential(nn.GroupNorm(8, in_channels), nn.SiLU(),
                                   nn.Conv2d(in_channels, out_channels, 3, padding=1))
        self.time_mlp = nn.Sequential(nn.SiLU(), nn.Linear(time_emb_dim, out_channels))
        self.label_proj = nn.Sequential(
            nn.SiLU(), nn.Linear(time_emb_dim, out_channels, bias=False)) if num_classes is not None else None
        self.conv2 = nn.Sequential(nn.GroupNorm(8, out_channels), nn.SiLU(), nn.Dropout(dropout),
                                   nn.Conv2d(out_channels, out_channels, 3, padding=1))
        if in_channels != out_channels:
            self.shortcut = nn.Conv2d(in_channels, out_channels, 1)
        else:
            self.shortcut = nn.Identity()


class AttentionBlock(_KernelOnly, nn.Module):
    """GN -> 1x1 qkv -> softmax(QK^T/sqrt(hd))V -> 1x1 proj -> +x (models/unet.py:75-99)."""

    def __init__(self, channels, num_heads=4):
        super().__init__()
        self.num_heads = num_heads
        self.norm = nn.GroupNorm(8, channels)
        self.qkv = nn.Conv2d(channels, channels * 3, 1)
        self.proj = nn.Conv2d(channels, channels, 1)


class Downsample(_KernelOnly, nn.Module):
    """3x3 stride-2 conv (models/unet.py:102-109)."""

    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=1)


class Upsample(_KernelOnly, nn.Module):
    """nearest x2 + 3x3 conv (models/unet.py:112-120); the upsample is folded into the conv's input indexing."""

    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)


def _resolve_dtype(compute_dtype):
    cd = compute_dtype or os.environ.get("DMC_COMPUTE_DTYPE", "fp32")
    cd = str(cd).lower()
    if cd in ("fp32", "float32", "f32"):
        return torch.float32
    if cd in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError(f"compute_dtype must be 'fp32' or 'bf16', got {compute_dtype!r}")


class UNet(nn.Module):
    """UNet model for diffusion (models/unet.py:123-292); same arguments as the reference."""

    def __init__(
        self,
        image_size: Tuple[int, int] = (32, 32),
        in_channels=3,
        model_channels=128,
        out_channels=3,
        num_res_blocks=2,
        attention_resolutions=(16, 8),
        dropout=0.1,
        channel_mult=(1, 2, 2, 2),
        num_classes=None,
        use_attention=True,
        compute_dtype=None,
    ):
        super().__init__()
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = attention_resolutions
        self.dropout = dropout
        self.channel_mult = channel_mult
        self.num_classes = num_classes
        self.use_attention = use_attention
        self.compute_dtype = _resolve_dtype(compute_dtype)

        time_emb_dim = model_channels * 4
        self.time_embed = nn.Sequential(
            TimeEmbedding(model_channels),
            nn.Linear(model_channels, time_emb_dim),
            nn.SiLU(),
            nn.Linear(time_emb_dim, time_emb_dim),
        )
        if num_classes is not None:
            self.label_embed = nn.Embedding(num_embeddings=num_classes + 1, embedding_dim=time_emb_dim, padding_idx=0)
        else:
            self.label_embed = None

        self.input_conv = nn.Conv2d(in_channels, model_channels, 3, padding=1)

        # identical construction order to the reference (parameter init consumes the RNG in this order)
        self.down_blocks = nn.ModuleList()
        ch = model_channels
        input_block_channels = [ch]
        resolution = list(image_size)
        for level, mult in enumerate(channel_mult):
            out_ch = model_channels * mult
            for _ in range(num_res_blocks):
                layers = [ResidualBlock(ch, out_ch, time_emb_dim, num_classes, dropout)]
                ch = out_ch
                if use_attention and (resolution[0] in attention_resolutions or resolution[1] in attention_resolutions):
                    layers.append(AttentionBlock(ch))
                self.down_blocks.append(nn.ModuleList(layers))
                input_block_channels.append(ch)
            if level != len(channel_mult) - 1:
                self.down_blocks.append(nn.ModuleList([Downsample(ch)]))
                input_block_channels.append(ch)
                resolution[0] //= 2
                resolution[1] //= 2

        self.middle_block = nn.ModuleList([
            ResidualBlock(ch, ch, time_emb_dim, num_classes, dropout),
            AttentionBlock(ch) if use_attention else nn.Identity(),
            ResidualBlock(ch, ch, time_emb_dim, num_classes, dropout),
        ])

        self.up_blocks = nn.ModuleList()
        for level, mult in enumerate(reversed(channel_mult)):
            for i in range(num_res_blocks + 1):
                ich = input_block_channels.pop()
                layers = [ResidualBlock(ch + ich, model_channels * mult, time_emb_dim, num_classes, dropout)]
                ch = model_channels * mult
                if use_attention and (resolution[0] in attention_resolutions or resolution[1] in attention_resolutions):
                    layers.append(AttentionBlock(ch))
                if level != len(channel_mult) - 1 and i == num_res_blocks:
                    layers.append(Upsample(ch))
                    resolution[0] *= 2
                    resolution[1] *= 2
                self.up_blocks.append(nn.ModuleList(layers))

        self.output = nn.Sequential(nn.GroupNorm(8, ch), nn.SiLU(), nn.Conv2d(ch, out_channels, 3, padding=1))
        self._executor = None

    # ------------------------------------------------------------------------------------------
    @property
    def executor(self):
        if self._executor is None:
            from ._unet_exec import UNetExecutor
            self._executor = UNetExecutor(self)
        return self._executor

    def set_compute_dtype(self, compute_dtype):
        self.compute_dtype = _resolve_dtype(compute_dtype)
        self._executor = None
        return self

    # Inference with one timestep for the whole batch may pass t of shape (1,) (the reference's broadcasting of
    # time_mlp(emb)[:, :, None, None] gives the same result): the time-embedding MLPs then run on one row, broadcast
    # by the convs' epilogues. Not with class labels, not with autograd. The samplers use it when this is set.
    shared_timestep = True

    def forward(self, x, t, y=None):
        """x: (B, C, H, W) f32, t: (B,) i64 (or (1,), see shared_timestep), y: (B,) i64 class labels or None ->
        eps (B, C_out, H, W) f32."""
        if not x.is_cuda:
            raise RuntimeError("UNet runs on the MI355X HIP kernels only: move the model and inputs to a cuda device")
        return self.executor.run(x, t, y if self.num_classes is not None else None)

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_executor"] = None
        return st


def unet_flops_per_image(model: UNet) -> float:
    """Analytic forward FLOPs per image (2*MACs of convs/linears/attention bmm), for roofline reporting."""
    from ._unet_exec import count_forward_flops
    return count_forward_flops(model)


__all__ = ["TimeEmbedding", "ResidualBlock", "AttentionBlock", "Downsample", "Upsample", "UNet", "math"]
