"""DiT (Diffusion Transformer) with the reference's API and parameter layout, executed by gfx950 HIP kernels.

Drop-in for models/dit.py of sunyzhi55/Diffusion_Models_Collection:
  * same classes (PatchEmbed :12, TimestepEmbedder :30, LabelEmbedder :58, DiTBlock :87, FinalLayer :135,
    DiT :154), same constructor signatures and the same nn.Module tree (nn.MultiheadAttention included), built in
    the same order and re-initialised by the same initialize_weights (:220-240), so under the same torch seed the
    parameters, every state_dict key and shape are identical and checkpoints interchange both ways;
  * DiT.forward(x[B,C,H,W] f32, t[B] i64, y[B] i64 | None) -> [B,C,H,W] f32 (:263-295).

The modules are parameter containers; the arithmetic is `_dit_exec.DiTExecutor` on libdmc.so: the patch
embedding, the attention in/out projections, the MLP and every block's adaLN modulation (all twelve plus the final
layer's stacked into one GEMM) on the implicit-GEMM kernels, the attention on the flash-attention kernels, and the
gated residuals + LayerNorm + modulation, GELU, timestep embedding and unpatchify in fused token-wise kernels.

Extra (optional) constructor argument: compute_dtype = "fp32" | "bf16" (as models/unet.py).
Dropout in training mode: the attention-probability dropout of nn.MultiheadAttention (inside the flash-attention
kernels, dmc_attn_fwd/bwd) and the two MLP dropouts (in the GELU and gated-residual kernels), each with a counter-hash
mask recomputed in the backward; the masks are not torch's RNG stream (statistically equivalent, not bitwise).
"""
import math
from typing import Tuple

import torch
import torch.nn as nn

from .unet import _resolve_dtype


class _KernelOnly:
    def forward(self, *args, **kwargs):
        raise RuntimeError(f"{type(self).__name__} is executed by the DiT HIP executor; call DiT.forward")


class PatchEmbed(_KernelOnly, nn.Module):
    """Image to patch embedding (dit.py:12-27): Conv2d(k=p, s=p)."""

    def __init__(self, img_size: Tuple[int, int] = (32, 32), patch_size=2, in_channels=3, embed_dim=768):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch_size
        self.h_tokens = img_size[0] // patch_size
        self.w_tokens = img_size[1] // patch_size
        self.num_patches = self.h_tokens * self.w_tokens
        self.proj = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)


class TimestepEmbedder(_KernelOnly, nn.Module):
    """Sinusoid [cos | sin] -> Linear -> SiLU -> Linear (dit.py:30-55)."""

    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(
            nn.Linear(frequency_embedding_size, hidden_size, bias=True),
            nn.SiLU(),
            nn.Linear(hidden_size, hidden_size, bias=True)
        )
        self.frequency_embedding_size = frequency_embedding_size


class LabelEmbedder(_KernelOnly, nn.Module):
    """Embedding(num_classes + 1, hidden, padding_idx=0), index 0 = null label (dit.py:58-84)."""

    def __init__(self, num_classes, hidden_size, dropout_prob=0.1):
        super().__init__()
        self.embedding_table = nn.Embedding(num_classes + 1, hidden_size, padding_idx=0)


class DiTBlock(_KernelOnly, nn.Module):
    """adaLN-zero transformer block (dit.py:87-132)."""

    def __init__(self, hidden_size, num_heads, mlp_ratio=4.0, dropout=0.1):
        super().__init__()
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.attn = nn.MultiheadAttention(hidden_size, num_heads, dropout=dropout, batch_first=True)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        mlp_hidden_dim = int(hidden_size * mlp_ratio)
        self.mlp = nn.Sequential(
            nn.Linear(hidden_size, mlp_hidden_dim),
            nn.GELU(),
            nn.Dropout(dropout),
            nn.Linear(mlp_hidden_dim, hidden_size),
            nn.Dropout(dropout)
        )
        self.adaLN_modulation = nn.Sequential(
            nn.SiLU(),
            nn.Linear(hidden_size, 6 * hidden_size, bias=True)
        )


class FinalLayer(_KernelOnly, nn.Module):
    """LayerNorm + modulation -> Linear(hidden, p*p*C) (dit.py:135-151)."""

    def __init__(self, hidden_size, patch_size, out_channels):
        super().__init__()
        self.norm_final = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.linear = nn.Linear(hidden_size, patch_size * patch_size * out_channels, bias=True)
        self.adaLN_modulation = nn.Sequential(
            nn.SiLU(),
            nn.Linear(hidden_size, 2 * hidden_size, bias=True)
        )


class DiT(nn.Module):
    """Diffusion Transformer (dit.py:154-295); same arguments as the reference."""

    def __init__(
        self,
        img_size: Tuple[int, int] = (32, 32),
        patch_size=2,
        in_channels=3,
        hidden_size=768,
        depth=12,
        num_heads=12,
        mlp_ratio=4.0,
        num_classes=None,
        dropout=0.1,
        compute_dtype=None,
    ):
        super().__init__()
        if isinstance(img_size, int):
            img_h = img_w = img_size
        else:
            img_h, img_w = img_size
        self.img_size = (img_h, img_w)
        self.patch_size = patch_size
        self.in_channels = in_channels
        self.out_channels = in_channels
        self.hidden_size = hidden_size
        self.num_heads = num_heads
        self.num_classes = num_classes
        self.dropout = dropout
        self.mlp_ratio = mlp_ratio
        self.compute_dtype = _resolve_dtype(compute_dtype)

        self.x_embedder = PatchEmbed(img_size, patch_size, in_channels, hidden_size)
        num_patches = self.x_embedder.num_patches
        self.h_tokens = self.x_embedder.h_tokens
        self.w_tokens = self.x_embedder.w_tokens
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches, hidden_size))
        self.t_embedder = TimestepEmbedder(hidden_size)
        if num_classes is not None:
            self.y_embedder = LabelEmbedder(num_classes, hidden_size, dropout_prob=0.0)
        else:
            self.y_embedder = None
        self.blocks = nn.ModuleList([
            DiTBlock(hidden_size, num_heads, mlp_ratio, dropout)
            for _ in range(depth)
        ])
        self.final_layer = FinalLayer(hidden_size, patch_size, self.out_channels)
        self.initialize_weights()
        self._executor = None

    def initialize_weights(self):
        # the reference's initialisation order (dit.py:220-240): xavier on every nn.Linear (post-order module
        # walk), pos_embed ~ N(0, 0.02), adaLN and the final projection zeroed
        def _basic_init(module):
            if isinstance(module, nn.Linear):
                torch.nn.init.xavier_uniform_(module.weight)
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0)
        self.apply(_basic_init)
        nn.init.normal_(self.pos_embed, std=0.02)
        for block in self.blocks:
            nn.init.constant_(block.adaLN_modulation[-1].weight, 0)
            nn.init.constant_(block.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.final_layer.adaLN_modulation[-1].weight, 0)
        nn.init.constant_(self.final_layer.adaLN_modulation[-1].bias, 0)
        nn.init.constant_(self.final_layer.linear.weight, 0)
        nn.init.constant_(self.final_layer.linear.bias, 0)

    @property
    def executor(self):
        if self._executor is None:
            from ._dit_exec import DiTExecutor
            self._executor = DiTExecutor(self)
        return self._executor

    def set_compute_dtype(self, compute_dtype):
        self.compute_dtype = _resolve_dtype(compute_dtype)
        self._executor = None

    def unpatchify(self, x):
        """(B, N, p*p*C) -> (B, C, H, W) (dit.py:248-261), on the device kernel."""
        from .. import kernels as K
        B = x.shape[0]
        p, h, w, C = self.patch_size, self.h_tokens, self.w_tokens, self.out_channels
        out = torch.empty(B, C, h * p, w * p, dtype=torch.float32, device=x.device)
        K.unpatchify(x.contiguous().float(), p * p * C, B, h, w, p, C, out)
        return out

    def forward(self, x, t, y=None):
        if not x.is_cuda:
            raise RuntimeError("DiT runs on the MI355X HIP kernels only: move the model and inputs to a cuda device")
        return self.executor.run(x, t, y if self.num_classes is not None else None)

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_executor"] = None
        return st
