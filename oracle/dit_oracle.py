"""CPU ORACLE — test infrastructure only. Never imported by the product path.

A from-scratch, functional fp32 restatement of the reference DiT forward (models/dit.py of
sunyzhi55/Diffusion_Models_Collection) over a state_dict, on plain PyTorch CPU ops (autograd supplies the
backward). Only tests/ and bench.py's cpu_baseline leg use it, as the checker and as a timed CPU baseline.

Pinned: tests/test_oracle.py checks it against the golden fixtures tests/golden/gen_golden.py produced by running
the reference DiT itself (dit_tiny_*.npz: forward outputs and every gradient; dit_s2.npz: the DiT-S/2 shape of
BASELINE config #4, output, grad_x and per-parameter gradient summaries).
"""
import math

import torch
import torch.nn.functional as F


def timestep_embedding(t, dim, max_period=10000):
    """models/dit.py:38-50: freqs = exp(-ln(max_period) * k / half), [cos(t f) | sin(t f)] (+ a zero column when
    dim is odd)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


class OracleDiT:
    """Walks the reference DiT by state_dict keys (models/dit.py:154-295)."""

    def __init__(self, sd, img_size=(32, 32), patch_size=2, in_channels=3, hidden_size=768, depth=12, num_heads=12,
                 mlp_ratio=4.0, num_classes=None, dropout=0.1):
        self.sd = sd
        if isinstance(img_size, int):
            img_size = (img_size, img_size)
        self.p = patch_size
        self.C = in_channels
        self.H = hidden_size
        self.depth = depth
        self.heads = num_heads
        self.num_classes = num_classes
        self.ht, self.wt = img_size[0] // patch_size, img_size[1] // patch_size

    def w(self, k):
        return self.sd[k]

    def mha(self, pre, h):
        """nn.MultiheadAttention(batch_first=True) self-attention, eval semantics: in_proj rows [q | k | v], heads
        split as [head][hd], softmax(q k^T / sqrt(hd)) v, out_proj."""
        B, L, H = h.shape
        hd = H // self.heads
        qkv = F.linear(h, self.w(pre + "in_proj_weight"), self.w(pre + "in_proj_bias"))
        q, k, v = qkv.split(H, dim=-1)
        q, k, v = (z.reshape(B, L, self.heads, hd).transpose(1, 2) for z in (q, k, v))
        a = torch.softmax((q @ k.transpose(-2, -1)) / math.sqrt(hd), dim=-1)
        o = (a @ v).transpose(1, 2).reshape(B, L, H)
        return F.linear(o, self.w(pre + "out_proj.weight"), self.w(pre + "out_proj.bias"))

    def block(self, i, x, c):
        """models/dit.py:111-132."""
        pre = f"blocks.{i}."
        mod = F.linear(F.silu(c), self.w(pre + "adaLN_modulation.1.weight"), self.w(pre + "adaLN_modulation.1.bias"))
        sh1, sc1, g1, sh2, sc2, g2 = mod.chunk(6, dim=-1)
        h = F.layer_norm(x, (self.H,), eps=1e-6)
        h = h * (1 + sc1[:, None]) + sh1[:, None]
        x = x + g1[:, None] * self.mha(pre + "attn.", h)
        h = F.layer_norm(x, (self.H,), eps=1e-6)
        h = h * (1 + sc2[:, None]) + sh2[:, None]
        h = F.linear(h, self.w(pre + "mlp.0.weight"), self.w(pre + "mlp.0.bias"))
        h = F.gelu(h)
        h = F.linear(h, self.w(pre + "mlp.3.weight"), self.w(pre + "mlp.3.bias"))
        return x + g2[:, None] * h

    def forward(self, x, t, y=None):
        """models/dit.py:263-295."""
        B = x.shape[0]
        p, C = self.p, self.C
        h = F.conv2d(x, self.w("x_embedder.proj.weight"), self.w("x_embedder.proj.bias"), stride=p)
        h = h.flatten(2).transpose(1, 2) + self.w("pos_embed")
        te = timestep_embedding(t, self.w("t_embedder.mlp.0.weight").shape[1])
        te = F.linear(te, self.w("t_embedder.mlp.0.weight"), self.w("t_embedder.mlp.0.bias"))
        c = F.linear(F.silu(te), self.w("t_embedder.mlp.2.weight"), self.w("t_embedder.mlp.2.bias"))
        if self.num_classes is not None and y is not None:
            c = c + F.embedding(torch.clamp(y, 0, self.num_classes), self.w("y_embedder.embedding_table.weight"),
                                padding_idx=0)
        for i in range(self.depth):
            h = self.block(i, h, c)
        mod = F.linear(F.silu(c), self.w("final_layer.adaLN_modulation.1.weight"),
                       self.w("final_layer.adaLN_modulation.1.bias"))
        shift, scale = mod.chunk(2, dim=-1)
        h = F.layer_norm(h, (self.H,), eps=1e-6) * (1 + scale[:, None]) + shift[:, None]
        h = F.linear(h, self.w("final_layer.linear.weight"), self.w("final_layer.linear.bias"))
        h = h.reshape(B, self.ht, self.wt, p, p, C)
        return torch.einsum("nhwpqc->nchpwq", h).reshape(B, C, self.ht * p, self.wt * p)


def make_oracle(state_dict, cfg, requires_grad=False):
    sd = {k: v.detach().float().cpu().clone().requires_grad_(requires_grad) for k, v in state_dict.items()}
    return OracleDiT(sd, **cfg), sd
