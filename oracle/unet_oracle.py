"""CPU ORACLE — test infrastructure only. Never imported by the product path.

A from-scratch, functional fp32 restatement of the reference UNet forward (models/unet.py of
sunyzhi55/Diffusion_Models_Collection) over a state_dict, on plain PyTorch CPU ops (autograd supplies the
backward). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker
and as the timed CPU baseline ("kind": "port").

Pinned: tests/test_oracle.py checks it against the golden fixtures in tests/golden/ that
tests/golden/gen_golden.py produced by running the reference itself (forward outputs, and the gradients of
every parameter and of the input).
"""
import math

import torch
import torch.nn.functional as F


def time_embedding(t, dim):
    """models/unet.py:18-25: exp(-i*ln(1e4)/(half-1)), args = t*f, cat(sin, cos)."""
    half = dim // 2
    step = math.log(10000) / (half - 1)
    freqs = torch.exp(torch.arange(half, device=t.device) * -step)
    args = t[:, None] * freqs[None, :]
    return torch.cat((args.sin(), args.cos()), dim=-1)


class OracleUNet:
    """Walks the reference module tree by state_dict key prefixes (models/unet.py:139-241 structure)."""

    def __init__(self, sd, image_size=(32, 32), in_channels=3, model_channels=128, out_channels=3,
                 num_res_blocks=2, attention_resolutions=(16, 8), dropout=0.1, channel_mult=(1, 2, 2, 2),
                 num_classes=None, use_attention=True):
        self.sd = sd
        self.mc = model_channels
        self.num_classes = num_classes
        self.dropout = dropout
        # rebuild the layer plan exactly as models/unet.py:186-235 does
        plan_down = []
        ch = model_channels
        ibc = [ch]
        res = list(image_size)
        for level, mult in enumerate(channel_mult):
            oc = model_channels * mult
            for _ in range(num_res_blocks):
                layers = [("res", ch, oc)]
                ch = oc
                if use_attention and (res[0] in attention_resolutions or res[1] in attention_resolutions):
                    layers.append(("attn", ch))
                plan_down.append(layers)
                ibc.append(ch)
            if level != len(channel_mult) - 1:
                plan_down.append([("down", ch)])
                ibc.append(ch)
                res = [res[0] // 2, res[1] // 2]
        plan_mid = [("res", ch, ch), ("attn", ch) if use_attention else ("id",), ("res", ch, ch)]
        plan_up = []
        for level, mult in enumerate(reversed(channel_mult)):
            for i in range(num_res_blocks + 1):
                ich = ibc.pop()
                layers = [("res", ch + ich, model_channels * mult)]
                ch = model_channels * mult
                if use_attention and (res[0] in attention_resolutions or res[1] in attention_resolutions):
                    layers.append(("attn", ch))
                if level != len(channel_mult) - 1 and i == num_res_blocks:
                    layers.append(("up", ch))
                    res = [res[0] * 2, res[1] * 2]
                plan_up.append(layers)
        self.plan_down, self.plan_mid, self.plan_up = plan_down, plan_mid, plan_up

    def p(self, name):
        return self.sd[name]

    def res_block(self, pre, x, temb, yemb, training):
        """models/unet.py:62-72."""
        h = F.silu(F.group_norm(x, 8, self.p(pre + "conv1.0.weight"), self.p(pre + "conv1.0.bias"), 1e-5))
        h = F.conv2d(h, self.p(pre + "conv1.2.weight"), self.p(pre + "conv1.2.bias"), padding=1)
        h = h + F.linear(F.silu(temb), self.p(pre + "time_mlp.1.weight"), self.p(pre + "time_mlp.1.bias"))[:, :, None,
                                                                                                             None]
        if yemb is not None and (pre + "label_proj.1.weight") in self.sd:
            h = h + F.linear(F.silu(yemb), self.p(pre + "label_proj.1.weight"))[:, :, None, None]
        h = F.silu(F.group_norm(h, 8, self.p(pre + "conv2.0.weight"), self.p(pre + "conv2.0.bias"), 1e-5))
        h = F.dropout(h, self.dropout, training)
        h = F.conv2d(h, self.p(pre + "conv2.3.weight"), self.p(pre + "conv2.3.bias"), padding=1)
        if (pre + "shortcut.weight") in self.sd:
            x = F.conv2d(x, self.p(pre + "shortcut.weight"), self.p(pre + "shortcut.bias"))
        return h + x

    def attn_block(self, pre, x, heads=4):
        """models/unet.py:84-99: channel index = which*C + head*hd + d."""
        B, C, H, W = x.shape
        hd = C // heads
        h = F.group_norm(x, 8, self.p(pre + "norm.weight"), self.p(pre + "norm.bias"), 1e-5)
        qkv = F.conv2d(h, self.p(pre + "qkv.weight"), self.p(pre + "qkv.bias"))
        qkv = qkv.reshape(B, 3, heads, hd, H * W).permute(1, 0, 2, 4, 3)
        q, k, v = qkv[0], qkv[1], qkv[2]
        a = torch.softmax(q @ k.transpose(-2, -1) / math.sqrt(hd), dim=-1)
        o = (a @ v).permute(0, 1, 3, 2).reshape(B, C, H, W)
        return x + F.conv2d(o, self.p(pre + "proj.weight"), self.p(pre + "proj.bias"))

    def layer(self, pre, spec, h, temb, yemb, training):
        kind = spec[0]
        if kind == "res":
            return self.res_block(pre, h, temb, yemb, training)
        if kind == "attn":
            return self.attn_block(pre, h)
        if kind == "down":   # models/unet.py:102-109
            return F.conv2d(h, self.p(pre + "conv.weight"), self.p(pre + "conv.bias"), stride=2, padding=1)
        if kind == "up":     # models/unet.py:112-120
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            return F.conv2d(h, self.p(pre + "conv.weight"), self.p(pre + "conv.bias"), padding=1)
        return h

    def forward(self, x, t, y=None, training=False):
        """models/unet.py:243-292."""
        e = time_embedding(t, self.mc)
        e = F.linear(e, self.p("time_embed.1.weight"), self.p("time_embed.1.bias"))
        temb = F.linear(F.silu(e), self.p("time_embed.3.weight"), self.p("time_embed.3.bias"))
        yemb = None
        if self.num_classes is not None and y is not None:
            yemb = F.embedding(torch.clamp(y, 0, self.num_classes), self.p("label_embed.weight"), padding_idx=0)
        h = F.conv2d(x, self.p("input_conv.weight"), self.p("input_conv.bias"), padding=1)
        hs = [h]
        for bi, layers in enumerate(self.plan_down):
            for li, spec in enumerate(layers):
                h = self.layer(f"down_blocks.{bi}.{li}.", spec, h, temb, yemb, training)
            hs.append(h)
        for li, spec in enumerate(self.plan_mid):
            h = self.layer(f"middle_block.{li}.", spec, h, temb, yemb, training)
        for bi, layers in enumerate(self.plan_up):
            h = torch.cat([h, hs.pop()], dim=1)
            for li, spec in enumerate(layers):
                h = self.layer(f"up_blocks.{bi}.{li}.", spec, h, temb, yemb, training)
        h = F.silu(F.group_norm(h, 8, self.p("output.0.weight"), self.p("output.0.bias"), 1e-5))
        return F.conv2d(h, self.p("output.2.weight"), self.p("output.2.bias"), padding=1)


def make_oracle(state_dict, cfg, requires_grad=False):
    sd = {k: v.detach().float().cpu().clone().requires_grad_(requires_grad) for k, v in state_dict.items()}
    return OracleUNet(sd, **cfg), sd
