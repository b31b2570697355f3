"""Executor of the DiT (models/dit.py of the reference, :87-295) on the gfx950 kernels, forward + backward.

Token rows [T = B * L, C] are the NHWC pixels of a [B, h_tokens, w_tokens, C] grid, so every Linear is a 1x1
implicit-GEMM conv (dmc_conv2d, MFMA) and the patch embedding the 2x2 stride-2 conv. Per forward:

  timestep embedding [cos|sin] -> Linear -> SiLU -> Linear (+ label embedding)            = c  [B, H]
  ONE GEMM for every block's adaLN_modulation and the final layer's (weights stacked)    = mod [B, 12*6H + 2H]
  patch conv (fp32) + pos_embed                                                          = x   (fp32 stream)
  per block:  h1 = LN(x) * (1 + scale_msa) + shift_msa            (dmc_ln_mod_fwd, fused with the previous
                                                                   block's gated MLP residual)
              qkv = h1 W_in^T + b -> flash attention (probability dropout in training) -> o W_out^T + b = ao
              x_mid = x + gate_msa * ao;  h2 = LN(x_mid) * (1 + scale_mlp) + shift_mlp   (one fused kernel)
              u = h2 W1^T + b1 -> a = Dropout(GELU(u)) -> mo = a W2^T + b2   (x_out = x_mid + gate_mlp * drop(mo)
                                                                              folded into the next LayerNorm)
  final: LN + modulation (fused with the last residual) -> Linear -> unpatchify (NCHW fp32)

The backward walks the tape in reverse with the same fused kernels (dmc_gate_bwd, dmc_ln_mod_bwd, dmc_gelu_bwd,
the conv dgrad/wgrad kernels, dmc_attn_bwd) and writes every parameter gradient into one flat fp32 buffer laid out
in the order the backward finishes them (data-parallel buckets, fused clip + AdamW + EMA: utils/trainer.py).
The residual stream stays fp32; GEMM operands are in the compute dtype (bf16 in perf mode).
"""
import math
import os

import torch

from .. import _lib as L
from .. import kernels as K
from ._unet_exec import Act, ExecCore, _PackCache, _seed_from_torch

# GELU + Dropout in fc1's epilogue (training with MLP dropout) and their backward in fc2's input-gradient epilogue
# (A/B: DMC_GELU_DROP_EPI=0 keeps dmc_gelu_fwd / dmc_gelu_bwd)
# measured slower on the DiT train step (erf/exp in the GEMM epilogue cost more than the separate HBM-bound pass:
# 6958 -> 6874 img/s forward, -> 6839 backward), so off by default
_GELU_EPI_BITS = int(os.environ.get("DMC_GELU_DROP_EPI", "0") or 0)   # bit 0: forward, bit 1: backward
# inference / dropout-free training: GELU in fc1's epilogue (DMC_GELU_EPI=0: conv + dmc_gelu_fwd, for A/B)
_GELU_EPI = os.environ.get("DMC_GELU_EPI", "1") not in ("", "0")
_GELU_DROP_EPI = bool(_GELU_EPI_BITS & 1)
_DGELU_EPI = bool(_GELU_EPI_BITS & 2)


class _W:
    """A weight holder for the pack cache (nn.MultiheadAttention keeps in_proj_weight as a bare Parameter)."""

    def __init__(self, weight):
        self.weight = weight


class DiTExecutor(ExecCore):
    def __init__(self, model):
        self._bind_model(model)
        self.dt = model.compute_dtype
        self.cdt = L.dtype_code(self.dt)
        self.chunk = L.chunk_for(self.dt)
        self.wgen = 0
        self.packs = _PackCache(self)
        self.params = list(model.parameters())
        self.pindex = {id(p): i for i, p in enumerate(self.params)}
        self.training_grad_scale = 1.0
        self.grad_hook = None
        self.seed_ptr = None
        H = model.hidden_size
        self.H = H
        self.blocks = list(model.blocks)
        self.in_proj = [_W(b.attn.in_proj_weight) for b in self.blocks]
        # stacked adaLN projections: block i's 6H rows at 6H*i, the final layer's 2H rows last
        self.ada = [b.adaLN_modulation[1] for b in self.blocks] + [model.final_layer.adaLN_modulation[1]]
        self.ada_off = [6 * H * i for i in range(len(self.blocks))] + [6 * H * len(self.blocks)]
        self.ada_total = 6 * H * len(self.blocks) + 2 * H
        p = model.patch_size
        if p * p > 16:
            raise L.DMCError(f"DiT: patch size {p} (the implicit-GEMM conv takes at most 16 taps)")
        self.patch_taps = [(i, j) for i in range(p) for j in range(p)]   # Conv2d(k=p, s=p) as p*p taps
        self._layout_grads()

    # ---------------------------------------------------------------------------------------
    def _block_params(self, b):
        return [b.mlp[3].weight, b.mlp[3].bias, b.mlp[0].weight, b.mlp[0].bias, b.attn.out_proj.weight,
                b.attn.out_proj.bias, b.attn.in_proj_weight, b.attn.in_proj_bias]

    def _layout_grads(self):
        """Flat gradient layout in backward-completion order: final linear, blocks last to first, pos_embed and
        the patch conv, the stacked adaLN weights and biases (rows in stacking order, so the stacked weight
        gradient lands in place), the timestep MLP, the label table."""
        m = self.m
        order = [m.final_layer.linear.weight, m.final_layer.linear.bias]
        for b in reversed(self.blocks):
            order += self._block_params(b)
        order += [m.pos_embed, m.x_embedder.proj.weight, m.x_embedder.proj.bias]
        order += [lin.weight for lin in self.ada] + [lin.bias for lin in self.ada]
        order += [m.t_embedder.mlp[2].weight, m.t_embedder.mlp[2].bias, m.t_embedder.mlp[0].weight,
                  m.t_embedder.mlp[0].bias]
        if m.y_embedder is not None:
            order.append(m.y_embedder.embedding_table.weight)
        assert len(order) == len(self.params) and {id(p) for p in order} == set(self.pindex), "DiT layout"
        self.order_ids = [id(p) for p in order]
        self.goff = [0] * len(self.params)
        off = 0
        for p in order:
            self.goff[self.pindex[id(p)]] = off
            off += p.numel()
        self.gtotal = off
        self.ada_w_off = self.goff[self.pindex[id(self.ada[0].weight)]]
        self.ada_b_off = self.goff[self.pindex[id(self.ada[0].bias)]]

    def _ada_pack(self, dtype=torch.float32):
        """Packed [ada_total][1][Kc] forward weight of all adaLN projections."""
        H = self.H
        Kc = L.kc_for(H, dtype)

        def jobs(buf):
            out, off = [], 0
            for lin in self.ada:
                co = lin.weight.shape[0]
                out.append((lin.weight, buf, off * Kc, L.PACK_FWD, co, H, 1, 1, Kc, -1))
                off += co
            return out

        return self.packs.get(("ada", dtype), tuple(lin.weight for lin in self.ada),
                              lambda: torch.zeros(self.ada_total * Kc, dtype=dtype, device=self.ada[0].weight.device),
                              jobs)

    def _ada_pack_dgrad(self, dtype=torch.float32):
        H = self.H
        Kt = L.kc_for(self.ada_total, dtype)

        def jobs(buf):
            out, off = [], 0
            for lin in self.ada:
                co = lin.weight.shape[0]
                out.append((lin.weight, buf, 0, L.PACK_DGRAD, co, H, 1, 1, Kt, off))
                off += co
            return out

        return self.packs.get(("ada_dg", dtype), tuple(lin.weight for lin in self.ada),
                              lambda: torch.zeros(H * Kt, dtype=dtype, device=self.ada[0].weight.device), jobs)

    def _ada_bias(self):
        def jobs(buf):
            out, off = [], 0
            for lin in self.ada:
                co = lin.bias.shape[0]
                out.append((lin.bias, buf, off, L.PACK_FWD, co, 1, 1, 1, 1, -1))
                off += co
            return out

        return self.packs.get("ada_b", tuple(lin.bias for lin in self.ada),
                              lambda: torch.empty(self.ada_total, dtype=torch.float32, device=self.ada[0].bias.device),
                              jobs)

    def _drop(self, site):
        if self._drop_spec is None:
            return None
        d = ((self._seed_base + 7919 * site) & 0xFFFFFFFF, self._drop_spec[0], self._drop_spec[1])
        if self.seed_ptr is not None:
            d = d + (self.seed_ptr,)
        return d

    # =========================================================================================
    def run(self, x, t, y=None):
        params = self.params
        need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
        if need_grad:
            return _DiTFunction.apply(self, x, t, y, *params)
        out, _ = self.forward(x, t, y, keep=False)
        return out

    def forward(self, x, t, y, keep):
        m = self.m
        self.device = x.device
        self.packs.refresh()
        dt = self.dt
        f32 = torch.float32
        B, Cin, Hi, Wi = x.shape
        p = m.patch_size
        ht, wt = m.h_tokens, m.w_tokens
        Lt = ht * wt
        T = B * Lt
        H = self.H
        heads = m.num_heads
        hd = H // heads
        x = x.contiguous().float()
        t = t.to(device=x.device, dtype=torch.long).contiguous()
        tape = [] if keep else None
        if m.training and m.dropout > 0:
            pd = float(m.dropout)
            self._drop_spec = (min(int(round(pd * 4294967296.0)), 4294967295), 1.0 / (1.0 - pd) if pd < 1 else 0.0)
            self._seed_base = 0 if self.seed_ptr is not None else _seed_from_torch()
        else:
            self._drop_spec = None

        # ---- conditioning: c = MLP(timestep embedding) (+ label embedding) ----
        te = m.t_embedder
        fdim = te.frequency_embedding_size
        tf = torch.empty(B, 1, 1, fdim, dtype=f32, device=x.device)
        K.timestep_embedding(t, fdim, tf.view(B, fdim))
        A0 = Act(tf, 1, 1, fdim)
        A1 = self._new(B, 1, 1, H, f32)
        self._conv([A0], te.mlp[0], K.TAPS1, 1, 1, H, bias=te.mlp[0].bias, out=A1.t, dtype=f32)
        c = self._new(B, 1, 1, H, f32)
        ye = None
        if m.y_embedder is not None and y is not None:
            y = y.to(device=x.device, dtype=torch.long).contiguous()
            ye = torch.empty(B, 1, 1, H, dtype=f32, device=x.device)
            K.embed_fwd(y, m.y_embedder.embedding_table.weight, ye.view(B, H))   # clamps y to [0, num_classes]
        self._conv([A1], te.mlp[2], K.TAPS1, 1, 1, H, pro=(L.PRO_SILU, None, None), bias=te.mlp[2].bias, resid=ye,
                   out=c.t, dtype=f32)
        mod = torch.empty(B, 1, 1, self.ada_total, dtype=f32, device=x.device)
        self._conv([c], None, K.TAPS1, 1, 1, self.ada_total, pro=(L.PRO_SILU, None, None), bias=self._ada_bias(),
                   out=mod, dtype=f32, w=self._ada_pack(f32), Kc=L.kc_for(H, f32))
        mod2 = mod.view(B, self.ada_total)
        ldm = self.ada_total

        # ---- patch embedding (fp32) + pos_embed: the fp32 residual stream ----
        c4 = L.chunk_for(f32)
        xin = Act(K.pack_input(f32, x, (Cin + c4 - 1) // c4 * c4), Hi, Wi, Cin)
        x0 = torch.empty(B, ht, wt, H, dtype=f32, device=x.device)
        self._conv([xin], m.x_embedder.proj, self.patch_taps, ht, wt, H, stride=p, bias=m.x_embedder.proj.bias,
                   out=x0, dtype=f32)
        K.add_bcast(x0, m.pos_embed, B, Lt * H)
        if keep:
            tape.append(("embed", t, y, tf, A1, c, ye, mod, xin))

        def ln(xs, br, off_gate, off_shift, off_scale, drop):
            """x_new = xs + gate * drop(br) (br given), then LN + modulation -> (x_new, h, mean, rstd)."""
            h = torch.empty(B, ht, wt, H, dtype=dt, device=x.device)
            mean = torch.empty(T, dtype=f32, device=x.device)
            rstd = torch.empty(T, dtype=f32, device=x.device)
            xo = None
            if br is not None:
                xo = torch.empty(B, ht, wt, H, dtype=f32, device=x.device)
            K.ln_mod_fwd(dt, xs, T, H, Lt, mod2, ldm, off_shift, off_scale, 1e-6, h, H, mean, rstd, br=br,
                         ld_br=H, off_gate=off_gate, drop=drop, x_out=xo)
            return (xo if xo is not None else xs), h, mean, rstd

        xcur = x0
        pend = None            # (mo, gate offset, drop) of the previous block's MLP branch, not yet added
        for i, blk in enumerate(self.blocks):
            mo_ = self.ada_off[i]
            if pend is None:
                x_in, h1, mean1, rstd1 = ln(xcur, None, 0, mo_, mo_ + H, None)
            else:
                x_in, h1, mean1, rstd1 = ln(xcur, pend[0], pend[1], mo_, mo_ + H, pend[2])
            A = Act(h1, ht, wt, H)
            qkv = self._new(B, ht, wt, 3 * H)
            self._conv([A], self.in_proj[i], K.TAPS1, ht, wt, 3 * H, bias=blk.attn.in_proj_bias, out=qkv.t)
            o = self._new(B, ht, wt, H)
            lse = torch.empty(B * heads * Lt, dtype=f32, device=x.device)
            d0 = self._drop(2 * len(self.blocks) + i)      # attention-probability dropout (MHA dropout=p)
            K.attn_fwd(dt, qkv.t, 3 * H, B, Lt, heads, hd, o.t, H, lse, drop=d0)
            ao = self._new(B, ht, wt, H)
            self._conv([o], blk.attn.out_proj, K.TAPS1, ht, wt, H, bias=blk.attn.out_proj.bias, out=ao.t)
            x_mid, h2, mean2, rstd2 = ln(x_in, ao.t, mo_ + 2 * H, mo_ + 3 * H, mo_ + 4 * H, None)
            Hm = blk.mlp[0].out_features
            d1 = self._drop(2 * i)
            a = self._new(B, ht, wt, Hm)
            u = self._new(B, ht, wt, Hm) if keep or d1 is not None else None
            if d1 is None and not _GELU_EPI:
                self._conv([Act(h2, ht, wt, H)], blk.mlp[0], K.TAPS1, ht, wt, Hm, bias=blk.mlp[0].bias,
                           out=(u.t if u is not None else a.t))
                K.gelu_fwd(dt, u.t if u is not None else a.t, T, Hm, Hm, a.t)
            elif d1 is None:
                # GELU in fc1's epilogue; the pre-activation is stored only when the backward needs it
                self._conv([Act(h2, ht, wt, H)], blk.mlp[0], K.TAPS1, ht, wt, Hm, bias=blk.mlp[0].bias, out=a.t,
                           act=L.ACT_GELU, y_pre=None if u is None else u.t)
            elif _GELU_DROP_EPI:
                # GELU + the MLP Dropout in fc1's epilogue (bitwise dmc_gelu_fwd of the stored pre-activation)
                self._conv([Act(h2, ht, wt, H)], blk.mlp[0], K.TAPS1, ht, wt, Hm, bias=blk.mlp[0].bias, out=a.t,
                           act=L.ACT_GELU_DROP, y_pre=u.t, drop=d1)
            else:
                self._conv([Act(h2, ht, wt, H)], blk.mlp[0], K.TAPS1, ht, wt, Hm, bias=blk.mlp[0].bias, out=u.t)
                K.gelu_fwd(dt, u.t, T, Hm, Hm, a.t, drop=d1)
            mo = self._new(B, ht, wt, H)
            self._conv([a], blk.mlp[3], K.TAPS1, ht, wt, H, bias=blk.mlp[3].bias, out=mo.t)
            d2 = self._drop(2 * i + 1)
            if keep:
                tape.append(("block", i, x_in, h1, mean1, rstd1, qkv, o, lse, ao, x_mid, h2, mean2, rstd2, u, a, mo,
                             d1, d2, d0))
            xcur = x_mid
            pend = (mo.t, mo_ + 5 * H, d2)
        # ---- final layer ----
        fo = self.ada_off[-1]
        x_fin, hf, meanf, rstdf = ln(xcur, pend[0], pend[1], fo, fo + H, pend[2])
        fl = m.final_layer.linear
        K_out = fl.out_features
        ldo = (K_out + 3) // 4 * 4
        otok = torch.empty(B, ht, wt, ldo, dtype=f32, device=x.device)
        self._conv([Act(hf, ht, wt, H)], fl, K.TAPS1, ht, wt, K_out, bias=fl.bias, out=otok, out_f32=True)
        out = torch.empty(B, m.out_channels, Hi, Wi, dtype=f32, device=x.device)
        K.unpatchify(otok, ldo, B, ht, wt, p, m.out_channels, out)
        if keep:
            tape.append(("final", x_fin, hf, meanf, rstdf, ldo))
        return out, tape

    # =========================================================================================
    def backward(self, tape, dout, x_requires_grad):
        m = self.m
        dt = self.dt
        f32 = torch.float32
        flat = getattr(self, "_flat", None)
        if flat is None or flat.device != dout.device or any(p.grad is not None for p in self.params):
            flat = torch.empty(self.gtotal, dtype=f32, device=dout.device)
        self._flat = flat
        self.flat = flat
        gv = lambda p: self._gview(flat, p)  # noqa: E731
        B = dout.shape[0]
        p = m.patch_size
        ht, wt = m.h_tokens, m.w_tokens
        Lt = ht * wt
        T = B * Lt
        H = self.H
        heads = m.num_heads
        hd = H // heads
        dev = dout.device
        emb = tape[0]
        mod = emb[7]
        mod2 = mod.view(B, self.ada_total)
        ldm = self.ada_total
        dmod = torch.empty(B, self.ada_total, dtype=f32, device=dev)
        hook = self.grad_hook
        pos = [0]

        def publish(final):
            if hook is None:
                return
            hook(flat, pos[0], final)

        # ---- final layer ----
        _, x_fin, hf, meanf, rstdf, ldo = tape[-1]
        fl = m.final_layer.linear
        K_out = fl.out_features
        ldq = (K_out + self.chunk - 1) // self.chunk * self.chunk
        dtok = torch.empty(B, ht, wt, ldq, dtype=dt, device=dev)
        K.patchify_grad(dt, dout.contiguous(), B, ht, wt, p, m.out_channels, dtok, ldq)
        self._wgrad([Act(hf, ht, wt, H)], dtok, ldq, K.TAPS1, ht, wt, K_out, gv(fl.weight), dbias=gv(fl.bias))
        dhf = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
        self._conv([Act(dtok, ht, wt, K_out)], fl, K.TAPS1, ht, wt, H, out=dhf, packmode=L.PACK_DGRAD,
                   Kc=L.kc_for(K_out, dt))
        dx = torch.zeros(B, ht, wt, H, dtype=f32, device=dev)
        fo = self.ada_off[-1]
        K.ln_mod_bwd(dt, dhf, H, x_fin, meanf, rstdf, mod2, ldm, fo + H, T, H, Lt, dx, dmod, fo + H, fo)
        pos[0] = self.goff[self.pindex[id(fl.bias)]] + fl.bias.numel()
        publish(False)

        # ---- blocks, last to first ----
        for rec in reversed(tape[1:-1]):
            (_, i, x_in, h1, mean1, rstd1, qkv, o, lse, ao, x_mid, h2, mean2, rstd2, u, a, mo, d1, d2, d0) = rec
            blk = self.blocks[i]
            mo_ = self.ada_off[i]
            Hm = blk.mlp[0].out_features
            # MLP branch: x_out = x_mid + gate_mlp * drop(mo)
            dmo = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
            K.gate_bwd(dt, dx, mo.t, H, mod2, ldm, mo_ + 5 * H, T, H, Lt, dmo, H, dmod, mo_ + 5 * H, drop=d2)
            self._wgrad([a], dmo, H, K.TAPS1, ht, wt, H, gv(blk.mlp[3].weight), dbias=gv(blk.mlp[3].bias))
            du = torch.empty(B, ht, wt, Hm, dtype=dt, device=dev)
            if _DGELU_EPI:
                # fc2's input gradient with the GELU (+ Dropout) backward in its epilogue (bitwise dmc_gelu_bwd)
                self._conv([Act(dmo, ht, wt, H)], blk.mlp[3], K.TAPS1, ht, wt, Hm, out=du, packmode=L.PACK_DGRAD,
                           act=L.ACT_DGELU, y_pre=u.t, drop=d1)
            else:
                da = torch.empty(B, ht, wt, Hm, dtype=dt, device=dev)
                self._conv([Act(dmo, ht, wt, H)], blk.mlp[3], K.TAPS1, ht, wt, Hm, out=da, packmode=L.PACK_DGRAD)
                K.gelu_bwd(dt, da, u.t, T, Hm, Hm, du, drop=d1)
            self._wgrad([Act(h2, ht, wt, H)], du, Hm, K.TAPS1, ht, wt, Hm, gv(blk.mlp[0].weight),
                        dbias=gv(blk.mlp[0].bias))
            dh2 = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
            self._conv([Act(du, ht, wt, Hm)], blk.mlp[0], K.TAPS1, ht, wt, H, out=dh2, packmode=L.PACK_DGRAD)
            K.ln_mod_bwd(dt, dh2, H, x_mid, mean2, rstd2, mod2, ldm, mo_ + 4 * H, T, H, Lt, dx, dmod, mo_ + 4 * H,
                         mo_ + 3 * H)
            # attention branch: x_mid = x_in + gate_msa * ao
            dao = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
            K.gate_bwd(dt, dx, ao.t, H, mod2, ldm, mo_ + 2 * H, T, H, Lt, dao, H, dmod, mo_ + 2 * H)
            op = blk.attn.out_proj
            self._wgrad([o], dao, H, K.TAPS1, ht, wt, H, gv(op.weight), dbias=gv(op.bias))
            do = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
            self._conv([Act(dao, ht, wt, H)], op, K.TAPS1, ht, wt, H, out=do, packmode=L.PACK_DGRAD)
            dqkv = torch.empty(B, ht, wt, 3 * H, dtype=dt, device=dev)
            K.attn_bwd(dt, qkv.t, 3 * H, o.t, do, H, lse, B, Lt, heads, hd, dqkv, 3 * H, drop=d0)
            self._wgrad([Act(h1, ht, wt, H)], dqkv, 3 * H, K.TAPS1, ht, wt, 3 * H, gv(blk.attn.in_proj_weight),
                        dbias=gv(blk.attn.in_proj_bias))
            dh1 = torch.empty(B, ht, wt, H, dtype=dt, device=dev)
            self._conv([Act(dqkv, ht, wt, 3 * H)], self.in_proj[i], K.TAPS1, ht, wt, H, out=dh1,
                       packmode=L.PACK_DGRAD)
            K.ln_mod_bwd(dt, dh1, H, x_in, mean1, rstd1, mod2, ldm, mo_ + H, T, H, Lt, dx, dmod, mo_ + H, mo_)
            pos[0] = self.goff[self.pindex[id(blk.attn.in_proj_bias)]] + blk.attn.in_proj_bias.numel()
            publish(False)

        # ---- pos_embed and the patch conv (fp32): dx is the gradient of x0 = conv(x) + pos ----
        _, t, y, tf, A1, c, ye, _, xin = emb
        K.batch_sum(dx, B, Lt * H, gv(m.pos_embed))
        pe = m.x_embedder.proj
        dxin = None
        if x_requires_grad:
            dxin = torch.empty(B, m.in_channels, ht * p, wt * p, dtype=f32, device=dev)
            K.patch_dgrad(dx, H, pe.weight.detach(), B, ht, wt, p, m.in_channels, H, dxin)
        self._wgrad([xin], dx, H, self.patch_taps, ht, wt, H, gv(pe.weight), stride=p, dtype=f32, dbias=gv(pe.bias))
        # ---- stacked adaLN: mod = SiLU(c) W_ada^T + b ----
        Ta = self.ada_total
        dw_a = flat[self.ada_w_off:self.ada_w_off + Ta * H]
        self._wgrad([c], dmod, Ta, K.TAPS1, 1, 1, Ta, dw_a, pro=(L.PRO_SILU, None, None), dtype=f32,
                    dbias=flat[self.ada_b_off:self.ada_b_off + Ta])
        dc = torch.empty(B, 1, 1, H, dtype=f32, device=dev)
        self._conv([Act(dmod.view(B, 1, 1, Ta), 1, 1, Ta)], None, K.TAPS1, 1, 1, H, out=dc, dtype=f32,
                   w=self._ada_pack_dgrad(f32), Kc=L.kc_for(Ta, f32), silu_pre=c.t, ld_silu=H)
        # ---- timestep MLP and label embedding: c = Linear2(SiLU(Linear1(tf))) + label_emb ----
        te = m.t_embedder
        self._wgrad([A1], dc, H, K.TAPS1, 1, 1, H, gv(te.mlp[2].weight), pro=(L.PRO_SILU, None, None), dtype=f32,
                    dbias=gv(te.mlp[2].bias))
        de1 = torch.empty(B, 1, 1, H, dtype=f32, device=dev)
        self._conv([Act(dc, 1, 1, H)], te.mlp[2], K.TAPS1, 1, 1, H, out=de1, dtype=f32, packmode=L.PACK_DGRAD,
                   silu_pre=A1.t, ld_silu=H)
        self._wgrad([Act(tf, 1, 1, tf.shape[-1])], de1, H, K.TAPS1, 1, 1, H, gv(te.mlp[0].weight), dtype=f32,
                    dbias=gv(te.mlp[0].bias))
        if m.y_embedder is not None:
            tab = m.y_embedder.embedding_table.weight
            if ye is not None:
                K.embed_bwd(y, tab.shape[0], dc.view(B, H), gv(tab))
            else:
                gv(tab).zero_()
        pos[0] = self.gtotal
        publish(True)
        grads = [self._gview(flat, q) for q in self.params]
        return dxin, grads


class _DiTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ex, x, t, y, *params):
        out, tape = ex.forward(x, t, y, keep=True)
        ctx.ex = ex
        ctx.tape = tape
        ctx.x_req = x.requires_grad
        return out

    @staticmethod
    def backward(ctx, dout):
        ex = ctx.ex
        dx, grads = ex.backward(ctx.tape, dout, ctx.x_req)
        ctx.tape = None
        return (None, dx, None, None, *grads)


def dit_flops_per_image(model) -> float:
    """2*MACs of one DiT forward per image (linears, patch conv, attention matmuls; the per-sample conditioning
    GEMMs included)."""
    H = model.hidden_size
    Lt = model.h_tokens * model.w_tokens
    p = model.patch_size
    Hm = model.blocks[0].mlp[0].out_features
    f = 2.0 * Lt * (model.in_channels * p * p) * H
    per_block = 2.0 * Lt * (H * 3 * H + H * H + H * Hm + Hm * H) + 2 * 2.0 * Lt * Lt * H
    f += len(model.blocks) * per_block
    f += 2.0 * Lt * H * model.final_layer.linear.out_features
    te = model.t_embedder
    f += 2.0 * (te.mlp[0].in_features * H + H * H) + 2.0 * H * (6 * H * len(model.blocks) + 2 * H)
    return f
