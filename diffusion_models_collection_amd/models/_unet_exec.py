"""Graph executor of the UNet on the gfx950 kernels (forward + hand-scheduled backward).

The reference runs UNet.forward (models/unet.py:243-292) as ~400 PyTorch eager ops and lets autograd
build the backward (~1000 ops). Here the network is walked once per call in the reference's order and
every layer is a handful of fused HIP kernels over NHWC activations:

  ResidualBlock   gn_stats(x) -> conv3x3[GN1+SiLU prologue; bias + temb epilogue] -> gn_stats(h1)
                  -> [1x1 shortcut conv] -> conv3x3[GN2+SiLU+dropout prologue; bias + residual epilogue]
  AttentionBlock  gn_stats(x) -> 1x1 qkv conv[GN prologue] -> fused flash attention -> 1x1 proj[+x]
  Downsample      stride-2 conv;  Upsample: conv with nearest-x2 folded into the input indexing
  up-path concat  never materialised: the consumer conv / GN read two sources (virtual concat)
  time MLP        sinusoid -> Linear -> SiLU -> Linear, then ONE GEMM for all 22 time_mlp (+label_proj)
                  projections (their weights are packed side by side)

The backward is hand-scheduled in reverse (a tape of forward records), recomputing GN/SiLU/dropout on the
fly (dropout masks come from a counter hash, never stored). Every parameter gradient is written straight
into one flat fp32 buffer (views are handed to autograd), which is also what the data-parallel
all-reduce works on.
"""
import contextlib
import ctypes
import math
import os
import weakref
from typing import List, Optional

import torch

from .. import _lib as L
from .. import kernels as K


class Act:
    """An NHWC activation [N, H, W, C] (contiguous, pitch C) plus its gradient buffer."""

    __slots__ = ("t", "H", "W", "C", "grad", "part")

    def __init__(self, t, H, W, C):
        self.t, self.H, self.W, self.C = t, H, W, C
        self.grad = None
        self.part = None    # GroupNorm partials written by the conv that produced t (dmc_conv_desc.gn_part)


# GroupNorm statistics from the conv epilogues (A/B: DMC_GN_PARTIALS=0 computes them with dmc_gn_stats passes)
_GN_PARTIALS = os.environ.get("DMC_GN_PARTIALS", "1") not in ("", "0")
# The GroupNorm backward's parameter column sums deferred to one dmc_colsum_batch per gradient segment (A/B switch
# DMC_GN_DEFER=0: one finish launch per GroupNorm)
_GN_DEFER = os.environ.get("DMC_GN_DEFER", "1") not in ("", "0")
# The weight-gradient slab reductions deferred to one dmc_wgrad_reduce_batch per gradient segment (A/B switch
# DMC_WG_DEFER=0: one reduce launch after each weight-gradient kernel)
_WG_DEFER = os.environ.get("DMC_WG_DEFER", "1") not in ("", "0")
# GroupNorm statistics + apply in one launch where a sample has at most this many elements (dmc_gn_stats_apply: the
# 4x4 levels); 0 = off. A module switch for same-box A/Bs (scripts/r5_gsa.sh), not an option. 16384 (the 8x8 levels
# too, in place of the conv-partial finalize + apply) measured neutral to slower
_GN_SMALL_FUSE = 8192


def _seed_from_torch():
    # dropout seeds follow torch's CPU generator (torch.manual_seed / set_seed semantics), no device sync
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


class _PackCache:
    """Weights repacked into the kernel layouts.

    An entry is (version, buffer, sources, jobs): `jobs` are dmc_pack_job specs writing `buffer` from the
    fp32 master `sources`. The version is the sources' torch version counters and pointers plus the
    executor's weight generation (bumped by the flat optimizer step, whose kernel writes the parameters
    behind torch's back). `refresh()` repacks every stale entry in ONE dmc_pack_weights launch; `get()`
    repacks a single stale entry (first use, or a weight changed outside a step).
    """

    def __init__(self, owner):
        self._owner = weakref.ref(owner)   # the executor owns the cache: no reference cycle back to it
        self.entries = {}
        self._batch = None

    def _ver(self, srcs):
        return (self._owner().wgen,) + tuple((s._version, s.data_ptr()) for s in srcs)

    def get(self, key, srcs, make_buf, make_jobs):
        v = self._ver(srcs)
        e = self.entries.get(key)
        if e is None or e[0] != v:
            buf = e[1] if e is not None and e[2] == tuple(id(s) for s in srcs) else make_buf()
            jobs = make_jobs(buf)
            K.PackBatch(jobs, buf.device).launch()
            e = (v, buf, tuple(id(s) for s in srcs), srcs, jobs)
            self.entries[key] = e
        return e[1]

    def refresh(self):
        stale = []
        for k, e in self.entries.items():
            v = self._ver(e[3])
            if e[0] != v:
                stale.append((k, e, v))
        if not stale:
            return
        # the cached job array holds raw source/destination pointers: key it on them
        key = tuple((k, e[1].data_ptr(), v[1:]) for k, e, v in stale)
        if self._batch is None or self._batch[0] != tuple((k, b, tuple(p for _, p in vv)) for k, b, vv in key):
            jobs = [j for _, e, _ in stale for j in e[4]]
            self._batch = (tuple((k, b, tuple(p for _, p in vv)) for k, b, vv in key),
                           K.PackBatch(jobs, stale[0][1][1].device))
        self._batch[1].launch()
        for k, e, v in stale:
            self.entries[k] = (v,) + e[1:]


class ExecCore:
    """What every backbone executor shares: weight packing through the pack cache, the generic implicit-GEMM conv
    / weight-gradient launchers over 1-2 NHWC sources, activation allocation and views of the flat gradient
    buffer. Subclasses set self.dt, self.packs, self.device, self.training_grad_scale, self.pindex, self.goff, and
    bind their model with _bind_model."""

    def _bind_model(self, model):
        self._mref = weakref.ref(model)

    @property
    def m(self):
        """The backbone, held weakly. model._executor -> executor is the only strong edge between the two (and the
        executor's pack cache / GradSync / graphed step refer back to it weakly too), so a dropped model frees its
        executor -- tape arenas, packed weights, flat gradients -- by reference counting at the `del`, never by the
        cyclic collector at an arbitrary later moment: round 5 saw such a collection free a dropped model's HIP graphs
        in the middle of another graph's capture and abort the process (tests/test_gpu_model.py
        test_dropped_model_frees_without_cyclic_gc)."""
        m = self._mref()
        if m is None:
            raise RuntimeError("the model this executor ran has been freed")
        return m

    def _gview(self, flat, p):
        i = self.pindex[id(p)]
        o = self.goff[i]
        return flat[o:o + p.numel()].view(p.shape)

    # ---------------------------------------------------------------------------------------
    def _wpack(self, conv, mode, Kc, dtype=None):
        dtype = dtype or self.dt
        w = conv.weight
        if w.dim() == 2:
            Cout, Cin, kh, kw = w.shape[0], w.shape[1], 1, 1
        else:
            Cout, Cin, kh, kw = w.shape
        ntaps = 16 if mode == L.PACK_UPDGRAD else kh * kw
        rows = Cout if mode == L.PACK_FWD else Cin

        def make_buf():
            return torch.empty(rows * ntaps * Kc, dtype=dtype, device=w.device)

        return self.packs.get((id(conv), mode, Kc, dtype), (w,), make_buf,
                              lambda buf: [(w, buf, 0, mode, Cout, Cin, kh, kw, Kc, -1)])

    def _conv(self, srcs, conv, taps, OH, OW, Cout, mode=L.MODE_NORMAL, stride=1, pro=None, drop=None,
              bias=None, addvec=None, ld_add=0, resid=None, out=None, out_f32=False, out_nchw=False,
              dtype=None, packmode=L.PACK_FWD, w=None, Kc=None, silu_pre=None, ld_silu=0, split=None,
              act=L.ACT_NONE, y_pre=None, stats=None):
        """Generic implicit-GEMM conv over 1-2 NHWC sources. pro = (kind, scale, shift), or (PRO_GN_SILU, gamma, beta,
        groups, eps): SiLU(GroupNorm(sources)) with the statistics taken inside the conv. stats = the output Act: in
        bf16 mode it gets the GroupNorm partials of the stored output (the next GroupNorm then needs no statistics
        pass over it, see _gn)."""
        dtype = dtype or self.dt
        gn_part = None
        if (stats is not None and _GN_PARTIALS and dtype == torch.bfloat16 and (OH * OW) % 64 == 0 and Cout % 8 == 0
                and split is None and not out_nchw and not out_f32):
            gn_part = torch.empty(srcs[0].t.shape[0] * OH * OW // 64 * (Cout // 8) * 2, dtype=torch.float32,
                                  device=srcs[0].t.device)
            stats.part = gn_part
        a = srcs[0]
        C1 = a.C
        C2 = srcs[1].C if len(srcs) > 1 else 0
        ld1 = a.t.shape[-1]
        ld2 = srcs[1].t.shape[-1] if len(srcs) > 1 else 0
        N = a.t.shape[0]
        if Kc is None:
            Kc = L.kc_for(C1 + C2, dtype)
        if w is None:
            w = self._wpack(conv, packmode, Kc, dtype)
        d = K.make_desc(dtype, N, a.H, a.W, C1, C2, ld1, ld2, Kc, OH, OW, Cout, taps, mode, stride)
        if pro is not None:
            K.set_prologue(d, pro[0], pro[1], pro[2], C1 + C2, drop, C1 + C2)
            if pro[0] == L.PRO_GN_SILU:
                d.pro_groups, d.pro_eps = pro[3], pro[4]
        elif drop is not None:
            if act not in (L.ACT_GELU_DROP, L.ACT_DGELU):
                raise ValueError("dropout needs a prologue (or the GELU-dropout epilogue)")
            K.set_prologue(d, L.PRO_NONE, drop=drop)    # the epilogue's dropout reads the drop_* fields
        ldy2 = 0
        y2 = None
        if split is not None:
            (y1, ldy1), (y2, ldy2), csplit = split
        else:
            y1 = out
            ldy1 = 0 if out_nchw else out.shape[-1]
            csplit = None
        K.set_epilogue(d, bias=bias, addvec=addvec, ld_add=ld_add, resid=resid,
                       ld_res=(0 if resid is None or out_nchw else resid.shape[-1]), silu_pre=silu_pre,
                       ld_silu=ld_silu, ldy1=ldy1, ldy2=ldy2, Csplit=csplit, out_f32=out_f32, out_nchw=out_nchw,
                       act=act, y_pre=y_pre, ld_pre=0 if y_pre is None else y_pre.shape[-1], gn_part=gn_part)
        K.conv(d, a.t, srcs[1].t if len(srcs) > 1 else None, w, y1, y2)
        return d

    def _wgrad(self, srcs, dy, ld_dy, taps, OH, OW, Cout, dw, mode=L.MODE_NORMAL, stride=1, pro=None, drop=None,
               dtype=None, dbias=None):
        """Weight gradient dw of a conv/linear; with dbias also its bias gradient (the pixel sums of dy), taken in
        the same kernel (include/dmc.h dmc_conv_desc.wg_bias) instead of a separate channel-sum pass."""
        dtype = dtype or self.dt
        a = srcs[0]
        C1 = a.C
        C2 = srcs[1].C if len(srcs) > 1 else 0
        N = a.t.shape[0]
        Kc = L.kc_for(C1 + C2, dtype)
        d = K.make_desc(dtype, N, a.H, a.W, C1, C2, a.t.shape[-1], srcs[1].t.shape[-1] if len(srcs) > 1 else 0, Kc,
                        OH, OW, Cout, taps, mode, stride)
        if pro is not None:
            K.set_prologue(d, pro[0], pro[1], pro[2], C1 + C2, drop, C1 + C2)
        K.wgrad(d, dy, ld_dy, a.t, srcs[1].t if len(srcs) > 1 else None, dw, self.training_grad_scale, dbias=dbias,
                defer=getattr(self, "_wg_defer", None))

    def _new(self, N, H, W, C, dtype=None):
        return Act(torch.empty(N, H, W, C, dtype=dtype or self.dt, device=self.device), H, W, C)



class UNetExecutor(ExecCore):
    def __init__(self, model):
        self._bind_model(model)
        self.dt = model.compute_dtype
        self.cdt = L.dtype_code(self.dt)
        self.chunk = L.chunk_for(self.dt)
        self._halo_pro_cache = {}   # shape -> dmc_conv_halo_prologue verdict
        self._gsa_cache = {}        # shape -> dmc_gn_stats_apply_ok verdict
        self.wgen = 0               # weight generation: bumped when a fused step rewrote the parameters
        self.packs = _PackCache(self)
        self.params = list(model.parameters())
        self.pindex = {id(p): i for i, p in enumerate(self.params)}
        # time-embedding projection layout: all ResidualBlocks' time_mlp (and label_proj) rows side by side
        self.res_blocks = [mod for mod in model.modules() if type(mod).__name__ == "ResidualBlock"]
        self.temb_off = {}
        off = 0
        for rb in self.res_blocks:
            self.temb_off[id(rb)] = off
            off += rb.out_channels
        self.temb_total = off
        self._layout_grads()
        self.daddvec = None
        self.training_grad_scale = 1.0
        self.grad_hook = None       # called as hook(flat_grad, lo, hi) when a range of grads is final
        self.seed_ptr = None        # device address of the dropout seed word (graph-captured training step)
        # the layer sequence of UNet.forward (models/unet.py:270-289): (layer, takes the [h, skip] concat, pushes a
        # skip) -- walked with one step of lookahead so each conv knows which GroupNorm reads its output next
        self.plan = []
        for block in model.down_blocks:
            for j, layer in enumerate(block):
                self.plan.append((layer, False, j == len(block) - 1))
        for layer in model.middle_block:
            if type(layer).__name__ != "Identity":
                self.plan.append((layer, False, False))
        for block in model.up_blocks:
            for j, layer in enumerate(block):
                self.plan.append((layer, j == 0, False))

    # ---------------------------------------------------------------------------------------
    def _layout_grads(self):
        """Flat fp32 gradient buffer layout.

        Slots follow the order in which the backward finishes them, so a prefix of the buffer is final early
        (data-parallel all-reduce buckets): reverse module order for the blocks, then the time embedding
        (its backward runs right after the last ResidualBlock's, before the input conv's, see backward()),
        with the 22 time_mlp weights, their biases and the label_proj weights side by side (the stacked
        projection GEMM's weight gradient lands in place with no copy), and the input conv LAST: the bucket
        still in flight when the backward ends is then only the input conv's 3.5K gradients.
        """
        m = self.m
        rbs = [mod for mod in m.modules() if type(mod).__name__ == "ResidualBlock"]
        tail = [rb.time_mlp[1].weight for rb in rbs] + [rb.time_mlp[1].bias for rb in rbs]
        if m.num_classes is not None:
            tail += [rb.label_proj[1].weight for rb in rbs]
        last = list(m.input_conv.parameters())
        tail_ids = {id(p) for p in tail + last}
        head = [p for p in reversed(self.params) if id(p) not in tail_ids]
        order = head + tail + last
        self.goff = [0] * len(self.params)
        off = 0
        for p in order:
            self.goff[self.pindex[id(p)]] = off
            off += p.numel()
        self.gtotal = off
        self.temb_w_off = self.goff[self.pindex[id(tail[0])]]
        self.temb_b_off = self.goff[self.pindex[id(tail[len(rbs)])]]
        self.temb_l_off = self.goff[self.pindex[id(tail[2 * len(rbs)])]] if m.num_classes is not None else None

    def _temb_lins(self, which):
        return [(rb.time_mlp[1] if which == 0 else rb.label_proj[1]) for rb in self.res_blocks]

    def _temb_pack(self, which, dtype):
        """Packed [sum Cout][1][Kc=512] weight of every block's time_mlp (which=0) / label_proj (which=1)."""
        lins = self._temb_lins(which)
        dim = lins[0].weight.shape[1]
        Kc = L.kc_for(dim, torch.float32)

        def jobs(buf):
            out, off = [], 0
            for lin in lins:
                co = lin.weight.shape[0]
                out.append((lin.weight, buf, off * Kc, L.PACK_FWD, co, dim, 1, 1, Kc, -1))
                off += co
            return out

        return self.packs.get(("temb", which), tuple(lin.weight for lin in lins),
                              lambda: torch.zeros(self.temb_total * Kc, dtype=torch.float32,
                                                  device=lins[0].weight.device), jobs)

    def _temb_pack_dgrad(self, which):
        """[dim][1][Kc >= sum Cout] dgrad pack of the row-concatenated projection weight: each Linear writes
        its own column block (koff) of the shared rows; the padding columns stay zero from allocation."""
        lins = self._temb_lins(which)
        dim = lins[0].weight.shape[1]
        Kt = L.kc_for(self.temb_total, torch.float32)

        def jobs(buf):
            out, off = [], 0
            for lin in lins:
                co = lin.weight.shape[0]
                out.append((lin.weight, buf, 0, L.PACK_DGRAD, co, dim, 1, 1, Kt, off))
                off += co
            return out

        return self.packs.get(("temb_dg", which), tuple(lin.weight for lin in lins),
                              lambda: torch.zeros(dim * Kt, dtype=torch.float32, device=lins[0].weight.device),
                              jobs)

    def _temb_bias(self):
        """All 22 time_mlp biases side by side (a 1x1 FWD 'pack' with Kc = 1 is a copy)."""
        lins = self._temb_lins(0)

        def jobs(buf):
            out, off = [], 0
            for lin in lins:
                co = lin.bias.shape[0]
                out.append((lin.bias, buf, off, L.PACK_FWD, co, 1, 1, 1, 1, -1))
                off += co
            return out

        return self.packs.get("temb_b", tuple(lin.bias for lin in lins),
                              lambda: torch.empty(self.temb_total, dtype=torch.float32, device=lins[0].bias.device),
                              jobs)

    # ---------------------------------------------------------------------------------------
    def _gn(self, srcs, gn, dtype=None):
        dtype = dtype or self.dt
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N = a.t.shape[0]
        C = a.C + (b.C if b else 0)
        if (all(s.part is not None for s in srcs) and (a.H * a.W) % 64 == 0 and C % gn.num_groups == 0
                and (C // gn.num_groups) % 8 == 0):
            # statistics from the producing convs' epilogue partials: no pass over the activation
            return K.gn_finalize(a.part, a.C, b.part if b else None, b.C if b else 0, N, a.H * a.W, gn.num_groups,
                                 gn.eps, gn.weight, gn.bias)
        return K.gn_stats(dtype, a.t, b.t if b else None, N, a.H * a.W, a.C, b.C if b else 0, a.t.shape[-1],
                          b.t.shape[-1] if b else 0, gn.num_groups, gn.eps, gn.weight, gn.bias)

    def _gn_apply_small(self, srcs, gn, silu, drop=None):
        """(stats, Act) of SiLU(GN(concat(srcs))) from ONE dmc_gn_stats_apply launch (bitwise _gn + _apply) where a
        sample is small enough for one block (the 4x4 levels); None elsewhere."""
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N, HW, C1, C2 = a.t.shape[0], a.H * a.W, a.C, (b.C if b else 0)
        if HW * (C1 + C2) > _GN_SMALL_FUSE or any(s.part is not None for s in srcs):
            return None     # (with conv partials the finalize path is taken, as before)
        key = (self.dt, N, HW, C1, C2, gn.num_groups, L.get_option("DMC_GN_STATS_SPLIT"))
        ok = self._gsa_cache.get(key)
        if ok is None:
            ok = self._gsa_cache[key] = K.gn_stats_apply_ok(self.dt, N, HW, C1, C2, gn.num_groups)
        if not ok:
            return None
        st, out = K.gn_stats_apply(self.dt, a.t, b.t if b else None, N, HW, C1, C2, a.t.shape[-1],
                                   b.t.shape[-1] if b else 0, gn.num_groups, gn.eps, gn.weight, gn.bias, silu=silu,
                                   drop=drop)
        return st, Act(out.view(N, a.H, a.W, C1 + C2), a.H, a.W, C1 + C2)

    def _apply(self, srcs, st, silu=True, drop=None):
        """Act of dropout(silu(GN(concat(srcs)))) materialised with dmc_gn_apply."""
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N = a.t.shape[0]
        C = a.C + (b.C if b else 0)
        out = K.gn_apply(self.dt, a.t, b.t if b else None, N, a.H * a.W, a.C, b.C if b else 0, a.t.shape[-1],
                         b.t.shape[-1] if b else 0, st[0], st[1], silu=silu, drop=drop)
        return Act(out.view(N, a.H, a.W, C), a.H, a.W, C)

    def _halo_pro_ok(self, srcs, Cout, st):
        """Whether dmc_conv2d runs the 3x3 conv of SiLU(GN(srcs)) on the halo kernel with the GN+SiLU applied
        to its resident halo (bf16 inference; dmc_conv_halo_prologue). Cached per shape and A/B switch."""
        if self.dt != torch.bfloat16:
            return False
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N = a.t.shape[0]
        key = (N, a.H, a.W, a.C, b.C if b else 0, a.t.shape[-1], b.t.shape[-1] if b else 0, Cout,
               L.get_option("DMC_HALO_PRO"))
        ok = self._halo_pro_cache.get(key)
        if ok is None:
            C1, C2 = a.C, (b.C if b else 0)
            d = K.make_desc(self.dt, N, a.H, a.W, C1, C2, key[5], key[6], L.kc_for(C1 + C2, self.dt), a.H, a.W, Cout,
                            K.TAPS3)
            K.set_prologue(d, L.PRO_AFFINE_SILU, st[0], st[1], C1 + C2)
            ok = self._halo_pro_cache[key] = K.conv_halo_prologue(d)
        return ok

    def _img_gn_ok(self, srcs, Cout, gn):
        """Whether dmc_conv2d runs the 3x3 conv of SiLU(GN(srcs)) on the small-map kernel with the GroupNorm
        statistics computed inside it (DMC_PRO_GN_SILU: no statistics / finalize / apply launch; bf16 inference at
        the 4x4 and 8x8 levels). Cached per shape and A/B switch."""
        if self.dt != torch.bfloat16 or gn.weight is None or gn.bias is None:
            return False
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N = a.t.shape[0]
        key = ("gn", N, a.H, a.W, a.C, b.C if b else 0, a.t.shape[-1], b.t.shape[-1] if b else 0, Cout,
               gn.num_groups, L.get_option("DMC_IMG_MASK"), L.get_option("DMC_IMG_GN"))
        ok = self._halo_pro_cache.get(key)
        if ok is None:
            C1, C2 = a.C, (b.C if b else 0)
            d = K.make_desc(self.dt, N, a.H, a.W, C1, C2, key[6], key[7], L.kc_for(C1 + C2, self.dt), a.H, a.W, Cout,
                            K.TAPS3)
            K.set_prologue(d, L.PRO_GN_SILU, gn.weight, gn.bias, C1 + C2)
            d.pro_groups, d.pro_eps = gn.num_groups, gn.eps
            lvl = 0 if a.H <= 4 else 1          # DMC_IMG_GN bit 0: the 4x4 levels, bit 1: the 8x8 levels
            ok = self._halo_pro_cache[key] = bool((L.get_option("DMC_IMG_GN") >> lvl) & 1) and K.conv_halo_prologue(d)
        return ok

    def _grad_target(self, act):
        """(buffer, accumulate) for writing a gradient contribution into act.grad."""
        if act.grad is None:
            act.grad = torch.empty_like(act.t)
            return act.grad, 0
        return act.grad, 1

    # =========================================================================================
    def run(self, x, t, y=None):
        params = self.params
        need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
        if need_grad:
            return _UNetFunction.apply(self, x, t, y, *params)
        out, _ = self.forward(x, t, y, keep=False)
        return out

    def forward(self, x, t, y, keep):
        m = self.m
        self.device = x.device
        self.packs.refresh()        # every weight the last step changed, repacked in one launch
        dt = self.dt
        N, Cin, H, W = x.shape
        x = x.contiguous().float()
        t = t.to(device=x.device, dtype=torch.long).contiguous()
        tape = [] if keep else None
        drop_on = m.training and m.dropout > 0
        if drop_on:
            p = float(m.dropout)
            self._drop = (min(int(round(p * 4294967296.0)), 4294967295), 1.0 / (1.0 - p) if p < 1 else 0.0)
            if self.seed_ptr is not None:
                # graph capture: the kernels add the step's seed from device memory (set per replay)
                self._seed_base = 0
            else:
                self._seed_base = _seed_from_torch()
        else:
            self._drop = None
        self._blk_idx = 0

        # ---- time embedding (fp32) ----
        f32 = torch.float32
        te = m.time_embed
        mc = te[0].dim
        tdim = te[1].out_features
        # a length-1 t at inference (the samplers' shared timestep, UNet.shared_timestep): the embedding rows are
        # computed once and broadcast to every image by the consuming epilogues (ld_add = 0)
        Nt = t.shape[0]
        if Nt != N and not (Nt == 1 and not keep and (m.num_classes is None or y is None)):
            raise ValueError(f"UNet: t has {Nt} entries for a batch of {N}")
        e0 = torch.empty(Nt, mc, dtype=f32, device=x.device)
        K.time_embed(t, mc, e0)
        A0 = Act(e0.view(Nt, 1, 1, mc), 1, 1, mc)
        A1 = self._new(Nt, 1, 1, tdim, f32)
        self._conv([A0], te[1], K.TAPS1, 1, 1, tdim, bias=te[1].bias, out=A1.t, dtype=f32)
        A2 = self._new(Nt, 1, 1, tdim, f32)
        self._conv([A1], te[3], K.TAPS1, 1, 1, tdim, pro=(L.PRO_SILU, None, None), bias=te[3].bias, out=A2.t,
                   dtype=f32)
        Ay = None
        if m.num_classes is not None and y is not None:
            y = y.to(device=x.device, dtype=torch.long).contiguous()
            ye = torch.empty(N, tdim, dtype=f32, device=x.device)
            K.embed_fwd(y, m.label_embed.weight, ye)
            Ay = Act(ye.view(N, 1, 1, tdim), 1, 1, tdim)
        addvec = torch.empty(Nt, 1, 1, self.temb_total, dtype=f32, device=x.device)
        Kt = L.kc_for(tdim, f32)
        self._conv([A2], None, K.TAPS1, 1, 1, self.temb_total, pro=(L.PRO_SILU, None, None), bias=self._temb_bias(),
                   out=addvec, dtype=f32, w=self._temb_pack(0, f32), Kc=Kt)
        if Ay is not None:
            self._conv([Ay], None, K.TAPS1, 1, 1, self.temb_total, pro=(L.PRO_SILU, None, None), resid=addvec,
                       out=addvec, dtype=f32, w=self._temb_pack(1, f32), Kc=Kt)
        self.addvec = addvec
        self._ld_add = self.temb_total if Nt == N else 0
        if keep:
            tape.append(("temb", t, y, A0, A1, A2, Ay, addvec))

        # ---- input ----
        ldx = (Cin + self.chunk - 1) // self.chunk * self.chunk
        xin = Act(K.pack_input(dt, x, ldx), H, W, Cin)
        h = self._new(N, H, W, m.model_channels)
        self._conv([xin], m.input_conv, K.TAPS3, H, W, m.model_channels, bias=m.input_conv.bias, out=h.t, stats=h)
        if keep:
            tape.append(("conv_in", xin, h, x.requires_grad))
        hs = [h]
        for i, (layer, cat, push) in enumerate(self.plan):
            srcs = [h, hs.pop()] if cat else [h]
            h = self._layer(srcs, layer, tape)
            if push:
                hs.append(h)
        # ---- output: GN -> SiLU -> conv3x3 -> NCHW fp32 ----
        gno, convo = m.output[0], m.output[2]
        sto = self._gn([h], gno)
        ao = self._apply([h], sto, silu=True)
        out = torch.empty(N, m.out_channels, H, W, dtype=f32, device=x.device)
        self._conv([ao], convo, K.TAPS3, H, W, m.out_channels, bias=convo.bias, out=out, out_f32=True, out_nchw=True)
        if keep:
            tape.append(("out", h, sto, ao))
        return out, tape

    def _layer(self, srcs, layer, tape):
        """One step of the plan."""
        name = type(layer).__name__
        if name == "ResidualBlock":
            return self._res_fwd(srcs, layer, tape)
        if name == "AttentionBlock":
            return self._attn_fwd(srcs[0], layer, tape)
        if name == "Downsample":
            a = srcs[0]
            OH, OW = (a.H + 2 - 3) // 2 + 1, (a.W + 2 - 3) // 2 + 1
            out = self._new(a.t.shape[0], OH, OW, a.C)
            self._conv([a], layer.conv, K.TAPS3, OH, OW, a.C, stride=2, bias=layer.conv.bias, out=out.t, stats=out)
            if tape is not None:
                tape.append(("down", layer, a, out))
            return out
        if name == "Upsample":
            a = srcs[0]
            out = self._new(a.t.shape[0], 2 * a.H, 2 * a.W, a.C)
            self._conv([a], layer.conv, K.TAPS3, 2 * a.H, 2 * a.W, a.C, mode=L.MODE_UPSAMPLE, bias=layer.conv.bias,
                       out=out.t, stats=out)
            if tape is not None:
                tape.append(("up", layer, a, out))
            return out
        raise TypeError(f"unexpected layer {name}")

    def _res_fwd(self, srcs, rb, tape):
        a = srcs[0]
        N, H, W = a.t.shape[0], a.H, a.W
        Cout = rb.out_channels
        gn1, conv1, gn2, conv2 = rb.conv1[0], rb.conv1[2], rb.conv2[0], rb.conv2[3]
        # a1 = SiLU(GN1(x)) materialised once (the 3x3 implicit GEMM reads every pixel 9x; the weight
        # gradient re-reads it in backward). Inference (no tape): where the halo kernel takes the conv, it
        # applies GN+SiLU to its LDS-resident halo instead and nothing is materialised.
        h1 = self._new(N, H, W, Cout)
        off = self.temb_off[id(rb)]
        gn_in1 = tape is None and self._img_gn_ok(srcs, Cout, gn1)
        fused = None if gn_in1 else self._gn_apply_small(srcs, gn1, True)
        st1 = None if gn_in1 else fused[0] if fused else self._gn(srcs, gn1)
        if gn_in1:
            # inference at 4x4 / 8x8: the conv takes GroupNorm statistics, affine and SiLU of its own images
            a1 = None
            self._conv(srcs, conv1, K.TAPS3, H, W, Cout, pro=(L.PRO_GN_SILU, gn1.weight, gn1.bias, gn1.num_groups,
                                                              gn1.eps), bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1)
        elif fused:
            a1 = fused[1]
            self._conv([a1], conv1, K.TAPS3, H, W, Cout, bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1)
        elif tape is None and self._halo_pro_ok(srcs, Cout, st1):
            a1 = None
            self._conv(srcs, conv1, K.TAPS3, H, W, Cout, pro=(L.PRO_AFFINE_SILU, st1[0], st1[1]), bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1)
        else:
            a1 = self._apply(srcs, st1, silu=True)
            self._conv([a1], conv1, K.TAPS3, H, W, Cout, bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1)
        if isinstance(rb.shortcut, torch.nn.Conv2d):
            s = torch.empty(N, H, W, Cout, dtype=self.dt, device=self.device)
            self._conv(srcs, rb.shortcut, K.TAPS1, H, W, Cout, bias=rb.shortcut.bias, out=s)
            resid = s
        else:
            resid = a.t
        drop = None
        if self._drop is not None:
            drop = ((self._seed_base + 7919 * self._blk_idx) & 0xFFFFFFFF, self._drop[0], self._drop[1])
            if self.seed_ptr is not None:
                drop = drop + (self.seed_ptr,)
        self._blk_idx += 1
        out = self._new(N, H, W, Cout)
        gn_in2 = tape is None and drop is None and self._img_gn_ok([h1], Cout, gn2)
        fused = None if gn_in2 else self._gn_apply_small([h1], gn2, True, drop)
        st2 = None if gn_in2 else fused[0] if fused else self._gn([h1], gn2)
        if gn_in2:
            a2 = None
            self._conv([h1], conv2, K.TAPS3, H, W, Cout, pro=(L.PRO_GN_SILU, gn2.weight, gn2.bias, gn2.num_groups,
                                                              gn2.eps), bias=conv2.bias, resid=resid, out=out.t, stats=out)
        elif fused:
            a2 = fused[1]
            self._conv([a2], conv2, K.TAPS3, H, W, Cout, bias=conv2.bias, resid=resid, out=out.t, stats=out)
        elif tape is None and drop is None and self._halo_pro_ok([h1], Cout, st2):
            a2 = None
            self._conv([h1], conv2, K.TAPS3, H, W, Cout, pro=(L.PRO_AFFINE_SILU, st2[0], st2[1]), bias=conv2.bias,
                       resid=resid, out=out.t, stats=out)
        else:
            a2 = self._apply([h1], st2, silu=True, drop=drop)
            self._conv([a2], conv2, K.TAPS3, H, W, Cout, bias=conv2.bias, resid=resid, out=out.t, stats=out)
        st1 = (st1, a1)
        st2 = (st2, a2)
        if tape is not None:
            tape.append(("res", rb, srcs, h1, st1, st2, drop, out))
        return out

    def _attn_fwd(self, a, ab, tape):
        N, H, W, C = a.t.shape[0], a.H, a.W, a.C
        Lq = H * W
        heads = ab.num_heads
        hd = C // heads
        qkv = self._new(N, H, W, 3 * C)
        fused = self._gn_apply_small([a], ab.norm, False)
        if fused:
            st, an = fused
        else:
            st = self._gn([a], ab.norm)
            an = self._apply([a], st, silu=False)      # GroupNorm output (no SiLU in AttentionBlock, :86)
        self._conv([an], ab.qkv, K.TAPS1, H, W, 3 * C, bias=ab.qkv.bias, out=qkv.t)
        st = (st, an)
        o = self._new(N, H, W, C)
        lse = torch.empty(N * heads * Lq, dtype=torch.float32, device=self.device)
        K.attn_fwd(self.dt, qkv.t, 3 * C, N, Lq, heads, hd, o.t, C, lse)
        out = self._new(N, H, W, C)
        self._conv([o], ab.proj, K.TAPS1, H, W, C, bias=ab.proj.bias, resid=a.t, out=out.t, stats=out)
        if tape is not None:
            tape.append(("attn", ab, a, st, qkv, o, lse, out))
        return out

    # =========================================================================================
    def backward(self, tape, dout, x_requires_grad):
        # The flat gradient buffer is reused across steps when no parameter still holds a gradient view of
        # it (optimizer.zero_grad(set_to_none=True)); with gradient accumulation a fresh one is used.
        flat = getattr(self, "_flat", None)
        if flat is None or flat.device != dout.device or any(p.grad is not None for p in self.params):
            flat = torch.empty(self.gtotal, dtype=torch.float32, device=dout.device)
        self._flat = flat
        self.flat = flat
        self.daddvec = None
        self._dx = None
        gv = lambda p: self._gview(flat, p)  # noqa: E731
        dx = None
        hook = self.grad_hook
        self._gn_defer = [] if _GN_DEFER else None
        if _WG_DEFER:
            if getattr(self, "_wg_arena", None) is None:
                self._wg_arena = K.WgradDefer()
            self._wg_arena.reset()      # nothing left over from a backward that raised part-way
            self._wg_defer = self._wg_arena
        if hook is not None:
            order = sorted(range(len(self.params)), key=lambda i: self.goff[i])
            final = [False] * len(self.params)
            cursor = 0
        recs = list(reversed(tape))
        # the time-embedding backward needs only the accumulated daddvec (complete after the last ResidualBlock):
        # run it before the input conv's, so its gradients (and all but the input conv's) are final earlier
        ti = next(i for i, r in enumerate(recs) if r[0] == "temb")
        ci = next(i for i, r in enumerate(recs) if r[0] == "conv_in")
        if ci < ti:
            recs.insert(ci, recs.pop(ti))
        try:
            for ri, rec in enumerate(recs):
                kind = rec[0]
                last = ri == len(recs) - 1
                self._backward_record(rec, dout, gv)
                if kind == "conv_in" and rec[3]:
                    dx = self._dx
                if hook is not None:
                    # this record's grads are final: publish the finished prefix of the flat buffer
                    for p in self._record_params(rec):
                        final[self.pindex[id(p)]] = True
                    while cursor < len(order) and final[order[cursor]]:
                        cursor += 1
                    hi = self.goff[order[cursor]] if cursor < len(order) else self.gtotal
                    if getattr(hook, "wants", None) is None or hook.wants(hi, last):
                        self._flush_gn()       # the deferred GroupNorm parameter sums and weight-gradient reductions
                    hook(flat, hi, last)
            self._flush_gn()
        except BaseException:
            if self._wg_defer is not None:
                self._wg_defer.reset()  # unflushed jobs point at buffers the caller may free or reuse
            raise
        finally:
            self._gn_defer = None
            self._wg_defer = None
        self.daddvec = None
        grads = [self._gview(flat, p) for p in self.params]
        return dx, grads

    def _record_params(self, rec):
        kind = rec[0]
        m = self.m
        if kind == "out":
            return list(m.output.parameters())
        if kind == "res":
            rb = rec[1]
            skip = {id(p) for p in rb.time_mlp.parameters()}
            if rb.label_proj is not None:
                skip |= {id(p) for p in rb.label_proj.parameters()}
            return [p for p in rb.parameters() if id(p) not in skip]
        if kind in ("attn", "down", "up"):
            return list(rec[1].parameters())
        if kind == "conv_in":
            return list(m.input_conv.parameters())
        # temb: the time embedding MLP, the label embedding and every block's time_mlp / label_proj
        ps = list(m.time_embed.parameters())
        if m.label_embed is not None:
            ps += list(m.label_embed.parameters())
        for rb in self.res_blocks:
            ps += list(rb.time_mlp.parameters())
            if rb.label_proj is not None:
                ps += list(rb.label_proj.parameters())
        return ps

    def _backward_record(self, rec, dout, gv):
        m = self.m
        dt = self.dt
        f32 = torch.float32
        kind = rec[0]
        if True:
            if kind == "out":
                _, h, (sc, sh, mr), ao = rec
                gno, convo = m.output[0], m.output[2]
                N, H, W = h.t.shape[0], h.H, h.W
                Co = m.out_channels
                ldo = (Co + self.chunk - 1) // self.chunk * self.chunk
                dy = K.pack_input(dt, dout.contiguous(), ldo)
                self._wgrad([ao], dy, ldo, K.TAPS3, H, W, Co, gv(convo.weight), dbias=gv(convo.bias))
                g = torch.empty(N, H, W, h.C, dtype=dt, device=dout.device)
                dya = Act(dy, H, W, Co)
                self._conv([dya], convo, K.TAPS3_DGRAD, H, W, h.C, out=g, packmode=L.PACK_DGRAD,
                           Kc=L.kc_for(Co, dt))
                buf, acc = self._grad_target(h)
                self._gn_bwd(dt, g, h.C, h.t, None, N, H * W, h.C, 0, h.t.shape[-1], 0, gno.num_groups, mr, gno.weight,
                         gno.bias, True, None, buf, None, h.C, 0, acc, 0, gv(gno.weight), gv(gno.bias))
            elif kind == "res":
                self._res_bwd(rec, gv)
            elif kind == "attn":
                self._attn_bwd(rec, gv)
            elif kind == "down":
                _, layer, a, out = rec
                N = a.t.shape[0]
                dy = out.grad
                self._wgrad([a], dy, out.C, K.TAPS3, out.H, out.W, out.C, gv(layer.conv.weight), stride=2,
                            dbias=gv(layer.conv.bias))
                buf, acc = self._grad_target(a)
                dya = Act(dy, out.H, out.W, out.C)
                self._conv([dya], layer.conv, K.TAPS3_DGRAD, a.H, a.W, a.C, mode=L.MODE_DILATE,
                           out=buf, resid=buf if acc else None, packmode=L.PACK_DGRAD)
            elif kind == "up":
                _, layer, a, out = rec
                N = a.t.shape[0]
                dy = out.grad
                if dt == torch.bfloat16:
                    # weight gradient over the materialised nearest-x2 input: the halo wgrad kernel (x halo
                    # in LDS for all 9 taps) on it is ~4x faster than the strided upsample-mode kernel,
                    # and the 2x2 replication costs one streaming pass
                    up = K.upsample2x(dt, a.t, a.t.shape[-1])
                    self._wgrad([Act(up, 2 * a.H, 2 * a.W, a.C)], dy, out.C, K.TAPS3, out.H, out.W, out.C,
                                gv(layer.conv.weight), dbias=gv(layer.conv.bias))
                else:
                    self._wgrad([a], dy, out.C, K.TAPS3, out.H, out.W, out.C, gv(layer.conv.weight),
                                mode=L.MODE_UPSAMPLE, dbias=gv(layer.conv.bias))
                buf, acc = self._grad_target(a)
                dya = Act(dy, out.H, out.W, out.C)
                self._conv([dya], layer.conv, K.TAPS_UPDGRAD, a.H, a.W, a.C, stride=2, out=buf,
                           resid=buf if acc else None, packmode=L.PACK_UPDGRAD)
            elif kind == "conv_in":
                _, xin, h, xg = rec
                N = h.t.shape[0]
                dy = h.grad
                conv = m.input_conv
                self._wgrad([xin], dy, h.C, K.TAPS3, h.H, h.W, h.C, gv(conv.weight), dbias=gv(conv.bias))
                if xg:
                    ldx = xin.t.shape[-1]
                    g = torch.empty(N, h.H, h.W, ldx, dtype=dt, device=dout.device)
                    self._conv([Act(dy, h.H, h.W, h.C)], conv, K.TAPS3_DGRAD, h.H, h.W, xin.C, out=g,
                               packmode=L.PACK_DGRAD)
                    self._dx = K.unpack_output(dt, g, ldx, N, xin.C, h.H, h.W)
            elif kind == "temb":
                self._temb_bwd(rec, self.daddvec, gv)

    def _res_bwd(self, rec, gv):
        _, rb, srcs, h1, (st1, a1), (st2, a2), drop, out = rec
        dt = self.dt
        a = srcs[0]
        N, H, W = a.t.shape[0], a.H, a.W
        Cout = rb.out_channels
        C1 = a.C
        C2 = srcs[1].C if len(srcs) > 1 else 0
        gn1, conv1, gn2, conv2 = rb.conv1[0], rb.conv1[2], rb.conv2[0], rb.conv2[3]
        dout = out.grad
        HW = H * W
        short_add = None   # an identity-shortcut gradient left for the GN1 backward to add (below)
        # conv2 (weight, bias) and its input gradient; a2 = dropout(SiLU(GN2(h1))) was kept from forward
        self._wgrad([a2], dout, Cout, K.TAPS3, H, W, Cout, gv(conv2.weight), dbias=gv(conv2.bias))
        g2 = torch.empty(N, H, W, Cout, dtype=dt, device=dout.device)
        self._conv([Act(dout, H, W, Cout)], conv2, K.TAPS3_DGRAD, H, W, Cout, out=g2, packmode=L.PACK_DGRAD)
        # shortcut
        if isinstance(rb.shortcut, torch.nn.Conv2d):
            sc = rb.shortcut
            self._wgrad(srcs, dout, Cout, K.TAPS1, H, W, Cout, gv(sc.weight), dbias=gv(sc.bias))
            if len(srcs) == 1:
                buf, acc = self._grad_target(a)
                self._conv([Act(dout, H, W, Cout)], sc, K.TAPS1, H, W, C1, out=buf, resid=buf if acc else None,
                           packmode=L.PACK_DGRAD)
            else:
                b = srcs[1]
                b1, acc1 = self._grad_target(a)
                b2, acc2 = self._grad_target(b)
                if acc1 or acc2:
                    # rare: pre-existing gradient on a concat source; go through a temporary
                    tmp = torch.empty(N, H, W, C1 + C2, dtype=dt, device=dout.device)
                    self._conv([Act(dout, H, W, Cout)], sc, K.TAPS1, H, W, C1 + C2, out=tmp, packmode=L.PACK_DGRAD)
                    self._scatter_add_concat(tmp, b1, acc1, b2, acc2, C1, C2)
                else:
                    self._conv([Act(dout, H, W, Cout)], sc, K.TAPS1, H, W, C1 + C2, packmode=L.PACK_DGRAD,
                               split=((b1, C1), (b2, C2), C1))
        else:
            if a.grad is None:
                a.grad = dout          # identity shortcut: alias (dout is dead after this block)
            elif len(srcs) == 1:
                # a.grad already holds a skip connection's gradient: the identity-shortcut gradient is added by the
                # GroupNorm backward below, which accumulates into a.grad anyway (round 6: one HBM pass fewer)
                short_add = dout
            else:
                K.add_(dt, a.grad, dout)
        # GN2 + SiLU + dropout backward -> dh1, with its pixel sums fused in: per (n, c) -> the time-embedding
        # add's gradient (daddvec slice), per c -> conv1's bias gradient
        off = self.temb_off[id(rb)]
        if self.daddvec is None:
            self.daddvec = torch.empty(N, self.temb_total, dtype=torch.float32, device=dout.device)
        dh1 = torch.empty(N, H, W, Cout, dtype=dt, device=dout.device)
        self._gn_bwd(dt, g2, Cout, h1.t, None, N, HW, Cout, 0, Cout, 0, gn2.num_groups, st2[2], gn2.weight, gn2.bias, True,
                 drop, dh1, None, Cout, 0, 0, 0, gv(gn2.weight), gv(gn2.bias), dx_sum_nc=self.daddvec[:, off:],
                 ld_sum_nc=self.temb_total, dx_sum_c=gv(conv1.bias))
        # conv1
        self._wgrad([a1], dh1, Cout, K.TAPS3, H, W, Cout, gv(conv1.weight))
        g1 = torch.empty(N, H, W, C1 + C2, dtype=dt, device=dout.device)
        x2 = srcs[1].t if len(srcs) > 1 else None
        self._conv([Act(dh1, H, W, Cout)], conv1, K.TAPS3_DGRAD, H, W, C1 + C2, out=g1, packmode=L.PACK_DGRAD)
        b1, acc1 = self._grad_target(a)
        if len(srcs) > 1:
            b2, acc2 = self._grad_target(srcs[1])
            ld2 = srcs[1].t.shape[-1]
        else:
            b2, acc2, ld2 = None, 0, 0
        self._gn_bwd(dt, g1, C1 + C2, a.t, srcs[1].t if len(srcs) > 1 else None, N, HW, C1, C2, a.t.shape[-1], ld2,
                 gn1.num_groups, st1[2], gn1.weight, gn1.bias, True, None, b1, b2, a.t.shape[-1], ld2, acc1, acc2,
                 gv(gn1.weight), gv(gn1.bias), add1=short_add, ld_add1=Cout if short_add is not None else 0)

    def _gn_bwd(self, *a, **kw):
        """K.gn_bwd with its parameter column sums (dgamma / dbeta / the bias sums) deferred to one batched launch
        per gradient segment (_flush_gn) -- 25 launches of ~4.7 us per B=128 training step became one."""
        return K.gn_bwd(*a, defer=getattr(self, "_gn_defer", None), **kw)

    def _flush_gn(self):
        if getattr(self, "_gn_defer", None):
            K.colsum_batch(self._gn_defer)
        if getattr(self, "_wg_defer", None) is not None:
            self._wg_defer.end_segment()

    def _scatter_add_concat(self, tmp, b1, acc1, b2, acc2, C1, C2):
        t1 = tmp[..., :C1].contiguous()
        t2 = tmp[..., C1:].contiguous()
        if acc1:
            K.add_(self.dt, b1, t1)
        else:
            b1.copy_(t1)
        if acc2:
            K.add_(self.dt, b2, t2)
        else:
            b2.copy_(t2)

    def _attn_bwd(self, rec, gv):
        _, ab, a, (st, an), qkv, o, lse, out = rec
        dt = self.dt
        N, H, W, C = a.t.shape[0], a.H, a.W, a.C
        HW = H * W
        heads = ab.num_heads
        hd = C // heads
        dout = out.grad
        # proj
        self._wgrad([o], dout, C, K.TAPS1, H, W, C, gv(ab.proj.weight), dbias=gv(ab.proj.bias))
        do = torch.empty(N, H, W, C, dtype=dt, device=dout.device)
        self._conv([Act(dout, H, W, C)], ab.proj, K.TAPS1, H, W, C, out=do, packmode=L.PACK_DGRAD)
        # residual: x gets dout
        if a.grad is None:
            a.grad = dout
        else:
            K.add_(dt, a.grad, dout)
        dqkv = torch.empty(N, H, W, 3 * C, dtype=dt, device=dout.device)
        K.attn_bwd(dt, qkv.t, 3 * C, o.t, do, C, lse, N, HW, heads, hd, dqkv, 3 * C)
        self._wgrad([an], dqkv, 3 * C, K.TAPS1, H, W, 3 * C, gv(ab.qkv.weight), dbias=gv(ab.qkv.bias))
        g = torch.empty(N, H, W, C, dtype=dt, device=dout.device)
        self._conv([Act(dqkv, H, W, 3 * C)], ab.qkv, K.TAPS1, H, W, C, out=g, packmode=L.PACK_DGRAD)
        self._gn_bwd(dt, g, C, a.t, None, N, HW, C, 0, C, 0, ab.norm.num_groups, st[2], ab.norm.weight, ab.norm.bias,
                 False, None, a.grad, None, C, 0, 1, 0, gv(ab.norm.weight), gv(ab.norm.bias))

    def _temb_bwd(self, rec, daddvec, gv):
        _, t, y, A0, A1, A2, Ay, addvec = rec
        m = self.m
        f32 = torch.float32
        te = m.time_embed
        N = daddvec.shape[0]
        tdim = A2.C
        T = self.temb_total
        dA = Act(daddvec.view(N, 1, 1, T), 1, 1, T)
        # stacked projection weights: dW[sumC][dim] -> the per-block slices are contiguous rows
        flat = self.flat
        dw_t = flat[self.temb_w_off:self.temb_w_off + T * tdim]
        self._wgrad([A2], daddvec, T, K.TAPS1, 1, 1, T, dw_t, pro=(L.PRO_SILU, None, None), dtype=f32,
                    dbias=flat[self.temb_b_off:self.temb_b_off + T])
        # d(silu(e2)) * silu'(e2) -> de2 (fused in the dgrad epilogue)
        de2 = torch.empty(N, 1, 1, tdim, dtype=f32, device=daddvec.device)
        self._conv([dA], None, K.TAPS1, 1, 1, tdim, out=de2, dtype=f32, w=self._temb_pack_dgrad(0),
                   Kc=L.kc_for(T, f32), silu_pre=A2.t, ld_silu=tdim)
        if Ay is not None:
            dw_l = flat[self.temb_l_off:self.temb_l_off + T * tdim]
            self._wgrad([Ay], daddvec, T, K.TAPS1, 1, 1, T, dw_l, pro=(L.PRO_SILU, None, None), dtype=f32)
            dye = torch.empty(N, 1, 1, tdim, dtype=f32, device=daddvec.device)
            self._conv([dA], None, K.TAPS1, 1, 1, tdim, out=dye, dtype=f32, w=self._temb_pack_dgrad(1),
                       Kc=L.kc_for(T, f32), silu_pre=Ay.t, ld_silu=tdim)
            K.embed_bwd(y, m.label_embed.weight.shape[0], dye.view(N, tdim), gv(m.label_embed.weight))
        # Linear2 (te[3]) on silu(e1)
        self._wgrad([A1], de2, tdim, K.TAPS1, 1, 1, tdim, gv(te[3].weight), pro=(L.PRO_SILU, None, None), dtype=f32,
                    dbias=gv(te[3].bias))
        de1 = torch.empty(N, 1, 1, tdim, dtype=f32, device=daddvec.device)
        self._conv([Act(de2, 1, 1, tdim)], te[3], K.TAPS1, 1, 1, tdim, out=de1, dtype=f32, packmode=L.PACK_DGRAD,
                   silu_pre=A1.t, ld_silu=tdim)
        # Linear1 (te[1]) on the sinusoid
        self._wgrad([A0], de1, tdim, K.TAPS1, 1, 1, tdim, gv(te[1].weight), dtype=f32, dbias=gv(te[1].bias))


class _UNetFunction(torch.autograd.Function):
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


def count_forward_flops(model) -> float:
    """2*MACs per image of the convs, linears and attention matmuls of one forward (for rooflines)."""
    flops = 0.0
    H, W = model.image_size
    mc = model.model_channels
    te = model.time_embed
    flops += 2 * (te[1].in_features * te[1].out_features + te[3].in_features * te[3].out_features)
    nres = 0

    def conv(cin, cout, h, w, k):
        return 2.0 * cin * cout * h * w * k * k

    flops += conv(model.in_channels, mc, H, W, 3)
    h, w = H, W
    chans = []

    def res(rb, h, w):
        f = conv(rb.in_channels, rb.out_channels, h, w, 3) + conv(rb.out_channels, rb.out_channels, h, w, 3)
        if rb.in_channels != rb.out_channels:
            f += conv(rb.in_channels, rb.out_channels, h, w, 1)
        f += 2 * rb.time_mlp[1].in_features * rb.out_channels
        return f

    def attn(ab, C, h, w):
        Lq = h * w
        return conv(C, 3 * C, h, w, 1) + conv(C, C, h, w, 1) + 2 * 2.0 * Lq * Lq * C

    for block in model.down_blocks:
        for layer in block:
            n = type(layer).__name__
            if n == "ResidualBlock":
                flops += res(layer, h, w)
                nres += 1
                C = layer.out_channels
            elif n == "AttentionBlock":
                flops += attn(layer, C, h, w)
            elif n == "Downsample":
                flops += conv(C, C, h // 2, w // 2, 3)
                h, w = h // 2, w // 2
        chans.append(C)
    for layer in model.middle_block:
        n = type(layer).__name__
        if n == "ResidualBlock":
            flops += res(layer, h, w)
        elif n == "AttentionBlock":
            flops += attn(layer, C, h, w)
    for block in model.up_blocks:
        for layer in block:
            n = type(layer).__name__
            if n == "ResidualBlock":
                flops += res(layer, h, w)
                C = layer.out_channels
            elif n == "AttentionBlock":
                flops += attn(layer, C, h, w)
            elif n == "Upsample":
                h, w = 2 * h, 2 * w
                flops += conv(C, C, h, w, 3)
    flops += conv(model.output[2].in_channels, model.out_channels, H, W, 3)
    return flops
