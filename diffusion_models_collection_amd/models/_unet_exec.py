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
from typing import List, Optional

import torch

from .. import _lib as L
from .. import kernels as K


class Act:
    """An NHWC activation [N, H, W, C] (contiguous, pitch C) plus its gradient buffer."""

    __slots__ = ("t", "H", "W", "C", "grad", "part", "fin")

    def __init__(self, t, H, W, C):
        self.t, self.H, self.W, self.C = t, H, W, C
        self.grad = None
        self.part = None    # GroupNorm partials written by the conv that produced t (dmc_conv_desc.gn_part)
        self.fin = None     # (GroupNorm, concat partner, (scale, shift, mean_rstd)) finalised by that conv (gn_fin)


# GroupNorm statistics from the conv epilogues (A/B: DMC_GN_PARTIALS=0 computes them with dmc_gn_stats passes)
_GN_PARTIALS = os.environ.get("DMC_GN_PARTIALS", "1") not in ("", "0")
# GroupNorm-backward sums from the input-gradient convs' epilogues (opt-in, DMC_GNB_PARTIALS=1). Measured on the
# B=128 train step: the dz recompute (sigmoid, dropout hash) in the MFMA kernels' epilogue costs what the removed
# gn_bwd_one / gn_bwd_partial passes saved (halo2 <7,3> 56 -> 66 us; train 8253 vs 8284 img/s, 8256 vs 8290)
_GNB_PARTIALS = _GN_PARTIALS and os.environ.get("DMC_GNB_PARTIALS", "0") not in ("", "0")
_GNB_DROP = os.environ.get("DMC_GNB_DROP", "1") not in ("", "0")   # ... also at the dropout sites
# The next GroupNorm's statistics finalised by the conv that produces its input (dmc_gn_fin: the producing launch's
# last block per image combines the epilogue partials) instead of a dmc_gn_finalize launch. Opt-in (DMC_GN_FIN=1):
# measured slower on MI355X (same box, B=128: train 8595 vs 8684 img/s, DDIM-50 621 vs 646) -- every block drains
# its stores before its arrival add, and the image's last block runs the combine on the kernel's critical path
_GN_FIN = _GN_PARTIALS and os.environ.get("DMC_GN_FIN", "0") not in ("", "0")

# GroupNorm statistics from epilogue partials finalised inside the apply launch (dmc_gn_apply_fin: each block
# combines its image's partials while its first rows load) instead of a dmc_gn_finalize launch before it. Opt-in
# (DMC_GN_APPLY_FIN=1): measured slower on MI355X (same box, B=128, 2 reps: train 8418/8470 vs 8648/8693 img/s,
# DDIM-50 599 vs 629; with the halo prologue off 558 vs 618) -- the 2048 blocks of an apply each repeat the
# per-image combine on their own critical path. A second form (partials loaded ahead of the rows, every group
# combined in one pass of 64/LG groups per wave) measured the same: train 8904/8898 vs 9140/9169, DDIM-50 649/646
# vs 676/672 (profiles/r4_ab_gemm_gn.txt).
_GN_APPLY_FIN = _GN_PARTIALS and os.environ.get("DMC_GN_APPLY_FIN", "0") not in ("", "0")
# The GroupNorm backward's parameter column sums deferred to one dmc_colsum_batch per gradient segment (A/B switch
# DMC_GN_DEFER=0: one finish launch per GroupNorm)
_GN_DEFER = os.environ.get("DMC_GN_DEFER", "1") not in ("", "0")
# Inference: the GroupNorm-prologue halo conv can combine the GroupNorm statistics itself from the producing convs'
# partials (dmc_conv_desc prologue DMC_PRO_GN_SILU, bitwise the finalize path), so those GroupNorms need no finalize
# launch. Opt-in (DMC_PRO_PART=1): every block combining its chunk's groups with the 64-lane tree costs more than the
# launch it saves -- DDIM-50 623/624 vs 666/673 img/s, CFG 370/371 vs 410/410 (profiles/r4_ab_gemm_gn.txt, r4ab16)
_PRO_PART = _GN_PARTIALS and os.environ.get("DMC_PRO_PART", "0") not in ("", "0")


class GnSt:
    """GroupNorm statistics (scale, shift, mean_rstd) of one site, computed lazily from the producing convs'
    partials: the apply that materialises the normalised activation finalises them in its own launch
    (K.gn_apply_fin); a consumer that needs them earlier (a conv prologue) triggers dmc_gn_finalize. Indexes and
    unpacks like the (scale, shift, mean_rstd) tuple of the other paths."""

    __slots__ = ("args", "bufs", "done")

    def __init__(self, args, N, C, G, dev):
        self.args = args          # (p1, C1, p2, C2, N, HW, G, eps, gamma, beta)
        self.bufs = (torch.empty(N * C, dtype=torch.float32, device=dev),
                     torch.empty(N * C, dtype=torch.float32, device=dev),
                     torch.empty(N * G * 2, dtype=torch.float32, device=dev))
        self.done = False

    def realize(self):
        if not self.done:
            K.gn_finalize(*self.args, out=self.bufs)
            self.done = True
        return self.bufs

    def __getitem__(self, i):
        return self.realize()[i]

    def __iter__(self):
        return iter(self.realize())

    def __len__(self):
        return 3


class GnbReq:
    """A request for the GroupNorm-backward sums from an input-gradient conv (ExecCore._gnb_epi): epi is the
    include/dmc.h dmc_gn_bwd_epi, part the sums; _conv sets part to None when its kernel would not fuse them."""

    def __init__(self, epi, part):
        self.epi, self.part = epi, part


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
        self.owner = owner
        self.entries = {}
        self._batch = None

    def _ver(self, srcs):
        return (self.owner.wgen,) + tuple((s._version, s.data_ptr()) for s in srcs)

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
    buffer. Subclasses set self.dt, self.packs, self.device, self.training_grad_scale, self.pindex, self.goff."""

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
              act=L.ACT_NONE, y_pre=None, stats=None, gnb=None, fin=None):
        """Generic implicit-GEMM conv over 1-2 NHWC sources. pro = (kind, scale, shift). stats = the output Act:
        in bf16 mode it gets the GroupNorm partials of the stored output (the next GroupNorm then needs no
        statistics pass over it, see _gn). gnb = the dmc_gn_bwd_epi from _gnb_epi when the output is the gradient
        a GroupNorm backward consumes: the conv also writes that backward's reduction sums. fin = (GroupNorm, concat
        partner Act or None) that reads this output next: where the kernel allows, the conv also finalises that
        GroupNorm's statistics (_attach_fin)."""
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
        if pro is not None and pro[0] == L.PRO_GN_SILU:
            gn = pro[3]
            K.set_prologue_gn(d, pro[1], pro[2], gn.num_groups, gn.eps, gn.weight, gn.bias)
        elif pro is not None:
            K.set_prologue(d, pro[0], pro[1], pro[2], C1 + C2, drop, C1 + C2)
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
        if fin is not None and gn_part is not None:
            self._attach_fin(d, fin, stats, N, OH * OW, Cout)
        if gnb is not None:
            if K.conv_fused(d) & L.FUSED_GN_BWD:
                d.gnb = ctypes.addressof(gnb.epi)
                d._keep_gnb = gnb
            else:
                gnb.part = None
        K.conv(d, a.t, srcs[1].t if len(srcs) > 1 else None, w, y1, y2)
        return d

    def _fin_counters(self, N):
        """A fresh set of N zeroed arrival counters for one gn_fin launch: slices of one buffer zeroed per forward
        (one fill launch; captured into the step's graph like every other launch)."""
        buf, i = self._fin_state
        if buf is None or (i + 1) * N > buf.numel():
            buf, i = torch.zeros(64 * N, dtype=torch.int32, device=self.device), 0
        self._fin_state = (buf, i + 1)
        return buf[i * N:(i + 1) * N]

    def _attach_fin(self, d, fin, out, N, HW, Cout):
        """Let the conv described by d finalise GroupNorm gn over [out | partner] (include/dmc.h dmc_gn_fin): out.fin
        then holds (gn, partner, (scale, shift, mean_rstd)) for _gn. Skipped (the finalize launch stays) where the
        kernel does not emit the partials or the group layout / partner partials do not allow it."""
        gn, partner = fin
        if not _GN_FIN or self.dt != torch.bfloat16:
            return
        C2 = partner.C if partner is not None else 0
        C, G = Cout + C2, gn.num_groups
        if C % G or (C // G) % 8 or C2 % 8 or (partner is not None and (partner.part is None or
                                                                          partner.H * partner.W != HW)):
            return
        if not K.conv_fused(d) & L.FUSED_GN_FIN:
            return
        dev = self.device
        mr = torch.empty(N * G * 2, dtype=torch.float32, device=dev)
        sc = torch.empty(N * C, dtype=torch.float32, device=dev)
        sh = torch.empty(N * C, dtype=torch.float32, device=dev)
        f = L.GnFin()
        ctr = self._fin_counters(N)
        f.counters, f.part2, f.C2, f.G, f.eps = ctr.data_ptr(), L.ptr(partner.part if partner else None), C2, G, gn.eps
        f.gamma, f.beta = L.ptr(gn.weight), L.ptr(gn.bias)
        f.mean_rstd, f.scale, f.shift = mr.data_ptr(), sc.data_ptr(), sh.data_ptr()
        d.gn_fin = ctypes.addressof(f)
        d._keep_fin = (f, ctr, partner)
        out.fin = (gn, partner, (sc, sh, mr))

    def _gnb_epi(self, x1, x2, C1, C2, ld1, ld2, mr, gn, silu, drop, N, HW):
        """(dmc_gn_bwd_epi, partials) for the input-gradient conv whose output g feeds gn_bwd over x = [x1 | x2]:
        the conv's epilogue (or one pass over g where its kernel cannot) writes gn_bwd's per-(64-pixel segment,
        channel) sums, so gn_bwd skips its reduction pass. None where gn_bwd reduces by itself; _conv also drops
        the request (req.part = None) where its kernel would need an extra pass for them."""
        C, G = C1 + C2, gn.num_groups
        if not (_GNB_PARTIALS and self.dt == torch.bfloat16 and HW % 64 == 0 and C % 8 == 0 and (C // G) % 8 == 0
                and (drop is None or _GNB_DROP)):
            return None
        return GnbReq(*K.gn_bwd_epi(x1, x2, C1, ld1, ld2, mr, gn.weight, gn.bias, G, silu, drop, N * HW, C))

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
        K.wgrad(d, dy, ld_dy, a.t, srcs[1].t if len(srcs) > 1 else None, dw, self.training_grad_scale, dbias=dbias)

    def _new(self, N, H, W, C, dtype=None):
        return Act(torch.empty(N, H, W, C, dtype=dtype or self.dt, device=self.device), H, W, C)



class UNetExecutor(ExecCore):
    def __init__(self, model):
        self.m = model
        self.dt = model.compute_dtype
        self.cdt = L.dtype_code(self.dt)
        self.chunk = L.chunk_for(self.dt)
        self._halo_pro_cache = {}   # shape -> dmc_conv_halo_prologue verdict
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
        # measured slower on MI355X (the overlapped kernels contend for LDS and CUs): opt-in only
        self.use_side = os.environ.get("DMC_SIDE_STREAM", "0") not in ("", "0")
        # DMC_SIDE_MAXHW > 0: only weight gradients on maps of at most that many pixels go to the side stream (the
        # 8x8 / 4x4 levels, whose latency-bound launches leave most CUs idle)
        self.side_maxhw = int(os.environ.get("DMC_SIDE_MAXHW", "0"))
        self.side = None
        self._side_reads = {}
        self._fin_state = (None, 0)
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
    def _next_gn(self, i, hs):
        """(GroupNorm, concat partner) that reads the output of plan step i (the step after it: a ResidualBlock's
        first GroupNorm -- over [h, skip] in the up path -- or an AttentionBlock's; the output GroupNorm after the
        last step), or None (a Down/Upsample conv reads it)."""
        if i + 1 >= len(self.plan):
            return (self.m.output[0], None)
        layer, cat, _ = self.plan[i + 1]
        name = type(layer).__name__
        if name == "ResidualBlock":
            return (layer.conv1[0], hs[-1] if cat else None)
        if name == "AttentionBlock":
            return (layer.norm, None)
        return None

    def _gn(self, srcs, gn, dtype=None):
        dtype = dtype or self.dt
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        if a.fin is not None and a.fin[0] is gn and a.fin[1] is b:
            return a.fin[2]          # finalised by the conv that produced a (dmc_gn_fin)
        N = a.t.shape[0]
        C = a.C + (b.C if b else 0)
        if (all(s.part is not None for s in srcs) and (a.H * a.W) % 64 == 0 and C % gn.num_groups == 0
                and (C // gn.num_groups) % 8 == 0):
            # statistics from the producing convs' epilogue partials: no pass over the activation
            if _GN_APPLY_FIN and self.dt == torch.bfloat16 and gn.num_groups <= 64 and C <= 2048:
                return GnSt((a.part, a.C, b.part if b else None, b.C if b else 0, N, a.H * a.W, gn.num_groups,
                             gn.eps, gn.weight, gn.bias), N, C, gn.num_groups, a.t.device)
            return K.gn_finalize(a.part, a.C, b.part if b else None, b.C if b else 0, N, a.H * a.W, gn.num_groups,
                                 gn.eps, gn.weight, gn.bias)
        return K.gn_stats(dtype, a.t, b.t if b else None, N, a.H * a.W, a.C, b.C if b else 0, a.t.shape[-1],
                          b.t.shape[-1] if b else 0, gn.num_groups, gn.eps, gn.weight, gn.bias)

    def _apply(self, srcs, st, silu=True, drop=None):
        """Act of dropout(silu(GN(concat(srcs)))) materialised with dmc_gn_apply."""
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        N = a.t.shape[0]
        C = a.C + (b.C if b else 0)
        if isinstance(st, GnSt) and not st.done:
            p1, C1, p2, C2, _, HW, G, eps, gamma, beta = st.args
            out, _ = K.gn_apply_fin(self.dt, a.t, b.t if b else None, N, HW, C1, C2, a.t.shape[-1],
                                    b.t.shape[-1] if b else 0, p1, p2, G, eps, gamma, beta, silu=silu, drop=drop,
                                    stats=st.bufs)
            st.done = True
            return Act(out.view(N, a.H, a.W, C), a.H, a.W, C)
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
            if st is None:   # shape query only (_pro_gn): any valid pointers
                st = (torch.empty(N * (C1 + C2), dtype=torch.float32, device=a.t.device),) * 2
            bufs = st.bufs if isinstance(st, GnSt) else st     # pointers only: no statistics launch here
            K.set_prologue(d, L.PRO_AFFINE_SILU, bufs[0], bufs[1], C1 + C2)
            ok = self._halo_pro_cache[key] = K.conv_halo_prologue(d)
        return ok

    def _pro_gn(self, srcs, gn, Cout):
        """pro = (PRO_GN_SILU, partials of srcs, gn) when the GroupNorm-prologue halo conv of SiLU(gn(srcs)) can
        combine gn's statistics itself from the producing convs' partials (no finalize launch), else None."""
        if not _PRO_PART or self.dt != torch.bfloat16 or any(s.part is None for s in srcs):
            return None
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else None
        if a.fin is not None and a.fin[0] is gn:
            return None                      # finalised by the producing conv already
        C, G, HW = a.C + (b.C if b else 0), gn.num_groups, a.H * a.W
        if C % G or (C // G) % 8 or C // G < 16 or HW % 64 or (HW // 64) * (C // G // 8) > 128:
            return None
        if not self._halo_pro_ok(srcs, Cout, None):
            return None
        return (L.PRO_GN_SILU, a.part, b.part if b else None, gn)

    def _grad_target(self, act):
        """(buffer, accumulate) for writing a gradient contribution into act.grad."""
        if act.grad is None:
            act.grad = torch.empty_like(act.t)
            return act.grad, 0
        self._guard(act.grad)
        return act.grad, 1

    # ---- weight-gradient side stream --------------------------------------------------------
    # The backward has two chains per layer: the input-gradient chain (dgrad conv -> GroupNorm backward ->
    # next layer), which is the critical path, and the weight/bias gradients, which only the optimizer
    # needs. The latter run on a second HIP stream so they fill the CUs the latency-bound GroupNorm and
    # small-M kernels leave idle. Hazards: (1) a side kernel reads tensors the main stream may free
    # (record_stream) or later accumulate into (an aliased gradient buffer: _guard makes the main stream
    # wait for the side reads first); (2) the flat gradient buffer is complete only after a join.
    @contextlib.contextmanager
    def _side(self, *reads):
        if not self.use_side or (self.side_maxhw > 0 and reads[0].dim() == 4
                                 and reads[0].shape[1] * reads[0].shape[2] > self.side_maxhw):
            yield
            return
        main = torch.cuda.current_stream()
        if self.side is None or self.side.device != main.device:
            self.side = torch.cuda.Stream(device=main.device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            yield
        ev = torch.cuda.Event()
        ev.record(self.side)
        for t in reads:
            t.record_stream(self.side)
            self._side_reads[t.untyped_storage().data_ptr()] = ev

    def _guard(self, t):
        """The main stream is about to write `t` in place: wait for pending side-stream reads of it."""
        if self._side_reads:
            ev = self._side_reads.pop(t.untyped_storage().data_ptr(), None)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)

    def _join_side(self):
        if self.use_side and self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        self._side_reads = {}

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
        self._fin_state = (None, 0)
        self._conv([xin], m.input_conv, K.TAPS3, H, W, m.model_channels, bias=m.input_conv.bias, out=h.t, stats=h,
                   fin=self._next_gn(-1, [h]))
        if keep:
            tape.append(("conv_in", xin, h, x.requires_grad))
        hs = [h]
        for i, (layer, cat, push) in enumerate(self.plan):
            srcs = [h, hs.pop()] if cat else [h]
            h = self._layer(srcs, layer, tape, self._next_gn(i, hs))
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

    def _layer(self, srcs, layer, tape, fin=None):
        """One step of the plan; fin = (GroupNorm, partner) that reads its output next (see _next_gn)."""
        name = type(layer).__name__
        if name == "ResidualBlock":
            return self._res_fwd(srcs, layer, tape, fin)
        if name == "AttentionBlock":
            return self._attn_fwd(srcs[0], layer, tape, fin)
        if name == "Downsample":
            a = srcs[0]
            OH, OW = (a.H + 2 - 3) // 2 + 1, (a.W + 2 - 3) // 2 + 1
            out = self._new(a.t.shape[0], OH, OW, a.C)
            self._conv([a], layer.conv, K.TAPS3, OH, OW, a.C, stride=2, bias=layer.conv.bias, out=out.t, stats=out,
                       fin=fin)
            if tape is not None:
                tape.append(("down", layer, a, out))
            return out
        if name == "Upsample":
            a = srcs[0]
            out = self._new(a.t.shape[0], 2 * a.H, 2 * a.W, a.C)
            self._conv([a], layer.conv, K.TAPS3, 2 * a.H, 2 * a.W, a.C, mode=L.MODE_UPSAMPLE, bias=layer.conv.bias,
                       out=out.t, stats=out, fin=fin)
            if tape is not None:
                tape.append(("up", layer, a, out))
            return out
        raise TypeError(f"unexpected layer {name}")

    def _res_fwd(self, srcs, rb, tape, fin=None):
        a = srcs[0]
        N, H, W = a.t.shape[0], a.H, a.W
        Cout = rb.out_channels
        gn1, conv1, gn2, conv2 = rb.conv1[0], rb.conv1[2], rb.conv2[0], rb.conv2[3]
        # a1 = SiLU(GN1(x)) materialised once (the 3x3 implicit GEMM reads every pixel 9x; the weight
        # gradient re-reads it in backward). Inference (no tape): where the halo kernel takes the conv, it
        # applies GN+SiLU to its LDS-resident halo instead and nothing is materialised.
        pg1 = self._pro_gn(srcs, gn1, Cout) if tape is None else None
        st1 = None if pg1 is not None else self._gn(srcs, gn1)
        h1 = self._new(N, H, W, Cout)
        off = self.temb_off[id(rb)]
        if pg1 is not None:
            a1 = None
            self._conv(srcs, conv1, K.TAPS3, H, W, Cout, pro=pg1, bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t,
                       stats=h1, fin=(gn2, None))
        elif tape is None and self._halo_pro_ok(srcs, Cout, st1):
            a1 = None
            self._conv(srcs, conv1, K.TAPS3, H, W, Cout, pro=(L.PRO_AFFINE_SILU, st1[0], st1[1]), bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1,
                       fin=(gn2, None))
        else:
            a1 = self._apply(srcs, st1, silu=True)
            self._conv([a1], conv1, K.TAPS3, H, W, Cout, bias=conv1.bias,
                       addvec=self.addvec.view(self.addvec.shape[0], -1)[:, off:], ld_add=self._ld_add, out=h1.t, stats=h1,
                       fin=(gn2, None))
        pg2 = self._pro_gn([h1], gn2, Cout) if tape is None and self._drop is None else None
        st2 = None if pg2 is not None else self._gn([h1], gn2)
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
        if pg2 is not None:
            a2 = None
            self._conv([h1], conv2, K.TAPS3, H, W, Cout, pro=pg2, bias=conv2.bias, resid=resid, out=out.t,
                       stats=out, fin=fin)
        elif tape is None and drop is None and self._halo_pro_ok([h1], Cout, st2):
            a2 = None
            self._conv([h1], conv2, K.TAPS3, H, W, Cout, pro=(L.PRO_AFFINE_SILU, st2[0], st2[1]), bias=conv2.bias,
                       resid=resid, out=out.t, stats=out, fin=fin)
        else:
            a2 = self._apply([h1], st2, silu=True, drop=drop)
            self._conv([a2], conv2, K.TAPS3, H, W, Cout, bias=conv2.bias, resid=resid, out=out.t, stats=out, fin=fin)
        st1 = (st1, a1)
        st2 = (st2, a2)
        if tape is not None:
            tape.append(("res", rb, srcs, h1, st1, st2, drop, out))
        return out

    def _attn_fwd(self, a, ab, tape, fin=None):
        N, H, W, C = a.t.shape[0], a.H, a.W, a.C
        Lq = H * W
        heads = ab.num_heads
        hd = C // heads
        st = self._gn([a], ab.norm)
        qkv = self._new(N, H, W, 3 * C)
        an = self._apply([a], st, silu=False)          # GroupNorm output (no SiLU in AttentionBlock, :86)
        self._conv([an], ab.qkv, K.TAPS1, H, W, 3 * C, bias=ab.qkv.bias, out=qkv.t)
        st = (st, an)
        o = self._new(N, H, W, C)
        lse = torch.empty(N * heads * Lq, dtype=torch.float32, device=self.device)
        K.attn_fwd(self.dt, qkv.t, 3 * C, N, Lq, heads, hd, o.t, C, lse)
        out = self._new(N, H, W, C)
        self._conv([o], ab.proj, K.TAPS1, H, W, C, bias=ab.proj.bias, resid=a.t, out=out.t, stats=out, fin=fin)
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
                    self._flush_gn()       # the deferred GroupNorm parameter sums of that prefix
                    self._join_side()      # the side stream's weight gradients of that prefix are written
                hook(flat, hi, last)
        self._flush_gn()
        self._gn_defer = None
        self._join_side()
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
                with self._side(ao.t, dy):
                    self._wgrad([ao], dy, ldo, K.TAPS3, H, W, Co, gv(convo.weight), dbias=gv(convo.bias))
                g = torch.empty(N, H, W, h.C, dtype=dt, device=dout.device)
                dya = Act(dy, H, W, Co)
                gnb = self._gnb_epi(h.t, None, h.C, 0, h.t.shape[-1], 0, mr, gno, True, None, N, H * W)
                self._conv([dya], convo, K.TAPS3_DGRAD, H, W, h.C, out=g, packmode=L.PACK_DGRAD,
                           Kc=L.kc_for(Co, dt), gnb=gnb)
                buf, acc = self._grad_target(h)
                self._gn_bwd(dt, g, h.C, h.t, None, N, H * W, h.C, 0, h.t.shape[-1], 0, gno.num_groups, mr, gno.weight,
                         gno.bias, True, None, buf, None, h.C, 0, acc, 0, gv(gno.weight), gv(gno.bias),
                         part=gnb and gnb.part)
            elif kind == "res":
                self._res_bwd(rec, gv)
            elif kind == "attn":
                self._attn_bwd(rec, gv)
            elif kind == "down":
                _, layer, a, out = rec
                N = a.t.shape[0]
                dy = out.grad
                with self._side(a.t, dy):
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
                with self._side(a.t, dy):
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
                with self._side(xin.t, dy):
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
        # conv2 (weight, bias) and its input gradient; a2 = dropout(SiLU(GN2(h1))) was kept from forward
        with self._side(a2.t, dout):
            self._wgrad([a2], dout, Cout, K.TAPS3, H, W, Cout, gv(conv2.weight), dbias=gv(conv2.bias))
        g2 = torch.empty(N, H, W, Cout, dtype=dt, device=dout.device)
        gnb2 = self._gnb_epi(h1.t, None, Cout, 0, Cout, 0, st2[2], gn2, True, drop, N, HW)
        self._conv([Act(dout, H, W, Cout)], conv2, K.TAPS3_DGRAD, H, W, Cout, out=g2, packmode=L.PACK_DGRAD,
                   gnb=gnb2)
        # shortcut
        if isinstance(rb.shortcut, torch.nn.Conv2d):
            sc = rb.shortcut
            with self._side(*[x.t for x in srcs], dout):
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
            else:
                self._guard(a.grad)
                K.add_(dt, a.grad, dout)
        # GN2 + SiLU + dropout backward -> dh1, with its pixel sums fused in: per (n, c) -> the time-embedding
        # add's gradient (daddvec slice), per c -> conv1's bias gradient
        off = self.temb_off[id(rb)]
        if self.daddvec is None:
            self.daddvec = torch.empty(N, self.temb_total, dtype=torch.float32, device=dout.device)
        dh1 = torch.empty(N, H, W, Cout, dtype=dt, device=dout.device)
        self._gn_bwd(dt, g2, Cout, h1.t, None, N, HW, Cout, 0, Cout, 0, gn2.num_groups, st2[2], gn2.weight, gn2.bias, True,
                 drop, dh1, None, Cout, 0, 0, 0, gv(gn2.weight), gv(gn2.bias), dx_sum_nc=self.daddvec[:, off:],
                 ld_sum_nc=self.temb_total, dx_sum_c=gv(conv1.bias), part=gnb2 and gnb2.part)
        # conv1
        with self._side(a1.t, dh1):
            self._wgrad([a1], dh1, Cout, K.TAPS3, H, W, Cout, gv(conv1.weight))
        g1 = torch.empty(N, H, W, C1 + C2, dtype=dt, device=dout.device)
        x2 = srcs[1].t if len(srcs) > 1 else None
        gnb1 = self._gnb_epi(a.t, x2, C1, C2, a.t.shape[-1], 0 if x2 is None else x2.shape[-1], st1[2], gn1,
                                    True, None, N, HW)
        self._conv([Act(dh1, H, W, Cout)], conv1, K.TAPS3_DGRAD, H, W, C1 + C2, out=g1, packmode=L.PACK_DGRAD,
                   gnb=gnb1)
        b1, acc1 = self._grad_target(a)
        if len(srcs) > 1:
            b2, acc2 = self._grad_target(srcs[1])
            ld2 = srcs[1].t.shape[-1]
        else:
            b2, acc2, ld2 = None, 0, 0
        self._gn_bwd(dt, g1, C1 + C2, a.t, srcs[1].t if len(srcs) > 1 else None, N, HW, C1, C2, a.t.shape[-1], ld2,
                 gn1.num_groups, st1[2], gn1.weight, gn1.bias, True, None, b1, b2, a.t.shape[-1], ld2, acc1, acc2,
                 gv(gn1.weight), gv(gn1.bias), part=gnb1 and gnb1.part)

    def _gn_bwd(self, *a, **kw):
        """K.gn_bwd with its parameter column sums (dgamma / dbeta / the bias sums) deferred to one batched launch
        per gradient segment (_flush_gn) -- 25 launches of ~4.7 us per B=128 training step became one."""
        return K.gn_bwd(*a, defer=getattr(self, "_gn_defer", None), **kw)

    def _flush_gn(self):
        if getattr(self, "_gn_defer", None):
            K.colsum_batch(self._gn_defer)

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
        with self._side(o.t, dout):
            self._wgrad([o], dout, C, K.TAPS1, H, W, C, gv(ab.proj.weight), dbias=gv(ab.proj.bias))
        do = torch.empty(N, H, W, C, dtype=dt, device=dout.device)
        self._conv([Act(dout, H, W, C)], ab.proj, K.TAPS1, H, W, C, out=do, packmode=L.PACK_DGRAD)
        # residual: x gets dout
        if a.grad is None:
            a.grad = dout
        else:
            self._guard(a.grad)
            K.add_(dt, a.grad, dout)
        dqkv = torch.empty(N, H, W, 3 * C, dtype=dt, device=dout.device)
        K.attn_bwd(dt, qkv.t, 3 * C, o.t, do, C, lse, N, HW, heads, hd, dqkv, 3 * C)
        with self._side(an.t, dqkv):
            self._wgrad([an], dqkv, 3 * C, K.TAPS1, H, W, 3 * C, gv(ab.qkv.weight), dbias=gv(ab.qkv.bias))
        g = torch.empty(N, H, W, C, dtype=dt, device=dout.device)
        gnb = self._gnb_epi(a.t, None, C, 0, C, 0, st[2], ab.norm, False, None, N, HW)
        self._conv([Act(dqkv, H, W, 3 * C)], ab.qkv, K.TAPS1, H, W, C, out=g, packmode=L.PACK_DGRAD, gnb=gnb)
        self._gn_bwd(dt, g, C, a.t, None, N, HW, C, 0, C, 0, ab.norm.num_groups, st[2], ab.norm.weight, ab.norm.bias,
                 False, None, a.grad, None, C, 0, 1, 0, gv(ab.norm.weight), gv(ab.norm.bias), part=gnb and gnb.part)

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
