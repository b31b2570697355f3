"""Tensor-level wrappers over the C ABI (include/dmc.h).

Every function takes torch tensors that already live on the GPU, launches on torch's current stream
and returns without synchronising. Activations are NHWC tensors [N, H, W, ld] (ld = channel pitch).
No function here has a CPU or PyTorch-op fallback.
"""
import ctypes

import torch

from . import _lib as L
from ._lib import LIB, check, ptr

TAPS3 = [(kh - 1, kw - 1) for kh in range(3) for kw in range(3)]      # forward 3x3, pad 1
TAPS3_DGRAD = [(1 - kh, 1 - kw) for kh in range(3) for kw in range(3)]  # input-gradient of a 3x3 conv
TAPS1 = [(0, 0)]
TAPS_UPDGRAD = [(u - 1, v - 1) for u in range(4) for v in range(4)]    # folded nearest-x2 + 3x3 (4x4, s2)


class Scratch:
    """Grow-only device scratch (wgrad slabs, GN partials, ...), one buffer per HIP stream: kernels of one
    stream run in order and may share it; kernels on another stream (the executor's weight-gradient side
    stream) get their own. A buffer is allocated while its stream is current, so the caching allocator
    never hands it to another stream while its kernels are pending."""

    def __init__(self):
        self.bufs = {}

    def get(self, nbytes: int, device) -> torch.Tensor:
        nbytes = max(int(nbytes), 256)
        key = L.stream()   # stream handles are unique across devices
        buf = self.bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(int(nbytes * 1.25) + 4096, dtype=torch.uint8, device=device)
            self.bufs[key] = buf
        return buf


SCRATCH = Scratch()


def make_desc(dtype, N, H, W, C1, C2, ld1, ld2, Kc, OH, OW, Cout, taps, mode=L.MODE_NORMAL, stride=1):
    d = L.ConvDesc()
    d.dtype = L.dtype_code(dtype)
    d.N, d.H, d.W = N, H, W
    d.C1, d.C2, d.ld1, d.ld2, d.Kc = C1, C2, ld1, ld2, Kc
    d.OH, d.OW, d.Cout = OH, OW, Cout
    d.ntaps, d.mode, d.stride = len(taps), mode, stride
    for i, (dy, dx) in enumerate(taps):
        d.tap_dy[i] = dy
        d.tap_dx[i] = dx
    d.Csplit = Cout
    d.drop_scale = 1.0
    return d


def drop_args(drop):
    """(seed, seed_base, thresh, scale) of a dropout spec (seed, thresh, scale[, seed_base]): seed_base is the
    device address of a uint32 added to seed in the kernels (a graph-captured step reads its seed there)."""
    if drop is None:
        return 0, None, 0, 1.0
    return drop[0], (drop[3] if len(drop) > 3 else None), drop[1], drop[2]


def set_prologue(d, kind=L.PRO_NONE, scale=None, shift=None, ld=0, drop=None, drop_ld=0):
    d.prologue = kind
    d._keep_pro = (scale, shift)   # the descriptor holds raw pointers: keep the tensors alive with it
    d.pro_scale = ptr(scale)
    d.pro_shift = ptr(shift)
    d.ld_pro = ld
    d.drop_seed, d.drop_seed_base, d.drop_thresh, d.drop_scale = drop_args(drop)
    d.drop_ld = drop_ld if drop is not None else 0


def set_epilogue(d, bias=None, addvec=None, ld_add=0, resid=None, ld_res=0, silu_pre=None, ld_silu=0,
                 ldy1=0, ldy2=0, Csplit=None, out_f32=False, out_nchw=False, act=L.ACT_NONE, y_pre=None, ld_pre=0,
                 gn_part=None):
    d._keep_epi = (bias, addvec, resid, silu_pre, y_pre, gn_part)   # keep what the raw pointers point at alive
    d.gn_part = ptr(gn_part)
    d.act = act
    d.y_pre = ptr(y_pre)
    d.ld_pre = ld_pre
    d.bias = ptr(bias)
    d.addvec = ptr(addvec)
    d.ld_add = ld_add
    d.resid = ptr(resid)
    d.ld_res = ld_res
    d.silu_pre = ptr(silu_pre)
    d.ld_silu = ld_silu
    d.ldy1, d.ldy2 = ldy1, ldy2
    d.Csplit = d.Cout if Csplit is None else Csplit
    d.out_f32 = int(out_f32)
    d.out_nchw = int(out_nchw)


class LayerProfile:
    """Opt-in (DMC_LAYER_PROF=1) per-call timing of the conv launches, keyed by kind and shape: HIP events on
    the launch stream around each call, read back by report(). Measurement tooling only."""

    def __init__(self):
        import os
        self.on = os.environ.get("DMC_LAYER_PROF", "0") not in ("", "0")
        self.pending = []

    def wrap(self, kind, d, fn):
        if not self.on:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        M = d.N * d.OH * d.OW
        key = (kind, d.dtype, d.N, d.H, d.W, d.C1 + d.C2, d.OH, d.OW, d.Cout, d.ntaps, d.mode)
        self.pending.append((key, 2.0 * M * d.Cout * d.ntaps * (d.C1 + d.C2), e0, e1))

    def report(self, steps=1):
        torch.cuda.synchronize()
        agg = {}
        for key, fl, e0, e1 in self.pending:
            a = agg.setdefault(key, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += e0.elapsed_time(e1)
            a[2] += fl
        self.pending = []
        rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
        tot = sum(v[1] for v in agg.values())
        lines = [f"conv launches: {tot / steps:.3f} ms/step"]
        for (kind, dt, N, H, W, Cin, OH, OW, Cout, nt, mode), (n, ms, fl) in rows:
            lines.append(f"{ms / steps * 1e3:8.1f} us/step  n/step {n / steps:4.1f}  avg {ms / n * 1e3:7.1f} us  "
                         f"{fl / (ms * 1e-3) / 1e12:7.1f} TF/s  {kind:5s} N{N} {H}x{W}x{Cin} -> {OH}x{OW}x{Cout} "
                         f"taps {nt} mode {mode}")
        return "\n".join(lines)


PROF = LayerProfile()


def conv(d, x1, x2, w, y1, y2=None):
    nbytes = LIB.dmc_conv2d_workspace(ctypes.byref(d))
    ws = SCRATCH.get(nbytes, y1.device) if nbytes else None
    PROF.wrap("conv", d, lambda: check(LIB.dmc_conv2d(ctypes.byref(d), ptr(x1), ptr(x2), ptr(w), ptr(y1), ptr(y2),
                                                      ptr(ws), nbytes, L.stream()), "dmc_conv2d"))


def conv_fused(d):
    """include/dmc.h dmc_conv2d_fused_epilogue: which optional outputs (L.FUSED_*) the kernel dmc_conv2d would run
    for `d` (with the workspace conv() passes) produces in its epilogue."""
    return LIB.dmc_conv2d_fused_epilogue(ctypes.byref(d), LIB.dmc_conv2d_workspace(ctypes.byref(d)))


def upsample2x(dtype, x, C):
    """Nearest x2 upsample of an NHWC [N, H, W, ld] activation's first C channels -> [N, 2H, 2W, C]."""
    N, H, W, ld = x.shape
    y = torch.empty(N, 2 * H, 2 * W, C, dtype=x.dtype, device=x.device)
    check(LIB.dmc_upsample2x_nhwc(L.dtype_code(dtype), ptr(x), N, H, W, C, ld, ptr(y), C, L.stream()),
          "dmc_upsample2x_nhwc")
    return y


def conv_halo_prologue(d):
    """True when dmc_conv2d applies d's GN-affine+SiLU prologue on the halo kernel's resident halo."""
    return bool(LIB.dmc_conv_halo_prologue(ctypes.byref(d)))


class WgradDefer:
    """Weight-gradient reductions deferred and batched (wgrad(defer=...) -> dmc_wgrad_reduce_batch).

    Each deferred call's fp32 partial sums get their own slice of a grow-only device arena and stay there until
    flush() reduces every pending job (<= 32 per launch) and recycles the arena. flush() runs every `every` jobs
    (DMC_WG_FLUSH_EVERY, default 3: the slabs are still in the 256 MB Infinity Cache when they are read back;
    3 measured best of 1-8 and of flushing only at the backward's segment ends: train 10,421 vs 10,365 img/s) and
    at every gradient-segment end (end_segment). When the pending jobs outgrow the arena they are flushed early
    and a larger arena is allocated; every arena ever allocated stays referenced (a captured HIP graph keeps
    using its addresses)."""

    def __init__(self):
        import os
        self.every = int(os.environ.get("DMC_WG_FLUSH_EVERY", "3"))
        self.arenas = []
        self.buf = None
        self.off = 0
        self.jobs = []

    def alloc(self, nbytes, device):
        nbytes = (max(int(nbytes), 256) + 255) // 256 * 256
        if self.buf is None or self.buf.device != device or self.off + nbytes > self.buf.numel():
            need = nbytes if self.buf is None or self.buf.device != device else self.off + nbytes
            self.flush()
            if self.buf is None or self.buf.device != device or need > self.buf.numel():
                self.buf = torch.empty(int(need * 1.25), dtype=torch.uint8, device=device)
                self.arenas.append(self.buf)
        ws = self.buf[self.off:self.off + nbytes]
        self.off += nbytes
        return ws

    def add(self, job):
        if job.splits == 0:
            return              # reduced inside the kernel (dmc_conv2d_wgrad_partial wrote dw directly)
        self.jobs.append(job)
        if self.every and len(self.jobs) >= self.every:
            self.flush()

    def flush(self):
        for k in range(0, len(self.jobs), 32):
            chunk = self.jobs[k:k + 32]
            arr = (L.WgradJob * len(chunk))(*chunk)
            check(LIB.dmc_wgrad_reduce_batch(arr, len(chunk), L.stream()), "dmc_wgrad_reduce_batch")
        self.jobs = []
        self.off = 0

    def end_segment(self):
        self.flush()

    def reset(self):
        """Drop every pending job unreduced and recycle the arena. A backward starts with this: one that
        raised part-way (an OOM, a capture error the caller survived) leaves jobs holding raw slab / dw pointers that
        the next backward's first flush would otherwise replay onto reused buffers."""
        self.jobs = []
        self.off = 0


def wgrad(d, dy, ld_dy, x1, x2, dw, scale=1.0, dbias=None, defer=None):
    """dmc_conv2d_wgrad: dw (and with dbias the bias gradient, the pixel sums of dy) from one pass over dy. With
    defer (a WgradDefer) only the partial-sum kernel runs now (dmc_conv2d_wgrad_partial); the reduction joins
    defer's batch."""
    d.wg_bias = ptr(dbias)
    d._keep_wgb = dbias
    nbytes = LIB.dmc_conv2d_wgrad_workspace(ctypes.byref(d))
    if defer is not None:
        ws = defer.alloc(nbytes, dy.device)
        job = L.WgradJob()
        PROF.wrap("wgrad", d, lambda: check(LIB.dmc_conv2d_wgrad_partial(
            ctypes.byref(d), ptr(dy), ld_dy, ptr(x1), ptr(x2), ptr(ws), ptr(dw), scale, ctypes.byref(job), L.stream()),
            "dmc_conv2d_wgrad_partial"))
        defer.add(job)
        return
    ws = SCRATCH.get(nbytes, dy.device)
    PROF.wrap("wgrad", d, lambda: check(LIB.dmc_conv2d_wgrad(ctypes.byref(d), ptr(dy), ld_dy, ptr(x1), ptr(x2), ptr(ws),
                                                             ptr(dw), scale, L.stream()), "dmc_conv2d_wgrad"))


def pack_weight(mode, dtype, w, Kc, out=None):
    """fp32 [Cout][Cin][kh][kw] (or [Cout][Cin] Linear) -> packed kernel layout."""
    w = w.detach()
    if w.dim() == 2:
        Cout, Cin, kh, kw = w.shape[0], w.shape[1], 1, 1
    else:
        Cout, Cin, kh, kw = w.shape
    ntaps = 16 if mode == L.PACK_UPDGRAD else kh * kw
    rows = Cout if mode == L.PACK_FWD else Cin
    if out is None:
        out = torch.empty(rows * ntaps * Kc, dtype=dtype, device=w.device)
    check(LIB.dmc_pack_weight(mode, L.dtype_code(dtype), ptr(w.contiguous()), Cout, Cin, kh, kw, Kc, ptr(out),
                              L.stream()), "dmc_pack_weight")
    return out


class PackBatch:
    """Device arrays of dmc_pack_job + their tiles for one dmc_pack_weights launch.

    jobs: list of (w fp32 tensor, dst tensor, dst element offset, mode, Cout, Cin, kh, kw, Kc, koff)."""

    def __init__(self, jobs, device):
        arr = (L.PackJob * len(jobs))()
        self.keep = []
        tiles = []
        for i, (w, dst, off, mode, Cout, Cin, kh, kw, Kc, koff) in enumerate(jobs):
            w = w.detach()
            if not w.is_contiguous():
                raise L.DMCError("pack job: master weight must be contiguous")
            self.keep.append(w)
            j = arr[i]
            j.w = w.data_ptr()
            j.dst = dst.data_ptr() + off * dst.element_size()
            j.dtype = L.dtype_code(dst.dtype)
            j.mode, j.Cout, j.Cin, j.kh, j.kw, j.Kc, j.koff = mode, Cout, Cin, kh, kw, Kc, koff
            n = LIB.dmc_pack_tiles(ctypes.byref(j), i, None, 0)
            buf = (ctypes.c_int * (3 * n))()
            LIB.dmc_pack_tiles(ctypes.byref(j), i, buf, n)
            tiles.append(torch.frombuffer(bytearray(buf), dtype=torch.int32))
        self.count = len(jobs)
        t = torch.cat(tiles)
        self.ntiles = t.numel() // 3
        self.jobs = torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(device)
        self.tiles = t.to(device)

    def launch(self):
        check(LIB.dmc_pack_weights(ptr(self.jobs), ptr(self.tiles), self.ntiles, L.stream()), "dmc_pack_weights")


def gn_stats(dtype, x1, x2, N, HW, C1, C2, ld1, ld2, G, eps, gamma, beta):
    C = C1 + C2
    dev = x1.device
    mr = torch.empty(N * G * 2, dtype=torch.float32, device=dev)
    sc = torch.empty(N * C, dtype=torch.float32, device=dev)
    sh = torch.empty(N * C, dtype=torch.float32, device=dev)
    ws = SCRATCH.get(LIB.dmc_gn_workspace(N, C, G, HW), dev)
    check(LIB.dmc_gn_stats(L.dtype_code(dtype), ptr(x1), ptr(x2), N, HW, C1, C2, ld1, ld2, G, eps, ptr(gamma),
                           ptr(beta), ptr(ws), ptr(mr), ptr(sc), ptr(sh), L.stream()), "dmc_gn_stats")
    return sc, sh, mr


def gn_finalize(p1, C1, p2, C2, N, HW, G, eps, gamma, beta, out=None):
    """GroupNorm (scale, shift, mean_rstd) from the producing convs' partials (dmc_conv_desc.gn_part); out: the
    three buffers to fill (allocated if None)."""
    dev = p1.device
    C = C1 + C2
    if out is None:
        out = (torch.empty(N * C, dtype=torch.float32, device=dev),
               torch.empty(N * C, dtype=torch.float32, device=dev),
               torch.empty(N * G * 2, dtype=torch.float32, device=dev))
    sc, sh, mr = out
    check(LIB.dmc_gn_finalize(ptr(p1), C1, ptr(p2), C2, N, HW, G, eps, ptr(gamma), ptr(beta), ptr(mr), ptr(sc),
                              ptr(sh), L.stream()), "dmc_gn_finalize")
    return sc, sh, mr


def gn_stats_apply_ok(dtype, N, HW, C1, C2, G):
    return bool(LIB.dmc_gn_stats_apply_ok(L.dtype_code(dtype), N, HW, C1, C2, G))


def gn_stats_apply(dtype, x1, x2, N, HW, C1, C2, ld1, ld2, G, eps, gamma, beta, silu=True, drop=None):
    """gn_stats + gn_apply in one launch (small samples, gn_stats_apply_ok): ((scale, shift, mean_rstd), a)."""
    C = C1 + C2
    dev = x1.device
    mr = torch.empty(N * G * 2, dtype=torch.float32, device=dev)
    sc = torch.empty(N * C, dtype=torch.float32, device=dev)
    sh = torch.empty(N * C, dtype=torch.float32, device=dev)
    out = torch.empty(N * HW * C, dtype=dtype, device=dev)
    seed, base, thresh, dscale = drop_args(drop)
    check(LIB.dmc_gn_stats_apply(L.dtype_code(dtype), ptr(x1), ptr(x2), N, HW, C1, C2, ld1, ld2, G, eps, ptr(gamma),
                                 ptr(beta), ptr(mr), ptr(sc), ptr(sh), int(silu), seed, base, thresh, dscale, ptr(out),
                                 C, L.stream()), "dmc_gn_stats_apply")
    return (sc, sh, mr), out


def gn_apply(dtype, x1, x2, N, HW, C1, C2, ld1, ld2, scale, shift, silu=True, drop=None, out=None):
    """a = dropout(silu(x*scale + shift)) materialised as [N*HW][C1+C2] (dtype)."""
    C = C1 + C2
    if out is None:
        out = torch.empty(N * HW * C, dtype=dtype, device=x1.device)
    seed, base, thresh, dscale = drop_args(drop)
    check(LIB.dmc_gn_apply(L.dtype_code(dtype), ptr(x1), ptr(x2), N, HW, C1, C2, ld1, ld2, ptr(scale), ptr(shift),
                           int(silu), seed, base, thresh, dscale, ptr(out), C, L.stream()), "dmc_gn_apply")
    return out


def gn_bwd(dtype, g, ld_g, x1, x2, N, HW, C1, C2, ld1, ld2, G, mr, gamma, beta, silu, drop, dx1, dx2, ld_dx1,
           ld_dx2, acc1, acc2, dgamma, dbeta, dx_sum_nc=None, ld_sum_nc=0, dx_sum_c=None, part=None, defer=None,
           add1=None, ld_add1=0):
    """GroupNorm(+SiLU+dropout) backward; optionally also the per-(n,c) / per-c pixel sums of dx (the bias and
    time-embedding gradients of the layer that produced x), fused into the dx pass. part: (sum dz, sum dz*xhat)
    partials from an earlier pass ([N*HW/64][C][2]), skipping the reduction. add1: a second operand added into dx1
    (single source, no pixel sums; folded into the one-pass kernel's dx pass on the deferred path)."""
    ws = SCRATCH.get(LIB.dmc_gn_workspace(N, C1 + C2, G, HW), g.device)
    seed, base, thresh, scale = drop_args(drop)
    if defer is not None:
        # the parameter column sums go to the caller's batch (colsum_batch) when the one-pass kernel takes the call
        C = C1 + C2
        a_keep = torch.empty(N * C * 2, dtype=torch.float32, device=g.device)
        s_keep = torch.empty(N * C, dtype=torch.float32, device=g.device) if dx_sum_c is not None else None
        flag = ctypes.c_int(0)
        check(LIB.dmc_gn_silu_bwd_deferred(
            L.dtype_code(dtype), ptr(g), ld_g, ptr(x1), ptr(x2), N, HW, C1, C2, ld1, ld2, G, ptr(mr), ptr(gamma),
            ptr(beta), int(silu), seed, base, thresh, scale, ptr(dx1), ptr(dx2), ld_dx1, ld_dx2, int(acc1), int(acc2),
            ptr(dgamma), ptr(dbeta), ptr(dx_sum_nc), ld_sum_nc, ptr(dx_sum_c), ptr(part), ptr(ws), ptr(a_keep),
            ptr(s_keep), ctypes.byref(flag), ptr(add1), int(ld_add1), L.stream()), "dmc_gn_silu_bwd_deferred")
        if flag.value:
            defer.append((a_keep, N, C, 2 * C, 2, dbeta, dgamma))
            if s_keep is not None:
                defer.append((s_keep, N, C, C, 1, dx_sum_c, None))
        return
    check(LIB.dmc_gn_silu_bwd(L.dtype_code(dtype), ptr(g), ld_g, ptr(x1), ptr(x2), N, HW, C1, C2, ld1, ld2, G, ptr(mr),
                              ptr(gamma), ptr(beta), int(silu), seed, base, thresh, scale, ptr(dx1), ptr(dx2), ld_dx1,
                              ld_dx2, int(acc1), int(acc2), ptr(dgamma), ptr(dbeta), ptr(dx_sum_nc), ld_sum_nc,
                              ptr(dx_sum_c), ptr(part), ptr(ws), L.stream()), "dmc_gn_silu_bwd")
    if add1 is not None:   # the immediate entry point has no extra operand: a separate add
        add_(dtype, dx1, add1)


def colsum_batch(jobs):
    """Launch the column sums gn_bwd(defer=jobs) left behind (dmc_colsum_batch, <= 56 per launch) and clear the
    list: out0[c] = sum_r in[r*ld + c*stride], out1 at +1 -- dgamma / dbeta / the bias sums."""
    for k in range(0, len(jobs), 56):
        chunk = jobs[k:k + 56]
        arr = (L.ColsumJob * len(chunk))()
        for j, (t, R, C, ld, stride, o0, o1) in enumerate(chunk):
            arr[j].in_, arr[j].R, arr[j].C, arr[j].ld, arr[j].stride = ptr(t), R, C, ld, stride
            arr[j].out0, arr[j].out1, arr[j].scale = ptr(o0), ptr(o1), 1.0
        check(LIB.dmc_colsum_batch(arr, len(chunk), L.stream()), "dmc_colsum_batch")
    jobs.clear()


def channel_sum(dtype, dy, N, HW, C, ld, out_nc=None, ld_out=0, out_c=None, scale=1.0):
    """Per-(n,c) and per-c pixel sums; wide tensors are processed in channel slices of <= 256 chunks."""
    step = 256 * L.chunk_for(dtype)
    esz = dy.element_size()
    for c0 in range(0, C, step):
        cs = min(step, C - c0)
        ws = SCRATCH.get(LIB.dmc_channel_sum_workspace(N, HW, cs), dy.device)
        onc = None if out_nc is None else out_nc.data_ptr() + 4 * c0
        oc = None if out_c is None else out_c.data_ptr() + 4 * c0
        check(LIB.dmc_channel_sum(L.dtype_code(dtype), dy.data_ptr() + esz * c0, N, HW, cs, ld, onc, ld_out, oc,
                                  scale, ptr(ws), L.stream()), "dmc_channel_sum")


def attn_fwd(dtype, qkv, ld_qkv, N, Lq, heads, hd, out, ld_out, lse, drop=None):
    """drop = (seed, thresh, scale[, seed_base]): attention-probability dropout (kernels.drop_args)."""
    seed, base, thresh, scale = drop_args(drop)
    check(LIB.dmc_attn_fwd(L.dtype_code(dtype), ptr(qkv), ld_qkv, N, Lq, heads, hd, ptr(out), ld_out, ptr(lse), seed,
                           base, thresh, scale, L.stream()), "dmc_attn_fwd")


def attn_bwd(dtype, qkv, ld_qkv, out, dout, ld_out, lse, N, Lq, heads, hd, dqkv, ld_dqkv, drop=None):
    ws = SCRATCH.get(LIB.dmc_attn_workspace(N, Lq, heads), qkv.device)
    seed, base, thresh, scale = drop_args(drop)
    check(LIB.dmc_attn_bwd(L.dtype_code(dtype), ptr(qkv), ld_qkv, ptr(out), ptr(dout), ld_out, ptr(lse), N, Lq, heads,
                           hd, ptr(dqkv), ld_dqkv, ptr(ws), seed, base, thresh, scale, L.stream()), "dmc_attn_bwd")


def time_embed(t, dim, out):
    check(LIB.dmc_time_embed(ptr(t), t.shape[0], dim, ptr(out), L.stream()), "dmc_time_embed")


def embed_fwd(y, table, out):
    check(LIB.dmc_embed_fwd(ptr(y), y.shape[0], table.shape[0], ptr(table), table.shape[1], ptr(out), L.stream()),
          "dmc_embed_fwd")


def embed_bwd(y, rows, dout, dtable):
    check(LIB.dmc_embed_bwd(ptr(y), y.shape[0], rows, ptr(dout), dout.shape[1], ptr(dtable), L.stream()),
          "dmc_embed_bwd")


def _same(ref, *ts, what):
    """Host-side operand validation before a launch: a shape the kernel does not expect is a Python error, never
    an out-of-bounds device access."""
    for t in ts:
        if t is not None and (t.shape != ref.shape or t.device != ref.device):
            raise L.DMCError(f"{what}: operand shape {tuple(t.shape)} on {t.device}, expected {tuple(ref.shape)} on "
                             f"{ref.device}")


def _steps(N, dev, *ts, what):
    for t in ts:
        if t is not None and (t.numel() != N or t.dtype != torch.long or t.device != dev or not t.is_contiguous()):
            raise L.DMCError(f"{what}: timesteps must be a contiguous int64 [{N}] tensor on {dev}, got "
                             f"{t.dtype} {tuple(t.shape)} on {t.device}")


def pack_input(dtype, x, ld, noise=None, t=None, a=None, b=None, out=None):
    N, C, H, W = x.shape
    _same(x, noise, what="dmc_pack_input")
    _steps(N, x.device, t, what="dmc_pack_input")
    if out is None:
        out = torch.empty(N, H, W, ld, dtype=dtype, device=x.device)
    check(LIB.dmc_pack_input(L.dtype_code(dtype), ptr(x), ptr(noise), ptr(t), ptr(a), ptr(b), N, C, H, W, ptr(out), ld,
                             L.stream()), "dmc_pack_input")
    return out


def unpack_output(dtype, src, ld, N, C, H, W, out=None):
    if out is None:
        out = torch.empty(N, C, H, W, dtype=torch.float32, device=src.device)
    check(LIB.dmc_unpack_output(L.dtype_code(dtype), ptr(src), ld, N, C, H, W, ptr(out), L.stream()),
          "dmc_unpack_output")
    return out


def add_(dtype, y, x):
    check(LIB.dmc_add(L.dtype_code(dtype), ptr(y), ptr(x), y.numel(), L.stream()), "dmc_add")


def q_sample(x0, noise, t, a, b, out=None):
    x0 = x0.contiguous()
    noise = noise.contiguous()
    if out is None:
        out = torch.empty_like(x0, dtype=torch.float32)
    N = x0.shape[0]
    _same(x0, noise, out, what="dmc_q_sample")
    _steps(N, x0.device, t, what="dmc_q_sample")
    check(LIB.dmc_q_sample(ptr(x0), ptr(noise), ptr(t), ptr(a), ptr(b), N, x0.numel() // max(N, 1), ptr(out),
                           L.stream()), "dmc_q_sample")
    return out


def loss_fwd(loss_type, pred, target):
    _same(pred, target, what="dmc_loss_fwd")
    n = pred.numel()
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    ws = SCRATCH.get(4096 * 4, pred.device)
    check(LIB.dmc_loss_fwd(L.LOSS[loss_type], ptr(pred), ptr(target), n, ptr(loss), ptr(ws), L.stream()),
          "dmc_loss_fwd")
    return loss


def loss_bwd(loss_type, pred, target, dloss):
    dpred = torch.empty_like(pred)
    check(LIB.dmc_loss_bwd(L.LOSS[loss_type], ptr(pred), ptr(target), pred.numel(), ptr(dloss), ptr(dpred),
                           L.stream()), "dmc_loss_bwd")
    return dpred


def ddim_step(x, eps, t, t_next, alphas_cumprod, eta=0.0, clip=True, x0=None, z=None, out=None):
    if out is None:
        out = torch.empty_like(x)
    N = x.shape[0]
    _same(x, eps, x0, z, out, what="dmc_ddim_step")
    _steps(N, x.device, t, t_next, what="dmc_ddim_step")
    check(LIB.dmc_ddim_step(ptr(x), ptr(eps), ptr(x0), ptr(t), ptr(t_next), ptr(alphas_cumprod), N, x.numel() // N,
                            float(eta), int(clip), ptr(z), ptr(out), L.stream()), "dmc_ddim_step")
    return out


def ddpm_step(x, eps, t, sra, srm1, c1, c2, logvar, clip=True, x0=None, z=None, out=None):
    if out is None:
        out = torch.empty_like(x)
    N = x.shape[0]
    _same(x, eps, x0, z, out, what="dmc_ddpm_step")
    _steps(N, x.device, t, what="dmc_ddpm_step")
    check(LIB.dmc_ddpm_step(ptr(x), ptr(eps), ptr(x0), ptr(t), ptr(sra), ptr(srm1), ptr(c1), ptr(c2), ptr(logvar), N,
                            x.numel() // N, int(clip), ptr(z), ptr(out), L.stream()), "dmc_ddpm_step")
    return out


def cfg_x0(x, ec, eu, scale, t, ta, tb, mode, p_threshold):
    N = x.shape[0]
    _same(x, ec, eu, what="dmc_cfg_x0")
    _steps(N, x.device, t, what="dmc_cfg_x0")
    eps = torch.empty_like(x)
    x0 = torch.empty_like(x)
    p = float(p_threshold) if p_threshold is not None else -1.0
    check(LIB.dmc_cfg_x0(ptr(x), ptr(ec), ptr(eu), float(scale), ptr(t), ptr(ta), ptr(tb), int(mode), N,
                         x.numel() // N, p, ptr(eps), ptr(x0), L.stream()), "dmc_cfg_x0")
    return eps, x0


class TensorRefs:
    """Device array of dmc_tensor_ref {a, b, n} for the multi-tensor kernels (uploaded once per pointer set)."""

    def __init__(self, pairs, device):
        self.key = tuple((a.data_ptr(), b.data_ptr() if b is not None else 0, a.numel()) for a, b in pairs)
        arr = (L.TensorRef * len(pairs))()
        for i, (a, b) in enumerate(pairs):
            arr[i].a = a.data_ptr()
            arr[i].b = b.data_ptr() if b is not None else None
            arr[i].n = a.numel()
        host = torch.frombuffer(bytearray(arr), dtype=torch.uint8)
        self.dev = host.to(device)
        self.count = len(pairs)


def ema_update(refs: TensorRefs, decay):
    check(LIB.dmc_ema_update(ptr(refs.dev), refs.count, float(decay), L.stream()), "dmc_ema_update")


def clip_grad_norm(refs: TensorRefs, max_norm):
    total = torch.empty((), dtype=torch.float32, device=refs.dev.device)
    ws = SCRATCH.get((16 * refs.count + 16) * 4, refs.dev.device)
    check(LIB.dmc_clip_grad_norm(ptr(refs.dev), refs.count, float(max_norm), ptr(total), ptr(ws), L.stream()),
          "dmc_clip_grad_norm")
    return total


def grad_norm_flat(g, max_norm):
    """(total_norm, clip coef) of a flat fp32 gradient buffer, both device scalars; no host sync."""
    out = torch.empty(2, dtype=torch.float32, device=g.device)
    ws = SCRATCH.get(1024 * 4, g.device)   # one partial per dmc_grad_norm_flat block
    check(LIB.dmc_grad_norm_flat(ptr(g), g.numel(), float(max_norm), ptr(out), out.data_ptr() + 4, ptr(ws),
                                 L.stream()), "dmc_grad_norm_flat")
    return out[0], out[1:]


def adamw_flat(p, g, m, v, ema, coef, wd_mul, lerp_w, beta2, omb2, eps, neg_step, bc2_sqrt, ema_decay, ema_om):
    check(LIB.dmc_adamw_flat(ptr(p), ptr(g), ptr(m), ptr(v), ptr(ema), p.numel(), ptr(coef), wd_mul, lerp_w, beta2,
                             omb2, eps, neg_step, bc2_sqrt, ema_decay, ema_om, L.stream()), "dmc_adamw_flat")


def adamw_flat_dev(p, g, m, v, ema, coef, hyper):
    """adamw_flat with the nine scalars (same order as adamw_flat's) read from the fp32 device tensor hyper."""
    check(LIB.dmc_adamw_flat_dev(ptr(p), ptr(g), ptr(m), ptr(v), ptr(ema), p.numel(), ptr(coef), ptr(hyper),
                                 L.stream()), "dmc_adamw_flat_dev")


# ---- DiT token-wise kernels (csrc/dmc_dit.hip) ----------------------------------------------------------------
def _mod_ptr(mod, off):
    """Device address of column `off` of the stacked modulation rows [B][ld_mod] (fp32)."""
    return None if mod is None else mod.data_ptr() + 4 * off


def ln_mod_fwd(dtype, x, T, C, L_, mod, ld_mod, off_shift, off_scale, eps, h, ld_h, mean, rstd, br=None, ld_br=0,
               off_gate=0, drop=None, x_out=None):
    seed, seed_base, thresh, scale = drop_args(drop)
    check(LIB.dmc_ln_mod_fwd(L.dtype_code(dtype), ptr(x), ptr(br), ld_br, _mod_ptr(mod, off_gate) if br is not None
                             else None, _mod_ptr(mod, off_shift), _mod_ptr(mod, off_scale), ld_mod, T, C, L_,
                             float(eps), seed, seed_base, thresh, scale, ptr(x_out), ptr(h), ld_h, ptr(mean),
                             ptr(rstd), L.stream()), "dmc_ln_mod_fwd")


def _rowsum_ws(T, C, L_, dev):
    n = LIB.dmc_dit_rowsum_workspace(T // L_, C, L_)
    return SCRATCH.get(n, dev) if n else None


def ln_mod_bwd(dtype, dh, ld_dh, x, mean, rstd, mod, ld_mod, off_scale, T, C, L_, dx, dmod, off_dscale, off_dshift):
    ws = _rowsum_ws(T, C, L_, dx.device)
    check(LIB.dmc_ln_mod_bwd(L.dtype_code(dtype), ptr(dh), ld_dh, ptr(x), ptr(mean), ptr(rstd),
                             _mod_ptr(mod, off_scale), ld_mod, T, C, L_, ptr(dx), _mod_ptr(dmod, off_dscale),
                             _mod_ptr(dmod, off_dshift), ptr(ws), L.stream()), "dmc_ln_mod_bwd")


def gate_bwd(dtype, dy, br, ld_br, mod, ld_mod, off_gate, T, C, L_, dbr, ld_dbr, dmod, off_dgate, drop=None):
    seed, seed_base, thresh, scale = drop_args(drop)
    ws = _rowsum_ws(T, C, L_, dy.device)
    check(LIB.dmc_gate_bwd(L.dtype_code(dtype), ptr(dy), ptr(br), ld_br, _mod_ptr(mod, off_gate), ld_mod, T, C, L_,
                           seed, seed_base, thresh, scale, ptr(dbr), ld_dbr, _mod_ptr(dmod, off_dgate), ptr(ws),
                           L.stream()), "dmc_gate_bwd")


def gelu_fwd(dtype, u, rows, C, ld, a, drop=None):
    seed, seed_base, thresh, scale = drop_args(drop)
    check(LIB.dmc_gelu_fwd(L.dtype_code(dtype), ptr(u), rows, C, ld, seed, seed_base, thresh, scale, ptr(a),
                           L.stream()), "dmc_gelu_fwd")


def gelu_bwd(dtype, da, u, rows, C, ld, du, drop=None):
    seed, seed_base, thresh, scale = drop_args(drop)
    check(LIB.dmc_gelu_bwd(L.dtype_code(dtype), ptr(da), ptr(u), rows, C, ld, seed, seed_base, thresh, scale, ptr(du),
                           L.stream()), "dmc_gelu_bwd")


def timestep_embedding(t, dim, out, max_period=10000.0):
    _steps(t.shape[0], out.device, t, what="dmc_timestep_embedding")
    check(LIB.dmc_timestep_embedding(ptr(t), t.shape[0], dim, float(max_period), ptr(out), L.stream()),
          "dmc_timestep_embedding")


def unpatchify(src, ld_src, B, ht, wt, p, C, out):
    check(LIB.dmc_unpatchify(ptr(src), ld_src, B, ht, wt, p, C, ptr(out), L.stream()), "dmc_unpatchify")


def patchify_grad(dtype, dout, B, ht, wt, p, C, out, ld_out):
    check(LIB.dmc_patchify_grad(L.dtype_code(dtype), ptr(dout), B, ht, wt, p, C, ptr(out), ld_out, L.stream()),
          "dmc_patchify_grad")


def add_bcast(x, v, rows, n):
    check(LIB.dmc_add_bcast(ptr(x), ptr(v), rows, n, L.stream()), "dmc_add_bcast")


def batch_sum(x, rows, n, out):
    check(LIB.dmc_batch_sum(ptr(x), rows, n, ptr(out), L.stream()), "dmc_batch_sum")


def patch_dgrad(dtok, ld, w, B, ht, wt, p, C, H, dx):
    check(LIB.dmc_patch_dgrad(ptr(dtok), ld, ptr(w), B, ht, wt, p, C, H, ptr(dx), L.stream()), "dmc_patch_dgrad")
