"""GPU numerics of each HIP kernel against a plain PyTorch fp32 CPU reference of the same op.

fp32 mode: the f32-input MFMA path is exact-f32 fma chains; tolerances are summation-order level.
bf16 mode: inputs are rounded to bf16 first, so the reference sees the same operands; tolerance covers
bf16 rounding of the output (rel ~4e-3) and of the prologue output (re-rounded to bf16 before the MFMA).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    from diffusion_models_collection_amd import _lib as L, kernels as K
    return L, K


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def tol(dt):
    return dict(rtol=1e-4, atol=1e-4) if dt == torch.float32 else dict(rtol=3e-2, atol=3e-2)


def rel_err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


def q(x, dt):
    """round to the storage dtype and back to fp32 (what the kernel actually sees)"""
    return x.to(dt).float()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["s1_concat_gn", "s2", "up", "1x1", "ragged_in", "ragged_in_generic", "narrow_out",
                                  "splitk_concat", "splitk_ragged"])
def test_conv_forward(dt, case, monkeypatch, dmc_opt):
    """splitk_*: small M with deep K, which both planners (bf16 LDS-DMA, fp32 register-staged) run as split-K
    over grid.z + epilogue kernel. ragged_in (3 input channels) and narrow_out (3 output channels) run the
    narrow-conv kernels; ragged_in_generic is the same conv on the tiled kernels (DMC_NO_NARROW)."""
    L, K = _lib()
    dmc_opt("DMC_NO_NARROW", 1 if case == "ragged_in_generic" else 0)
    torch.manual_seed(0)
    N, H, W = 2, 8, 8
    C1, C2, Cout = 32, 16, 48
    taps, mode, stride, k, OH, OW = K.TAPS3, L.MODE_NORMAL, 1, 3, H, W
    if case == "splitk_concat":
        N, C1, C2, Cout = 4, 192, 64, 256
    elif case == "splitk_ragged":
        N, C1, C2, Cout = 3, 320, 0, 200
    elif case == "s2":
        C2, stride, OH, OW = 0, 2, 4, 4
    elif case == "up":
        C2, mode, OH, OW = 0, L.MODE_UPSAMPLE, 16, 16
    elif case == "1x1":
        taps, k = K.TAPS1, 1
    elif case.startswith("ragged_in"):
        C1, C2 = 3, 0
    elif case == "narrow_out":
        Cout = 3
    ld1 = C1 if not case.startswith("ragged_in") else L.chunk_for(dt)
    x1 = torch.randn(N, C1, H, W)
    x2 = torch.randn(N, C2, H, W) if C2 else None
    w = torch.randn(Cout, C1 + C2, k, k) / math.sqrt((C1 + C2) * k * k)
    bias = torch.randn(Cout)
    addv = torch.randn(N, Cout)
    use_gn = case == "s1_concat_gn"
    sc = torch.rand(N, C1 + C2) + 0.5
    sh = torch.randn(N, C1 + C2) * 0.1
    # reference (fp32 CPU) on dtype-rounded inputs
    xr = q(x1, dt) if x2 is None else torch.cat([q(x1, dt), q(x2, dt)], 1)
    if use_gn:
        xr = q(F.silu(xr * sc[:, :, None, None] + sh[:, :, None, None]), dt)
    if mode == L.MODE_UPSAMPLE:
        xr = F.interpolate(xr, scale_factor=2, mode="nearest")
    yr = F.conv2d(xr, q(w, dt), bias, stride=stride, padding=k // 2)
    yr = yr + addv[:, :, None, None]
    resid = torch.randn(N, Cout, OH, OW)
    yr = yr + q(resid, dt)
    # kernel
    # padding channels of a narrow source hold garbage: the kernels must not read them into the sum
    x1d = torch.full((N, H, W, ld1), 1e4, dtype=dt, device=DEV)
    x1d[..., :C1] = nhwc(x1).to(dt).to(DEV)
    x2d = nhwc(x2).to(dt).to(DEV) if x2 is not None else None
    Kc = L.kc_for(C1 + C2, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w.to(DEV), Kc)
    d = K.make_desc(dt, N, H, W, C1, C2, ld1, C2, Kc, OH, OW, Cout, taps, mode, stride)
    if use_gn:
        K.set_prologue(d, L.PRO_AFFINE_SILU, sc.to(DEV), sh.to(DEV), C1 + C2)
    y = torch.empty(N, OH, OW, Cout, dtype=dt, device=DEV)
    rd = nhwc(resid).to(dt).to(DEV)
    K.set_epilogue(d, bias=bias.to(DEV), addvec=addv.to(DEV), ld_add=Cout, resid=rd, ld_res=Cout, ldy1=Cout)
    if case.startswith("splitk"):
        import ctypes
        assert L.LIB.dmc_conv2d_workspace(ctypes.byref(d)) > 0   # the planner does choose split-K here
    K.conv(d, x1d, x2d, wp, y)
    torch.cuda.synchronize()
    got = nchw(y.float().cpu())
    assert rel_err(got, yr) < (1e-5 if dt == torch.float32 else 2e-2), rel_err(got, yr)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_upsample2x_nhwc_bitwise(dt):
    """Nearest x2 upsample (models/unet.py:118) of an NHWC activation with a padded channel pitch: bitwise equal
    to torch's nearest interpolate of the same values."""
    L, K = _lib()
    torch.manual_seed(4)
    N, H, W, C, ld = 3, 5, 7, 40, 48
    x = torch.randn(N, H, W, ld).to(dt).to(DEV)
    y = K.upsample2x(dt, x, C)
    torch.cuda.synchronize()
    ref = F.interpolate(x[..., :C].permute(0, 3, 1, 2).float(), scale_factor=2, mode="nearest")
    assert torch.equal(y.permute(0, 3, 1, 2).float(), ref)


@pytest.mark.parametrize("case", ["c32_two_sources", "c16_wide", "c32_384", "c8_multi_image", "c64_rows",
                                  "c64_two_sources"])
def test_conv3x3_halo_gn_silu_prologue(case, monkeypatch, dmc_opt):
    """Inference prologue on the halo kernel: conv(SiLU(x*scale+shift)) with the GroupNorm affine + SiLU
    applied to the LDS-resident halo equals, BITWISE, dmc_gn_apply materialisation followed by the plain halo
    conv (same op sequence and bf16 rounding), and the fp32 torch reference within bf16 tolerance. c64_*: the
    64-pixel rows of BASELINE config #5's 64x64 level (halo tiles of 9 pieces, conv3x3_halo2_kernel<9,2,true>),
    the plan its DDIM-100 sampling loop runs (models/unet.py:34-38 at image_size (64, 64))."""
    L, K = _lib()
    dmc_opt("DMC_NO_SPLITK", 1)   # small N: keep the planner on the halo kernel
    dmc_opt("DMC_HALO_PRO", 1)    # the halo prologue path (default on)
    dt = torch.bfloat16
    torch.manual_seed(11)
    N, H, C1, C2, Cout = {"c32_two_sources": (2, 32, 128, 64, 128), "c16_wide": (3, 16, 256, 0, 256),
                          "c32_384": (2, 32, 256, 128, 128), "c8_multi_image": (8, 8, 128, 64, 128),
                          "c64_rows": (2, 64, 128, 0, 128), "c64_two_sources": (2, 64, 128, 128, 128)}[case]
    # tiles of several 8x8 images are not taken (a lane's scale/shift row would differ per piece): the conv
    # then runs the register-staged prologue kernel, equal to the materialised path within bf16 rounding
    halo = case != "c8_multi_image"
    W, Cin, G = H, C1 + C2, 8
    x = q(torch.randn(N, Cin, H, W) * 1.4 + 0.3, dt)
    gamma, beta = torch.rand(Cin) + 0.5, torch.randn(Cin)
    w = q(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), dt)
    bias = torch.randn(Cout)
    xd = nhwc(x).to(dt).to(DEV)
    x1d, x2d = (xd[..., :C1].contiguous(), xd[..., C1:].contiguous()) if C2 else (xd, None)
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w.to(DEV), Kc)
    sc, sh, _ = K.gn_stats(dt, x1d, x2d, N, H * W, C1, C2, C1, C2, G, 1e-5, gamma.to(DEV), beta.to(DEV))
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, Kc, H, W, Cout, K.TAPS3)
    K.set_prologue(d, L.PRO_AFFINE_SILU, sc, sh, Cin)
    K.set_epilogue(d, bias=bias.to(DEV), ldy1=Cout)
    assert K.conv_halo_prologue(d) == halo
    y = torch.full((N, H, W, Cout), float("nan"), dtype=dt, device=DEV)
    K.conv(d, x1d, x2d, wp, y)
    a = K.gn_apply(dt, x1d, x2d, N, H * W, C1, C2, C1, C2, sc, sh, silu=True).view(N, H, W, Cin)
    d0 = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, Kc, H, W, Cout, K.TAPS3)
    K.set_epilogue(d0, bias=bias.to(DEV), ldy1=Cout)
    y0 = torch.full((N, H, W, Cout), float("nan"), dtype=dt, device=DEV)
    K.conv(d0, a, None, wp, y0)
    torch.cuda.synchronize()
    if halo:
        assert torch.equal(y, y0), (y.float() - y0.float()).abs().max().item()
    else:
        assert rel_err(y.float(), y0.float()) < 1e-2
    yr = F.conv2d(F.silu(F.group_norm(x, G, gamma, beta, 1e-5)), w, bias, padding=1)
    assert rel_err(nchw(y.float().cpu()), yr) < 2e-2
    dmc_opt("DMC_HALO_PRO", 0)
    assert not K.conv_halo_prologue(d)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["s1", "s2", "up", "1x1_concat_split"])
def test_conv_dgrad_wgrad(dt, case):
    """input- and weight-gradient kernels vs autograd of F.conv2d (fp32 CPU)."""
    L, K = _lib()
    torch.manual_seed(1)
    N, H, W, Cin, Cout = 2, 8, 8, 32, 48
    k, stride, OH, OW, mode = 3, 1, H, W, L.MODE_NORMAL
    if case == "s2":
        stride, OH, OW = 2, 4, 4
    elif case == "up":
        OH, OW, mode = 16, 16, L.MODE_UPSAMPLE
    elif case.startswith("1x1"):
        k = 1
    x = q(torch.randn(N, Cin, H, W), dt).requires_grad_(True)
    w = q(torch.randn(Cout, Cin, k, k) / math.sqrt(Cin * k * k), dt).requires_grad_(True)
    xi = F.interpolate(x, scale_factor=2, mode="nearest") if mode == L.MODE_UPSAMPLE else x
    y = F.conv2d(xi, w, stride=stride, padding=k // 2)
    g = q(torch.randn_like(y), dt)
    y.backward(g)
    gd = nhwc(g).to(dt).to(DEV)
    xd = nhwc(x.detach()).to(dt).to(DEV)
    # dgrad
    dx = torch.zeros(N, H, W, Cin, dtype=dt, device=DEV)
    src = K.Act if hasattr(K, "Act") else None
    if case == "s1" or case.startswith("1x1"):
        pm, taps, dmode, dstride = L.PACK_DGRAD, (K.TAPS3_DGRAD if k == 3 else K.TAPS1), L.MODE_NORMAL, 1
    elif case == "s2":
        pm, taps, dmode, dstride = L.PACK_DGRAD, K.TAPS3_DGRAD, L.MODE_DILATE, 1
    else:
        pm, taps, dmode, dstride = L.PACK_UPDGRAD, K.TAPS_UPDGRAD, L.MODE_NORMAL, 2
    Kc = L.kc_for(Cout, dt)
    wp = K.pack_weight(pm, dt, w.detach().to(DEV), Kc)
    d = K.make_desc(dt, N, OH, OW, Cout, 0, Cout, 0, Kc, H, W, Cin, taps, dmode, dstride)
    if case == "1x1_concat_split":
        d1 = torch.empty(N, H, W, 24, dtype=dt, device=DEV)
        d2 = torch.empty(N, H, W, 8, dtype=dt, device=DEV)
        K.set_epilogue(d, ldy1=24, ldy2=8, Csplit=24)
        K.conv(d, gd, None, wp, d1, d2)
        dx = torch.cat([d1, d2], -1)
    else:
        K.set_epilogue(d, ldy1=Cin)
        K.conv(d, gd, None, wp, dx)
    # wgrad
    dw = torch.empty_like(w, device=DEV)
    dw_desc = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, L.kc_for(Cin, dt), OH, OW, Cout,
                          K.TAPS3 if k == 3 else K.TAPS1, mode, stride)
    db = torch.full((Cout,), float("nan"), device=DEV)
    K.wgrad(dw_desc, gd, Cout, xd, None, dw, dbias=db)    # + the bias gradient from the same kernel
    torch.cuda.synchronize()
    e1 = rel_err(nchw(dx.float().cpu()), x.grad)
    e2 = rel_err(dw.cpu(), w.grad)
    lim = 1e-5 if dt == torch.float32 else 2e-2
    assert e1 < lim and e2 < (1e-5 if dt == torch.float32 else 1e-2), (e1, e2)
    assert rel_err(db.cpu(), g.sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", ["fwd32_concat", "fwd16_ragged_cout", "dgrad32", "fwd8_multi_image", "fallback_4x4",
                                  "fwd8_concat_b128", "fwd64_rows"])
def test_conv3x3_halo_kernel(case, monkeypatch, dmc_opt):
    """bf16 3x3 stride-1 convs on the LDS-halo kernel (conv3x3_halo2_kernel: 128-pixel tiles of whole rows or
    whole images, two blocks per CU) vs an fp32 reference and vs the per-tap kernel (DMC_NO_HALO) on the same
    inputs; its weight-gradient twin (wgrad3x3_halo2_kernel) likewise."""
    L, K = _lib()
    # at these small M the planner would split K over the LDS-DMA kernel instead; the halo kernel is what the
    # B=128 model runs, so keep split-K off here to exercise it
    dmc_opt("DMC_NO_SPLITK", 1)
    dt = torch.bfloat16
    torch.manual_seed(5)
    N, H, C1, C2, Cout, taps, pm = 2, 32, 64, 64, 128, K.TAPS3, L.PACK_FWD
    if case == "fwd16_ragged_cout":
        N, H, C1, C2, Cout = 3, 16, 128, 0, 200
    elif case == "dgrad32":
        N, H, C1, C2, Cout, taps, pm = 1, 32, 192, 0, 64, K.TAPS3_DGRAD, L.PACK_DGRAD
    elif case == "fwd8_multi_image":
        N, H, C1, C2, Cout = 8, 8, 128, 64, 128   # 4 whole 8x8 images per 256-pixel tile (7 halo pieces/wave)
    elif case == "fwd8_concat_b128":
        # the UNet's 8x8 up blocks at B=128: 7 halo pieces per wave AND several 256-pixel tiles per wgrad block
        # (round 2 fix: the 7th piece of the next tile's halo was never issued -> NaN weight gradients)
        N, H, C1, C2, Cout = 128, 8, 256, 256, 256
    elif case == "fwd64_rows":
        N, H, C1, C2, Cout = 16, 64, 128, 0, 128  # 64-wide rows: 4-row tiles, 396 halo pixels (HP = 7)
    elif case == "fallback_4x4":
        N, H, C1, C2, Cout = 8, 4, 64, 0, 128     # halo of 16 images exceeds the LDS budget: per-tap kernel
    W = H
    Cin = C1 + C2
    x = q(torch.randn(N, Cin, H, W), dt)
    if pm == L.PACK_DGRAD:
        # dgrad of a conv Cout<-Cin is a conv over the gradient with flipped/transposed weights
        w = q(torch.randn(Cin, Cout, 3, 3) / math.sqrt(Cin * 9), dt)   # forward weight [C_fwd_out=Cin][Cout]
        yr = torch.nn.grad.conv2d_input((N, Cout, H, W), w, x, padding=1)
        wp = K.pack_weight(pm, dt, w.to(DEV), L.kc_for(Cin, dt))
    else:
        w = q(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), dt)
        yr = F.conv2d(x, w, padding=1)
        wp = K.pack_weight(pm, dt, w.to(DEV), L.kc_for(Cin, dt))
    bias = torch.randn(Cout)
    yr = yr + bias[:, None, None]
    xd = nhwc(x).to(dt).to(DEV)
    x1d, x2d = (xd[..., :C1].contiguous(), xd[..., C1:].contiguous()) if C2 else (xd, None)
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(Cin, dt), H, W, Cout, taps)
    K.set_epilogue(d, bias=bias.to(DEV), ldy1=Cout)
    outs = []
    for no_halo in ("0", "1"):
        dmc_opt("DMC_NO_HALO", int(no_halo))
        y = torch.full((N, H, W, Cout), float("nan"), dtype=dt, device=DEV)
        K.conv(d, x1d, x2d, wp, y)
        torch.cuda.synchronize()
        outs.append(nchw(y.float().cpu()))
    assert rel_err(outs[0], yr) < 2e-2, rel_err(outs[0], yr)
    assert rel_err(outs[0], outs[1]) < 1e-2
    if pm == L.PACK_FWD:
        # weight gradient of the same conv: halo wgrad kernel vs autograd and vs the per-tap wgrad kernel
        g = q(torch.randn(N, Cout, H, W), dt)
        wr = torch.nn.grad.conv2d_weight(x, w.shape, g, padding=1)
        gd = nhwc(g).to(dt).to(DEV)
        dws = []
        for no_halo in ("0", "1"):
            dmc_opt("DMC_NO_HALO", int(no_halo))
            dw = torch.full(tuple(w.shape), float("nan"), device=DEV)
            db = torch.full((Cout,), float("nan"), device=DEV)
            K.wgrad(d, gd, Cout, x1d, x2d, dw, dbias=db)
            torch.cuda.synchronize()
            dws.append(dw.cpu())
            # the bias gradient (halo kernel: dy fragments x an all-ones MFMA operand) = the pixel sums of dy
            assert rel_err(db.cpu(), g.sum((0, 2, 3))) < 1e-5, (no_halo, rel_err(db.cpu(), g.sum((0, 2, 3))))
        assert rel_err(dws[0], wr) < 1e-2, rel_err(dws[0], wr)
        assert rel_err(dws[0], dws[1]) < 1e-3, rel_err(dws[0], dws[1])


@pytest.mark.parametrize("case", ["in32", "in16_dgrad", "out32_nchw", "out64", "out8_multi_image"])
def test_conv3x3_narrow_halo_kernels(case, dmc_opt):
    """The halo'd narrow convs (conv3x3_nin_kernel: <= 8 input channels, the UNet's input conv and the input gradient
    of its output conv, through the shared LDS epilogue with the GroupNorm partials; conv3x3_nout_kernel: <= 16 output
    channels, the output conv with its NCHW fp32 store) vs the fp32 torch reference and vs the global-fragment narrow
    kernels (DMC_NO_NHALO=1) on the same inputs."""
    L, K = _lib()
    dt = torch.bfloat16
    torch.manual_seed(13)
    N, H, Cin, Cout, taps, pm, nchw_out = {"in32": (8, 32, 3, 128, K.TAPS3, L.PACK_FWD, False),
                                            "in16_dgrad": (8, 16, 3, 256, K.TAPS3_DGRAD, L.PACK_DGRAD, False),
                                            "out32_nchw": (8, 32, 128, 3, K.TAPS3, L.PACK_FWD, True),
                                            "out64": (4, 64, 128, 3, K.TAPS3, L.PACK_FWD, False),
                                            "out8_multi_image": (16, 8, 64, 3, K.TAPS3, L.PACK_FWD, True)}[case]
    W = H
    x = q(torch.randn(N, Cin, H, W), dt)
    if pm == L.PACK_DGRAD:
        w = q(torch.randn(Cin, Cout, 3, 3) / math.sqrt(Cin * 9), dt)
        yr = torch.nn.grad.conv2d_input((N, Cout, H, W), w, x, padding=1)
    else:
        w = q(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), dt)
        yr = F.conv2d(x, w, padding=1)
    bias = torch.randn(Cout)
    yr = yr + bias[:, None, None]
    ld1 = 8 if Cin < 8 else Cin
    xd = torch.full((N, H, W, ld1), 1e4, dtype=dt, device=DEV)   # padding channels hold garbage
    xd[..., :Cin] = nhwc(x).to(dt).to(DEV)
    wp = K.pack_weight(pm, dt, w.to(DEV), L.kc_for(Cin, dt))
    stats = Cin < 8 and H * W % 64 == 0
    outs, parts = [], []
    for no_nhalo in (0, 1):
        dmc_opt("DMC_NO_NHALO", no_nhalo)
        d = K.make_desc(dt, N, H, W, Cin, 0, ld1, 0, L.kc_for(Cin, dt), H, W, Cout, taps)
        part = torch.full((N * H * W // 64 * (Cout // 8) * 2,), float("nan"), device=DEV) if stats else None
        if nchw_out:
            y = torch.full((N, Cout, H, W), float("nan"), device=DEV)
            K.set_epilogue(d, bias=bias.to(DEV), out_f32=True, out_nchw=True, gn_part=part)
        else:
            y = torch.full((N, H, W, Cout), float("nan"), dtype=dt, device=DEV)
            K.set_epilogue(d, bias=bias.to(DEV), ldy1=Cout, gn_part=part)
        K.conv(d, xd, None, wp, y)
        torch.cuda.synchronize()
        outs.append(y.float().cpu() if nchw_out else nchw(y.float().cpu()))
        parts.append(part.cpu() if stats else None)
    assert rel_err(outs[0], yr) < 2e-2, rel_err(outs[0], yr)
    assert rel_err(outs[0], outs[1]) < 1e-2, rel_err(outs[0], outs[1])
    if stats:
        p0, p1 = parts[0].view(-1, 2), parts[1].view(-1, 2)
        assert torch.isfinite(p0).all()
        assert rel_err(p0[:, 0], p1[:, 0]) < 2e-2 and rel_err(p0[:, 1], p1[:, 1]) < 2e-2


@pytest.mark.parametrize("case", ["f8_256", "f8_concat512", "d8_512out", "f4_256", "f4_concat512", "d4_512out"])
def test_conv3x3_small_kernel(case, dmc_opt):
    """The small-map 3x3 conv (round 6: conv3x3_img_kernel, whole-image tiles over the full K; it replaced round 4's
    conv3x3_small_kernel) at the UNet's B=128 shapes -- forward (one source and the up path's 256+256 concat) and
    the input gradient with 512 output channels -- with the full epilogue (bias, time embedding, residual) and, at
    8x8, the GroupNorm partials: vs the fp32 torch reference, and vs the split-K LDS-DMA path (DMC_IMG_MASK=0) on
    the same inputs."""
    L, K = _lib()
    dt = torch.bfloat16
    torch.manual_seed(9)
    H = 8 if case[1] == "8" else 4
    N = 128
    C1, C2, Cout, taps, pm = 256, 0, 256, K.TAPS3, L.PACK_FWD
    if "concat512" in case:
        C2 = 256
    elif case.startswith("d"):
        Cout, taps, pm = 512, K.TAPS3_DGRAD, L.PACK_DGRAD
    W, Cin = H, C1 + C2
    x = q(torch.randn(N, Cin, H, W), dt)
    if pm == L.PACK_DGRAD:
        w = q(torch.randn(Cin, Cout, 3, 3) / math.sqrt(Cin * 9), dt)   # the forward conv Cout -> Cin
        yr = torch.nn.grad.conv2d_input((N, Cout, H, W), w, x, padding=1)
    else:
        w = q(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), dt)
        yr = F.conv2d(x, w, padding=1)
    wp = K.pack_weight(pm, dt, w.to(DEV), L.kc_for(Cin, dt))
    bias, addv = torch.randn(Cout), torch.randn(N, Cout)
    resid = q(torch.randn(N, Cout, H, W), dt)
    yr = yr + bias[:, None, None] + addv[:, :, None, None] + resid
    xd = nhwc(x).to(dt).to(DEV)
    x1d, x2d = (xd[..., :C1].contiguous(), xd[..., C1:].contiguous()) if C2 else (xd, None)
    rd = nhwc(resid).to(dt).to(DEV)
    outs, parts = [], []
    for mask in (15, 0):
        dmc_opt("DMC_IMG_MASK", mask)
        d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(Cin, dt), H, W, Cout, taps)
        part = torch.full((N * H * W // 64 * (Cout // 8) * 2,), float("nan"), device=DEV) if H == 8 else None
        K.set_epilogue(d, bias=bias.to(DEV), addvec=addv.to(DEV), ld_add=Cout, resid=rd, ld_res=Cout, ldy1=Cout,
                       gn_part=part)
        y = torch.full((N, H, W, Cout), float("nan"), dtype=dt, device=DEV)
        K.conv(d, x1d, x2d, wp, y)
        torch.cuda.synchronize()
        outs.append(nchw(y.float().cpu()))
        parts.append(None if part is None else part.cpu())
    assert rel_err(outs[0], yr) < 2e-2, rel_err(outs[0], yr)
    assert rel_err(outs[0], outs[1]) < 1e-2, rel_err(outs[0], outs[1])
    if H == 8:
        # (mean, M2) per (64-pixel segment, 8-channel chunk) of the stored bf16 output, both paths
        p0, p1 = parts[0].view(-1, 2), parts[1].view(-1, 2)
        assert torch.isfinite(p0).all()
        assert rel_err(p0[:, 0], p1[:, 0]) < 2e-2 and rel_err(p0[:, 1], p1[:, 1]) < 2e-2
        yv = outs[0].permute(0, 2, 3, 1).reshape(N, 64, Cout // 8, 8)           # [segment][pixel][chunk][8]
        mean = yv.mean(dim=(1, 3)).reshape(-1)
        m2 = ((yv - yv.mean(dim=(1, 3), keepdim=True)) ** 2).sum(dim=(1, 3)).reshape(-1)
        assert rel_err(p0[:, 0], mean) < 1e-4 and rel_err(p0[:, 1], m2) < 1e-4


@pytest.mark.parametrize("shape", [(64, 8, 8, 256, 256), (128, 32, 32, 128, 0), (96, 16, 16, 136, 120),
                                   (64, 4, 4, 512, 0)])
def test_groupnorm_stats_one_block_per_sample(shape, monkeypatch, dmc_opt):
    """bf16 at N >= 64: statistics of a sample in one 1024-thread block, finalised in the same launch
    (gn_stats_one), vs torch fp32 group_norm statistics of the same bf16 values and vs the split path."""
    L, K = _lib()
    torch.manual_seed(5)
    N, H, W, C1, C2 = shape
    G, C = 8, C1 + C2
    x = q(torch.randn(N, C, H, W) * 1.5 + 0.7, torch.bfloat16)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    xd = nhwc(x).to(torch.bfloat16).to(DEV)
    x1, x2 = xd[..., :C1].contiguous(), (xd[..., C1:].contiguous() if C2 else None)
    outs = []
    for split in ("0", "1"):
        dmc_opt("DMC_GN_STATS_SPLIT", int(split))
        sc, sh, mr = K.gn_stats(torch.bfloat16, x1, x2, N, H * W, C1, C2, C1, C2, G, 1e-5, gamma.to(DEV),
                                beta.to(DEV))
        torch.cuda.synchronize()
        outs.append((sc.cpu(), sh.cpu(), mr.cpu()))
    xv = x.view(N, G, -1).double()
    mean, var = xv.mean(-1), xv.var(-1, unbiased=False)
    rstd = (var + 1e-5).rsqrt()
    for sc, sh, mr in outs:
        m = mr.view(N, G, 2)
        torch.testing.assert_close(m[..., 0].double(), mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(m[..., 1].double(), rstd, rtol=1e-4, atol=1e-5)
        sc_ref = (rstd.repeat_interleave(C // G, 1) * gamma.double())
        torch.testing.assert_close(sc.view(N, C).double(), sc_ref, rtol=1e-4, atol=1e-5)
        sh_ref = beta.double() - mean.repeat_interleave(C // G, 1) * sc_ref
        torch.testing.assert_close(sh.view(N, C).double(), sh_ref, rtol=1e-4, atol=1e-4)
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("case", [(128, 4, 4, 256, 0, 32, True, 0.0), (64, 4, 4, 256, 256, 32, True, 0.1),
                                  (128, 4, 4, 512, 0, 32, False, 0.0), (64, 2, 2, 768, 256, 8, True, 0.3)])
def test_gn_stats_apply_bitwise(case):
    """dmc_gn_stats_apply (statistics + SiLU / dropout apply of a small sample in one launch, the UNet's 4x4 levels)
    is BITWISE dmc_gn_stats followed by dmc_gn_apply: scale, shift, mean_rstd and the applied activation; the
    shape gate rejects samples above 8192 elements and fp32."""
    L, K = _lib()
    torch.manual_seed(11)
    N, H, W, C1, C2, G, silu, p = case
    C, HW = C1 + C2, H * W
    x = (torch.randn(N, H, W, C) * 1.3 + 0.4).to(torch.bfloat16).to(DEV)
    x1, x2 = x[..., :C1].contiguous(), (x[..., C1:].contiguous() if C2 else None)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    drop = None
    if p > 0:
        thresh = int(p * 2 ** 32)
        drop = (1234567, thresh, 1.0 / (1.0 - p))
    assert K.gn_stats_apply_ok(torch.bfloat16, N, HW, C1, C2, G)
    (sc, sh, mr), a = K.gn_stats_apply(torch.bfloat16, x1, x2, N, HW, C1, C2, C1, C2, G, 1e-5, gamma, beta, silu=silu,
                                       drop=drop)
    sc0, sh0, mr0 = K.gn_stats(torch.bfloat16, x1, x2, N, HW, C1, C2, C1, C2, G, 1e-5, gamma, beta)
    a0 = K.gn_apply(torch.bfloat16, x1, x2, N, HW, C1, C2, C1, C2, sc0, sh0, silu=silu, drop=drop)
    torch.cuda.synchronize()
    for u, v in ((sc, sc0), (sh, sh0), (mr, mr0), (a, a0)):
        assert torch.equal(u, v)
    assert not K.gn_stats_apply_ok(torch.bfloat16, N, 64, 256, 0, 32)
    assert not K.gn_stats_apply_ok(torch.float32, N, HW, C1, C2, G)
    assert not K.gn_stats_apply_ok(torch.bfloat16, 32, HW, C1, C2, G)


@pytest.mark.parametrize("shape", [(64, 8, 8, 256, 256), (128, 16, 16, 256, 0), (64, 4, 4, 384, 128)])
def test_groupnorm_backward_one_block_per_sample(shape, monkeypatch, dmc_opt):
    """bf16 at N >= 64 and HW*C <= 64K: the per-channel sums and apply coefficients of a sample in one
    1024-thread block (gn_bwd_one) vs torch fp32 autograd of SiLU(GN(x)), and vs the partial+final path, with
    dropout and the fused dx pixel sums."""
    L, K = _lib()
    torch.manual_seed(6)
    N, H, W, C1, C2 = shape
    G, C, dt = 8, C1 + C2, torch.bfloat16
    x = q(torch.randn(N, C, H, W) * 1.3 + 0.4, dt).requires_grad_(True)
    gamma = (torch.rand(C) + 0.5).requires_grad_(True)
    beta = torch.randn(C).requires_grad_(True)
    a = F.silu(F.group_norm(x, G, gamma, beta, 1e-5))
    gout = q(torch.randn_like(a), dt)
    a.backward(gout)
    xd = nhwc(x.detach()).to(dt).to(DEV)
    x1, x2 = xd[..., :C1].contiguous(), (xd[..., C1:].contiguous() if C2 else None)
    gd, gm_d, bt_d = nhwc(gout).to(dt).to(DEV), gamma.detach().to(DEV), beta.detach().to(DEV)
    _, _, mr = K.gn_stats(dt, x1, x2, N, H * W, C1, C2, C1, C2, G, 1e-5, gm_d, bt_d)
    res = {}
    for split in ("0", "1"):
        dmc_opt("DMC_GN_BWD_SPLIT", int(split))
        for drop in (None, (7, 1 << 30, 4.0 / 3.0)):   # (seed, thresh, scale): keep prob 0.75
            dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if C2 else None)
            dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            K.gn_bwd(dt, gd, C, x1, x2, N, H * W, C1, C2, C1, C2, G, mr, gm_d, bt_d, True, drop, dx1, dx2, C1, C2,
                     0, 0, dg, db)
            torch.cuda.synchronize()
            dx = torch.cat([dx1, dx2], -1) if C2 else dx1
            res[(split, drop is None)] = (dx.float().cpu(), dg.cpu(), db.cpu())
    dxk, dgk, dbk = res[("0", True)]
    assert rel_err(nchw(dxk), x.grad) < 2e-2
    assert rel_err(dgk, gamma.grad) < 1e-4 and rel_err(dbk, beta.grad) < 1e-4
    for nodrop in (True, False):
        for u, v in zip(res[("0", nodrop)], res[("1", nodrop)]):
            assert rel_err(u, v) < 1e-2, (nodrop, rel_err(u, v))
    # dropout changes the result (keep prob 0.75), identically on both paths
    assert rel_err(res[("0", False)][0], dxk) > 1e-2


@pytest.mark.parametrize("shape", [(128, 32, 32, 128, 0), (128, 16, 16, 256, 256), (64, 8, 8, 256, 256),
                                   (128, 4, 4, 256, 0), (128, 16, 16, 384, 0), (96, 8, 8, 512, 0),
                                   (64, 16, 16, 32, 0), (64, 8, 8, 96, 0)])
def test_groupnorm_backward_fused_one_pass(shape, dmc_opt):
    """bf16 at N >= 64: the one-pass GroupNorm backward (gn_bwd_fused: a channel slice of a sample per 1024-thread
    block, x and g held in registers between the reduction and the dx pass) vs the two-pass kernels
    (DMC_GN_BWD_FUSED=0) and torch fp32 autograd: dx with dropout and accumulation, dgamma / dbeta, and the fused
    per-(n, c) / per-c pixel sums of the stored dx. The last two shapes have 4 and 12 channels per group (not whole
    8-channel chunks: the planner must keep them off the one-pass kernel, whose threads take one group's
    statistics per chunk)."""
    L, K = _lib()
    torch.manual_seed(8)
    N, H, W, C1, C2 = shape
    G, C, dt, HW = 8, C1 + C2, torch.bfloat16, shape[1] * shape[2]
    x = q(torch.randn(N, C, H, W) * 1.3 + 0.4, dt).requires_grad_(True)
    gamma = (torch.rand(C) + 0.5).requires_grad_(True)
    beta = torch.randn(C).requires_grad_(True)
    a = F.silu(F.group_norm(x, G, gamma, beta, 1e-5))
    gout = q(torch.randn_like(a), dt)
    a.backward(gout)
    xd = nhwc(x.detach()).to(dt).to(DEV)
    x1, x2 = xd[..., :C1].contiguous(), (xd[..., C1:].contiguous() if C2 else None)
    gd, gm_d, bt_d = nhwc(gout).to(dt).to(DEV), gamma.detach().to(DEV), beta.detach().to(DEV)
    _, _, mr = K.gn_stats(dt, x1, x2, N, HW, C1, C2, C1, C2, G, 1e-5, gm_d, bt_d)
    prev = q(torch.randn(N, H, W, C), dt).to(dt).to(DEV)
    res = {}
    for fused in (4, 0):
        dmc_opt("DMC_GN_BWD_FUSED", fused)
        for drop in (None, (11, 1 << 30, 4.0 / 3.0)):
            dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if C2 else None)
            dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            K.gn_bwd(dt, gd, C, x1, x2, N, HW, C1, C2, C1, C2, G, mr, gm_d, bt_d, True, drop, dx1, dx2, C1, C2,
                     0, 0, dg, db)
            out = [(torch.cat([dx1, dx2], -1) if C2 else dx1).float().cpu(), dg.cpu(), db.cpu()]
            if not C2:   # single source: accumulate into dx and the fused pixel sums
                dxs = prev.clone()
                snc = torch.full((N, C + 8), -7.0, device=DEV)
                sc_ = torch.empty(C, device=DEV)
                K.gn_bwd(dt, gd, C, x1, None, N, HW, C, 0, C, 0, G, mr, gm_d, bt_d, True, drop, dxs, None, C, 0, 1, 0,
                         dg, db, dx_sum_nc=snc, ld_sum_nc=C + 8, dx_sum_c=sc_)
                torch.cuda.synchronize()
                ref_nc = dxs.float().sum((1, 2))
                tag = f"fused={fused} drop={drop is not None}"
                assert rel_err(snc[:, :C], ref_nc) < 1e-4, (tag, rel_err(snc[:, :C], ref_nc),
                                                            (snc[:, :C] == -7.0).float().mean().item())
                assert (snc[:, C:] == -7.0).all(), tag
                assert rel_err(sc_, ref_nc.sum(0)) < 1e-4, (tag, rel_err(sc_, ref_nc.sum(0)))
                assert rel_err(dxs.float().cpu(), out[0] + prev.float().cpu()) < 1e-2
                out.append(snc[:, :C].cpu())
            res[(fused, drop is None)] = out
    dxk, dgk, dbk = res[(4, True)][:3]
    assert rel_err(nchw(dxk), x.grad) < 2e-2
    assert rel_err(dgk, gamma.grad) < 1e-4 and rel_err(dbk, beta.grad) < 1e-4
    for nodrop in (True, False):
        for u, v in zip(res[(4, nodrop)], res[(0, nodrop)]):
            assert rel_err(u, v) < 1e-2, (nodrop, rel_err(u, v))
    assert rel_err(res[(4, False)][0], dxk) > 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(128, 32, 32, 128), (128, 8, 8, 256), (16, 8, 8, 128)])
def test_gn_bwd_extra_operand(shape, dt):
    """dmc_gn_silu_bwd_deferred(add1=...): the identity-shortcut gradient added into the accumulated dx1 by the
    GroupNorm backward (round 6) vs the same call followed by a separate add (the executor's former order). bf16 on
    the one-pass kernel: one rounding instead of two, so within bf16 last-bit flips; fp32 / small batches take the
    other kernels plus the add launch, which is the separate add: bitwise."""
    L, K = _lib()
    torch.manual_seed(17)
    N, H, W, C = shape
    G, HW = 8, H * W
    x = (torch.randn(N, H, W, C) * 1.3 + 0.4).to(dt).to(DEV)
    g = torch.randn(N, H, W, C).to(dt).to(DEV)
    add = torch.randn(N, H, W, C).to(dt).to(DEV)
    prev = torch.randn(N, H, W, C).to(dt).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    _, _, mr = K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, G, 1e-5, gamma, beta)
    drop = (5, 1 << 29, 1.0 / 0.875)
    outs = []
    for fold in (False, True):
        dx = prev.clone()
        if not fold:
            K.add_(dt, dx, add)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        jobs = []
        K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, G, mr, gamma, beta, True, drop, dx, None, C, 0, 1, 0, dg, db,
                 defer=jobs, add1=add if fold else None, ld_add1=C if fold else 0)
        K.colsum_batch(jobs)
        torch.cuda.synchronize()
        outs.append((dx.float(), dg, db))
    (a, dga, dba), (b, dgb, dbb) = outs
    assert torch.equal(dga, dgb) and torch.equal(dba, dbb)
    fused = dt == torch.bfloat16 and N >= 64
    if fused:
        # reference: the GroupNorm gradient alone (no accumulation), summed with prev and add in fp32
        alone = torch.empty_like(prev)
        K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, G, mr, gamma, beta, True, drop, alone, None, C, 0, 0, 0,
                 torch.empty(C, device=DEV), torch.empty(C, device=DEV))
        torch.cuda.synchronize()
        ref = prev.float() + add.float() + alone.float()
        # one bf16 rounding of the three-term sum instead of two: no further from the fp32 sum than the separate add
        assert rel_err(b, ref) <= rel_err(a, ref) * 1.02, (rel_err(b, ref), rel_err(a, ref))
        assert rel_err(b, a) < 1e-2, rel_err(b, a)
    else:
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(128, 32, 32, 128), (128, 8, 8, 256), (64, 4, 4, 512)])
def test_gn_bwd_deferred_column_sums_bitwise(shape):
    """dmc_gn_silu_bwd_deferred + dmc_colsum_batch (the parameter column sums of several GroupNorm backwards in one
    launch) give BITWISE the dgamma / dbeta / per-c dx sums of the immediate dmc_gn_silu_bwd, and the same dx and
    per-(n, c) sums."""
    L, K = _lib()
    torch.manual_seed(9)
    N, H, W, C = shape
    G, dt, HW = 8, torch.bfloat16, H * W
    x = (torch.randn(N, H, W, C) * 1.3 + 0.4).to(dt).to(DEV)
    g = torch.randn(N, H, W, C).to(dt).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    _, _, mr = K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, G, 1e-5, gamma, beta)
    drop = (5, 1 << 29, 1.0 / 0.875)
    outs = []
    jobs = []
    for defer in (None, jobs):
        dx = torch.empty_like(x)
        dg, db, sc_ = (torch.full((C,), -3.0, device=DEV) for _ in range(3))
        snc = torch.empty(N, C, device=DEV)
        K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, G, mr, gamma, beta, True, drop, dx, None, C, 0, 0, 0, dg, db,
                 dx_sum_nc=snc, ld_sum_nc=C, dx_sum_c=sc_, defer=defer)
        if defer is not None:
            assert len(jobs) == 2                      # the one-pass kernel took it: A and the dx sums deferred
            assert (dg == -3.0).all() and (sc_ == -3.0).all()
            K.colsum_batch(jobs)
            assert not jobs
        torch.cuda.synchronize()
        outs.append((dx, dg, db, sc_, snc))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_groupnorm_stats_and_backward(dt):
    L, K = _lib()
    torch.manual_seed(2)
    N, H, W, C1, C2, G = 3, 8, 8, 48, 48, 8    # group 3 straddles the two sources (12 ch/group)
    x = q(torch.randn(N, C1 + C2, H, W) * 2 + 0.5, dt).requires_grad_(True)
    gamma = torch.rand(C1 + C2).requires_grad_(True)
    beta = torch.randn(C1 + C2).requires_grad_(True)
    z = F.group_norm(x, G, gamma, beta, 1e-5)
    a = F.silu(z)
    gout = q(torch.randn_like(a), dt)
    a.backward(gout)
    xd = nhwc(x.detach()).to(dt).to(DEV)
    x1, x2 = xd[..., :C1].contiguous(), xd[..., C1:].contiguous()
    sc, sh, mr = K.gn_stats(dt, x1, x2, N, H * W, C1, C2, C1, C2, G, 1e-5, gamma.detach().to(DEV),
                            beta.detach().to(DEV))
    torch.cuda.synchronize()
    zr = z.detach()
    mean = x.detach().view(N, G, -1).mean(-1)
    torch.testing.assert_close(mr.view(N, G, 2)[..., 0].cpu(), mean, rtol=1e-5, atol=1e-5)
    zk = xd.float().cpu().permute(0, 3, 1, 2) * sc.view(N, -1, 1, 1).cpu() + sh.view(N, -1, 1, 1).cpu()
    torch.testing.assert_close(zk, zr, rtol=1e-4, atol=1e-4)
    dx1 = torch.empty_like(x1)
    dx2 = torch.empty_like(x2)
    dg = torch.empty(C1 + C2, device=DEV)
    db = torch.empty(C1 + C2, device=DEV)
    K.gn_bwd(dt, nhwc(gout).to(dt).to(DEV), C1 + C2, x1, x2, N, H * W, C1, C2, C1, C2, G, mr, gamma.detach().to(DEV),
             beta.detach().to(DEV), True, None, dx1, dx2, C1, C2, 0, 0, dg, db)
    torch.cuda.synchronize()
    dxk = nchw(torch.cat([dx1, dx2], -1).float().cpu())
    assert rel_err(dxk, x.grad) < (1e-4 if dt == torch.float32 else 2e-2)
    assert rel_err(dg.cpu(), gamma.grad) < 1e-4 and rel_err(db.cpu(), beta.grad) < 1e-4
    # single source with dropout, accumulation and the fused pixel sums of the stored dx
    xs = xd.contiguous()
    scs, shs, mrs = K.gn_stats(dt, xs, None, N, H * W, C1 + C2, 0, C1 + C2, 0, G, 1e-5, gamma.detach().to(DEV),
                               beta.detach().to(DEV))
    prev = q(torch.randn(N, H, W, C1 + C2), dt).to(dt).to(DEV)
    dxs = prev.clone()
    snc = torch.full((N, 100), -7.0, device=DEV)
    sc_ = torch.empty(C1 + C2, device=DEV)
    drop = (7, 1 << 30, 4.0 / 3.0)   # (seed, thresh, scale): keep prob 0.75
    K.gn_bwd(dt, nhwc(gout).to(dt).to(DEV), C1 + C2, xs, None, N, H * W, C1 + C2, 0, C1 + C2, 0, G, mrs,
             gamma.detach().to(DEV), beta.detach().to(DEV), True, drop, dxs, None, C1 + C2, 0, 1, 0, dg, db,
             dx_sum_nc=snc, ld_sum_nc=100, dx_sum_c=sc_)
    dx0 = torch.empty_like(xs)
    K.gn_bwd(dt, nhwc(gout).to(dt).to(DEV), C1 + C2, xs, None, N, H * W, C1 + C2, 0, C1 + C2, 0, G, mrs,
             gamma.detach().to(DEV), beta.detach().to(DEV), True, drop, dx0, None, C1 + C2, 0, 0, 0, dg, db)
    torch.cuda.synchronize()
    assert rel_err(dxs.float(), dx0.float() + prev.float()) < (1e-5 if dt == torch.float32 else 1e-2)
    ref_nc = dxs.float().sum((1, 2))
    torch.testing.assert_close(snc[:, :C1 + C2], ref_nc, rtol=1e-4, atol=1e-3)
    assert (snc[:, C1 + C2:] == -7.0).all()
    torch.testing.assert_close(sc_, ref_nc.sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("path", ["auto", "staged", "hg4"])
@pytest.mark.parametrize("Lq,hd", [(16, 64), (64, 64), (256, 64), (1024, 64), (64, 8), (100, 16)])
def test_attention_fwd_bwd(dt, Lq, hd, path, monkeypatch, dmc_opt):
    """auto: row-resident kernels for L <= 256 (one head per block at this batch), staged above; staged: the
    64-row-tile kernels everywhere (DMC_ATTN_STAGED); hg4: resident blocks owning 4 heads where they fit."""
    L, K = _lib()
    dmc_opt("DMC_ATTN_STAGED", 1 if path == "staged" else 0)
    dmc_opt("DMC_ATTN_HG", 4 if path == "hg4" else 0)
    torch.manual_seed(3)
    N, heads = 2, 4
    C = heads * hd
    qkv = q(torch.randn(N, Lq, 3 * C), dt).requires_grad_(True)
    # reference: models/unet.py:88-96 channel layout
    t = qkv.view(N, Lq, 3, heads, hd).permute(2, 0, 3, 1, 4)
    qq, kk, vv = t[0], t[1], t[2]
    p = torch.softmax(qq @ kk.transpose(-2, -1) / math.sqrt(hd), -1)
    o = (p @ vv).permute(0, 2, 1, 3).reshape(N, Lq, C)
    do = q(torch.randn_like(o), dt)
    o.backward(do)
    qd = qkv.detach().to(dt).to(DEV).contiguous()
    od = torch.empty(N, Lq, C, dtype=dt, device=DEV)
    lse = torch.empty(N * heads * Lq, device=DEV)
    K.attn_fwd(dt, qd, 3 * C, N, Lq, heads, hd, od, C, lse)
    dq = torch.empty_like(qd)
    K.attn_bwd(dt, qd, 3 * C, od, do.to(dt).to(DEV), C, lse, N, Lq, heads, hd, dq, 3 * C)
    torch.cuda.synchronize()
    lim = 1e-4 if dt == torch.float32 else 3e-2
    assert rel_err(od.float().cpu(), o.detach()) < lim
    assert rel_err(dq.float().cpu(), qkv.grad) < (2e-4 if dt == torch.float32 else 5e-2)


def _hash_u32(x, seed):
    """csrc/dmc_common.h hash_u32 in numpy uint32 arithmetic (test-side reconstruction of the dropout mask)."""
    import numpy as np
    with np.errstate(over="ignore"):
        x = (x ^ np.uint32(seed)).astype(np.uint32)
        x = (x * np.uint32(0x9E3779B1)).astype(np.uint32); x ^= x >> np.uint32(16)
        x = (x * np.uint32(0x85EBCA6B)).astype(np.uint32); x ^= x >> np.uint32(13)
        x = (x * np.uint32(0xC2B2AE35)).astype(np.uint32); x ^= x >> np.uint32(16)
    return x


def drop_keep_np(idx, seed, thresh):
    """dmc_common.h drop_keep over an int64 index array (low 32 bits, seed mix of drop_seed_mix)."""
    import numpy as np
    with np.errstate(over="ignore"):
        mix = _hash_u32(np.zeros(1, np.uint32), np.uint32((seed * 0x27d4eb2f + 1) & 0xFFFFFFFF))[0]
    return _hash_u32((idx.astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32) ^ mix, seed) >= np.uint32(thresh)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("path", ["auto", "staged"])
@pytest.mark.parametrize("Lq", [64, 256, 320])
def test_attention_probability_dropout(dt, path, Lq, dmc_opt):
    """Attention-probability dropout (dmc_attn_fwd/bwd drop_* arguments, the DiT's nn.MultiheadAttention(dropout=p)):
    O = (softmax(QK^T/sqrt(hd)) * M / (1-p)) V with the counter-hash mask M[(n*heads+h)*L+q)*L+key] rebuilt on the
    host, forward and the q/k/v gradients vs torch autograd of that formula."""
    import numpy as np
    L, K = _lib()
    dmc_opt("DMC_ATTN_STAGED", 1 if path == "staged" else 0)
    torch.manual_seed(4)
    N, heads, hd = 2, 3, 64
    C = heads * hd
    p_drop, seed = 0.25, 12345
    thresh = int(round(p_drop * 4294967296.0))
    scale = 1.0 / (1.0 - p_drop)
    idx = np.arange(N * heads * Lq * Lq, dtype=np.int64)
    mask = torch.from_numpy(drop_keep_np(idx, seed, thresh).reshape(N, heads, Lq, Lq).astype(np.float32))
    assert 0.7 < mask.mean().item() < 0.8
    qkv = q(torch.randn(N, Lq, 3 * C), dt).requires_grad_(True)
    t = qkv.view(N, Lq, 3, heads, hd).permute(2, 0, 3, 1, 4)
    qq, kk, vv = t[0], t[1], t[2]
    pr = torch.softmax(qq @ kk.transpose(-2, -1) / math.sqrt(hd), -1)
    o = ((pr * mask * scale) @ vv).permute(0, 2, 1, 3).reshape(N, Lq, C)
    do = q(torch.randn_like(o), dt)
    o.backward(do)
    qd = qkv.detach().to(dt).to(DEV).contiguous()
    od = torch.empty(N, Lq, C, dtype=dt, device=DEV)
    lse = torch.empty(N * heads * Lq, device=DEV)
    drop = (seed, thresh, scale)
    K.attn_fwd(dt, qd, 3 * C, N, Lq, heads, hd, od, C, lse, drop=drop)
    dq = torch.empty_like(qd)
    K.attn_bwd(dt, qd, 3 * C, od, do.to(dt).to(DEV), C, lse, N, Lq, heads, hd, dq, 3 * C, drop=drop)
    torch.cuda.synchronize()
    lim = 1e-4 if dt == torch.float32 else 3e-2
    assert rel_err(od.float().cpu(), o.detach()) < lim, rel_err(od.float().cpu(), o.detach())
    assert rel_err(dq.float().cpu(), qkv.grad) < (2e-4 if dt == torch.float32 else 5e-2), rel_err(dq.float().cpu(),
                                                                                                      qkv.grad)


def test_elementwise_and_multitensor():
    L, K = _lib()
    torch.manual_seed(4)
    # loss fwd/bwd
    pred = torch.randn(4, 3, 8, 8, device=DEV)
    tgt = torch.randn(4, 3, 8, 8, device=DEV)
    for lt, fn in (("l2", F.mse_loss), ("l1", F.l1_loss), ("huber", F.smooth_l1_loss)):
        pc = pred.cpu().requires_grad_(True)
        ref = fn(tgt.cpu(), pc)
        ref.backward()
        got = K.loss_fwd(lt, pred, tgt)
        g = K.loss_bwd(lt, pred, tgt, torch.ones((), device=DEV))
        torch.testing.assert_close(got.cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(g.cpu(), pc.grad, rtol=1e-5, atol=1e-7)
    # EMA + clip
    ps = [torch.randn(n, device=DEV) for n in (10, 1000, 33333)]
    es = [torch.randn_like(p) for p in ps]
    es_ref = [e.clone().cpu() for e in es]
    refs = K.TensorRefs(list(zip(es, ps)), DEV)
    K.ema_update(refs, 0.999)
    for e, p, r in zip(es, ps, es_ref):
        r.mul_(0.999).add_(p.cpu(), alpha=1 - 0.999)
        torch.testing.assert_close(e.cpu(), r, rtol=1e-6, atol=1e-7)
    gs = [torch.randn(n, device=DEV) for n in (10, 1000, 33333)]
    gref = [g.cpu().clone().requires_grad_(False) for g in gs]
    tot = K.clip_grad_norm(K.TensorRefs([(g, None) for g in gs], DEV), 1.0)
    params = [torch.zeros_like(g, requires_grad=True) for g in gref]
    for p, g in zip(params, gref):
        p.grad = g
    tr = torch.nn.utils.clip_grad_norm_(params, 1.0)
    torch.testing.assert_close(tot.cpu(), tr, rtol=1e-5, atol=1e-6)
    for g, p in zip(gs, params):
        torch.testing.assert_close(g.cpu(), p.grad, rtol=1e-5, atol=1e-7)


def test_quantile_threshold_matches_torch():
    L, K = _lib()
    torch.manual_seed(5)
    N = 5
    x = torch.randn(N, 3, 32, 32, device=DEV) * 2
    ec = torch.randn_like(x)
    eu = torch.randn_like(x)
    t = torch.tensor([999, 500, 10, 0, 250], device=DEV)
    ac = torch.cumprod(1 - torch.linspace(1e-4, 0.02, 1000), 0).to(DEV)
    eps, x0 = K.cfg_x0(x, ec, eu, 3.0, t, ac, None, 0, 0.995)
    e_ref = eu.cpu() + 3.0 * (ec.cpu() - eu.cpu())
    at = ac.cpu()[t.cpu()].view(N, 1, 1, 1)
    x0r = (x.cpu() - torch.sqrt(1 - at) * e_ref) / torch.sqrt(at)
    s = torch.quantile(x0r.reshape(N, -1).abs(), 0.995, dim=1)
    s = torch.maximum(s, torch.ones_like(s)).view(N, 1, 1, 1)
    x0r = torch.clamp(x0r, -s, s) / s
    torch.testing.assert_close(eps.cpu(), e_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(x0.cpu(), x0r, rtol=1e-5, atol=1e-5)


def test_pack_weights_batch_matches_single_packs():
    """One dmc_pack_weights launch over mixed jobs == the per-weight dmc_pack_weight packs (all modes,
    bf16/fp32 destinations, column-block (koff) jobs of a row concatenation, a Kc=1 bias copy)."""
    L, K = _lib()
    torch.manual_seed(11)
    w3 = torch.randn(24, 16, 3, 3, device=DEV)
    w1 = torch.randn(40, 24, device=DEV)
    lins = [torch.randn(co, 32, device=DEV) for co in (8, 16, 24)]
    bias = [torch.randn(co, device=DEV) for co in (8, 16, 24)]
    bf = torch.bfloat16
    Kc3, Kc1 = L.kc_for(16, bf), L.kc_for(24, torch.float32)
    refs = {
        "fwd": K.pack_weight(L.PACK_FWD, bf, w3, Kc3),
        "dg": K.pack_weight(L.PACK_DGRAD, bf, w3, L.kc_for(24, bf)),
        "up": K.pack_weight(L.PACK_UPDGRAD, bf, w3, L.kc_for(24, bf)),
        "lin": K.pack_weight(L.PACK_FWD, torch.float32, w1, Kc1),
        "cat_dg": K.pack_weight(L.PACK_DGRAD, torch.float32, torch.cat(lins, 0), 64),
    }
    outs = {k: torch.full_like(v, 7.0) for k, v in refs.items()}
    outs["cat_dg"].zero_()     # koff jobs never touch the padding columns: zero from allocation
    bcat = torch.empty(48, device=DEV)
    jobs = [(w3, outs["fwd"], 0, L.PACK_FWD, 24, 16, 3, 3, Kc3, -1),
            (w3, outs["dg"], 0, L.PACK_DGRAD, 24, 16, 3, 3, L.kc_for(24, bf), -1),
            (w3, outs["up"], 0, L.PACK_UPDGRAD, 24, 16, 3, 3, L.kc_for(24, bf), -1),
            (w1, outs["lin"], 0, L.PACK_FWD, 40, 24, 1, 1, Kc1, -1)]
    off = 0
    for wl, b in zip(lins, bias):
        jobs.append((wl, outs["cat_dg"], 0, L.PACK_DGRAD, wl.shape[0], 32, 1, 1, 64, off))
        jobs.append((b, bcat, off, L.PACK_FWD, wl.shape[0], 1, 1, 1, 1, -1))
        off += wl.shape[0]
    K.PackBatch(jobs, DEV).launch()
    for k in refs:
        assert torch.equal(outs[k], refs[k]), k
    assert torch.equal(bcat, torch.cat(bias))


@pytest.mark.parametrize("n", [4099, 1 << 20])
def test_flat_grad_norm_and_adamw_match_torch(n):
    """dmc_grad_norm_flat + dmc_adamw_flat (clip, AdamW, EMA) vs clip_grad_norm_ + torch.optim.AdamW + the
    reference EMA (utils/trainer.py:198-202), 3 steps, ragged n."""
    L, K = _lib()
    torch.manual_seed(5)
    p = torch.randn(n, device=DEV)
    ema = p.clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    pr = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([pr], lr=1e-3, weight_decay=1e-2, foreach=True)
    er = ema.clone()
    lr, (b1, b2), eps, wd, d = 1e-3, (0.9, 0.999), 1e-8, 1e-2, 0.99
    for t in range(1, 4):
        g = torch.randn(n, device=DEV) * (0.01 if t == 2 else 1.0)
        total, coef = K.grad_norm_flat(g, 1.0)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        K.adamw_flat(p, g, m, v, ema, coef, 1 - lr * wd, 1 - b1, b2, 1 - b2, eps, (lr / bc1) * -1, bc2 ** 0.5,
                     d, 1 - d)
        pr.grad = g.clone()
        tr = torch.nn.utils.clip_grad_norm_([pr], 1.0)
        opt.step()
        er.mul_(d).add_(pr.detach(), alpha=1 - d)
        torch.testing.assert_close(total, tr, rtol=1e-5, atol=0)
        torch.testing.assert_close(p, pr.detach(), rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(m, opt.state[pr]["exp_avg"], rtol=1e-5, atol=1e-8)
        torch.testing.assert_close(v, opt.state[pr]["exp_avg_sq"], rtol=1e-5, atol=1e-10)
        torch.testing.assert_close(ema, er, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("Cin,Cout", [(4992, 512), (512, 4992)])
def test_conv_fp32_gemm_splitk_silu_pre(Cin, Cout):
    """The time-embedding GEMMs (1x1 'conv' over N=128 rows, fp32): split-K register-staged kernel with the
    SiLU-derivative (silu_pre) and bias epilogue, vs torch fp32."""
    import ctypes
    L, K = _lib()
    torch.manual_seed(8)
    N = 128
    x = torch.randn(N, Cin)
    w = torch.randn(Cout, Cin) / math.sqrt(Cin)
    bias = torch.randn(Cout)
    z = torch.randn(N, Cout)
    sg = torch.sigmoid(z)
    ref = (x @ w.t() + bias) * sg * (1 + z * (1 - sg))
    Kc = L.kc_for(Cin, torch.float32)
    wp = K.pack_weight(L.PACK_FWD, torch.float32, w.to(DEV), Kc)
    xd = torch.zeros(N, 1, 1, Kc, device=DEV)
    xd[..., :Cin] = x.view(N, 1, 1, Cin).to(DEV)
    y = torch.empty(N, 1, 1, Cout, device=DEV)
    d = K.make_desc(torch.float32, N, 1, 1, Cin, 0, Kc, 0, Kc, 1, 1, Cout, K.TAPS1)
    K.set_epilogue(d, bias=bias.to(DEV), silu_pre=z.to(DEV), ld_silu=Cout, ldy1=Cout)
    if Cin > 1024:
        assert L.LIB.dmc_conv2d_workspace(ctypes.byref(d)) > 0
    K.conv(d, xd, None, wp, y)
    torch.cuda.synchronize()
    assert rel_err(y.view(N, Cout).cpu(), ref) < 1e-5


@pytest.mark.parametrize("case", ["halo2_3x3", "glds1x1", "splitk_small", "fp32_reg", "concat_two"])
def test_conv_epilogue_groupnorm_partials(case, dmc_opt):
    """dmc_conv_desc.gn_part + dmc_gn_finalize (the conv epilogue's GroupNorm partials: in-kernel on the halo and
    LDS-DMA paths, one pass over the output elsewhere) give the statistics dmc_gn_stats computes over the stored
    output: mean / rstd and the folded scale / shift within 2e-5 (fp32 summation order)."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(11)
    dt = torch.float32 if case == "fp32_reg" else torch.bfloat16
    # (the halo cases need >= 240 256x128 tiles: fewer take the split-K path, whose partials come from one pass)
    N, H, W, Cin, Cout, taps = {"glds1x1": (8, 16, 16, 256, 256, K.TAPS1),
                                "halo2_3x3": (32, 32, 32, 128, 256, K.TAPS3),
                                "splitk_small": (2, 8, 8, 256, 256, K.TAPS3), "fp32_reg": (2, 16, 16, 64, 128, K.TAPS3),
                                "concat_two": (4, 16, 16, 128, 128, K.TAPS3)}[case]
    G = 8

    def conv_with_part(cout, seed):
        g = torch.Generator().manual_seed(seed)
        x = (torch.randn(N, H, W, Cin, generator=g) + 0.5).to(DEV).to(dt)
        w = (torch.randn(cout, Cin, int(len(taps) ** 0.5), int(len(taps) ** 0.5), generator=g) * 0.05).to(DEV)
        b = (torch.randn(cout, generator=g) + 2.0).to(DEV)        # a large mean: tests the M2 form
        Kc = L.kc_for(Cin, dt)
        wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
        y = torch.empty(N, H, W, cout, dtype=dt, device=DEV)
        part = torch.empty(N * H * W // 64 * (cout // 8) * 2, device=DEV)
        d = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, Kc, H, W, cout, taps)
        K.set_epilogue(d, bias=b, ldy1=cout, gn_part=part)
        K.conv(d, x, None, wp, y)
        return y, part

    y1, p1 = conv_with_part(Cout, 1)
    if case == "splitk_small":
        # the split-K epilogue emits the partials in its pass: bitwise the separate pass's (DMC_NO_SKGN=1)
        dmc_opt("DMC_NO_SKGN", 1)
        y1s, p1s = conv_with_part(Cout, 1)
        dmc_opt("DMC_NO_SKGN", 0)
        torch.cuda.synchronize()
        assert torch.equal(y1, y1s) and torch.equal(p1, p1s)
    if case == "halo2_3x3":
        d = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, L.kc_for(Cin, dt), H, W, Cout, taps)
        K.set_epilogue(d, ldy1=Cout)
        assert K.conv_fused(d) & L.FUSED_GN_STATS, case
    y2, p2, C2 = (None, None, 0)
    if case == "concat_two":
        y2, p2 = conv_with_part(256, 2)
        C2 = 256
    gamma = torch.randn(Cout + C2, generator=gen).to(DEV)
    beta = torch.randn(Cout + C2, generator=gen).to(DEV)
    sc, sh, mr = K.gn_finalize(p1, Cout, p2, C2, N, H * W, G, 1e-5, gamma, beta)
    rsc, rsh, rmr = K.gn_stats(dt, y1, y2, N, H * W, Cout, C2, Cout, C2, G, 1e-5, gamma, beta)
    torch.cuda.synchronize()
    for got, ref in ((mr, rmr), (sc, rsc), (sh, rsh)):
        assert rel_err(got, ref) < 2e-5, (case, rel_err(got, ref))


@pytest.mark.parametrize("N,H,C1,C2,Cout", [(128, 16, 256, 0, 768), (128, 8, 256, 0, 768), (128, 32, 256, 0, 128),
                                           (128, 16, 256, 256, 256), (128, 16, 768, 0, 256), (64, 8, 512, 0, 256)])
def test_gemm1x1_persistent_bitwise(N, H, C1, C2, Cout, dmc_opt):
    """The persistent 1x1 GEMM (gemm1x1_persist_kernel: tiles streamed through one LDS-DMA ring across tile
    boundaries, bias epilogue from the accumulators) is BITWISE the per-tile LDS-DMA kernel (DMC_GEMM1X1=0): same
    fragments, same K order, same rounding; and both match an fp32 torch GEMM of the bf16 operands."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(N + H + C1 + C2 + Cout)
    dt = torch.bfloat16
    x1 = torch.randn(N, H, H, C1, generator=gen).to(dt).to(DEV)
    x2 = torch.randn(N, H, H, C2, generator=gen).to(dt).to(DEV) if C2 else None
    w = (torch.randn(Cout, C1 + C2, 1, 1, generator=gen) * 0.05).to(DEV)
    b = torch.randn(Cout, generator=gen).to(DEV)
    Kc = L.kc_for(C1 + C2, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    outs = []
    for on in (1, 0):
        dmc_opt("DMC_GEMM1X1", on)
        y = torch.full((N, H, H, Cout), 7.0, device=DEV, dtype=dt)
        d = K.make_desc(dt, N, H, H, C1, C2, C1, C2, Kc, H, H, Cout, K.TAPS1)
        K.set_epilogue(d, bias=b, ldy1=Cout)
        K.conv(d, x1, x2, wp, y)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    xs = torch.cat([x1, x2], -1) if C2 else x1
    ref = xs.float().reshape(-1, C1 + C2) @ w.view(Cout, -1).to(dt).float().t() + b
    assert rel_err(outs[0].float().reshape(-1, Cout), ref) < 1e-2


@pytest.mark.parametrize("N,H,C1,Cout,inplace", [(128, 16, 256, 256, False), (128, 8, 256, 256, False),
                                                  (128, 32, 256, 128, True), (128, 16, 256, 512, True)])
def test_gemm1x1_persistent_residual_bitwise(N, H, C1, Cout, inplace, dmc_opt):
    """Round 6: the persistent 1x1 GEMM with the residual epilogue (the attention output projection x + proj(h) of
    models/unet.py:97-99, and the 1x1 input gradients that accumulate into an existing gradient, the residual then
    being the output itself) is BITWISE the per-tile LDS-DMA kernel (DMC_GEMM1X1=0: same fragments, same K order,
    (acc + bias) + residual rounded once) and matches an fp32 torch GEMM. (Same-box A/B of the residual form against
    the per-tile kernel for these layers: train 10,841 / 10,838 vs 10,865 / 10,836 img/s -- neutral.)"""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(N + H + C1 + Cout + int(inplace))
    dt = torch.bfloat16
    x1 = torch.randn(N, H, H, C1, generator=gen).to(dt).to(DEV)
    w = (torch.randn(Cout, C1, 1, 1, generator=gen) * 0.05).to(DEV)
    b = torch.randn(Cout, generator=gen).to(DEV)
    r0 = torch.randn(N, H, H, Cout, generator=gen).to(dt).to(DEV)
    Kc = L.kc_for(C1, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    outs = []
    for on in (1, 0):
        dmc_opt("DMC_GEMM1X1", on)
        if inplace:
            y = r0.clone()
            res = y
        else:
            y = torch.full((N, H, H, Cout), 7.0, device=DEV, dtype=dt)
            res = r0
        d = K.make_desc(dt, N, H, H, C1, 0, C1, 0, Kc, H, H, Cout, K.TAPS1)
        K.set_epilogue(d, bias=b, resid=res, ld_res=Cout, ldy1=Cout)
        K.conv(d, x1, None, wp, y)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = x1.float().reshape(-1, C1) @ w.view(Cout, -1).to(dt).float().t() + b + r0.float().reshape(-1, Cout)
    assert rel_err(outs[0].float().reshape(-1, Cout), ref) < 1e-2


@pytest.mark.parametrize("N,H,Cin,C1,C2", [(64, 32, 128, 128, 128), (64, 32, 128, 256, 128), (128, 16, 256, 256, 256),
                                          (32, 32, 128, 192, 64)])
def test_gemm1x1_persistent_split_output_bitwise(N, H, Cin, C1, C2, dmc_opt):
    """Round 6: the persistent 1x1 GEMM writing a split output (the 1x1 shortcut's input gradient into the two
    sources of a concat, models/unet.py:70 on the up path: y1 = channels [0, Csplit), y2 = the rest) is BITWISE the
    per-tile LDS-DMA kernel (DMC_GEMM1X1=0). (32, 32, 128, 192, 64): a split that is not a multiple of 128 keeps the
    per-tile kernel on both arms."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(N + H + C1 + C2)
    dt = torch.bfloat16
    Cout = C1 + C2
    x1 = torch.randn(N, H, H, Cin, generator=gen).to(dt).to(DEV)
    w = (torch.randn(Cout, Cin, 1, 1, generator=gen) * 0.05).to(DEV)
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    outs = []
    for on in (1, 0):
        dmc_opt("DMC_GEMM1X1", on)
        y1 = torch.full((N, H, H, C1), 7.0, device=DEV, dtype=dt)
        y2 = torch.full((N, H, H, C2), 7.0, device=DEV, dtype=dt)
        d = K.make_desc(dt, N, H, H, Cin, 0, Cin, 0, Kc, H, H, Cout, K.TAPS1)
        K.set_epilogue(d, ldy1=C1, ldy2=C2, Csplit=C1)
        K.conv(d, x1, None, wp, y1, y2)
        outs.append((y1, y2))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = x1.float().reshape(-1, Cin) @ w.view(Cout, -1).to(dt).float().t()
    got = torch.cat([outs[0][0], outs[0][1]], -1).float().reshape(-1, Cout)
    assert rel_err(got, ref) < 1e-2


@pytest.mark.parametrize("shape", [(32, 32, 32, 256, 0), (64, 16, 16, 128, 128)])
@pytest.mark.parametrize("silu,dropout", [(True, False), (True, True), (False, False)])
def test_gn_bwd_with_precomputed_partials(shape, silu, dropout):
    """dmc_gn_silu_bwd(part=...): the per-(64-pixel segment, channel) sums of dz and dz * xhat supplied from an
    earlier pass (here an fp64 host restatement with the counter-hash dropout mask) give the dx / dgamma / dbeta of
    the kernel's own reduction (summation order only)."""
    import numpy as np
    from diffusion_models_collection_amd import kernels as K
    N, H, W, C1, C2 = shape
    C, G, dt, HW = C1 + C2, 8, torch.bfloat16, H * W
    gen = torch.Generator().manual_seed(21)
    xs = (torch.randn(N, H, W, C, generator=gen) * 1.3 + 0.4).to(dt).to(DEV)
    x1 = xs[..., :C1].contiguous()
    x2 = xs[..., C1:].contiguous() if C2 else None
    gamma = (torch.rand(C, generator=gen) + 0.5).to(DEV)
    beta = torch.randn(C, generator=gen).to(DEV)
    _, _, mr = K.gn_stats(dt, x1, x2, N, HW, C1, C2, C1, C2, G, 1e-5, gamma, beta)
    drop = (7, 1 << 30, 4.0 / 3.0) if dropout else None
    g = torch.randn(N, H, W, C, generator=gen).to(dt).to(DEV)
    gv = g.double().cpu().view(N * HW, C)
    if dropout:
        idx = np.arange(N * HW * C, dtype=np.int64)
        keep = torch.from_numpy(drop_keep_np(idx, 7, 1 << 30).reshape(N * HW, C))
        gv = torch.where(keep, gv * (4.0 / 3.0), torch.zeros_like(gv))
    xv = xs.double().cpu().view(N, HW, C)
    m = mr.double().cpu().view(N, G, 2)
    mean = m[..., 0].repeat_interleave(C // G, 1).unsqueeze(1)
    rstd = m[..., 1].repeat_interleave(C // G, 1).unsqueeze(1)
    xh = ((xv - mean) * rstd).view(N * HW, C)
    dz = gv
    if silu:
        z = xh * gamma.double().cpu() + beta.double().cpu()
        sg = torch.sigmoid(z)
        dz = gv * sg * (1 + z * (1 - sg))
    part = torch.stack([dz.view(-1, 64, C).sum(1), (dz * xh).view(-1, 64, C).sum(1)], -1).float().contiguous().to(DEV)
    outs = []
    for pp in (part, None):
        dx1, dx2 = torch.empty_like(x1), (torch.empty_like(x2) if C2 else None)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        K.gn_bwd(dt, g, C, x1, x2, N, HW, C1, C2, C1, C2, G, mr, gamma, beta, silu, drop, dx1, dx2, C1, C2, 0, 0,
                 dg, db, part=pp)
        outs.append((torch.cat([dx1, dx2], -1) if C2 else dx1, dg, db))
    torch.cuda.synchronize()
    # bf16 dx: the two paths are different kernels (gn_bwd_apply's folded coefficients vs gn_bwd_fused's
    # sc * dz + ku * (x - mean) + kw, fp32 contraction chosen by the compiler), so last-bit flips of the bf16 rounding
    # (2^-8 relative each) are expected on a fraction of the elements: 3e-3 in the norm
    for a, b in zip(outs[0], outs[1]):
        assert rel_err(a.float(), b.float()) < (3e-3 if a.dtype == dt else 1e-5), (rel_err(a.float(), b.float()))


@pytest.mark.parametrize("case", ["linear", "concat", "ragged", "split_tail"])
def test_wgrad1x1_glds(case):
    """1x1 / Linear weight gradients (wgrad1x1_glds_kernel: both operands LDS-DMA'd as 64-pixel stages, 2-stage
    ring; the register-staged generic kernel where the shape does not fit it) and the bias gradient from the same
    launch vs an fp32 matmul of the same bf16 operands."""
    L, K = _lib()
    dt = torch.bfloat16
    torch.manual_seed(7)
    N, H, W, C1, C2, Cout = {"linear": (16, 16, 16, 384, 0, 1152), "concat": (8, 16, 16, 256, 128, 256),
                             "ragged": (4, 8, 8, 96, 0, 200), "split_tail": (3, 8, 8, 64, 0, 64)}[case]
    M = N * H * W
    x1 = torch.randn(M, C1).to(dt)
    x2 = torch.randn(M, C2).to(dt) if C2 else None
    g = torch.randn(M, Cout).to(dt)
    xs = torch.cat([x1, x2], 1) if C2 else x1
    ref_w = (g.float().t() @ xs.float())                           # [Cout, Cin]
    Cin = C1 + C2
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(Cin, dt), H, W, Cout, K.TAPS1)
    dw = torch.full((Cout, Cin, 1, 1), float("nan"), device=DEV)
    db = torch.full((Cout,), float("nan"), device=DEV)
    K.wgrad(d, g.to(DEV).view(N, H, W, Cout), Cout, x1.to(DEV).view(N, H, W, C1),
            x2.to(DEV).view(N, H, W, C2) if C2 else None, dw, dbias=db)
    torch.cuda.synchronize()
    assert rel_err(dw.cpu().view(Cout, Cin), ref_w) < 1e-5
    assert rel_err(db.cpu(), g.float().sum(0)) < 1e-5


@pytest.mark.parametrize("case", ["s1_8", "s1_4_concat", "s2", "up"])
def test_wgrad_small_maps_and_taps(case):
    """3x3 weight gradients off the halo kernel (the register-staged kernel: stride 1 at the 8x8 / 4x4 levels,
    stride 2, nearest-x2 upsample folded into the indexing) and the bias gradient, vs autograd of F.conv2d on the
    same bf16 values (fp32 CPU)."""
    L, K = _lib()
    dt = torch.bfloat16
    torch.manual_seed(3)
    N, H, W, C1, C2, Cout, stride, mode = {
        "s1_8": (4, 8, 8, 256, 0, 256, 1, L.MODE_NORMAL), "s1_4_concat": (8, 4, 4, 128, 128, 256, 1, L.MODE_NORMAL),
        "s2": (2, 16, 16, 128, 0, 128, 2, L.MODE_NORMAL), "up": (2, 8, 8, 128, 0, 128, 1, L.MODE_UPSAMPLE)}[case]
    Cin = C1 + C2
    x = q(torch.randn(N, Cin, H, W), dt).requires_grad_(True)
    w = q(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), dt).requires_grad_(True)
    xi = F.interpolate(x, scale_factor=2, mode="nearest") if mode == L.MODE_UPSAMPLE else x
    y = F.conv2d(xi, w, stride=stride, padding=1)
    g = q(torch.randn_like(y), dt)
    y.backward(g)
    OH, OW = y.shape[2], y.shape[3]
    gd = nhwc(g).to(dt).to(DEV)
    xd = nhwc(x.detach()).to(dt).to(DEV)
    x1, x2 = (xd[..., :C1].contiguous(), xd[..., C1:].contiguous()) if C2 else (xd, None)
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(Cin, dt), OH, OW, Cout, K.TAPS3, mode, stride)
    dw = torch.full_like(w, float("nan"), device=DEV)
    db = torch.full((Cout,), float("nan"), device=DEV)
    K.wgrad(d, gd, Cout, x1, x2, dw, dbias=db)
    torch.cuda.synchronize()
    assert rel_err(dw.cpu(), w.grad) < 1e-5
    assert rel_err(db.cpu(), g.float().sum((0, 2, 3))) < 1e-5


def test_wgrad_pipe_narrow_output_padded_dy():
    """The pipelined 3x3 weight gradient of the UNet's output conv (Cout = 3, dy in a pitch of 8): the dy pitch
    padding holds NaN here, and must not reach the weight or bias gradients (it feeds only accumulator rows that are
    never stored). Against an fp32 torch reference of the same bf16 operands."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    N, H, W, Cin, Cout = 16, 32, 32, 128, 3
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(N, H, W, Cin, generator=gen).to(torch.bfloat16)
    g = torch.randn(N, H, W, Cout, generator=gen).to(torch.bfloat16)
    gp = torch.full((N, H, W, 8), float("nan"), dtype=torch.bfloat16)
    gp[..., :Cout] = g
    d = K.make_desc(torch.bfloat16, N, H, W, Cin, 0, Cin, 0, L.kc_for(Cin, torch.bfloat16), H, W, Cout, K.TAPS3)
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=DEV)
    db = torch.full((Cout,), float("nan"), device=DEV)
    K.wgrad(d, gp.to(DEV), 8, x.to(DEV), None, dw, dbias=db)
    torch.cuda.synchronize()
    xr, gr = x.permute(0, 3, 1, 2).float(), g.permute(0, 3, 1, 2).float()
    wr = torch.nn.grad.conv2d_weight(xr, (Cout, Cin, 3, 3), gr, padding=1)
    assert torch.isfinite(dw).all() and torch.isfinite(db).all()
    assert rel_err(dw.cpu(), wr) < 1e-5
    assert rel_err(db.cpu(), gr.sum((0, 2, 3))) < 1e-5


def test_wgrad_partial_reduce_batch_bitwise():
    """dmc_conv2d_wgrad_partial + ONE dmc_wgrad_reduce_batch over the jobs of several layers (the pipelined 3x3 kernel
    with its bias, a two-source 1x1, the generic kernel on a stride-2 conv, an fp32 Linear-shaped 1x1), partial sums in
    slices of one arena (K.WgradDefer), equal dmc_conv2d_wgrad of each layer bitwise; an arena too small for the
    segment flushes early and grows, with the same results."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(11)
    bf, f32 = torch.bfloat16, torch.float32
    # (dtype, N, H, W, C1, C2, Cout, taps, stride, bias)
    cases = [(bf, 16, 32, 32, 128, 0, 128, K.TAPS3, 1, True), (bf, 8, 8, 8, 256, 128, 256, K.TAPS1, 1, True),
             (bf, 4, 16, 16, 128, 0, 128, K.TAPS3, 2, False), (f32, 128, 1, 1, 512, 0, 256, K.TAPS1, 1, True)]
    layers = []
    for dt, N, H, W, C1, C2, Cout, taps, stride, bias in cases:
        OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
        x1 = torch.randn(N, H, W, C1, generator=gen).to(dt).to(DEV)
        x2 = torch.randn(N, H, W, C2, generator=gen).to(dt).to(DEV) if C2 else None
        dy = torch.randn(N, OH, OW, Cout, generator=gen).to(dt).to(DEV)
        kh = 3 if len(taps) == 9 else 1
        d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(C1 + C2, dt), OH, OW, Cout, taps, L.MODE_NORMAL, stride)
        layers.append((d, dy, Cout, x1, x2, (Cout, C1 + C2, kh, kh), bias))

    def run(defer):
        outs = []
        for d, dy, Cout, x1, x2, wshape, bias in layers:
            dw = torch.full(wshape, float("nan"), device=DEV)
            db = torch.full((Cout,), float("nan"), device=DEV) if bias else None
            K.wgrad(d, dy, Cout, x1, x2, dw, 0.5, dbias=db, defer=defer)
            outs.append((dw, db))
        if defer is not None:
            defer.end_segment()
        torch.cuda.synchronize()
        return outs

    ref = run(None)
    small = K.WgradDefer()
    small.buf = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)   # forces early flushes and a regrow
    one_batch = K.WgradDefer()
    one_batch.every = 0                                                 # all four jobs in one launch
    for defer in (one_batch, K.WgradDefer(), small, small):
        got = run(defer)
        for (a, ab), (b, bb) in zip(ref, got):
            assert torch.equal(a, b)
            assert ab is None or torch.equal(ab, bb)
    assert small.buf.numel() > (1 << 20)


@pytest.mark.parametrize("shape", [(128, 32, 32, 128, 0, 128), (64, 32, 32, 128, 128, 128), (128, 16, 16, 256, 0, 256),
                                   (32, 16, 16, 256, 128, 256), (128, 8, 8, 256, 256, 256), (6, 8, 8, 128, 64, 192),
                                   (3, 16, 16, 128, 0, 200), (128, 4, 4, 256, 0, 256), (32, 4, 4, 256, 256, 256),
                                   (4, 4, 4, 128, 64, 64)])
def test_wgrad_pipe_kernel(shape, dmc_opt):
    """The pipelined 3x3 weight gradient (wgrad3x3_pipe_kernel: x-fragment addresses fixed per lane with the k-step
    and tap row shifts as immediates, double-buffered 128-pixel halos, [split][kk][co] slab) against the round-4 halo
    kernel (DMC_WG_PIPE=0) and an fp32 torch reference of the same bf16 operands: weight and bias gradients, two
    sources (virtual concat), ragged Cout, the B=128 split plans; and bitwise reproducible run to run."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    N, H, W, C1, C2, Cout = shape
    gen = torch.Generator().manual_seed(N + H + C1 + C2 + Cout)
    dt = torch.bfloat16
    x = torch.randn(N, H, W, C1 + C2, generator=gen).to(dt)
    g = torch.randn(N, H, W, Cout, generator=gen).to(dt)
    x1d = x[..., :C1].contiguous().to(DEV)
    x2d = x[..., C1:].contiguous().to(DEV) if C2 else None
    gd = g.to(DEV)
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(C1 + C2, dt), H, W, Cout, K.TAPS3)
    res = []
    for pipe in (1, 1, 0):
        dmc_opt("DMC_WG_PIPE", pipe)
        dw = torch.full((Cout, C1 + C2, 3, 3), float("nan"), device=DEV)
        db = torch.full((Cout,), float("nan"), device=DEV)
        K.wgrad(d, gd, Cout, x1d, x2d, dw, dbias=db)
        torch.cuda.synchronize()
        res.append((dw.cpu(), db.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])   # deterministic
    xr = x.permute(0, 3, 1, 2).float()
    gr = g.permute(0, 3, 1, 2).float()
    wr = torch.nn.grad.conv2d_weight(xr, (Cout, C1 + C2, 3, 3), gr, padding=1)
    assert rel_err(res[0][0], wr) < 1e-5, rel_err(res[0][0], wr)
    assert rel_err(res[0][0], res[2][0]) < 1e-5
    assert rel_err(res[0][1], gr.sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("case", ["halo2_32", "halo2_16", "glds_up"])
@pytest.mark.parametrize("shared_t", [False, True])
def test_reg_epilogue_bitwise_lds_staged(case, shared_t, dmc_opt):
    """The register epilogue (DMC_REG_EPI=3, default: bias, time-embedding row, residual and the GroupNorm partials
    straight from the accumulators, lane-pair exchanges for 16-byte stores) against the LDS-staged epilogue
    (DMC_REG_EPI=0) on the halo conv (32x32 and 16x16 tiles) and the LDS-DMA GEMM (the nearest-x2 upsample conv),
    with bias, a per-image or shared (ld_add = 0) time-embedding row and a residual: the stored outputs are bitwise
    equal (same additions in the same order), the GroupNorm partials equal up to their fp32 combine order."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    dt = torch.bfloat16
    # batch sizes that give the non-split plans (>= 240 tiles of 256 x 128), whose epilogues these are
    N, H, W, Cin, Cout, mode = {"halo2_32": (64, 32, 32, 128, 128, L.MODE_NORMAL),
                                "halo2_16": (128, 16, 16, 256, 256, L.MODE_NORMAL),
                                "glds_up": (64, 16, 16, 128, 128, L.MODE_UPSAMPLE)}[case]
    OH, OW = (2 * H, 2 * W) if mode == L.MODE_UPSAMPLE else (H, W)
    gen = torch.Generator().manual_seed(21)
    x = torch.randn(N, H, W, Cin, generator=gen).to(dt).to(DEV)
    w = (torch.randn(Cout, Cin, 3, 3, generator=gen) * 0.03).to(DEV)
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    bias = torch.randn(Cout, generator=gen).to(DEV)
    tv = torch.randn(1 if shared_t else N, Cout, generator=gen).to(DEV)
    resid = torch.randn(N, OH, OW, Cout, generator=gen).to(dt).to(DEV)
    outs = {}
    for reg in (3, 0):
        dmc_opt("DMC_REG_EPI", reg)
        d = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, Kc, OH, OW, Cout, K.TAPS3, mode)
        y = torch.full((N, OH, OW, Cout), float("nan"), dtype=dt, device=DEV)
        part = torch.full((N * OH * OW // 64 * (Cout // 8) * 2,), float("nan"), device=DEV)
        K.set_epilogue(d, bias=bias, addvec=tv, ld_add=0 if shared_t else Cout, resid=resid, ld_res=Cout,
                       ldy1=Cout, gn_part=part)
        K.conv(d, x, None, wp, y)
        torch.cuda.synchronize()
        fused = K.conv_fused(d) & L.FUSED_GN_STATS
        outs[reg] = (y.cpu(), part.cpu(), fused)
    (y3, p3, f3), (y0, p0, f0) = outs[3], outs[0]
    assert torch.isfinite(y3.float()).all()
    assert torch.equal(y3, y0)
    if f3 and f0:   # both epilogues emitted the partials
        assert torch.isfinite(p3).all() and torch.allclose(p3, p0, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", ["pro32", "pro32_concat", "pro16", "pro64", "lds_epi32"])
def test_lds_dma_plain_store_stress_bitwise(case, dmc_opt):
    """VERDICT r5 #8 ("LDS-DMA and plain LDS stores"): round 4's per-block GroupNorm combine in the
    prologue conv (DMC_PRO_PART, removed in round 5) corrupted single tiles intermittently at 32x32 -- a block-shared
    LDS array written by plain stores while the chunk's halo LDS-DMA was still in flight. The shipped kernels that
    mix plain LDS stores with LDS-DMA are the GroupNorm+SiLU prologue halo conv (each wave rewrites its own halo
    pieces after draining its own DMA, while OTHER waves' halo / weight DMA may still land in other regions) and the
    LDS-staged epilogue (after the last weight slice's wait). Such a race shows as rare, launch-to-launch differences:
    64 back-to-back launches of each on the B=128 benchmark shapes must all be bitwise equal to the first, and (the
    prologue cases) to the materialised GroupNorm-apply + plain halo conv."""
    L, K = _lib()
    dt = torch.bfloat16
    torch.manual_seed(21)
    N, H, C1, C2, Cout = {"pro32": (128, 32, 128, 0, 128), "pro32_concat": (128, 32, 256, 128, 128),
                          "pro16": (128, 16, 256, 0, 256), "pro64": (32, 64, 128, 0, 128),
                          "lds_epi32": (128, 32, 128, 0, 128)}[case]
    pro = case.startswith("pro")
    if not pro:
        dmc_opt("DMC_REG_EPI", 0)         # every tile through the LDS-staged epilogue (with GroupNorm partials)
    W, Cin, G = H, C1 + C2, 8
    xd = (torch.randn(N, H, W, Cin, device=DEV) * 1.3 + 0.2).to(dt)
    x1d, x2d = (xd[..., :C1].contiguous(), xd[..., C1:].contiguous()) if C2 else (xd, None)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / math.sqrt(Cin * 9)
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    bias = torch.randn(Cout, device=DEV)
    addv = torch.randn(N, Cout, device=DEV)
    resid = torch.randn(N, H, W, Cout, device=DEV).to(dt)
    gamma, beta = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV)
    sc, sh, _ = K.gn_stats(dt, x1d, x2d, N, H * W, C1, C2, C1, C2, G, 1e-5, gamma, beta)
    gpart = torch.empty(N * H * W // 64 * (Cout // 8) * 2, dtype=torch.float32, device=DEV)
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, Kc, H, W, Cout, K.TAPS3)
    if pro:
        K.set_prologue(d, L.PRO_AFFINE_SILU, sc, sh, Cin)
        assert K.conv_halo_prologue(d)
    K.set_epilogue(d, bias=bias, addvec=addv, ld_add=Cout, resid=resid, ld_res=Cout, ldy1=Cout,
                   gn_part=None if pro else gpart)
    outs, parts = [], []
    ys = [torch.empty(N, H, W, Cout, dtype=dt, device=DEV) for _ in range(4)]
    for i in range(64):
        y = ys[i % 4]
        K.conv(d, x1d, x2d, wp, y)
        if i % 4 == 3 or i == 0:
            torch.cuda.synchronize()
        if i == 0:
            ref, pref = y.clone(), (None if pro else gpart.clone())
        elif i % 4 == 3:
            for yy in ys:
                outs.append(torch.equal(yy, ref))
            if not pro:
                parts.append(torch.equal(gpart, pref))
    torch.cuda.synchronize()
    assert all(outs), f"{outs.count(False)} of {len(outs)} launches differ from the first"
    assert all(parts)
    if pro:
        a = K.gn_apply(dt, x1d, x2d, N, H * W, C1, C2, C1, C2, sc, sh, silu=True).view(N, H, W, Cin)
        d0 = K.make_desc(dt, N, H, W, Cin, 0, Cin, 0, Kc, H, W, Cout, K.TAPS3)
        K.set_epilogue(d0, bias=bias, addvec=addv, ld_add=Cout, resid=resid, ld_res=Cout, ldy1=Cout)
        y0 = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
        K.conv(d0, a, None, wp, y0)
        torch.cuda.synchronize()
        assert torch.equal(ref, y0)


@pytest.mark.parametrize("size", ["bn16", "bn32"])
@pytest.mark.parametrize("case", ["f4", "f4_concat", "d4", "f8", "f8_concat", "d8"])
def test_conv3x3_img_kernel(case, size, dmc_opt):
    """Round 6 whole-image small-map conv (conv3x3_img_kernel, DMC_IMG_MASK): bf16 3x3 stride-1 forward (with the
    ResBlock conv2 epilogue: bias + time embedding + residual) and input gradient (flipped / transposed pack) at the
    UNet's 4x4 and 8x8 levels, one and two (virtual concat) sources, against the fp32 torch reference of the same
    bf16 operands (models/unet.py:34-60 at the two deepest levels). The batch picks the channel tile: few images
    give 16-channel tiles, many 32 (the planner's ~256-block rule)."""
    L, K = _lib()
    dmc_opt("DMC_IMG_MASK", 15)
    dt = torch.bfloat16
    torch.manual_seed(31)
    H = 4 if case.endswith("4") or "4_" in case else 8
    N = (16 if H == 4 else 4) if size == "bn16" else (256 if H == 4 else 128)
    if size == "bn32" and case == "d8":
        N = 64   # 8x8 with 512 output channels: one round of 256 blocks (more rounds keep the split-K plan)
    dgrad = case.startswith("d")
    C1, C2, Cout = {"f": (256, 0, 256), "f_concat": (256, 256, 256), "d": (256, 0, 512)}[
        case[0] + ("_concat" if "concat" in case else "")]
    x1 = torch.randn(N, C1, H, H)
    x2 = torch.randn(N, C2, H, H) if C2 else None
    xr = q(x1, dt) if x2 is None else torch.cat([q(x1, dt), q(x2, dt)], 1)
    if dgrad:   # dx = conv_transpose(dy, w) of the forward conv Cout -> C1 (w: [C1, Cout, 3, 3])
        w = torch.randn(C1, Cout, 3, 3) / math.sqrt(C1 * 9)
        yr = F.conv_transpose2d(xr, q(w, dt), padding=1)
    else:
        w = torch.randn(Cout, C1 + C2, 3, 3) / math.sqrt((C1 + C2) * 9)
        bias, addv, resid = torch.randn(Cout), torch.randn(N, Cout), torch.randn(N, Cout, H, H)
        yr = F.conv2d(xr, q(w, dt), bias, padding=1) + addv[:, :, None, None] + q(resid, dt)
    x1d = nhwc(x1).to(dt).to(DEV)
    x2d = nhwc(x2).to(dt).to(DEV) if x2 is not None else None
    Kc = L.kc_for(C1 + C2, dt)
    wp = K.pack_weight(L.PACK_DGRAD if dgrad else L.PACK_FWD, dt, w.to(DEV), Kc)
    d = K.make_desc(dt, N, H, H, C1, C2, C1, C2, Kc, H, H, Cout, K.TAPS3_DGRAD if dgrad else K.TAPS3)
    if dgrad:
        K.set_epilogue(d, ldy1=Cout)
    else:   # at 8x8 the epilogue also emits the next GroupNorm's partials (64-pixel segment = one image)
        part = torch.full((N * H * H // 64 * (Cout // 8) * 2,), float("nan"), device=DEV) if H == 8 else None
        K.set_epilogue(d, bias=bias.to(DEV), addvec=addv.to(DEV), ld_add=Cout, resid=nhwc(resid).to(dt).to(DEV),
                       ld_res=Cout, ldy1=Cout, gn_part=part)
    y = torch.empty(N, H, H, Cout, dtype=dt, device=DEV)
    K.conv(d, x1d, x2d, wp, y)
    torch.cuda.synchronize()
    got = nchw(y.float().cpu())
    e = rel_err(got, yr)
    assert e < 1e-2, e
    if not dgrad and H == 8:   # (mean, M2) of the stored bf16 values per (64-pixel segment, 8-channel chunk)
        v = y.float().view(N * H * H // 64, 64, Cout // 8, 8).permute(0, 2, 1, 3).reshape(-1, 512)
        m = v.mean(1)
        m2 = ((v - m[:, None]) ** 2).sum(1)
        p2 = part.view(-1, 2)
        assert torch.allclose(p2[:, 0], m, rtol=1e-4, atol=1e-5)
        assert torch.allclose(p2[:, 1], m2, rtol=1e-4, atol=1e-3)
    # the same launch twice: bitwise reproducible
    y2 = torch.empty_like(y)
    K.conv(d, x1d, x2d, wp, y2)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)


@pytest.mark.parametrize("case", ["c4", "c4_concat", "c8", "c8_concat"])
def test_conv3x3_img_gn_silu_prologue(case, dmc_opt):
    """Round 6: DMC_PRO_GN_SILU on the whole-image small-map conv -- conv(SiLU(GroupNorm(x))) with the GroupNorm
    statistics of each image computed inside the conv from its LDS chunks (no statistics / finalize / apply launch),
    the ResBlock inference chain of models/unet.py:34-38 / :50-60 at the 4x4 and 8x8 levels (one source, or the
    up-path concat whose 512 channels make 64-channel groups), against torch's fp32 group_norm -> silu -> bf16 ->
    conv2d on the same bf16 operands."""
    L, K = _lib()
    dmc_opt("DMC_IMG_MASK", 15)
    dt = torch.bfloat16
    torch.manual_seed(41)
    H = 4 if case.startswith("c4") else 8
    N = 128
    C1, C2, Cout, G = (256, 256, 256, 8) if "concat" in case else (256, 0, 256, 8)
    x1 = torch.randn(N, C1, H, H) * 1.7 + 0.3
    x2 = torch.randn(N, C2, H, H) * 0.8 - 0.2 if C2 else None
    xr = q(x1, dt) if x2 is None else torch.cat([q(x1, dt), q(x2, dt)], 1)
    gamma, beta = torch.rand(C1 + C2) + 0.5, torch.randn(C1 + C2) * 0.3
    a = q(F.silu(F.group_norm(xr, G, gamma, beta, 1e-5)), dt)
    w = torch.randn(Cout, C1 + C2, 3, 3) / math.sqrt((C1 + C2) * 9)
    bias, addv, resid = torch.randn(Cout), torch.randn(N, Cout), torch.randn(N, Cout, H, H)
    yr = F.conv2d(a, q(w, dt), bias, padding=1) + addv[:, :, None, None] + q(resid, dt)
    x1d = nhwc(x1).to(dt).to(DEV)
    x2d = nhwc(x2).to(dt).to(DEV) if x2 is not None else None
    Kc = L.kc_for(C1 + C2, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w.to(DEV), Kc)
    d = K.make_desc(dt, N, H, H, C1, C2, C1, C2, Kc, H, H, Cout, K.TAPS3)
    K.set_prologue(d, L.PRO_GN_SILU, gamma.to(DEV), beta.to(DEV), C1 + C2)
    d.pro_groups, d.pro_eps = G, 1e-5
    assert K.conv_halo_prologue(d)
    K.set_epilogue(d, bias=bias.to(DEV), addvec=addv.to(DEV), ld_add=Cout, resid=nhwc(resid).to(dt).to(DEV),
                   ld_res=Cout, ldy1=Cout)
    y = torch.empty(N, H, H, Cout, dtype=dt, device=DEV)
    K.conv(d, x1d, x2d, wp, y)
    torch.cuda.synchronize()
    got = nchw(y.float().cpu())
    e = rel_err(got, yr)
    assert e < 1e-2, e
    # a descriptor the small-map kernel cannot take is refused, not silently run another way
    d2 = K.make_desc(dt, N, 16, 16, 256, 0, 256, 0, L.kc_for(256, dt), 16, 16, 256, K.TAPS3)
    K.set_prologue(d2, L.PRO_GN_SILU, gamma[:256].to(DEV), beta[:256].to(DEV), 256)
    d2.pro_groups, d2.pro_eps = G, 1e-5
    assert not K.conv_halo_prologue(d2)
    with pytest.raises(RuntimeError):
        K.conv(d2, torch.zeros(N, 16, 16, 256, dtype=dt, device=DEV), None,
               K.pack_weight(L.PACK_FWD, dt, torch.zeros(256, 256, 3, 3, device=DEV), L.kc_for(256, dt)),
               torch.empty(N, 16, 16, 256, dtype=dt, device=DEV))


@pytest.mark.parametrize("shape", [(128, 4, 4, 256, 0, 256), (128, 4, 4, 256, 256, 256), (64, 4, 4, 128, 0, 64)])
@pytest.mark.parametrize("deferred", [False, True])
def test_wgrad_img4_kernel(shape, deferred, dmc_opt):
    """Round 6 whole-image 4x4 weight gradient (wgrad3x3_img4_kernel, DMC_WG_IMG4): every pixel of the batch in one
    block per 16 co x 16 ci tile, no slab and no reduction job (a deferred call leaves nothing to flush), the bias
    gradient from a ones-MFMA: against the fp32 torch reference of the same bf16 operands and the pipelined slab
    kernel (DMC_WG_IMG4=0), one and two (virtual concat) sources, bitwise reproducible run to run
    (models/unet.py:34-60 conv weights at the 4x4 level)."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    N, H, W, C1, C2, Cout = shape
    gen = torch.Generator().manual_seed(7 + N + C2)
    dt = torch.bfloat16
    x = torch.randn(N, H, W, C1 + C2, generator=gen).to(dt)
    g = torch.randn(N, H, W, Cout, generator=gen).to(dt)
    x1d = x[..., :C1].contiguous().to(DEV)
    x2d = x[..., C1:].contiguous().to(DEV) if C2 else None
    gd = g.to(DEV)
    d = K.make_desc(dt, N, H, W, C1, C2, C1, C2, L.kc_for(C1 + C2, dt), H, W, Cout, K.TAPS3)
    res = []
    for img in (1, 1, 0):
        dmc_opt("DMC_WG_IMG4", img)
        dw = torch.full((Cout, C1 + C2, 3, 3), float("nan"), device=DEV)
        db = torch.full((Cout,), float("nan"), device=DEV)
        if deferred:
            defer = K.WgradDefer()
            K.wgrad(d, gd, Cout, x1d, x2d, dw, scale=0.5, dbias=db, defer=defer)
            if img:
                assert not defer.jobs      # reduced in the kernel: nothing deferred
            defer.flush()
        else:
            K.wgrad(d, gd, Cout, x1d, x2d, dw, scale=0.5, dbias=db)
        torch.cuda.synchronize()
        res.append((dw.cpu(), db.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])   # deterministic
    xr = x.permute(0, 3, 1, 2).float()
    gr = g.permute(0, 3, 1, 2).float()
    wr = 0.5 * torch.nn.grad.conv2d_weight(xr, (Cout, C1 + C2, 3, 3), gr, padding=1)
    assert rel_err(res[0][0], wr) < 1e-5, rel_err(res[0][0], wr)
    assert rel_err(res[0][0], res[2][0]) < 1e-5
    assert rel_err(res[0][1], 0.5 * gr.sum((0, 2, 3))) < 1e-5
