"""Numerics of the DiT token-wise kernels (csrc/dmc_dit.hip) and the conv GELU epilogue against plain PyTorch fp32
references of the same ops (models/dit.py of the reference, :111-132 and :98-104).

Tolerances: fp32 1e-5 relative to the tensor's max magnitude; bf16 outputs within 1e-2 (one bf16 rounding); the
fused GELU epilogue is bitwise equal to conv + dmc_gelu_fwd on the stored pre-activation."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def _mod(B, C, gen):
    # [B, ld_mod] fp32 modulation rows: shift at 0, scale at C, gate at 2C (ld padded)
    return (torch.randn(B, 3 * C + 8, generator=gen) * 0.5).to(DEV)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,L,branch", [(384, 256, True), (64, 64, False), (1152, 16, True)])
def test_ln_mod_fwd_bwd(dt, C, L, branch):
    from diffusion_models_collection_amd import kernels as K
    gen = torch.Generator().manual_seed(3)
    B = 3
    T = B * L
    x = torch.randn(T, C, generator=gen).to(DEV)
    br = torch.randn(T, C, generator=gen).to(DEV).to(dt) if branch else None
    mod = _mod(B, C, gen)
    ld = mod.shape[1]
    h = torch.empty(T, C, dtype=dt, device=DEV)
    mean = torch.empty(T, device=DEV)
    rstd = torch.empty(T, device=DEV)
    xo = torch.empty(T, C, device=DEV) if branch else None
    K.ln_mod_fwd(dt, x, T, C, L, mod, ld, 0, C, 1e-6, h, C, mean, rstd, br=br, ld_br=C, off_gate=2 * C, x_out=xo)
    # torch reference (fp32, autograd)
    xr = x.clone().requires_grad_(True)
    brr = br.float().clone().requires_grad_(True) if branch else None
    modr = mod.clone().requires_grad_(True)
    sh = modr[:, :C].repeat_interleave(L, 0)
    sc = modr[:, C:2 * C].repeat_interleave(L, 0)
    xn = xr + modr[:, 2 * C:3 * C].repeat_interleave(L, 0) * brr if branch else xr
    hr = torch.nn.functional.layer_norm(xn, (C,), eps=1e-6) * (1 + sc) + sh
    lim = 1e-5 if dt == torch.float32 else 1e-2
    assert rel(h, hr) < lim, rel(h, hr)
    if branch:
        assert rel(xo, xn) < 1e-6
    if C > 512:
        return   # ln_mod_bwd: C <= 512
    dh = torch.randn(T, C, generator=gen).to(DEV)
    (hr * dh).sum().backward()
    dx = torch.zeros(T, C, device=DEV)
    dmod = torch.zeros_like(mod)
    K.ln_mod_bwd(dt, dh.to(dt), C, xo if branch else x, mean, rstd, mod, ld, C, T, C, L, dx, dmod, C, 0)
    # dx = gradient of the LayerNorm input xn, which equals xr.grad (xn = xr + gate * branch)
    lim = 1e-4 if dt == torch.float32 else 2e-2
    assert rel(dx, xr.grad) < lim, rel(dx, xr.grad)
    assert rel(dmod[:, :C], modr.grad[:, :C]) < lim
    assert rel(dmod[:, C:2 * C], modr.grad[:, C:2 * C]) < lim
    if branch:
        # gate_bwd: d(branch) = dy * gate, dgate = token sum of dy * branch
        dbr = torch.empty(T, C, dtype=dt, device=DEV)
        dmod2 = torch.zeros_like(mod)
        K.gate_bwd(dt, xr.grad.contiguous(), br, C, mod, ld, 2 * C, T, C, L, dbr, C, dmod2, 2 * C)
        assert rel(dbr, brr.grad) < (1e-5 if dt == torch.float32 else 1e-2)
        assert rel(dmod2[:, 2 * C:3 * C], modr.grad[:, 2 * C:3 * C]) < 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gelu_fwd_bwd(dt):
    from diffusion_models_collection_amd import kernels as K
    gen = torch.Generator().manual_seed(4)
    u = (torch.randn(777, 96, generator=gen) * 3).to(DEV).to(dt)
    a = torch.empty_like(u)
    K.gelu_fwd(dt, u, 777, 96, 96, a)
    ur = u.float().clone().requires_grad_(True)
    ar = torch.nn.functional.gelu(ur)
    assert rel(a, ar) < (1e-6 if dt == torch.float32 else 8e-3)
    da = torch.randn(777, 96, generator=gen).to(DEV)
    (ar * da).sum().backward()
    du = torch.empty_like(u)
    K.gelu_bwd(dt, da.to(dt), u, 777, 96, 96, du)
    assert rel(du, ur.grad) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt,M", [(torch.bfloat16, 65536), (torch.bfloat16, 512), (torch.float32, 4096)])
def test_conv_gelu_epilogue_bitwise(dt, M):
    """act=GELU in the conv epilogue (LDS-DMA kernel at large M, split-K at small M, register kernel in fp32):
    the activation equals dmc_gelu_fwd of the separately stored pre-activation bitwise, and the stored
    pre-activation equals the plain conv output bitwise."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    gen = torch.Generator().manual_seed(5)
    Cin, Cout = 384, 1536
    x = torch.randn(M, Cin, generator=gen).to(DEV).to(dt)
    w = (torch.randn(Cout, Cin, generator=gen) * 0.05).to(DEV)
    b = torch.randn(Cout, generator=gen).to(DEV)
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)

    def run(act, y_pre=None, drop=None):
        y = torch.empty(M, Cout, dtype=dt, device=DEV)
        d = K.make_desc(dt, M, 1, 1, Cin, 0, Cin, 0, Kc, 1, 1, Cout, K.TAPS1)
        if drop is not None:
            K.set_prologue(d, L.PRO_NONE, drop=drop)
        K.set_epilogue(d, bias=b, ldy1=Cout, act=act, y_pre=y_pre, ld_pre=Cout if y_pre is not None else 0)
        K.conv(d, x, None, wp, y)
        return y

    plain = run(L.ACT_NONE)
    pre = torch.empty_like(plain)
    fused = run(L.ACT_GELU, pre)
    ref = torch.empty_like(plain)
    K.gelu_fwd(dt, plain, M, Cout, Cout, ref)
    torch.cuda.synchronize()
    assert torch.equal(pre, plain)
    assert torch.equal(fused, ref)
    fused2 = run(L.ACT_GELU)          # without the pre-activation copy
    assert torch.equal(fused2, ref)
    # GELU + the MLP Dropout (p = 0.1, a device seed base as in the graphed step): bitwise dmc_gelu_fwd with the
    # same dropout of the stored pre-activation
    base = torch.tensor([77], dtype=torch.int32, device=DEV)
    drop = (1234, int(0.1 * 2 ** 32), 1.0 / 0.9, base.data_ptr())
    pre_d = torch.empty_like(plain)
    fused_d = run(L.ACT_GELU_DROP, pre_d, drop)
    ref_d = torch.empty_like(plain)
    K.gelu_fwd(dt, plain, M, Cout, Cout, ref_d, drop=drop)
    torch.cuda.synchronize()
    assert torch.equal(pre_d, plain)
    assert torch.equal(fused_d, ref_d)
    zero = (fused_d == 0).float().mean().item()
    assert 0.07 < zero < 0.13, zero
    # DGELU: an input-gradient-shaped conv whose epilogue applies dmc_gelu_bwd with the stored pre-activation
    for dr in (None, drop):
        dgel = run(L.ACT_DGELU, pre_d, dr)
        ref_b = torch.empty_like(plain)
        K.gelu_bwd(dt, plain, pre_d, M, Cout, Cout, ref_b, drop=dr)
        torch.cuda.synchronize()
        assert torch.equal(dgel, ref_b)


def test_timestep_embedding_batch_sum_patch_dgrad():
    from diffusion_models_collection_amd import kernels as K
    from oracle.dit_oracle import timestep_embedding
    t = torch.tensor([0, 1, 17, 500, 999], dtype=torch.long)
    out = torch.empty(5, 256, device=DEV)
    K.timestep_embedding(t.to(DEV), 256, out)
    # 1e-4: cos/sin of arguments t*f up to ~1000, where one ulp of the fp32 argument (exp of the frequencies on
    # the GPU vs the host's vectorised exp) moves the result by ~6e-5
    assert rel(out, timestep_embedding(t, 256)) < 1e-4
    gen = torch.Generator().manual_seed(6)
    x = torch.randn(7, 1000, generator=gen).to(DEV)
    s = torch.empty(1000, device=DEV)
    K.batch_sum(x, 7, 1000, s)
    assert rel(s, x.sum(0)) < 1e-6
    # patch embedding input gradient: conv_transpose2d with stride = kernel = p
    B, C, H, p, ht, wt = 2, 3, 64, 2, 4, 5
    dtok = torch.randn(B, ht, wt, H, generator=gen).to(DEV)
    w = torch.randn(H, C, p, p, generator=gen).to(DEV)
    dx = torch.empty(B, C, ht * p, wt * p, device=DEV)
    K.patch_dgrad(dtok, H, w, B, ht, wt, p, C, H, dx)
    ref = torch.nn.functional.conv_transpose2d(dtok.permute(0, 3, 1, 2), w, stride=p)
    assert rel(dx, ref) < 1e-5
