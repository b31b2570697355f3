"""CPU tests: the C-ABI library loads and exports every declared symbol; host-side API parity with the
reference (constructors, tables, timesteps, state_dict layout, error behaviour). No GPU compute here."""
import re
from pathlib import Path

import pytest
import torch

from conftest import ROOT, load_golden


def _ensure_lib():
    lib = ROOT / "diffusion_models_collection_amd" / "libdmc.so"
    if not lib.exists():
        from diffusion_models_collection_amd.build import build
        build()
    return lib


def test_library_exports_header_symbols():
    _ensure_lib()
    import ctypes
    hdr = (ROOT / "include" / "dmc.h").read_text()
    names = sorted(set(re.findall(r"^\s*(?:int|long|void|size_t|const char\*)\s+(dmc_\w+)\s*\(", hdr, re.M)))
    assert len(names) >= 29, names
    lib = ctypes.CDLL(str(ROOT / "diffusion_models_collection_amd" / "libdmc.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from diffusion_models_collection_amd import _lib
    assert set(names) == set(_lib.EXPORTS), set(names) ^ set(_lib.EXPORTS)
    assert _lib.LIB.dmc_version() == 1


def test_descriptor_validation_errors():
    """Bad descriptors are rejected on the host with a message (no launch happens)."""
    _ensure_lib()
    from diffusion_models_collection_amd import kernels as K, _lib as L
    d = K.make_desc(torch.float32, 1, 4, 4, 6, 0, 8, 0, 32, 4, 4, 8, K.TAPS3)   # C1=6 not multiple of 4
    K.set_prologue(d, L.PRO_AFFINE_SILU)
    with pytest.raises(L.DMCError, match="multiples"):
        L.check(L.LIB.dmc_conv2d(__import__("ctypes").byref(d), None, None, None, None, None, None, 0, None),
                    "conv")
    with pytest.raises(L.DMCError, match="head dim"):
        L.check(L.LIB.dmc_attn_fwd(0, None, 768, 1, 16, 4, 100, None, 256, None, 0, None, 0, 1.0, None), "attn")


def test_schedule_op_sequence_reproduces_fixture():
    """With this host's torch sqrt/log/cos as primitives, the product's explicit op sequence reproduces all 36
    fixture tables bit for bit (the op order is the reference's). Only meaningful on a host whose torch
    CPU transcendentals give the fixture host's bits; elsewhere it is skipped (the product never uses them)."""
    import numpy as np
    from diffusion_models_collection_amd.diffusion import _schedule as S
    g = load_golden("schedules")
    probe = S.TorchPrims.sqrt(g["linear/alphas_cumprod"].numpy())
    if not np.array_equal(probe, g["linear/sqrt_alphas_cumprod"].numpy()):
        pytest.skip("this host's torch CPU sqrt (MKL VML) differs from the fixture host's")
    for kind in ("linear", "cosine", "quadratic"):
        t = S.build_tables(1000, 1e-4, 0.02, kind, prims=S.TorchPrims)
        for name, v in t.items():
            if f"{kind}/{name}" in g:
                assert np.array_equal(v.view(np.int32), g[f"{kind}/{name}"].numpy().view(np.int32)), (kind, name)


def test_schedule_log_cos_rounding_margin():
    """log / cos go through the host libm in double and are rounded once to fp32. For every argument
    the three schedules pass to them, the double result lies more than 64 double ulps away from the nearest fp32
    rounding boundary (midpoint between adjacent fp32 values), so any libm accurate to 64 ulps produces the same
    fp32 table bits: the tables are host-independent under that (weak) accuracy assumption."""
    import math
    import numpy as np
    from diffusion_models_collection_amd.diffusion import _schedule as S
    args = {"log": [], "cos": []}

    class Rec(S.IEEE):
        @staticmethod
        def log(x):
            args["log"].extend(np.asarray(x, np.float32).ravel().tolist())
            return S.IEEE.log(x)

        @staticmethod
        def cos(x):
            args["cos"].extend(np.asarray(x, np.float32).ravel().tolist())
            return S.IEEE.cos(x)

    for kind in ("linear", "cosine", "quadratic"):
        S.build_tables(1000, 1e-4, 0.02, kind, prims=Rec)
    assert args["log"] and args["cos"]
    worst = math.inf
    for name, fn in (("log", math.log), ("cos", math.cos)):
        for v in args[name]:
            d = fn(float(v))
            f = np.float32(d)
            if float(f) == d or d == 0.0:
                continue
            other = np.nextafter(f, np.float32(np.inf) if d > float(f) else np.float32(-np.inf))
            mid = (float(f) + float(other)) / 2.0
            margin = abs(d - mid) / math.ulp(d)
            worst = min(worst, margin)
            assert margin > 64, (name, v, d, margin)
    print(f"worst log/cos margin to an fp32 rounding boundary: {worst:.3g} double ulps")


def test_schedule_tables_host_independent_and_pinned():
    """Product tables: IEEE op sequence (identical on every host), pinned against the fixture per
    conftest.check_schedule_vs_fixture; DDIM timesteps bit-exact for every fixture (T, S)."""
    import numpy as np
    from conftest import check_schedule_vs_fixture
    from diffusion_models_collection_amd.diffusion import DDPM, DDIM
    from diffusion_models_collection_amd.diffusion import _schedule as S
    g = load_golden("schedules")
    for kind in ("linear", "quadratic"):
        d = DDPM(1000, 1e-4, 0.02, kind, device="cpu")
        check_schedule_vs_fixture({k: getattr(d, k).numpy() for k in S.build_tables(10, 1e-4, 0.02, kind)}, kind)
    for kind in ("linear", "cosine", "quadratic"):
        d = DDPM(1000, 1e-4, 0.02, kind, device="cpu")
        dd = DDIM(1000, 50, 1e-4, 0.02, kind, device="cpu")
        assert torch.equal(dd.alphas_cumprod, d.alphas_cumprod)
        # the cosine betas pass through cos(): MKL vs correctly rounded, a relative difference only
        assert torch.allclose(d.betas, g[f"{kind}/betas"], rtol=1e-3, atol=0), kind
    # linspace + fma emulation and the double-accumulated cumprod are exact (no transcendental involved)
    assert np.array_equal(S.linspace_f32(0, 1000, 1001), torch.linspace(0, 1000, 1001).numpy())
    for k, v in g.items():
        if k.startswith("ddim_ts/"):
            _, T, Sn = k.split("/")
            dd = DDIM(int(T), int(Sn), device="cpu")
            assert torch.equal(dd.inference_timesteps, v), k
    dd = DDIM(1000, 10, device="cpu")
    dd.set_inference_steps(50)
    assert dd.inference_timesteps[:3].tolist() == [999, 979, 958]


def test_errors_match_reference():
    from diffusion_models_collection_amd.diffusion import DDPM, DDIM
    with pytest.raises(ValueError, match="Unknown beta schedule"):
        DDPM(beta_schedule="sigmoid", device="cpu")
    with pytest.raises(ValueError, match="Unknown beta schedule"):
        DDIM(beta_schedule="sigmoid", device="cpu")
    d = DDIM(device="cpu")
    with pytest.raises(ValueError, match="requires class labels"):
        d.sample_with_cfg(None, (1, 3, 8, 8), None)
    with pytest.raises(ValueError, match="p_threshold"):
        d.sample_with_cfg(None, (1, 3, 8, 8), torch.zeros(1, dtype=torch.long), p_threshold=1.5)
    from diffusion_models_collection_amd.diffusion.ddpm import diffusion_loss
    with pytest.raises(ValueError, match="Unknown loss type"):
        diffusion_loss(torch.zeros(1), torch.zeros(1), "l3")


@pytest.mark.parametrize("name", ["unet_tiny_uncond", "unet_tiny_cond", "unet_tiny_l3"])
def test_state_dict_layout_matches_reference(name):
    from test_oracle import TINY
    from diffusion_models_collection_amd.models import UNet
    g = load_golden(name)
    ref = {k[len("param/"):]: v for k, v in g.items() if k.startswith("param/")}
    torch.manual_seed(1234)   # same seed the fixture generator used -> identical initialisation
    m = UNet(**TINY[name])
    sd = m.state_dict()
    assert list(sd) == list(ref)
    for k in sd:
        assert sd[k].shape == ref[k].shape, k
        assert torch.equal(sd[k], ref[k]), k
    m.load_state_dict(ref)


def test_cifar_unet_param_count_and_flops():
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.models.unet import unet_flops_per_image
    m = UNet()
    assert sum(p.numel() for p in m.parameters()) == 37064707
    assert len(m.state_dict()) == 334
    assert abs(unet_flops_per_image(m) / 1e9 - 12.632) < 0.01


def test_forward_refuses_cpu_tensors():
    from diffusion_models_collection_amd.models import UNet
    m = UNet(image_size=(8, 8), model_channels=16, channel_mult=(1,), attention_resolutions=())
    with pytest.raises(RuntimeError, match="MI355X"):
        m(torch.zeros(1, 3, 8, 8), torch.zeros(1, dtype=torch.long))
    with pytest.raises(RuntimeError, match="executed by the UNet HIP executor"):
        m.input_conv.weight.sum() and m.down_blocks[0][0](torch.zeros(1))


def test_dropin_registry_imports():
    import importlib
    import sys
    sys.path.insert(0, str(ROOT / "dropin"))
    try:
        for mod in ("models", "diffusion", "utils", "utils.trainer", "utils.helpers"):
            sys.modules.pop(mod, None)
        models = importlib.import_module("models")
        diffusion = importlib.import_module("diffusion")
        trainer = importlib.import_module("utils.trainer")
        helpers = importlib.import_module("utils.helpers")
        assert models.UNet.__module__.startswith("diffusion_models_collection_amd")
        assert hasattr(models, "DiT") and hasattr(models, "DiM")
        assert diffusion.DDPM.__module__.startswith("diffusion_models_collection_amd")
        assert trainer.DiffusionTrainer.__module__.startswith("diffusion_models_collection_amd")
        assert helpers.resolve_image_size(32) == (32, 32)
        assert models.DiT.__module__.startswith("diffusion_models_collection_amd")
        with pytest.raises(NotImplementedError):
            models.DiM()
    finally:
        sys.path.remove(str(ROOT / "dropin"))
        for mod in ("models", "diffusion", "utils", "utils.trainer", "utils.helpers"):
            sys.modules.pop(mod, None)


def test_launch_option_table():
    """include/dmc.h dmc_set_option / dmc_get_option / dmc_reset_options: the planners' A/B table (read from the
    environment once) is changed only through these calls; unknown names are errors."""
    _ensure_lib()
    from diffusion_models_collection_amd import _lib as L
    try:
        assert L.get_option("DMC_WG_BLOCKS") == 512
        L.set_option("DMC_NO_HALO", 1)
        assert L.get_option("DMC_NO_HALO") == 1
        L.reset_options(from_env=False)
        assert L.get_option("DMC_NO_HALO") == 0
        assert L.get_option("DMC_NOT_AN_OPTION") == -1
        with pytest.raises(L.DMCError, match="unknown option"):
            L.set_option("DMC_NOT_AN_OPTION", 1)
    finally:
        L.reset_options(from_env=False)


def test_integration_lists_every_option():
    """INTEGRATION.md §3 documents the complete launch-option table: every option the library knows (the kOpts table
    of csrc/dmc_elem.hip) is listed there with its default, and every listed launch option is one the library
    accepts (dmc_get_option != -1). The executor switches are the DMC_* names the Python package reads."""
    import re
    _ensure_lib()
    from diffusion_models_collection_amd import _lib as L
    src = (ROOT / "diffusion_models_collection_amd" / "csrc" / "dmc_elem.hip").read_text()
    table = src[src.index("constexpr OptDef kOpts"):]
    table = table[:table.index("};")]
    lib_opts = set(re.findall(r'"(DMC_[A-Z0-9_]+)"', table))
    doc = (ROOT / "INTEGRATION.md").read_text()
    launch = doc[doc.index("Launch options (measurement A/B only"):doc.index("Executor and package switches")]
    exec_ = doc[doc.index("Executor and package switches"):doc.index("Fused epilogue activation")]
    doc_launch = set(re.findall(r"^\| `(DMC_[A-Z0-9_]+)`", launch, re.M))
    doc_exec = set(re.findall(r"^\| `(DMC_[A-Z0-9_]+)`", exec_, re.M))
    assert doc_launch == lib_opts, (sorted(lib_opts - doc_launch), sorted(doc_launch - lib_opts))
    for name in lib_opts:
        assert L.get_option(name) != -1, name
    py_read = set()
    for f in (ROOT / "diffusion_models_collection_amd").rglob("*.py"):
        py_read |= set(re.findall(r'environ\.get\("(DMC_[A-Z0-9_]+)"', f.read_text()))
        py_read |= set(re.findall(r'environ\["(DMC_[A-Z0-9_]+)"\]', f.read_text()))
    assert py_read <= doc_exec, sorted(py_read - doc_exec)
    assert len(doc_launch | doc_exec) <= 45


def test_wgrad_pipe_lds_swizzle_conflict_free():
    """scripts/swizzle_check.py: the x-halo and dy images of wgrad3x3_pipe_kernel are bank-conflict free for every
    tap / k-step / lane group of ds_read_b64_tr_b16, and every fragment address is its set's base + an immediate."""
    import runpy
    mod = runpy.run_path(str(ROOT / "scripts" / "swizzle_check.py"))
    for ow in (32, 16, 8, 4):
        assert mod["check_x"](ow) == 0, ow
    assert mod["check_dy"]() == 0
