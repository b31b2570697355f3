"""CPU test (no GPU): the inline-asm LDS reads of the conv kernels are never used before their wait.

DESIGN.md section 3 "LDS hazards". The halo GroupNorm+SiLU prologue and the small-map conv's in-kernel GroupNorm
read LDS with inline asm (plain reads would make hipcc drain the in-flight chunk DMA). Round 6 found hipcc
scheduling uses of such reads before the asm s_waitcnt (all outputs NaN); the fix ties every result to the wait.
This test compiles dmc_conv.hip and dmc_wgrad.hip (the 4x4 weight gradient's asm transposed reads with partial
lgkmcnt waits) for gfx950 to assembly and checks every asm ds_read (scripts/lds_asm_check.py),
and checks the checker on a hand-made bad sequence."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))
import lds_asm_check  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"


def test_checker_flags_a_premature_use():
    bad = """k:
\t;;#ASMSTART
\tds_read_b128 v[4:7], v196
\t;;#ASMEND
\tv_lshlrev_b32_e32 v86, 16, v4
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
"""
    good = bad.replace("\tv_lshlrev_b32_e32 v86, 16, v4\n", "") + "\tv_lshlrev_b32_e32 v86, 16, v4\n"
    assert len(lds_asm_check.check(bad)) == 1
    assert lds_asm_check.check(good) == []


@pytest.mark.skipif(not Path(HIPCC).exists() and shutil.which("hipcc") is None, reason="hipcc not available")
@pytest.mark.parametrize("unit", ["dmc_conv.hip", "dmc_wgrad.hip"])
def test_conv_kernels_asm_lds_reads_wait_before_use(unit, tmp_path):
    src = ROOT / "diffusion_models_collection_amd" / "csrc" / unit
    out = tmp_path / "conv.s"
    cmd = [HIPCC if Path(HIPCC).exists() else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-I", str(ROOT / "include"), "-I", str(src.parent), "--offload-device-only", "-S", "-o", str(out),
           str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    assert text.count(";;#ASMSTART") > 20 and "ds_read_b" in text
    viol = lds_asm_check.check(text)
    assert viol == [], viol[:5]
