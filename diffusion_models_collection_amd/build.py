"""Build libdmc.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

    python -m diffusion_models_collection_amd.build          # incremental
    python -m diffusion_models_collection_amd.build --force  # rebuild everything

The shared object lands next to this file (diffusion_models_collection_amd/libdmc.so) so it travels with
the repo snapshot to the GPU box; objects go to build/ at the repo root.
"""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
BUILD = ROOT / "build"
LIB = PKG / "libdmc.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DMC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["dmc_conv.hip", "dmc_wgrad.hip", "dmc_norm.hip", "dmc_attn.hip", "dmc_elem.hip", "dmc_dit.hip", "dmc_data.hip"]
# the element-wise and data files restate torch op sequences: no FMA contraction there
EXTRA = {"dmc_elem.hip": ["-ffp-contract=off"], "dmc_data.hip": ["-ffp-contract=off"]}
COMMON = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-I", str(INCLUDE), "-I", str(CSRC)]


def _stale(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    jobs = []
    for src in SOURCES:
        s = CSRC / src
        o = BUILD / (Path(src).stem + ".o")
        if force or _stale(o, [s] + headers):
            jobs.append([HIPCC] + COMMON + EXTRA.get(src, []) + ["-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print("[dmc build]", " ".join(cmd[-3:]), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {cmd[-3]}:\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=min(len(jobs), 4) or 1) as ex:
        list(ex.map(run, jobs))
    objs = [BUILD / (Path(s).stem + ".o") for s in SOURCES]
    if force or jobs or _stale(LIB, objs):
        # link to a temporary name and rename: a snapshot of the tree never holds a half-written library
        tmp = LIB.with_name(LIB.name + ".tmp")
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
        run(cmd)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force))
    sys.exit(0)
