"""Weight-ring depth sweep of conv3x3_halo5_kernel on the roofline layer (per-launch HIP events)."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402
import halo_ab  # noqa: E402
for ws in (3, 4):
    L.set_option("DMC_HALO_WS", ws)
    print("WS", ws, end=": ")
    halo_ab.run("r128_32")
