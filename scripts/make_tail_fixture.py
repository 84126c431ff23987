"""Writes tests/golden/nsc_tail_vjp_lower.npz: layer 2's lower-spline parameters of the bench's
config-3 flow after 27 Adam steps (saved by scripts/diag_train_nan.py in r06_g1, the state whose
step went non-finite) and the lower-spline input that did it (dim 6, y = 3.0040803 at B = 3:
the extrapolated map's F_theta is exactly 0 there; scripts/diag_nan_cpu.py)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
st = torch.load(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out/r06_g1/nan_state_t0.pt",
                weights_only=True, map_location="cpu")
p = st["params"]
l = 2
uw, uh, ud = (p[9 * l + 6].numpy(), p[9 * l + 7].numpy(), p[9 * l + 8].numpy())
np.savez(ROOT / "tests/golden/nsc_tail_vjp_lower.npz", uw=uw.astype(np.float32), uh=uh.astype(np.float32),
         ud=ud.astype(np.float32), y_fail=np.float32(3.004080295562744), dim_fail=np.int32(6), bound=np.float32(3.0),
         step=np.int32(st["step"]))
print(uw.shape, uh.shape, ud.shape)
