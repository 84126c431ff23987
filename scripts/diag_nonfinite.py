"""diagnostic: non-finite rows of the config-3 headline flow at 2^20 rows.

Run under the NAZ_DEBUG_NONFINITE library to name the first offending (workgroup, layer, stage):
    NAZ_LIB=$PWD/naz_amd/lib/libnazhip_debug.so python scripts/diag_nonfinite.py [trials]
(build it with `python -m naz_amd.build debug -DNAZ_DEBUG_NONFINITE`).  Prints one JSON line."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from naz_amd import _lib  # noqa: E402
from oracle import naz_oracle as O  # noqa: E402
from tests.test_gpu_parity import _config3_flow  # noqa: E402

DEV = "cuda"
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 3
f, spec, state = _config3_flow()
f = f.to(DEV)
B = 1 << 20
g = torch.Generator(device=DEV).manual_seed(0)
x = torch.as_tensor(O.gaussian_mixture(B, 16, seed=0), device=DEV)
c = torch.randn(B, 32, device=DEV, generator=g)
rec = (C.c_int64 * 5)()
debug = _lib.lib().naz_debug_nonfinite(rec, 1) == 0
out = {"lib": str(_lib.LIB_PATH), "debug_build": debug, "trials": []}
with torch.no_grad():
    for trial in range(trials):
        lp = f.log_prob(x, condition=c)
        bad = torch.nonzero(~torch.isfinite(lp)).reshape(-1)
        t = {"nonfinite_rows": int(bad.numel()), "rows": bad[:8].tolist()}
        if debug:
            _lib.check(_lib.lib().naz_debug_nonfinite(rec, 1), "debug_nonfinite")
            t["record"] = dict(zip(["hit", "workgroup", "layer", "stage", "row"], list(rec)))
        out["trials"].append(t)
print(json.dumps(out))
