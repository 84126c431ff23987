"""Device helpers with naz's signature (naz/utils.py:7-23).

naz hard-wires CUDA and imports JAX at import time; here ``device`` is the current
HIP device when one is visible and the CPU otherwise, so the package (and its host
logic tests) import on a GPU-less host.  Compute still requires the HIP device.
"""
import torch


def set_device(tensor, device="cuda", dtype=torch.float32):
    """Convert a list / array / tensor to a torch tensor on ``device`` (naz/utils.py:7-21)."""
    if device == "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("naz_amd.set_device: no HIP device visible")
        device = f"cuda:{torch.cuda.current_device()}"
    elif device != "cpu" and not isinstance(device, torch.device):
        raise ValueError(f"unknown device {device!r}")
    return torch.as_tensor(tensor, dtype=dtype, device=torch.device(device))


def _default_device() -> torch.device:
    try:
        if torch.cuda.is_available():
            return torch.device(f"cuda:{torch.cuda.current_device()}")
    except Exception:  # pragma: no cover
        pass
    return torch.device("cpu")


device = _default_device()
