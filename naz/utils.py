"""naz.utils (src/naz/utils.py:7-23) -> naz_amd.utils."""
from naz_amd.utils import device, set_device

__all__ = ["device", "set_device"]
