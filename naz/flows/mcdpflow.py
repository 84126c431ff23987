"""naz.flows.mcdpflow (src/naz/flows/mcdpflow.py) -> naz_amd.flows.mcdpflow."""
from naz_amd.flows.mcdpflow import MCDPNormalizingFlow

__all__ = ["MCDPNormalizingFlow"]
