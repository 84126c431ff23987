"""naz.flows.flow (src/naz/flows/flow.py) -> naz_amd.flows.flow."""
from naz_amd.flows.flow import NormalizingFlow, flow_makers
from naz_amd.flows.transforms import bounding_transform, inverse_bounding_transform
from naz_amd.utils import device, set_device

__all__ = ["NormalizingFlow", "flow_makers", "bounding_transform", "inverse_bounding_transform", "device",
           "set_device"]
