"""naz_amd — MI355X-native (gfx950) implementation of naz's normalizing-flow hot path.

Public surface mirrors the reference package ``naz`` (AnaryaRay1/naz):
``naz_amd.flows.NormalizingFlow``, ``naz_amd.flows.flow.flow_makers``,
``naz_amd.utils.{set_device, device}``, ``naz_amd.trainers.train_flows.train``.
All compute goes through ``naz_amd/lib/libnazhip.so`` (C ABI: include/naz_hip.h).
"""
__version__ = "0.1.0"
