"""ctypes binding of libnazhip.so (the C ABI in include/naz_hip.h).

The library is the ONLY compute path of naz_amd: if it is missing, or a tensor is
not on a HIP device, calls raise — there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("NAZ_LIB", Path(__file__).resolve().parent / "lib" / "libnazhip.so"))

LAYOUT_DENSE, LAYOUT_ARN = 0, 1
RQS_FAST = 16  # NAZ_RQS_FAST: OR into the spline layout for the select-first hardware-math evaluator
LD_PERDIM, LD_ROWSUM, LD_ROWSUM_ADD, LD_ROWSUM_SUB = 0, 1, 2, 3
ACT = {"identity": 0, "tanh": 1, "relu": 2, "softplus": 3, "sigmoid": 4}
MFMA_BF16X6, MFMA_F32, MFMA_F16X3 = 0, 1, 2

_f, _i, _i64, _vp = C.POINTER(C.c_float), C.c_int, C.c_int64, C.c_void_p


class CouplingDesc(C.Structure):
    _fields_ = [("D", C.c_int), ("C", C.c_int), ("S", C.c_int), ("K", C.c_int), ("L", C.c_int), ("H", C.c_int),
                ("act", C.c_int), ("has_lower", C.c_int), ("bound", C.c_float), ("mfma_mode", C.c_int),
                ("reserved", C.c_int * 6)]


class ArDesc(C.Structure):
    _fields_ = [("D", C.c_int), ("C", C.c_int), ("H", C.c_int), ("K", C.c_int), ("L", C.c_int), ("act", C.c_int),
                ("bound", C.c_float), ("n_hidden", C.c_int), ("kind", C.c_int), ("flags", C.c_int),
                ("reserved", C.c_int * 5)]


class CnfDesc(C.Structure):
    _fields_ = [("D", C.c_int), ("C", C.c_int), ("n_hidden", C.c_int), ("H", C.c_int * 4), ("act", C.c_int),
                ("mfma_mode", C.c_int), ("reserved", C.c_int * 7)]


class FlowDesc(C.Structure):
    _fields_ = [("kind", C.c_int), ("coupling", CouplingDesc), ("ar", ArDesc), ("reserved", C.c_int * 8)]


FLOW_COUPLING, FLOW_AR = 1, 2

# name -> (restype, argtypes); every symbol declared in include/naz_hip.h
SIGNATURES = {
    "naz_last_error": (C.c_char_p, []),
    "naz_abi_version": (C.c_int, []),
    "naz_image_attach": (C.c_int, [_vp, _i64, _vp]),
    "naz_image_release": (C.c_int, [_vp]),
    "naz_tuning": (C.c_int, [C.c_char_p, _i]),
    "naz_debug_nonfinite": (C.c_int, [C.POINTER(C.c_int64), _i]),
    "naz_rqs_fwd": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i, _i64, _i, _i, _i, C.c_float, _vp]),
    "naz_rqs_inv": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i, _i64, _i, _i, _i, C.c_float, _vp]),
    "naz_spline_elementwise": (C.c_int, [_i, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i, _i, C.c_float,
                                         _vp]),
    "naz_linear_act": (C.c_int, [_vp, _i64, _i, _vp, _i64, _i, _vp, _vp, _vp, _vp, _i64, _i64, _i, _i, _vp]),
    "naz_gemm_dact": (C.c_int, [_vp, _i64, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i, _i64, _i, _vp]),
    "naz_made_affine_inv1": (C.c_int, [_vp, _i64, _i, _i, _i, _vp, _i64, _i64, _vp, _i64, _i64, _i, _vp, _i64, _i64,
                                       _vp, _i64, _i, _i64, _i, _i, _vp]),
    "naz_made_packed_floats": (_i64, [_i, _i, _i, _i]),
    "naz_made_affine_fwd": (C.c_int, [_vp, _i64, _i, _i, _i, _i, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64,
                                      _vp, _i64, _i, _i64, _i, _i, _vp]),
    "naz_linear_act_batched": (C.c_int, [_vp, _i64, _i64, _i, _vp, _i64, _i64, _i, _vp, _i64, _vp, _vp, _i64, _vp,
                                         _i64, _i64, _i64, _i, _i, _i, _vp]),
    "naz_affine_ar": (C.c_int, [_i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i, _i64, _i, _vp]),
    "naz_base_log_prob": (C.c_int, [_vp, _i64, _vp, _i64, _i, _i, _vp]),
    "naz_bounding_fwd": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _i, _vp]),
    "naz_bounding_inv": (C.c_int, [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i, _vp]),
    "naz_rqs_bwd": (C.c_int, [_i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i, _vp, _i64, _vp, _i64, _i64, _i, _i, _i,
                              C.c_float, _vp]),
    "naz_gemm": (C.c_int, [_i, _i, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i, _i,
                           _i, _vp, _vp]),
    "naz_affine_ar_bwd": (C.c_int, [_i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _i64,
                                    _i, _vp]),
    "naz_maf_dim_vjp": (C.c_int, [_i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                                  _i64, _i, _i, _vp]),
    "naz_colsum": (C.c_int, [_vp, _i64, _i64, _i, _vp, _vp]),
    "naz_act_bwd": (C.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i, _i, _vp]),
    "naz_base_log_prob_bwd": (C.c_int, [_vp, _i64, _vp, _vp, _i64, _i64, _i, _vp]),
    "naz_dropout": (C.c_int, [_vp, _i64, _vp, _i64, _i64, _i, C.c_float, C.c_uint64, _vp]),
    "naz_coupling_bwd_packed_bytes": (C.c_int64, [C.POINTER(CouplingDesc)]),
    "naz_coupling_pack_bwd": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _vp]),
    "naz_coupling_log_prob_train": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "naz_coupling_bwd_layer": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _vp, _i, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp, _i64, _vp]),
    "naz_coupling_dp3_columns": (C.c_int, [C.POINTER(CouplingDesc), _vp]),
    "naz_coupling_layer_fwd": (C.c_int, [C.POINTER(CouplingDesc), _vp, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i,
                                         _i64, _vp]),
    "naz_coupling_layer_inv": (C.c_int, [C.POINTER(CouplingDesc), _vp, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i,
                                         _i64, _vp]),
    "naz_cnf_supported": (C.c_int, [C.POINTER(CnfDesc)]),
    "naz_cnf_param_count": (C.c_int64, [C.POINTER(CnfDesc)]),
    "naz_cnf_packed_bytes": (C.c_int64, [C.POINTER(CnfDesc)]),
    "naz_cnf_pack": (C.c_int, [C.POINTER(CnfDesc), _vp, _vp, _vp]),
    "naz_cnf_integrate": (C.c_int, [C.POINTER(CnfDesc), _vp, _vp, _i64, _vp, _i64, _vp, _i64, C.c_float, C.c_float,
                                    _i, _vp, _i64, _vp, _i, _i64, _vp]),
    "naz_cnf_integrate_dopri5": (C.c_int, [C.POINTER(CnfDesc), _vp, _vp, _i64, _vp, _i64, _vp, _i64, C.c_float,
                                           C.c_float, C.c_float, C.c_float, _i, _vp, _i64, _vp, _i, _vp, _i64, _vp]),
    "naz_cnf_dopri5_global_workspace_bytes": (C.c_int64, [C.POINTER(CnfDesc), _i64]),
    "naz_cnf_integrate_dopri5_global": (C.c_int, [C.POINTER(CnfDesc), _vp, _vp, _i64, _vp, _i64, _vp, _i64, C.c_float,
                                                  C.c_float, C.c_float, C.c_float, _i, _vp, _i64, _vp, _i, _vp, _vp,
                                                  _i64, _vp]),
    "naz_gemm_jvp_bwd": (C.c_int, [_vp, _i64, _i, _vp, _i64, _vp, _i64, _vp, _i64, _i, _i64, _i, _vp]),
    "naz_ar_flow_supported": (C.c_int, [C.POINTER(ArDesc)]),
    "naz_ar_flow_packed_bytes": (C.c_int64, [C.POINTER(ArDesc)]),
    "naz_ar_flow_degrees": (C.c_int, [C.POINTER(ArDesc), _vp]),
    "naz_ar_flow_pack_host": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _vp]),
    "naz_ar_flow_workspace_bytes": (C.c_int64, [C.POINTER(ArDesc), _i64, _i64]),
    "naz_ar_flow_log_prob": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64,
                                       _vp]),
    "naz_ar_flow_fwd_packed_bytes": (C.c_int64, [C.POINTER(ArDesc)]),
    "naz_ar_flow_pass0_floats": (C.c_int64, [C.POINTER(ArDesc)]),
    "naz_ar_flow_pack": (C.c_int, [C.POINTER(ArDesc), _vp, _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _vp]),
    "naz_ar_flow_log_prob_batched": (C.c_int, [C.POINTER(ArDesc), _vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _i64,
                                               _i64, _i64, _i, _vp, _i64, _vp]),
    "naz_ar_flow_pack_fwd": (C.c_int, [C.POINTER(ArDesc), _vp, _i64, _vp, _i64, _i64, _vp, _vp]),
    "naz_ar_flow_sample_batched": (C.c_int, [C.POINTER(ArDesc), _vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _i64,
                                             _i64, _vp, _i64, _i64, _i64, _vp]),
    "naz_ar_flow_pack_fwd_host": (C.c_int, [C.POINTER(ArDesc), _vp, _vp]),
    "naz_wgrad_batched": (C.c_int, [_i64, _i, _i, _i, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64,
                                    _vp]),
    "naz_ar_flow_log_prob_train": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64,
                                             _vp]),
    "naz_ar_flow_bwd_packed_bytes": (C.c_int64, [C.POINTER(ArDesc)]),
    "naz_ar_flow_bwd_dims": (C.c_int, [C.POINTER(ArDesc), _vp]),
    "naz_ar_flow_pack_bwd": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _vp, _vp]),
    "naz_ar_flow_bwd_layer": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _vp, _i, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                        _i64, _vp]),
    "naz_ar_flow_sample": (C.c_int, [C.POINTER(ArDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64,
                                     _vp]),
    "naz_flow_packed_bytes": (C.c_int64, [C.POINTER(FlowDesc)]),
    "naz_workspace_bytes": (C.c_int64, [C.POINTER(FlowDesc), _i64]),
    "naz_flow_log_prob": (C.c_int, [C.POINTER(FlowDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64,
                                    _vp]),
    "naz_flow_sample": (C.c_int, [C.POINTER(FlowDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64,
                                  _vp]),
    "naz_coupling_supported": (C.c_int, [C.POINTER(CouplingDesc)]),
    "naz_coupling_param_count": (C.c_int64, [C.POINTER(CouplingDesc)]),
    "naz_coupling_packed_bytes": (C.c_int64, [C.POINTER(CouplingDesc)]),
    "naz_coupling_pack": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _vp]),
    "naz_coupling_log_prob": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64,
                                        _vp]),
    "naz_coupling_sample": (C.c_int, [C.POINTER(CouplingDesc), _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _vp,
                                      _i64, _vp]),
}

_lib = None


class NazLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the HIP library; raise if it has not been built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise NazLibraryError(
                f"naz_amd: HIP library {LIB_PATH} is missing — build it with `python -m naz_amd.build` "
                "(there is no CPU fallback)")
        L = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_LOCAL", 0))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().naz_last_error().decode(errors="replace")
        raise RuntimeError(f"naz_amd {what}: {msg or f'error code {rc}'}")
