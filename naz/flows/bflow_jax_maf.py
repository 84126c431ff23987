"""naz.flows.bflow_jax_maf (src/naz/flows/bflow_jax_maf.py) -> naz_amd.flows.bflow_maf.

The flow construction and its log_prob / sampler (torch_to_jax, the conditional MADE, the
affine MAF, make_normalizing_flow: :26-225) are built, batched over weight draws.  The
NumPyro / optax drivers around them (train_maf, bayesian_normalizing_flow, the HMC / SVI /
prior trainers, calibrate, compute_bic: :227-476) are JAX front ends outside the hot path
(SURVEY.md §2); they exist so the scripts import, and raise NotImplementedError when called."""
from naz_amd.flows.bflow_maf import (MAFSpec, make_conditional_autoregressive_nn,
                                     make_masked_affine_autoregressive_transform, make_normalizing_flow, ravel,
                                     torch_to_jax, unravel)
from naz_amd.flows.transforms import bounding_transform, inverse_bounding_transform

__all__ = ["MAFSpec", "make_conditional_autoregressive_nn", "make_masked_affine_autoregressive_transform",
           "make_normalizing_flow", "ravel", "torch_to_jax", "unravel", "bounding_transform",
           "inverse_bounding_transform", "train_maf", "bayesian_normalizing_flow", "train_bayesian_flow_hmc",
           "train_bayesian_flow_prior", "train_bayesian_flow_svi", "train_bayesian_flow", "calibrate",
           "compute_bic"]


def _jax_only(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"naz_amd: {name} is a JAX/NumPyro driver outside the log_prob hot path; the "
                                  "flow's lp / lp_batched / lp_and_grad / sampler_batched are built")
    f.__name__ = name
    return f


for _n in ("train_maf", "bayesian_normalizing_flow", "train_bayesian_flow_hmc", "train_bayesian_flow_prior",
           "train_bayesian_flow_svi", "train_bayesian_flow", "calibrate", "compute_bic"):
    globals()[_n] = _jax_only(_n)
del _n
