"""naz.trainers.train_flows (src/naz/trainers/train_flows.py) -> naz_amd.trainers.train_flows.

train / get_params / set_params / predict / train_lightning are built.  The Pyro inference
trainers (train_hmc :280-323, train_svi :325-356, train_importance :358-380) are front ends
outside the log_prob hot path and raise NotImplementedError when called."""
from naz_amd.trainers.train_flows import get_params, predict, set_params, train, train_lightning

__all__ = ["get_params", "predict", "set_params", "train", "train_lightning", "train_hmc", "train_svi",
           "train_importance"]


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"naz_amd: {name} (Pyro MCMC/VI over the flow weights) is outside the "
                                  "log_prob hot path; use naz.flows.bflow_jax_maf's batched lp / lp_and_grad")
    f.__name__ = name
    return f


train_hmc = _out_of_scope("train_hmc")
train_svi = _out_of_scope("train_svi")
train_importance = _out_of_scope("train_importance")
