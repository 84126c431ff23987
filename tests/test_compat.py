"""CPU: the ``naz`` import-compatible package and the reference-flow exporter (SURVEY.md §8f
rank 4).  No GPU: flows are constructed on the CPU and only their parameters are compared."""
from types import SimpleNamespace

import numpy as np
import torch

from oracle import naz_oracle as O


def test_naz_paths_the_examples_import():
    # examples/papers/2506.05657/*.py and eposydon/*.py (grep 'from naz'): these must import unchanged
    from naz.flows.flow import NormalizingFlow  # noqa: F401
    from naz.utils import set_device, device  # noqa: F401
    from naz.trainers.train_flows import train, train_lightning, predict, get_params, set_params  # noqa: F401
    from naz.flows.bflow_jax_maf import (make_conditional_autoregressive_nn,  # noqa: F401
                                         make_masked_affine_autoregressive_transform, make_normalizing_flow,
                                         train_maf, bayesian_normalizing_flow, train_bayesian_flow_hmc,
                                         train_bayesian_flow_prior, train_bayesian_flow, torch_to_jax, calibrate,
                                         compute_bic, train_bayesian_flow_svi, bounding_transform)
    from naz.flows.transforms import masked_affine_autoregressive, neural_spline_autoregressive  # noqa: F401
    from naz.flows.continuous_transforms import continuous_free_form  # noqa: F401
    import naz_amd
    assert NormalizingFlow.__module__.startswith("naz_amd")
    import pytest
    with pytest.raises(NotImplementedError):
        train_maf(None, None, None)


def _duck_maf(spec, state):
    """A stand-in for a pickled pyro maf: flow.flow_dist.transforms[i].nn.{layers, masks,
    permutation} — exactly the fields torch_to_jax reads (bflow_jax_maf.py:26-46)."""
    from naz_amd.nn import create_mask
    ts = []
    for l in range(spec["L"]):
        p = f"layers.{l}."
        n_lin = len(spec["hidden"]) + 1
        lins = [SimpleNamespace(weight=torch.as_tensor(state[p + f"nn.layers.{i}.weight"]),
                                bias=torch.as_tensor(state[p + f"nn.layers.{i}.bias"])) for i in range(n_lin)]
        perm = torch.as_tensor(state[p + "nn.permutation"])
        masks, _ = create_mask(spec["D"], spec["C"], spec["hidden"], perm, 2)
        ts.append(SimpleNamespace(nn=SimpleNamespace(layers=lins, masks=masks, permutation=perm)))
    return SimpleNamespace(flow_dist=SimpleNamespace(transforms=ts))


def test_exporter_roundtrip_duck_typed_flow(tmp_path):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    spec = dict(flow_type="maf", D=3, C=2, hidden=[16, 16], L=3)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=11).items()}
    exported = fio.state_from_reference_flow(_duck_maf(spec, state))
    np.savez(tmp_path / "m.npz", **exported)
    f = NormalizingFlow("maf", None, 3, 2, [16, 16], 3)
    fio.load_npz(f, tmp_path / "m.npz")
    with np.load(tmp_path / "m.npz", allow_pickle=False) as z:
        fio.check_masks(f, {k: z[k] for k in z.files})
    back = fio.export_state(f)
    for k, v in state.items():
        np.testing.assert_array_equal(back[k], np.asarray(v, dtype=back[k].dtype), err_msg=k)
