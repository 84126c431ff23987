"""CPU: host logic of naz_amd — MADE masks, weight exchange, API surface (no kernels)."""
import pickle

import numpy as np
import pytest
import torch

from naz_amd import nn as nnz
from naz_amd.flows import NormalizingFlow, flow_makers
from naz_amd.flows import io as fio
from oracle import naz_oracle as O


@pytest.mark.parametrize("D,C,hidden,mult", [(4, 0, [16, 16], 2), (5, 3, [20], 23), (16, 32, [128, 128], 23),
                                             (2, 0, [150, 150, 150], 2)])
def test_masks_match_oracle(D, C, hidden, mult):
    perm = torch.randperm(D, generator=torch.Generator().manual_seed(D + C))
    a, askip = nnz.create_mask(D, C, hidden, perm, mult)
    b, bskip = O.create_mask(D, C, hidden, perm, mult)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(askip, bskip)


def test_flow_makers_and_signature():
    assert set(flow_makers) == {"maf", "nsa", "nsc", "cnf"}
    f = NormalizingFlow("nsa", None, 4, 2, [32, 32], 3, 8)
    assert f.conditional and len(f.flow_dist.transforms) == 3
    for t in f.flow_dist.transforms:  # train_flows.get_params / set_params walk these
        names = [n for n, _ in t.named_parameters()]
        assert "nn.layers.0.weight" in names and "nn.layers.2.bias" in names
        assert hasattr(t.nn, "masks") and hasattr(t.nn, "mask_skip") and hasattr(t.nn, "permutation")
    g = NormalizingFlow("maf", None, 2, 0, [16, 16], 3)
    assert not g.conditional and len(g.flow_dist.transforms) == 1  # torch wraps a single compose transform


def test_fused_plan_binds_keyword_maker_arguments():
    """count_bins / split_dim / hidden_dim passed by keyword pick the same fused plan as the
    positional form (they raised at construction)."""
    from naz_amd.flows.flow import _FusedAR, _FusedCoupling
    a = NormalizingFlow("nsa", None, 4, 2, [128, 128], 8, count_bins=8)
    assert isinstance(a._plan, _FusedAR)
    b = NormalizingFlow("nsc", None, 16, 32, [128, 128], 8, 8, split_dim=8)
    assert isinstance(b._plan, _FusedCoupling)
    c = NormalizingFlow("maf", None, 2, 2, hidden_dim=[150, 150, 150], num_layers=16)
    assert isinstance(c._plan, _FusedAR)


@pytest.mark.parametrize("ft,args", [("nsc", (6, 2, [32, 32], 3, 4, 2)), ("nsa", (4, 2, [32, 32], 2, 8)),
                                     ("maf", (3, 2, [16, 16], 3))])
def test_state_roundtrip_and_oracle_masks(ft, args, tmp_path):
    f = NormalizingFlow(ft, None, *args)
    st = fio.export_state(f)
    g = NormalizingFlow(ft, None, *args)
    fio.save_npz(f, tmp_path / "w.npz")
    fio.load_npz(g, tmp_path / "w.npz")
    st2 = fio.export_state(g)
    assert st.keys() == st2.keys()
    for k in st:
        np.testing.assert_array_equal(st[k], st2[k])
    if ft != "nsc":  # product masks after import == oracle masks from the same permutation
        spec = dict(flow_type=ft, D=args[0], C=args[1], hidden=args[2], L=args[3],
                    K=args[4] if ft == "nsa" else 8)
        mult = 3 * spec["K"] - 1 if ft == "nsa" else 2
        for l, t in enumerate(g.flow_dist.transforms if g.conditional else g.flow_dist.transforms[0]):
            om, _ = O.create_mask(spec["D"], spec["C"], spec["hidden"], torch.as_tensor(st[f"layers.{l}.nn.permutation"]),
                                  mult)
            for lin, m in zip(t.nn.layers, om):
                assert torch.equal(lin.mask.cpu(), m)


def test_pickle_whole_model():
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 2, 8, 8)
    g = pickle.loads(pickle.dumps(f))
    assert g.fused
    for (n1, p1), (n2, p2) in zip(f.named_parameters(), g.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2)


def test_unsupported_options_fail_loudly():
    with pytest.raises(NotImplementedError):
        NormalizingFlow("nsc", None, 4, 2, [16, 16], 2, 8, 2, use_batchnorm=True)
    with pytest.raises(NotImplementedError):  # MC dropout in the CNF vector field
        NormalizingFlow("cnf", None, 4, 2, [16, 16], 2, dropout_p=0.1)
    # a CNF shape without a fused solve kernel runs the per-layer solve (flows/cnf_adjoint.py), e.g.
    # naz's POSYDON CNF (eposydon/train_cnf_mle.py:91): it constructs, it does not fall back silently
    f = NormalizingFlow("cnf", None, 4, 2, [16, 16], 2)
    assert not any(t._plan.fused for t in f.transforms)
    f = NormalizingFlow("cnf", None, 4, 5, [128] * 4, 1)
    assert not f.transforms[0]._plan.fused
