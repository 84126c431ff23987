"""GPU: the generic whole-flow entries (naz_flow_log_prob / naz_flow_sample) give
bitwise the kind-specific launches' results (coupling: naz_coupling_*, AR: naz_ar_flow_*)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_flow_entries_equal_kind_specific_launches():
    from naz_amd import ops
    from naz_amd.flows import NormalizingFlow
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1)
    cases = [("nsc", (16, 32, [128, 128], 4, 8, 8)), ("maf", (2, 2, [150, 150, 150], 5)),
             ("nsa", (16, 32, [128, 128], 3, 8))]
    for ftype, args in cases:
        f = NormalizingFlow(ftype, None, *args).to("cuda")
        assert f.fused, ftype
        D, C = args[0], args[1]
        x = torch.randn(1000, D, generator=g).cuda()
        c = torch.randn(1000, C, generator=g).cuda()
        plan = f._plan
        packed = plan.packed()
        with torch.no_grad():
            lp = f.log_prob(x, condition=c)
        lp_gen = ops.flow_log_prob(ops.flow_desc(plan.desc), packed, x, c)
        assert torch.equal(lp, lp_gen), ftype
        if ftype == "nsc":
            y_ref, ld_ref = ops.coupling_sample(plan.desc, packed, x, c, with_logdet=True)
            y, ld = ops.flow_sample(ops.flow_desc(plan.desc), packed, x, c)
            assert torch.equal(y, y_ref) and torch.equal(ld, ld_ref)
