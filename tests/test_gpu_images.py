"""GPU: the packed-image contract of ABI 3 (include/naz_hip.h "Packed images") and the caller-owned
workspace of the autoregressive log_prob entries.

Every launch entry resolves its image through the library's registry before launching, so a
foreign, truncated, mis-tagged or wrong-kind image is a clean error (RuntimeError from the entry's
status), never an out-of-bounds LDS-DMA; the wide MAF inverse takes its per-wave scratch from the
caller (naz_ar_flow_workspace_bytes) instead of allocating it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _flows():
    from naz_amd.flows import NormalizingFlow
    torch.manual_seed(3)
    nsc = NormalizingFlow("nsc", None, 16, 32, [128, 128], 2, 8, 8).to(DEV)
    maf = NormalizingFlow("maf", None, 2, 2, [150] * 3, 3).to(DEV)
    return nsc, maf


def _cnf():
    from naz_amd import ops
    d = ops.cnf_desc(4, 2, [32, 32], mfma="f32")
    g = torch.Generator().manual_seed(2)
    flat = (torch.randn(ops.cnf_param_count(d), generator=g) * 0.1).to(DEV)
    return d, ops.cnf_pack(d, flat)


def _raises(fn, *pat):
    with pytest.raises(RuntimeError) as e:
        fn()
        torch.cuda.synchronize()
    msg = str(e.value)
    assert any(p in msg for p in pat), msg
    torch.cuda.synchronize()  # nothing launched: the device is untouched


def test_every_entry_refuses_a_foreign_image():
    """Each image-taking entry, handed an image of another kind (the CNF vector field's) or plain
    memory, returns an error naming the problem before any launch; with its own image it runs."""
    from naz_amd import ops
    nsc, maf = _flows()
    dcnf, cimg = _cnf()
    junk = torch.zeros(1 << 20, device=DEV)
    B = 300
    x16, c32 = torch.randn(B, 16, device=DEV), torch.randn(B, 32, device=DEV)
    x2, c2 = torch.randn(B, 2, device=DEV), torch.randn(B, 2, device=DEV)
    cimgs, aimg = nsc._plan.packed(), maf._plan.packed()
    cd, ad = nsc._plan.desc, maf._plan.desc  # (read after packed(): it resolves the MFMA image mode)
    states = torch.empty((cd.L + 1, B, 16), device=DEV)
    ld = torch.zeros(B, device=DEV)
    entries = {
        "coupling_log_prob": lambda img: ops.coupling_log_prob(cd, img, x16, c32),
        "coupling_sample": lambda img: ops.coupling_sample(cd, img, x16, c32),
        "coupling_layer": lambda img: ops.coupling_layer(cd, img, 1, x16, c32, True, ld),
        "coupling_log_prob_train": lambda img: ops.coupling_log_prob_train(cd, img, x16, c32, None, None, states),
        "flow_log_prob": lambda img: ops.flow_log_prob(ops.flow_desc(cd), img, x16, c32),
        "ar_flow_log_prob": lambda img: ops.ar_flow_log_prob(ad, img, x2, c2),
        "ar_flow_log_prob_train": lambda img: ops.ar_flow_log_prob_train(
            ad, img, x2, c2, torch.empty((ad.L, B, 2), device=DEV)),
        "ar_flow_sample": lambda img: ops.ar_flow_sample(ad, img, x2, c2),
        "cnf_integrate": lambda img: ops.cnf_integrate(dcnf, img, x2.repeat(1, 2), torch.randn(B, 4, device=DEV),
                                                       0.0, 1.0, 2, context=c2),
    }
    for name, fn in entries.items():
        foreign = cimg if not name.startswith("cnf") else cimgs
        _raises(lambda: fn(foreign), "image", name)
        _raises(lambda: fn(junk), "is not a packed image")
    # an address inside a registered image (not at a draw boundary) is not an image either
    _raises(lambda: ops.coupling_log_prob(cd, cimgs[64:], x16, c32), "is not a packed image")
    # the entries still run on their own images
    with torch.no_grad():
        lp = nsc.log_prob(x16, condition=c32)
    assert torch.equal(ops.coupling_log_prob(cd, cimgs, x16, c32), lp)
    assert torch.isfinite(ops.ar_flow_log_prob(ad, aimg, x2, c2)).all()


def test_descriptor_and_layer_mismatch_is_refused():
    """An image packed for one descriptor, used with another (other layer count, other bins, other
    MFMA image mode) is refused: tag or size mismatch."""
    from naz_amd import ops
    nsc, _ = _flows()
    img = nsc._plan.packed()
    cd = nsc._plan.desc
    x, c = torch.randn(200, 16, device=DEV), torch.randn(200, 32, device=DEV)
    for field, value in (("L", cd.L + 1), ("L", cd.L - 1), ("K", 4), ("H", 64), ("mfma_mode", 2)):
        d2 = ops.coupling_desc(cd.D, cd.C, cd.S, cd.K, cd.L, cd.H)
        for f in ("D", "C", "S", "K", "L", "H", "act", "has_lower", "bound", "mfma_mode"):
            setattr(d2, f, getattr(cd, f))
        setattr(d2, field, value)
        if not ops.coupling_supported(d2):
            continue
        _raises(lambda: ops.coupling_log_prob(d2, img, x, c), "another descriptor", "layers")


def test_truncated_and_mistagged_host_images():
    """Host-packed images enter the registry through naz_image_attach, which reads the header back:
    a buffer shorter than the header announces, a header of another layout version or a bad magic
    are refused at attach; a corrupted layout tag is refused at launch."""
    from naz_amd import ops
    _, maf = _flows()
    d = maf._plan.desc
    good = maf._plan.packed()
    host = good.cpu()
    n = host.numel()
    L = ops.lib()
    trunc = host[: n // 2].to(DEV)
    assert L.naz_image_attach(trunc.data_ptr(), trunc.numel() * 4, None) != 0
    assert b"announces" in L.naz_last_error()
    bad_magic = host.clone()
    bad_magic[0:1].view(torch.int32)[0] = 12345
    bm = bad_magic.to(DEV)
    assert L.naz_image_attach(bm.data_ptr(), bm.numel() * 4, None) != 0
    assert b"no packed-image header" in L.naz_last_error()
    old = host.clone()
    old[1:2].view(torch.int32)[0] = 2
    ov = old.to(DEV)
    assert L.naz_image_attach(ov.data_ptr(), ov.numel() * 4, None) != 0
    assert b"layout version" in L.naz_last_error()
    tag = host.clone()
    tag[3:4].view(torch.int32)[0] ^= 0x5A5A
    tg = ops.attach_image(tag.to(DEV), "attach")
    x, c = torch.randn(500, 2, device=DEV), torch.randn(500, 2, device=DEV)
    _raises(lambda: ops.ar_flow_log_prob(d, tg, x, c), "another descriptor")
    ok = ops.attach_image(host.to(DEV), "attach")
    assert torch.equal(ops.ar_flow_log_prob(d, ok, x, c), ops.ar_flow_log_prob(d, good, x, c))


def test_batched_draw_ranges_and_pass0_flag():
    """A multi-draw image set is one registry record: draw p (or a run of draws from p) resolves,
    a draw range past the set or a different draw stride is refused, and an image packed with
    pass-0 constants only runs with pass0_const = 1."""
    from naz_amd import ops
    _, maf = _flows()
    d = maf._plan.desc
    g = torch.Generator().manual_seed(9)
    per = 2 * 150 + 2 * 150 + 150 + 2 * (150 * 150 + 150) + 4 * 150 + 4  # W0 | b0 | 2 x (W, b) | Wout | bout
    flat = (torch.randn(4, d.L * per, generator=g) * 0.05).to(DEV)
    perm = np.tile(np.array([1, 0], np.int32), (d.L, 1))
    imgs = ops.ar_flow_pack_batched(d, flat, perm)
    x = torch.randn(300, 2, device=DEV)
    ctx = torch.randn(2, device=DEV)
    full = ops.ar_flow_log_prob_batched(d, imgs, x, ctx)
    part = ops.ar_flow_log_prob_batched(d, imgs[1:3], x, ctx)
    assert torch.equal(part, full[1:3])
    one = ops.ar_flow_log_prob(d, imgs[2], x, ctx.reshape(1, 2).expand(300, 2))
    assert torch.equal(one, full[2])
    L = ops.lib()
    out = torch.empty(5 * 300, device=DEV)
    rc = L.naz_ar_flow_log_prob_batched(d, imgs.data_ptr(), imgs.stride(0), x.data_ptr(), 2, 0, ctx.data_ptr(), 0,
                                        out.data_ptr(), 300, 300, 5, 0, None, 0, None)
    assert rc != 0 and b"draws" in L.naz_last_error()
    rc = L.naz_ar_flow_log_prob_batched(d, imgs.data_ptr(), imgs.stride(0) + 64, x.data_ptr(), 2, 0, ctx.data_ptr(),
                                        0, out.data_ptr(), 300, 300, 2, 0, None, 0, None)
    assert rc != 0 and b"draws" in L.naz_last_error()
    _raises(lambda: ops.ar_flow_log_prob_batched(d, imgs, x, ctx, pass0_const=True), "pass-0")


def test_wide_maf_workspace_is_caller_owned():
    """The wide MLE MAF's inverse (made_ar_wide.h) keeps its hidden layers in the caller's workspace:
    too little (or none) is an error before any launch; the exact size
    (naz_ar_flow_workspace_bytes) gives the ops path's result bit for bit."""
    from naz_amd import ops
    from naz_amd.flows import NormalizingFlow
    torch.manual_seed(5)
    f = NormalizingFlow("maf", None, 4, 2, [512] * 5, 2).to(DEV)
    assert f.fused
    d, img = f._plan.desc, f._plan.packed()
    B = 1000
    x, c = torch.randn(B, 4, device=DEV), torch.randn(B, 2, device=DEV)
    ref = ops.ar_flow_log_prob(d, img, x, c)
    L = ops.lib()
    need = int(L.naz_ar_flow_workspace_bytes(d, B, 1))
    assert need == ((B + 63) // 64) * 4 * 128 * 1024
    out = torch.empty(B, device=DEV)
    args = (d, img.data_ptr(), x.data_ptr(), 4, c.data_ptr(), 2, None, None, out.data_ptr(), B)
    assert L.naz_ar_flow_log_prob(*args, None, 0, None) != 0 and b"workspace" in L.naz_last_error()
    ws = torch.empty(need, dtype=torch.uint8, device=DEV)
    assert L.naz_ar_flow_log_prob(*args, ws.data_ptr(), need - 16, None) != 0
    assert L.naz_ar_flow_log_prob(*args, ws.data_ptr(), need, torch.cuda.current_stream().cuda_stream) == 0
    assert torch.equal(out, ref)
    fd = ops.flow_desc(d)
    assert int(L.naz_workspace_bytes(fd, B)) == need
