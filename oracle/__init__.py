"""TEST INFRASTRUCTURE ONLY — CPU oracle for the naz normalizing-flow hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker / the timed
CPU baseline.  The product package ``naz_amd`` never imports it: its compute
path is the HIP library and fails loudly when that library is missing.

Contents
--------
naz_oracle   pure-torch (CPU, any float dtype) restatement of the pyro-ppl 1.9
             semantics naz's hot path delegates to (SURVEY.md §8a rows a1–a9).
jax_maf_np   numpy restatement of the reference's own in-tree JAX affine MAF
             (``src/naz/flows/bflow_jax_maf.py:48-225``) — an independent second
             statement of the affine path used to cross-check ``naz_oracle``.
gen_golden   writes the committed fixtures under ``tests/golden/``.

Parity status: the reference's arithmetic lives in
``pyro-ppl`` (unpinned, not installed, not vendored) and the reference ships no
tests or fixtures, so the spline / coupling / autoregressive arithmetic is
**parity unpinned** by the reference itself.  The affine MAF is pinned against
the reference's in-tree JAX restatement (read as text, re-stated in numpy).
"""
