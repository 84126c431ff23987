"""Import-compatible front for naz_amd: the module paths naz's own scripts import
(``naz.flows.flow``, ``naz.flows.transforms``, ``naz.flows.continuous_transforms``,
``naz.flows.mcdpflow``, ``naz.flows.bflow_jax_maf``, ``naz.trainers.train_flows``,
``naz.utils``) re-export the MI355X implementation in ``naz_amd``, so front ends written
against naz (e.g. examples/papers/2506.05657/train_mle_all_data.py:1-20, 62-76) run unchanged.
Every name here is a re-export; the implementations and their reference citations live in
``naz_amd``."""
