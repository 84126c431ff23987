"""naz.flows -> naz_amd.flows."""
