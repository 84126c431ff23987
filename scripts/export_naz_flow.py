"""Export a trained reference naz flow to naz_amd's canonical .npz.

Run where the reference's stack (pyro-ppl, torch) is installed, on a flow YOU pickled with
naz (train_mle_all_data.py:77-82 writes them with pickle.dump):

    python scripts/export_naz_flow.py model.pkl model.npz [--spec '{"flow_type": "maf", ...}']

Unpickling executes code from the file: only run it on your own trained models.  The .npz
holds plain arrays (no pickle) and loads into naz_amd with

    flow = naz_amd.flows.NormalizingFlow('maf', None, D, C, hidden, L)
    naz_amd.flows.io.load_npz(flow, 'model.npz')
"""
import argparse
import json
import pickle
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from naz_amd.flows.io import state_from_reference_flow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pickle_in")
    ap.add_argument("npz_out")
    ap.add_argument("--spec", default=None, help="optional JSON spec stored next to the weights (spec/* keys)")
    a = ap.parse_args()
    with open(a.pickle_in, "rb") as f:
        ref_flow = pickle.load(f)  # the user's own model file (see the module docstring)
    state = state_from_reference_flow(ref_flow)
    if a.spec:
        for k, v in json.loads(a.spec).items():
            state["spec/" + k] = np.asarray(v)
    np.savez(a.npz_out, **state)
    print(f"wrote {len(state)} arrays to {a.npz_out}")


if __name__ == "__main__":
    main()
