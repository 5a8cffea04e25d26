"""Shared fixture plumbing for the parity tests (CPU and GPU): the catalogue side-car of the
golden vectors and the joint content/CF item space the hybrid cases run in."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def catalog_json():
    with open(os.path.join(GOLDEN, "catalog.json")) as f:
        return json.load(f)


def hybrid_space(golden):
    """Content rows + CF item factors scattered into the content row space (+ CF-only sets
    appended as rows that are absent from the content side).

    Returns X (content features), present (content item space), F (CF factors),
    cf_present (CF item space), rated (per-user rated bitmap), n (joint rows), n_rows
    (content rows)."""
    g1, g3 = golden("g1_content.npz"), golden("g3_cf.npz")
    cat = catalog_json()
    rows = list(cat["row_set_nums"])
    pos = {s: i for i, s in enumerate(rows)}
    extra = [s for s in cat["cf_columns"] if s not in pos]
    for s in extra:
        pos[s] = len(pos)
    n = len(pos)
    X = np.zeros((n, g1["feat_matrix"].shape[1]))
    X[: len(rows)] = g1["feat_matrix"]
    present = np.zeros(n, bool)
    present[: len(rows)] = True
    F = np.zeros((n, g3["item_factors"].shape[1]))
    cf_present = np.zeros(n, bool)
    cols = [pos[s] for s in cat["cf_columns"]]
    F[cols] = g3["item_factors"]
    cf_present[cols] = True
    rated = np.zeros((g3["rated"].shape[0], n), bool)
    rated[:, cols] = g3["rated"]
    return X, present, F, cf_present, rated, n, len(rows)


def constraint_pairs(kw):
    """create_constraint_set(**kw) -> [(constraint_type value, value)] for the oracle."""
    from brickrec.constraints import create_constraint_set_values
    return [(c.constraint_type.value, c.value) for c in create_constraint_set_values(**kw)]
