import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "brickbrain-rec-engine_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbrickrec on the device)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load


def pytest_sessionfinish(session, exitstatus):
    """Near-tie gate counts of every parity test that ran (tests/_parity.py RECORDS) ->
    gpurun_out/parity_gates.json (BB_GATE_OUT overrides), so a -q run keeps them."""
    mod = sys.modules.get("_parity")
    recs = getattr(mod, "RECORDS", None)
    if not recs:
        return
    import json
    out = os.environ.get("BB_GATE_OUT", os.path.join(ROOT, "gpurun_out", "parity_gates.json"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"exitstatus": int(exitstatus), "gates": recs}, f, indent=1)
