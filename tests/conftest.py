import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dist-svgd_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


# worst parity error seen per test (tests record into it; written at session end)
PARITY = {}
INFO = {}


def record_parity(err, **info):
    """Keep the worst error of the running test; optional counters (e.g. the
    auction's round count) go to the "info" section of the dump."""
    key = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    PARITY[key] = max(PARITY.get(key, 0.0), float(err))
    if info:
        INFO[key] = info


def pytest_sessionfinish(session, exitstatus):
    if not PARITY:
        return
    import json
    import time
    out = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_%d.json" % int(time.time())), "w") as f:
            doc = dict(sorted(PARITY.items()))
            if INFO:
                doc["info"] = dict(sorted(INFO.items()))
            json.dump(doc, f, indent=1)
    except OSError:
        pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")


@pytest.fixture
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    return load
