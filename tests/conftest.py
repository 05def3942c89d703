import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


def pytest_terminal_summary(terminalreporter):
    """The margin of every logits parity check of the run (tests/grad_check.py), printed
    even under -q: err = max |GPU - fp64|, bar = the asserted bound, d32 = max |GPU - the
    CPU-fp32 reference|, floor = the CPU-fp32 reference's own error."""
    from tests.grad_check import LOGITS_MARGINS
    if not LOGITS_MARGINS:
        return
    tr = terminalreporter
    tr.write_line("logits parity margins (err/bar <= 1 passes):")
    for tag, err, bar, d32, floor in LOGITS_MARGINS:
        tr.write_line(f"  {tag:40s} err {err:.3e} bar {bar:.3e} err/bar {err / bar:.2f}  "
                      f"vs CPU-fp32 {d32:.3e}  CPU-fp32 floor {floor:.3e}")
    from tests.grad_check import WELL_CONDITIONED
    over = [m for m in LOGITS_MARGINS if m[3] > 1e-4]
    wc = [m for m in LOGITS_MARGINS if m[4] <= WELL_CONDITIONED]
    tr.write_line(f"logits checks: {len(LOGITS_MARGINS)}; more than 1e-4 from the CPU-fp32 "
                  f"reference: {len(over)} ({', '.join(m[0] for m in over) or 'none'}); in the "
                  f"well-conditioned regime (CPU-fp32 floor <= {WELL_CONDITIONED:g}): {len(wc)}, of "
                  f"them above 1e-4: {sum(m[3] > 1e-4 for m in wc)}")
