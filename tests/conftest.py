"""pytest configuration: the ``gpu`` marker and import paths.

``-m "not gpu"`` runs here (no GPU): oracle vs golden fixtures, host logic, the
C-ABI library's exports.  ``-m gpu`` runs on an MI355X box: parity of libpiadmm
against the oracle and the golden fixtures, through the C-ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libpiadmm kernels)")
