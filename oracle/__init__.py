"""Oracle package: CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
See oracle/piadmm_oracle.py for what is restated and how parity is pinned.
"""
