"""Oracle package -- TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
See oracle/zk_oracle.h for what it restates and how it is pinned.
"""
