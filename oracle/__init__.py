"""Parity oracle -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package never imports it.  See
depth_pro_oracle.py for what it restates and how it is pinned to the
reference (tests/golden/).
"""
