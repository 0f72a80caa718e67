"""Parity oracle — TEST INFRASTRUCTURE ONLY (see raft_oracle.py header).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
