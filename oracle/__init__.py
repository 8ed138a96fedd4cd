"""CPU oracle for the hot path -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  See dx_oracle.py (NumPy scalar restatement) and
dx_oracle.c (C restatement, built into oracle/_build/libdxoracle.so).
"""
