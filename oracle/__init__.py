"""CPU oracle for the hot path -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The oracle is dx_oracle.py: a scalar NumPy restatement of
the reference (pinned by the golden fixtures the reference itself produced)
plus a restatement of the build's own device Philox streams (pinned by the
Random123 known-answer vectors).  The reference is pure Python, so there is
no compiled reference build (oracle/_ref) and no C restatement.
"""
