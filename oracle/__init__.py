"""CPU oracle for the RP-Style-Transfer hot path — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product (rp-style-transfer_amd/) must never import it. See restate.py.
"""
