"""CPU oracle of the reference swarm step path — TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
