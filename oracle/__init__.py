"""ORACLE / TEST INFRASTRUCTURE ONLY: CPU restatements used as the checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
