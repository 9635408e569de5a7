"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see s2s_oracle.py header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
