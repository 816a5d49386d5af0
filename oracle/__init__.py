"""ORACLE package — test infrastructure (CPU restatement of the reference hot path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product path (robust-nerf_amd/noisy_src) never does.
"""
