"""ORACLE / TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's secret-scanning path used as the parity
checker.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this package; the product (trivy_amd/) never does.
"""
