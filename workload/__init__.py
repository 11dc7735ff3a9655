"""Synthetic workloads for the BASELINE.json configs (bench.py and tests).
Not part of the product package: trivy_amd/ never imports this."""
