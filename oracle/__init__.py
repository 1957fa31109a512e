"""ORACLE package — test infrastructure only (see oracle/fedavg_oracle.py header).

Never imported by the product package ``fedlesscan_amd``.
"""
