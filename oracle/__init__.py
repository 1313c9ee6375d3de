"""Parity oracle -- TEST INFRASTRUCTURE ONLY (see crc32c_oracle.py header).

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package ``revel_amd`` never imports it.
"""
