"""ORACLE — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
and only as the checker. The product package never imports it.
"""
