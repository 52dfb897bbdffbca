"""ORACLE — test infrastructure only.

Nothing under ``oracle/`` is part of the product. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker (never as the thing measured or shipped).
"""
