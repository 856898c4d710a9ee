"""CPU oracle for the Retina flow-aggregation path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker; the product (``retina_amd``) never
imports it.
"""
