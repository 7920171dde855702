"""CPU oracle for the omega-mi355x hot path.

TEST INFRASTRUCTURE ONLY. Nothing under ``oracle/`` is part of the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as
the checker (or as the timed CPU baseline), never as a fallback for the HIP path.

Parity pin: the restatement in :mod:`oracle.omega_ref` is checked against golden vectors in
``tests/golden/`` that ``oracle/gen_golden.py`` produced by importing the reference itself
(``/root/reference``, numpy 2.2.6 / scipy 1.15.3) in the build container.
"""
