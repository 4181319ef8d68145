"""CPU oracle for the DLSA hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference algorithm
(Vicky-Lamperouge/dlsa, read-only at /root/reference).  It exists to *check*
the MI355X product path, never to run it:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import it;
* nothing under ``dlsa_amd/`` imports it -- the product path fails loudly
  when the HIP library is missing instead of falling back to this code.

Pinning: every function here is checked against golden vectors produced by
the reference itself (``tests/golden/make_golden.py`` imports
``/root/reference`` through a small compatibility shim and records its
outputs in ``tests/golden/*.npz``; ``tests/test_oracle_golden.py`` asserts
the agreement).  See DESIGN.md section "Oracle".
"""

from .dlsa_oracle import (  # noqa: F401
    dummy_design,
    expand_codes,
    simulate_logistic_arrays,
    simulate_logistic,
    simulate_counter,
    systematic_partition,
    logistic_fit,
    logistic_fit_partitions,
    dlsa_mapred,
    lars_lsa,
    dlsa,
    ols_fit,
    logistic_loglik,
    column_moments,
)
