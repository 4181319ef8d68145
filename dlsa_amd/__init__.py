"""dlsa_amd -- Distributed Least Squares Approximation on AMD MI355X.

Drop-in for the estimation path of the reference ``dlsa`` package
(Vicky-Lamperouge/dlsa): ``models.logistic_model`` (map), ``dlsa.dlsa_mapred``
(combine), ``dlsa.dlsa`` and ``lsa.lars_lsa`` (adaptive-lasso / DBIC
selection), with the per-partition fits running as hand-written gfx950 HIP
kernels (libdlsa_hip.so, C-ABI in include/dlsa_hip.h).
"""

__version__ = "0.1.0"

from ._hip import DlsaHipError  # noqa: F401
