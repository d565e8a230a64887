"""CPU oracle for the wrlife/tf_depth_estimation hot path -- TEST INFRASTRUCTURE ONLY.

This package is a float64 (or float32) PyTorch-CPU / NumPy *restatement* of the reference's
TensorFlow-1 graph: the conv/deconv encoder-decoders (`nets_optflow_depth.py`, `nets_depth.py`,
`nets_optflow_depth_pairtest.py`), the geometry / warp library (`utils_lr.py`, `utils.py`), the
per-config loss loops (`train_depth_only.py`, `train_optflow_combine.py`,
`train_depth_then_cam_lr.py`, `refine_depth.py`) and TF's Adam.  Every function cites the
reference file:line it follows.

Rules (see DESIGN.md "Oracle"):
  * Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may import
    this package, and only as the checker / CPU baseline.  The product package
    `tf_depth_estimation_amd` never imports it and has no CPU fallback.
  * Parity status: the reference ships no fixtures, golden outputs or tests, and TensorFlow 1.x is
    not importable in this container.  The restatement is pinned by
    known-answer tests derived from the reference formulas, by cross-checks against
    independent NumPy loop implementations of the TF-1 op semantics, and by float64
    finite-difference gradient checks (tests/test_oracle_*.py).  Against TensorFlow itself the
    oracle is therefore **parity unpinned**.
"""
