"""Monotonic Alignment Search for CFM training (§8f rank 3).

Drop-in for the reference's `maximum_path(neg_cent, mask)` (train_standalone.py:280-325), which
copies the log-prior to the host and runs a numba / Python DP there (train_standalone.py:646). Here
the same recurrence runs on the GPU (`mt_maximum_path`, csrc/mt_mas.hip): inputs stay in HBM, the
result is bit-identical to the reference (tests/test_mas.py against tests/golden/g7_mas.npz).
"""
from matcha_hip.runtime import maximum_path

__all__ = ["maximum_path"]
