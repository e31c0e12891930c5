"""MI355X-native LDPC belief-propagation Monte-Carlo engine.

Drop-in for the decoding hot path of roryhighnam/iib_project_ldpc_codes
(message_passing.c behind parallel_simulator.py), plus batched soft decoding
(sum-product / min-sum), on-device channels and a multi-GPU Monte-Carlo driver.
All compute runs in libldpc_mi355x.so (hand-written HIP for gfx950).
"""
from . import _native  # noqa: F401
from ._native import LdpcError  # noqa: F401
from .graph import TannerGraph  # noqa: F401

__all__ = ["TannerGraph", "LdpcError"]
