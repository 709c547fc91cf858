"""aec_amd — MI355X (gfx950) drop-in for the Stage-2 AEC inference path of
SZU-Speech/Acoustic-Echo-Cancellation (Stage2_lhm/).

Public surface (mirrors the reference):
  * ``Little_net(conf, erb_bands, nlms=None)``      scripts/network/ERB.py:203 (+ build-defined FD-NLMS)
  * ``EquivalentRectangularBandwidth(...).filters`` scripts/network/ERB.py:10
  * ``speech_conf`` / ``erb_conf`` / ``net_conf``   scripts/configs.py:1-46
  * ``dccrn.DCCRN(config)`` / ``dccrn2.DCCRN(config)`` scripts/network/dccrn.py:453, dccrn2.py:10 (CRN, eval)
The compute runs in ``libaec_hip.so`` (C ABI: include/aec_hip.h, include/aec_crn.h).
"""
from .configs import speech_conf, erb_conf, train_conf, nlms_conf, net_conf  # noqa: F401
from .erb import EquivalentRectangularBandwidth, erb_matrix     # noqa: F401
from .little_net import Little_net                              # noqa: F401
from . import dccrn, dccrn2                                     # noqa: F401  (DCCRN v1 / v2 drop-ins)

WIN_SIZE = 512
HOP_SIZE = 256


def num_frames(n: int) -> int:
    """T = N//256 + 1 (attention_ccrn.py:48-49)."""
    return n // HOP_SIZE + 1


def out_len(n: int) -> int:
    """256*(N//256) (attention_ccrn.py:92,99)."""
    return HOP_SIZE * (n // HOP_SIZE)
