"""CPU-side guard on the code generation of the MX-folded fused stream kernels
(crn_stream_enc_kernel<*, true>, crn_stream_dec_kernel<*, true>): hipcc
cross-compiles crn_stream.hip for gfx950 here and tests/isa_check.py reads the
assembly.  The workarounds it guards (keep_live,
the accumulator pins, mx_drain) depend on the compiler's
scheduling and register allocation, so a toolchain change that undoes them is
caught on the build host instead of as NaN / last-bit errors on the GPU box.

Checks per kernel (isa_check.check_kernel): no MFMA inside a lane-divergent
exec region; no scaled MFMA whose destination overlaps its A / B operand; in
the encoder fold, no scaled-MFMA operand register rewritten before the
three-`s_nop 15` drain.  The second test compiles the same source with every
workaround removed (-DCRN_NO_CODEGEN_GUARDS) and requires the check to flag it,
so a check that silently stopped seeing anything would fail too."""
import os

import pytest

import isa_check as I

pytestmark = pytest.mark.skipif(not os.path.exists(I.HIPCC), reason='hipcc not installed')


def test_fused_stream_codegen_guards():
    res = I.check_source()
    assert len(res) == 12, sorted(res)           # enc TAPS 0..8 + dec MODE 0..2, MX-folded instantiations
    bad = {k: v for k, v in res.items() if v}
    assert not bad, {k: v[:3] for k, v in bad.items()}


def test_check_flags_a_build_without_the_workarounds():
    res = I.check_source(('CRN_NO_CODEGEN_GUARDS',))
    flagged = [k for k, v in res.items() if v]
    assert any('enc_kernel' in k for k in flagged), 'the check no longer sees the missing drain / pins'
