"""Static checks of the gfx950 code object of the fused per-hop stream kernels
(crn_stream.hip), run on the CPU build host (hipcc cross-compiles the device
code; nothing here touches a GPU).

Two code-generation traps of these kernels were found on the GPU (DESIGN.md
§14.4) and are held off by source-level workarounds whose effect depends on the
compiler version:

* an MFMA whose destination registers overlap its own A or B operand (under
  448-VGPR pressure the allocator gave a first-stage MFMA vdst = a[56:59] with
  srcB = a[56:63]: NaN outputs) -- held off by `keep_live`;
* MFMAs sunk into a lane-divergent `exec` region (the operand moves of the
  masked-off lanes no longer ran: last-bit errors) -- held off by the empty
  `asm volatile` accumulator pins before the lane-divergent epilogues;
* the scale operands of `v_mfma_scale_*` still read after issue, which the
  compiler's hazard recognizer does not pad for -- held off by `mx_drain`
  (three `s_nop 15` after every run of scaled MFMAs).

check_kernel() finds each of these in the assembly of one kernel.
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, 'acoustic-echo-cancellation_amd', 'csrc')
HIPCC = '/opt/rocm/bin/hipcc'

_REG = re.compile(r'^([va])(?:\[(\d+):(\d+)\]|(\d+))$')


def compile_asm(src='crn_stream.hip', defines=()):
    """Device assembly of one source, with the library's own flags."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'k.s')
        subprocess.run([HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++17', '-fno-slp-vectorize',
                        '--cuda-device-only', '-S', f'-I{CSRC}', f'-I{os.path.join(REPO, "include")}',
                        *[f'-D{x}' for x in defines], os.path.join(CSRC, src), '-o', out],
                       check=True, capture_output=True)
        return open(out).read()


def kernels(asm, pattern):
    """{mangled name: [instruction lines]} of the kernels whose name matches."""
    res, cur = {}, None
    for line in asm.split('\n'):
        m = re.match(r'^(_Z\w+):', line)
        if m:
            cur = m.group(1) if re.search(pattern, m.group(1)) else None
            if cur:
                res[cur] = []
            continue
        if cur is None:
            continue
        t = line.strip()
        if t.startswith('.Lfunc_end'):
            cur = None
            continue
        if not t or t.startswith((';', '.')) or t.endswith(':'):
            continue
        res[cur].append(t.split(';')[0].strip())
    return res


def regs(op):
    """(file, first, last) of a register operand, or None."""
    m = _REG.match(op.strip())
    if not m:
        return None
    if m.group(4) is not None:
        i = int(m.group(4))
        return m.group(1), i, i
    return m.group(1), int(m.group(2)), int(m.group(3))


def _overlap(a, b):
    return a and b and a[0] == b[0] and a[1] <= b[2] and b[1] <= a[2]


def operands(ins):
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    ops = [o.strip() for o in re.split(r',(?![^\[]*\])', parts[1])]
    return parts[0], ops


def check_kernel(lines, war=True):
    """Violations in one kernel's instruction stream: (kind, index, instruction).

    * mfma-in-divergent-exec: any MFMA while a lane-divergent exec mask is in
      force (inside an s_and_saveexec ... s_or_b64 exec region);
    * scaled-mfma-dst-overlaps-src: a v_mfma_scale_* whose destination shares a
      register with its A or B operand (plain bf16 MFMAs with vdst == srcA and
      C = 0 are the compiler's normal, correct allocation and are not flagged);
    * scaled-operand-rewritten-before-drain: an instruction other than an MFMA
      writes a register that a scaled MFMA reads (A, B or a scale operand)
      before three `s_nop 15` have followed the latest scaled MFMA (mx_drain;
      the scale operands are still read after issue and the compiler's
      hazard recognizer does not pad for it)."""
    bad = []
    stack = []              # exec masks saved by the divergent regions we are inside (None: unsaved narrowing)
    pending = []            # operand registers of scaled MFMAs not yet drained
    nops = 0
    for i, ins in enumerate(lines):
        op, ops = operands(ins)
        if op == 's_and_saveexec_b64':
            stack.append(ops[0])
        elif op in ('s_and_b64', 's_andn2_b64') and ops and ops[0] == 'exec':
            stack.append(None)
        elif op == 's_or_b64' and ops[:2] == ['exec', 'exec']:
            saved = ops[2]
            while stack:
                if stack.pop() == saved:
                    break
        elif op == 's_mov_b64' and ops and ops[0] == 'exec':
            stack.clear()
        if op.startswith('v_mfma'):
            if stack:
                bad.append(('mfma-in-divergent-exec', i, ins))
            if op.startswith('v_mfma_scale'):
                dst, sa, sb = (regs(o) for o in ops[:3])
                if _overlap(dst, sa) or _overlap(dst, sb):
                    bad.append(('scaled-mfma-dst-overlaps-src', i, ins))
                pending += [r for r in (sa, sb, regs(ops[4]), regs(ops[5])) if r]
                nops = 0
            continue
        if not pending or not war:
            continue
        if op == 's_nop' and ops and ops[0] == '15':
            nops += 1
            if nops >= 3:
                pending = []
            continue
        if ops and not op.startswith(('ds_write', 'global_store', 'buffer_store', 'scratch_store', 'flat_store')):
            r = regs(ops[0])
            if r and any(_overlap(r, d) for d in pending):
                bad.append(('scaled-operand-rewritten-before-drain', i, ins))
                pending = []
    return bad


GUARDED = r'crn_stream_(enc|dec)_kernelILi\d+ELb1E'


def check_source(defines=()):
    """{kernel: violations} of the MX-folded fused stream kernels.  The drain
    (operand-rewrite) check applies to the encoder fold, whose MX level runs
    as one straight run of scaled MFMAs closed by mx_drain; the decoder fold's
    K-stage loop reuses operand registers between stages under the compiler's
    own hazard model, so there only the overlap and exec checks apply."""
    ks = kernels(compile_asm('crn_stream.hip', defines), GUARDED)
    return {k: check_kernel(v, war='enc_kernel' in k) for k, v in ks.items()}
