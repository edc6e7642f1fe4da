"""Build-time ISA check of libasr_hip.so (round 5).

gfx950 hazard found this round (tools/ubench/pk_hazard.hip, profiles/
r05_pk_hazard.txt): a packed-FP32 VALU instruction (v_pk_{add,mul,fma}_f32)
whose LOW lane reads the HIGH dword of its second source (op_sel:[x,1,..])
intermittently returns 0 in lanes 48-63 of the wave while waves of other
work-groups with memory traffic share the SIMD.  That was the co-residency
fault of the backward recurrence (rounds 3-4).  Measured clean under the same
load: op_sel on src0 (op_sel:[1,0]), the broadcast forms (op_sel_hi:[0,1] /
[1,0]) and the unselected forms.  src2 of v_pk_fma_f32 was not measured and is
treated like src1.  The library is compiled so that the compiler does not
form such instructions (csrc/Makefile), and this script proves it on the built
code objects: every packed-FP32 instruction is counted and any high-dword
selection on src1 / src2 is an error.

usage: python tools/isa_check.py [lib.so]   (exit 1 on a finding, or when no code
object / no packed-FP32 instruction was found: the check would be vacuous)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'pytorch_end2end_speech_recognition_amd', 'libasr_hip.so')
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


def code_objects(path):
    """Every gfx950 device code object in the .so's offload bundles."""
    data = open(path, 'rb').read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from('<Q', data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tlen].decode(errors='replace')
            p += 24 + tlen
            if 'gfx950' in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


PK = re.compile(r'\bv_pk_(add|mul|fma)_f32\b(.*)$')


def crossing(operands):
    """True when op_sel routes the HIGH dword of src1 (or src2) into the low lane."""
    m = re.search(r'op_sel:\[([01,]+)\]', operands)
    sel = [int(x) for x in m.group(1).split(',')] if m else []
    return any(sel[i] == 1 for i in (1, 2) if i < len(sel))


def scan(path=LIB, counts=None):
    findings, total = [], 0
    cos = code_objects(path)
    if counts is not None:
        counts['code_objects'] = len(cos)
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(cos):
            f = os.path.join(d, 'co%d.o' % k)
            open(f, 'wb').write(co)
            txt = subprocess.run([OBJDUMP, '-d', '--no-show-raw-insn', f], capture_output=True,
                                 text=True, check=True).stdout
            kern = '?'
            for line in txt.splitlines():
                if line.endswith('>:'):
                    kern = line.split('<', 1)[-1][:-2]
                    continue
                m = PK.search(line)
                if m:
                    total += 1
                    if crossing(m.group(2)):
                        findings.append((kern, line.strip()))
    return findings, total


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else LIB
    counts = {}
    findings, total = scan(path, counts)
    print('%s: %d gfx950 code objects, %d packed-FP32 instructions, %d selecting a src1 / '
          'src2 high dword' % (os.path.basename(path), counts['code_objects'], total,
                               len(findings)))
    for kern, line in findings[:40]:
        print('  %s: %s' % (kern[:90], line))
    if not counts['code_objects'] or not total:
        # nothing scanned (a changed bundle format or triple, or a build without
        # the recurrence's packed math): the gate would be vacuous -- fail it
        print('isa_check: no gfx950 code object or no packed-FP32 instruction found; '
              'the hazard check did not run (ADVICE r05)')
        return 1
    return 1 if findings else 0


if __name__ == '__main__':
    sys.exit(main())
