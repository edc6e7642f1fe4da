"""The persistent hot-path kernels of the bf16 bench configs use no scratch
(private segment 0): a register spill in a persistent pass costs far more than
its bytes suggest (round 6: a 12-B spill in the production decoder backward,
from carrying both the conv-feature load and the recompute path in one
instantiation, made att4x320 14.2 -> 18.9 ms / step).  Read from the gfx950
code objects' AMDGPU metadata in the built objects (CPU only)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, 'pytorch_end2end_speech_recognition_amd', 'csrc', 'build')
LLVM = '/opt/rocm/lib/llvm/bin'

# (object, kernel-name regex) that must be spill-free: the bf16 production
# decoder passes (SA/SE/SD/SK = 128/640/320/201, F32 = false, both conv-feature
# variants), every BLSTM recurrence and CTC lattice instantiation
HOT = [
    ('decoder', r'attdec_fwd_persistILi10ELi2ELi128ELi640ELi320ELi201ELb0E'),
    ('decoder', r'attdec_bwd_persistILi10ELi2ELi128ELi640ELi320ELi201ELb0ELb[01]E'),
    ('lstm_xg', r'lstm_fwd_xgx'),
    ('lstm_xg', r'lstm_bwd_xg'),
    ('ctc', r'ctc_lattice'),
]


def _kernels(obj, tmp_path):
    src = os.path.join(BUILD, obj + '.o')
    if not os.path.exists(src):
        pytest.skip('%s not built (run __graft_entry__.build())' % src)
    fat = str(tmp_path / (obj + '.fatbin'))
    co = str(tmp_path / (obj + '.co'))
    subprocess.check_call([os.path.join(LLVM, 'llvm-objcopy'), '--dump-section=.hip_fatbin=' + fat,
                           src])
    subprocess.check_call([os.path.join(LLVM, 'clang-offload-bundler'), '--type=o', '--unbundle',
                           '--input=' + fat, '--output=' + co,
                           '--targets=hipv4-amdgcn-amd-amdhsa--gfx950'])
    notes = subprocess.check_output([os.path.join(LLVM, 'llvm-readelf'), '--notes', co]).decode()
    out, name = {}, None
    for line in notes.splitlines():
        m = re.match(r'\s+\.name:\s+(\S+)', line)
        if m:
            name = m.group(1)
            continue
        m = re.match(r'\s+\.private_segment_fixed_size:\s+(\d+)', line)
        if m and name is not None:
            out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, 'clang-offload-bundler')),
                    reason='ROCm LLVM tools absent')
@pytest.mark.parametrize('obj,pat', HOT)
def test_hot_kernels_spill_free(obj, pat, tmp_path):
    ks = _kernels(obj, tmp_path)
    hits = {k: v for k, v in ks.items() if re.search(pat, k)}
    assert hits, 'no kernel matching %s in %s.o' % (pat, obj)
    spilled = {k: v for k, v in hits.items() if v}
    assert not spilled, 'scratch bytes / lane: %s' % spilled
