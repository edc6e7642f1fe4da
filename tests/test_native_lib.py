"""CPU checks of the C ABI boundary: the library loads and exports every symbol
declared in include/asr_hip.h, and the ctypes table mirrors the header.  No
compute calls (no GPU here)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'asr_hip.h')


def _declared():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(asr_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_entry_points():
    names = _declared()
    assert 'asr_ctc_forward' in names and 'asr_version' in names


def test_ctypes_table_mirrors_header():
    from pytorch_end2end_speech_recognition_amd import _native
    assert sorted(_native.SIGNATURES) == _declared()


def _prototypes():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    out = {}
    for m in re.finditer(r'\b(asr_[a-z0-9_]+)\s*\(([^)]*)\)\s*;', src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ('', 'void') else args.count(',') + 1
    return out


def test_ctypes_argument_counts_match_header():
    from pytorch_end2end_speech_recognition_amd import _native
    protos = _prototypes()
    for name, (_, args) in _native.SIGNATURES.items():
        assert len(args) == protos[name], (name, len(args), protos[name])


def test_library_loads_and_exports_every_symbol():
    from pytorch_end2end_speech_recognition_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.fail('libasr_hip.so not built (run __graft_entry__.build())')
    lib = _native.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.asr_version().decode().startswith('asr_hip')


def test_workspace_query_without_gpu():
    from pytorch_end2end_speech_recognition_amd import _native
    n = _native.query('asr_ctc_workspace_bytes', 1000, 32, 29, 125)
    assert n >= 2 * 32 * 1000 * 256 * 4


def test_gemm_split_plan_without_gpu():
    """Split-K is chosen from shapes only: the encoder's dW_hh product (two
    2048x512 outputs, K = B*T = 32000) splits; the gate GEMM does not."""
    import ctypes
    from pytorch_end2end_speech_recognition_amd import _native as N

    def prob(M, Nn, K, dtype=N.ASR_DT_BF16):
        g = N.Gemm()
        g.M, g.N, g.K, g.batch = M, Nn, K, 1
        g.a.dtype = g.b.dtype = dtype
        return g

    def nbytes(*ps):
        arr = (N.Gemm * len(ps))(*ps)
        return N.query('asr_gemm_workspace_bytes', ctypes.cast(arr, ctypes.c_void_p), len(ps))

    n = nbytes(prob(2048, 512, 32000), prob(2048, 512, 32000))
    assert n >= 2 * 2 * 2048 * 512 * 4
    assert nbytes(prob(32000, 4096, 1024)) == 0
    assert nbytes(prob(300, 29, 123)) == 0
    # f32 operands of a large enough product get bf16 staging copies (bf16 mode
    # converts them once and takes the fast kernels): M*K + N*K bf16 elements
    assert nbytes(prob(4032, 320, 640, N.ASR_DT_F32)) >= (4032 + 320) * 640 * 2
    assert nbytes(prob(300, 29, 123, N.ASR_DT_F32)) == 0   # too small: generic kernel


def test_bad_args_raise_runtime_error():
    from pytorch_end2end_speech_recognition_amd import _native
    with pytest.raises(RuntimeError):
        _native.call('asr_ctc_forward', None, 29, 29000, 1000, 32, 29, None, None, None, 10,
                     0, 1, None, None, 1.0, None, 0, None)


def test_no_packed_fp32_src1_high_dword_selects():
    """The gfx950 co-residency hazard: no v_pk_{add,mul,fma}_f32
    in the built library routes src1's / src2's high dword into the low lane
    (op_sel:[x,1,..]); tools/ubench/pk_hazard.hip measured that form returning
    0 in lanes 48-63 beside other work-groups' memory traffic."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import isa_check
    from pytorch_end2end_speech_recognition_amd import _native
    findings, total = isa_check.scan(_native.LIB_PATH)
    assert total > 0
    assert not findings, findings[:5]
