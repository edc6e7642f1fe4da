"""The bf16 GEMM kernels of csrc/gemm.hip (no vendor library on the path):
plain products in all four operand layouts, padded leading dimensions,
alpha/beta, one bias and the summed bias pair (nn.LSTM's b_ih + b_hh), a launch
that mixes a plain problem with a row-mapped one, the 256 x 256 8-wave kernel
and its ring variant over ragged shapes and split-K.  Small-integer operands
make bf16 products with f32 accumulation exact, so the results must equal
float64 bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from pytorch_end2end_speech_recognition_amd import native_ops
    return native_ops


def _store(rng, rows, cols, ld):
    a = np.zeros((rows, ld), np.float32)
    a[:, :cols] = rng.randint(-3, 4, (rows, cols))
    return a


@pytest.mark.parametrize('at,bt', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('nbias', [0, 1, 2])
def test_plain_gemm_exact(at, bt, nbias, cuda_dev):
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(10 * at + bt + 100 * nbias)
        M, Nn, K = 2048, 1024, 1032
        pad = 8
        sa = _store(rng, K if at else M, M if at else K, (M if at else K) + pad)
        sb = _store(rng, K if bt else Nn, Nn if bt else K, (Nn if bt else K) + pad)
        A = (sa[:, :M].T if at else sa[:, :K]).astype(np.float64)
        Bm = (sb[:, :Nn].T if bt else sb[:, :K]).astype(np.float64)
        ad = torch.from_numpy(sa).to(torch.bfloat16).to(cuda_dev)
        bd = torch.from_numpy(sb).to(torch.bfloat16).to(cuda_dev)
        ldc = Nn + 4
        c0 = rng.randint(-4, 5, (M, ldc)).astype(np.float32)
        C = torch.from_numpy(c0).to(cuda_dev)
        b1 = rng.randint(-8, 9, Nn).astype(np.float32)
        b2 = rng.randint(-8, 9, Nn).astype(np.float32)
        kw = {}
        if nbias >= 1:
            kw['bias'] = torch.from_numpy(b1).to(cuda_dev)
        if nbias == 2:
            kw['bias2'] = torch.from_numpy(b2).to(cuda_dev)
        p = ops.gemm_problem(ops.operand(ad, at, ops.rowmap(sa.shape[1])),
                             ops.operand(bd, bt, ops.rowmap(sb.shape[1])), C, ops.rowmap(ldc),
                             M, Nn, K, alpha=0.5, beta=1.0, **kw)
        ops.run_gemm([p], cuda_dev)
        torch.cuda.synchronize()
        ref = c0.astype(np.float64).copy()
        ref[:, :Nn] += 0.5 * A @ Bm.T
        if nbias >= 1:
            ref[:, :Nn] += b1
        if nbias == 2:
            ref[:, :Nn] += b2
        np.testing.assert_array_equal(C.cpu().numpy(), ref)
    finally:
        ops.set_compute_dtype('fp32')


def test_plain_and_mapped_problems_in_one_launch(cuda_dev):
    """nprob = 2: a plain product next to a subsampled-row product (t_mul = 2)
    that also needs a split-K slab."""
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(3)
        M, Nn, K = 4096, 1024, 1024
        a = rng.randint(-3, 4, (M, K)).astype(np.float32)
        b = rng.randint(-3, 4, (Nn, K)).astype(np.float32)
        ad = torch.from_numpy(a).to(torch.bfloat16).to(cuda_dev)
        bd = torch.from_numpy(b).to(torch.bfloat16).to(cuda_dev)
        C1 = torch.zeros(M, Nn, device=cuda_dev)
        p1 = ops.gemm_problem(ops.operand(ad, 0, ops.rowmap(K)), ops.operand(bd, 0, ops.rowmap(K)),
                              C1, ops.rowmap(Nn), M, Nn, K)
        # dW-shaped: C2[Nn2][K] = sum over every other row t of g[t] x[t]
        Tn, N2 = 4096, 256
        g = rng.randint(-3, 4, (2 * Tn, 64)).astype(np.float32)
        x = rng.randint(-3, 4, (2 * Tn, N2)).astype(np.float32)
        gd = torch.from_numpy(g).to(torch.bfloat16).to(cuda_dev)
        xd = torch.from_numpy(x).to(torch.bfloat16).to(cuda_dev)
        C2 = torch.zeros(64, N2, device=cuda_dev)
        p2 = ops.gemm_problem(ops.operand(gd, 1, ops.rowmap(64, t_mul=2, t_add=1)),
                              ops.operand(xd, 1, ops.rowmap(N2, t_mul=2, t_add=1)), C2,
                              ops.rowmap(N2), 64, N2, Tn)
        ops.run_gemm([p1, p2], cuda_dev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C1.cpu().numpy(), a.astype(np.float64) @ b.T)
        ref2 = g[1::2].T.astype(np.float64) @ x[1::2]
        np.testing.assert_array_equal(C2.cpu().numpy(), ref2)
    finally:
        ops.set_compute_dtype('fp32')


def test_linear_bf16_staged_padded(cuda_dev):
    """LinearFn in bf16 mode above the staging threshold with an output width
    that is not a multiple of 8 (the word-level CTC head, V = 10001): operands
    staged in bf16 with zero-padded pitches; y, dx, dW, db vs float64 of the
    same bf16-rounded values."""
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(11)
        M, K, Nout = 2048, 640, 1001            # 2 M N K = 2.6e9 >= _STAGE_FLOPS
        x = rng.randn(M, K).astype(np.float32)
        w = (rng.randn(Nout, K) * 0.05).astype(np.float32)
        b = rng.randn(Nout).astype(np.float32)
        dy = rng.randn(M, Nout).astype(np.float32)
        xd = torch.from_numpy(x).to(cuda_dev).requires_grad_(True)
        wd = torch.from_numpy(w).to(cuda_dev).requires_grad_(True)
        bd = torch.from_numpy(b).to(cuda_dev).requires_grad_(True)
        y = ops.linear(xd, wd, bd)
        y.backward(torch.from_numpy(dy).to(cuda_dev))
        torch.cuda.synchronize()

        def r(a):
            return torch.from_numpy(a).to(torch.bfloat16).double().numpy()
        xr, wr, dyr = r(x), r(w), r(dy)
        ref_y = xr @ wr.T + b
        ref_dx = dyr @ wr
        ref_dw = dyr.T @ xr
        for got, ref in ((y, ref_y), (xd.grad, ref_dx), (wd.grad, ref_dw)):
            g = got.detach().cpu().double().numpy()
            assert np.abs(g - ref).max() / (np.abs(ref).max() + 1e-9) < 1e-3
        np.testing.assert_allclose(bd.grad.cpu().numpy(), dy.sum(0), rtol=1e-4, atol=1e-3)
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('M,K,Nout', [(2048, 640, 1001), (4160, 320, 320), (999, 960, 33)])
def test_linear_staging_one_launch_bitwise(M, K, Nout, cuda_dev, monkeypatch):
    """A staged bf16 linear layer converts its input, weight and zero pad rows
    in one launch (asr_convert_rows_bf16_multi): y, dx, dW, db equal the
    one-conversion-per-launch path (ASR_LINEAR_MULTI=0) bit for bit, padded
    (Nout % 8 != 0) and dense output widths."""
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(M + K + Nout)
        x = rng.randn(M, K).astype(np.float32)
        w = (rng.randn(Nout, K) * 0.05).astype(np.float32)
        b = rng.randn(Nout).astype(np.float32)
        dy = rng.randn(M, Nout).astype(np.float32)
        outs = {}
        for multi in ('0', '1'):
            monkeypatch.setenv('ASR_LINEAR_MULTI', multi)
            xd = torch.from_numpy(x).to(cuda_dev).requires_grad_(True)
            wd = torch.from_numpy(w).to(cuda_dev).requires_grad_(True)
            bd = torch.from_numpy(b).to(cuda_dev).requires_grad_(True)
            y = ops.linear(xd, wd, bd)
            y.backward(torch.from_numpy(dy).to(cuda_dev))
            torch.cuda.synchronize()
            outs[multi] = [t.detach().cpu() for t in (y, xd.grad, wd.grad, bd.grad)]
        for name, a1, a0 in zip(('y', 'dx', 'dW', 'db'), outs['1'], outs['0']):
            assert torch.equal(a1, a0), name
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('M,N,K', [(529, 389, 3000), (256, 256, 64), (300, 260, 200),
                                    (1024, 512, 8000)])
def test_kmajor_256_tiles_exact(M, N, K, cuda_dev, monkeypatch):
    """K-major x K-major products with M, N >= 256 take the 256 x 256 kernel
    (gemm_bf16_kk256, opt-in by ASR_GEMM_KK256=1): ragged edges, a single
    k-tile, a K that is not a multiple of the 32-deep k-tile, split-K chunks;
    alpha / beta / bias."""
    monkeypatch.setenv('ASR_GEMM_KK256', '1')
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(M + N + K)
        a = rng.randint(-3, 4, (K, M + 8)).astype(np.float32)     # stored [K][M(+pad)]
        b = rng.randint(-3, 4, (K, N + 16)).astype(np.float32)
        c0 = rng.randint(-4, 5, (M, N)).astype(np.float32)
        bias = rng.randint(-8, 9, N).astype(np.float32)
        ad = torch.from_numpy(a).to(torch.bfloat16).to(cuda_dev)
        bd = torch.from_numpy(b).to(torch.bfloat16).to(cuda_dev)
        C = torch.from_numpy(c0).to(cuda_dev)
        bias_d = torch.from_numpy(bias).to(cuda_dev)
        p = ops.gemm_problem(ops.operand(ad, 1, ops.rowmap(M + 8)),
                             ops.operand(bd, 1, ops.rowmap(N + 16)), C, ops.rowmap(N), M, N, K,
                             alpha=2.0, beta=1.0, bias=bias_d)
        ops.run_gemm([p], cuda_dev)
        torch.cuda.synchronize()
        ref = 2.0 * (a[:, :M].T.astype(np.float64) @ b[:, :N]) + c0 + bias
        np.testing.assert_array_equal(C.cpu().numpy(), ref)
    finally:
        ops.set_compute_dtype('fp32')


def test_kmajor_256_tiles_two_problems_rowmapped(cuda_dev, monkeypatch):
    """The dW_hh launch shape: two problems side by side, the second reading
    column offsets, the B operand through a shifted per-utterance row map
    (h_{t-1}: t_add = -1, rows past the utterance read as zeros)."""
    monkeypatch.setenv('ASR_GEMM_KK256', '1')
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(5)
        Bu, T, H = 4, 700, 256
        g = rng.randint(-3, 4, (Bu * T, 8 * H)).astype(np.float32)
        y = rng.randint(-3, 4, (Bu * T, 2 * H)).astype(np.float32)
        gd = torch.from_numpy(g).to(torch.bfloat16).to(cuda_dev)
        yd = torch.from_numpy(y).to(torch.bfloat16).to(cuda_dev)
        C = torch.zeros(2, 4 * H, H, device=cuda_dev)
        R = ops.rowmap
        hp_f = R(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=-1, t_limit=T)
        hp_r = R(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=1, t_limit=T)
        ops.run_gemm([
            ops.gemm_problem(ops.operand(gd, 1, R(8 * H)), ops.operand(yd, 1, hp_f), C, R(H),
                             4 * H, H, Bu * T, beta=1.0),
            ops.gemm_problem(ops.operand(gd, 1, R(8 * H), offset=4 * H),
                             ops.operand(yd, 1, hp_r, offset=H), C, R(H), 4 * H, H, Bu * T,
                             beta=1.0, c_offset=4 * H * H),
        ], cuda_dev)
        torch.cuda.synchronize()
        y3 = y.reshape(Bu, T, 2 * H).astype(np.float64)
        hf = np.zeros_like(y3[:, :, :H]); hf[:, 1:] = y3[:, :-1, :H]
        hr = np.zeros_like(y3[:, :, H:]); hr[:, :-1] = y3[:, 1:, H:]
        g64 = g.astype(np.float64)
        ref_f = g64[:, :4 * H].T @ hf.reshape(-1, H)
        ref_r = g64[:, 4 * H:].T @ hr.reshape(-1, H)
        got = C.cpu().numpy()
        np.testing.assert_array_equal(got[0], ref_f)
        np.testing.assert_array_equal(got[1], ref_r)
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('ring', ['0', '1'])
@pytest.mark.parametrize('at,bt', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K', [(256, 256, 64), (529, 389, 3000), (300, 260, 200),
                                    (1024, 512, 8000), (777, 1030, 1000)])
def test_gemm_8wave_256_tiles_exact(at, bt, M, N, K, ring, cuda_dev, monkeypatch):
    """The 8-wave 256 x 256 kernel (gemm_bf16_8w) in every operand layout:
    ragged M / N / K (partial tiles and a K that is not a multiple of the
    64-deep k-tile), a single k-tile, split-K (long K, few tiles), padded
    leading dimensions, alpha / beta / bias pair; both forms (two 64-deep
    buffers: ASR_GEMM_8R=0, and the 32-deep five-slot ring, the default).  Exact on small
    integers."""
    monkeypatch.setenv('ASR_GEMM_8W', '1')
    monkeypatch.setenv('ASR_GEMM_8R', ring)
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(M * 7 + N * 3 + K + 11 * at + 13 * bt)
        pa, pb = 8, 16
        sa = _store(rng, K if at else M, M if at else K, (M if at else K) + pa)
        sb = _store(rng, K if bt else N, N if bt else K, (N if bt else K) + pb)
        A = (sa[:, :M].T if at else sa[:, :K]).astype(np.float64)
        Bm = (sb[:, :N].T if bt else sb[:, :K]).astype(np.float64)
        c0 = rng.randint(-4, 5, (M, N)).astype(np.float32)
        b1 = rng.randint(-8, 9, N).astype(np.float32)
        b2 = rng.randint(-8, 9, N).astype(np.float32)
        ad = torch.from_numpy(sa).to(torch.bfloat16).to(cuda_dev)
        bd = torch.from_numpy(sb).to(torch.bfloat16).to(cuda_dev)
        C = torch.from_numpy(c0).to(cuda_dev)
        p = ops.gemm_problem(ops.operand(ad, at, ops.rowmap(sa.shape[1])),
                             ops.operand(bd, bt, ops.rowmap(sb.shape[1])), C, ops.rowmap(N),
                             M, N, K, alpha=2.0, beta=1.0,
                             bias=torch.from_numpy(b1).to(cuda_dev),
                             bias2=torch.from_numpy(b2).to(cuda_dev))
        ops.run_gemm([p], cuda_dev)
        torch.cuda.synchronize()
        ref = 2.0 * (A @ Bm.T) + c0 + b1 + b2
        np.testing.assert_array_equal(C.cpu().numpy(), ref)
    finally:
        ops.set_compute_dtype('fp32')


def _mapped_rows(store, rpb, stride_b, stride_t, t_mul, t_add, t_limit, nrows, ncols):
    """Rows 0..nrows-1 of an operand read through asr_rowmap_t (zero where the
    mapped frame falls outside [0, t_limit))."""
    out = np.zeros((nrows, ncols), np.float64)
    flat = store.reshape(-1)
    for r in range(nrows):
        b, t = (r // rpb, r % rpb) if rpb > 0 else (0, r)
        tp = t * t_mul + t_add
        if 0 <= tp < (t_limit if t_limit > 0 else 1 << 30):
            off = b * stride_b + tp * stride_t
            out[r] = flat[off:off + ncols]
    return out


@pytest.mark.parametrize('stagef', ['1', '0'])
def test_fast_kernel_mapped_k_rows_exact(stagef, cuda_dev, monkeypatch):
    """The 128 x 128 kernel (N < 256) on weight-gradient-shaped products whose
    K rows come through a grouped row map (utterance groups, frame stride 2,
    offset 1, frame limit: the pyramidal-subsampling and shifted-h operands),
    with the division-free staging (StageF) and without it."""
    monkeypatch.setenv('ASR_GEMM_STAGEF', stagef)
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(7)
        M, Nn = 320, 200
        rpb, T, t_mul, t_add, t_limit = 37, 80, 2, 1, 60
        nb = 9
        K = nb * rpb
        lda, ldb = M + 8, Nn + 8
        sa = _store(rng, nb * T, M, lda)
        sb = _store(rng, nb * T, Nn, ldb)
        A = _mapped_rows(sa, rpb, T * lda, lda, t_mul, t_add, t_limit, K, M)
        Bm = _mapped_rows(sb, rpb, T * ldb, ldb, t_mul, t_add, t_limit, K, Nn)
        ad = torch.from_numpy(sa).to(torch.bfloat16).to(cuda_dev)
        bd = torch.from_numpy(sb).to(torch.bfloat16).to(cuda_dev)
        C = torch.zeros(M, Nn, device=cuda_dev)
        p = ops.gemm_problem(
            ops.operand(ad, 1, ops.rowmap(lda, T * lda, rpb, t_mul, t_add, t_limit)),
            ops.operand(bd, 1, ops.rowmap(ldb, T * ldb, rpb, t_mul, t_add, t_limit)),
            C, ops.rowmap(Nn), M, Nn, K)
        ops.run_gemm([p], cuda_dev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C.cpu().numpy(), A.T @ Bm)
        # R-mode operand with mapped rows (M rows through the same kind of map)
        Mr = nb * rpb
        A2 = _mapped_rows(sa, rpb, T * lda, lda, t_mul, t_add, t_limit, Mr, 64)
        sb2 = _store(rng, Nn, 64, 64)
        bd2 = torch.from_numpy(sb2).to(torch.bfloat16).to(cuda_dev)
        C2 = torch.zeros(Mr, Nn, device=cuda_dev)
        p2 = ops.gemm_problem(
            ops.operand(ad, 0, ops.rowmap(lda, T * lda, rpb, t_mul, t_add, t_limit)),
            ops.operand(bd2, 0, ops.rowmap(64)), C2, ops.rowmap(Nn), Mr, Nn, 64)
        ops.run_gemm([p2], cuda_dev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C2.cpu().numpy(), A2 @ sb2.astype(np.float64).T)
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('M,N,K,dtype,kind', [
    (2048, 1024, 512, 'bf16', '8-wave'),        # both extents >= 256: 256 x 256 kernel
    (2048, 200, 512, 'bf16', '128x128'),        # N < 256: 128 x 128 fast kernel
    (192, 160, 32768, 'bf16', 'split-K'),       # few tiles, long K: slabs + splitk_reduce
    (600, 300, 96, 'fp32', 'generic'),          # f32 operands, parity mode
])
def test_dropout_epilogue_matches_separate_pass(M, N, K, dtype, kind, cuda_dev):
    """Dropout's backward fused into the producing GEMM (asr_gemm_t.drop_p):
    the result equals the product written plainly and then masked by
    asr_dropout over the same tensor (same seed), bit for bit, on every kernel
    family, including a row-mapped (scattered) C inside a larger tensor."""
    from pytorch_end2end_speech_recognition_amd import _native as NL
    ops = _ops()
    ops.set_compute_dtype(dtype)
    try:
        rng = np.random.RandomState(M + N + K)
        tdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
        a = torch.from_numpy(rng.randint(-3, 4, (M, K)).astype(np.float32)).to(tdt).to(cuda_dev)
        b = torch.from_numpy(rng.randint(-3, 4, (N, K)).astype(np.float32)).to(tdt).to(cuda_dev)
        # C rows scattered as rows 2t+1 of a [2M, N] tensor ('drop' subsampling's layout)
        cmap = ops.rowmap(N, stride_b=2 * M * N, rows_per_b=M, t_mul=2, t_add=1, t_limit=2 * M)
        p, seed = 0.3, 987654321
        plain = torch.zeros(2 * M, N, device=cuda_dev)
        fused = torch.zeros(2 * M, N, device=cuda_dev)
        for c, drop in ((plain, None), (fused, (p, seed))):
            prob = ops.gemm_problem(ops.operand(a, 0, ops.rowmap(K)), ops.operand(b, 0, ops.rowmap(K)),
                                    c, cmap, M, N, K, drop=drop)
            ops.run_gemm([prob], cuda_dev)
        ref = torch.empty_like(plain)
        NL.call('asr_dropout', NL.ptr(plain), NL.ptr(ref), plain.numel(), p, seed,
                NL.stream_handle(cuda_dev))
        torch.cuda.synchronize()
        assert torch.equal(fused, ref), kind
        assert (fused[1::2] == 0).float().mean().item() > 0.2      # the mask is applied
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('M,N,K,atrans,btrans', [(5000, 64, 576, 0, 0), (4391, 40, 200, 0, 0),
                                                 (6000, 64, 1152, 1, 0), (4096, 17, 72, 1, 0),
                                                 (576, 64, 70000, 1, 1), (4100, 48, 264, 0, 1)])
def test_n64_kernel_exact(M, N, K, atrans, btrans, cuda_dev, monkeypatch):
    """The 256 x 64 kernel (products with N <= 64, B stored [N][K]: the
    64-channel VGG convolutions) on small-integer bf16 operands, exact in f32:
    both A layouts, N below 64, K not a multiple of the 64-deep k-tile, M not a
    multiple of the 256-row tile, bias pair and beta; equal to the 128 x 128
    kernel's result (ASR_GEMM_N64=0) bit for bit."""
    ops = _ops()
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(M + N + K)
        a_np = rng.randint(-3, 4, (M, K)).astype(np.float32)
        b_np = rng.randint(-3, 4, (N, K)).astype(np.float32)
        bias = torch.from_numpy(rng.randint(-2, 3, N).astype(np.float32)).to(cuda_dev)
        c0 = rng.randint(-2, 3, (M, N)).astype(np.float32)
        a_st = a_np.T.copy() if atrans else a_np
        b_st = b_np.T.copy() if btrans else b_np
        a = torch.from_numpy(a_st).to(torch.bfloat16).to(cuda_dev)
        b = torch.from_numpy(b_st).to(torch.bfloat16).to(cuda_dev)
        from pytorch_end2end_speech_recognition_amd import _native as NL
        outs = []
        for n64 in ('1', '0'):
            monkeypatch.setenv('ASR_GEMM_N64', n64)
            c = torch.from_numpy(c0).to(cuda_dev)
            p = ops.gemm_problem(ops.operand(a, atrans, ops.rowmap(M if atrans else K)),
                                 ops.operand(b, btrans, ops.rowmap(N if btrans else K)), c,
                                 ops.rowmap(N), M, N, K, bias=bias, beta=1.0)
            NL.call('asr_gemm_set_n64_kmode', 1)
            try:
                ops.run_gemm([p], cuda_dev)
            finally:
                NL.call('asr_gemm_set_n64_kmode', 0)
            torch.cuda.synchronize()
            outs.append(c.cpu().numpy())
        ref = a_np.astype(np.float64) @ b_np.astype(np.float64).T + bias.cpu().numpy() + c0
        np.testing.assert_array_equal(outs[0], ref)
        np.testing.assert_array_equal(outs[0], outs[1])
    finally:
        ops.set_compute_dtype('fp32')


def _f32_run(ops, dev, probs_fn, fast, monkeypatch):
    monkeypatch.setenv('ASR_GEMM_F32FAST', fast)
    probs, outs = probs_fn()
    ops.run_gemm(probs, dev)
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in outs]


@pytest.mark.parametrize('at,bt', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K', [(600, 389, 1032), (128, 128, 32), (300, 260, 203),
                                    (192, 160, 32768), (1030, 777, 1001), (5000, 64, 576),
                                    (4391, 40, 198), (64, 576, 20000), (37, 300, 401)])
@pytest.mark.parametrize('stages', ['2', '3'])
def test_f32_fast_kernel_exact(at, bt, M, N, K, stages, cuda_dev, monkeypatch):
    """gemm_f32_fast (fp32 mode: LDS-DMA staging, v_mfma_f32_16x16x4_f32) in
    every operand layout and all three tile shapes (128 x 128; 256 x 64 for
    N <= 64; 64 x 256 for M <= 64): ragged M / N, K not a multiple of the
    32-deep k-tile and not of 4 (the straddling chunk zero-filled in LDS), a
    single k-tile, split-K (few tiles, long K), padded leading dimensions
    (16-B aligned rows), alpha / beta / bias pair.  Small integers: exact, so
    equal to float64 bit for bit (and to gemm_kernel<false>,
    ASR_GEMM_F32FAST=0).  stages: the double buffer and the three-stage ring."""
    monkeypatch.setenv('ASR_GEMM_F32_STAGES', stages)
    ops = _ops()
    ops.set_compute_dtype('fp32')
    rng = np.random.RandomState(M * 5 + N * 3 + K + 17 * at + 19 * bt)

    def ld(cols, pad):
        return (cols + 3) // 4 * 4 + pad
    sa = _store(rng, K if at else M, M if at else K, ld(M if at else K, 4))
    sb = _store(rng, K if bt else N, N if bt else K, ld(N if bt else K, 12))
    # garbage past each row's end (inside the padding): must not reach C
    sa[:, (M if at else K):] = 1e30
    sb[:, (N if bt else K):] = -1e30
    A = (sa[:, :M].T if at else sa[:, :K]).astype(np.float64)
    Bm = (sb[:, :N].T if bt else sb[:, :K]).astype(np.float64)
    c0 = rng.randint(-4, 5, (M, N)).astype(np.float32)
    b1 = rng.randint(-8, 9, N).astype(np.float32)
    b2 = rng.randint(-8, 9, N).astype(np.float32)
    ad, bd = torch.from_numpy(sa).to(cuda_dev), torch.from_numpy(sb).to(cuda_dev)
    bias, bias2 = torch.from_numpy(b1).to(cuda_dev), torch.from_numpy(b2).to(cuda_dev)

    def probs():
        C = torch.from_numpy(c0).to(cuda_dev)
        return [ops.gemm_problem(ops.operand(ad, at, ops.rowmap(sa.shape[1])),
                                 ops.operand(bd, bt, ops.rowmap(sb.shape[1])), C, ops.rowmap(N),
                                 M, N, K, alpha=2.0, beta=1.0, bias=bias, bias2=bias2)], [C]
    got = _f32_run(ops, cuda_dev, probs, '1', monkeypatch)[0]
    ref = 2.0 * (A @ Bm.T) + c0 + b1 + b2
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got, _f32_run(ops, cuda_dev, probs, '0', monkeypatch)[0])


def test_f32_fast_kernel_mapped_rows_exact(cuda_dev, monkeypatch):
    """gemm_f32_fast with row-mapped operands (utterance groups, frame stride
    2, offset 1, frame limit) in K mode (weight-gradient shape) and R mode, and
    two problems in one launch: exact against float64."""
    ops = _ops()
    ops.set_compute_dtype('fp32')
    rng = np.random.RandomState(71)
    M, Nn = 320, 200
    rpb, T, t_mul, t_add, t_limit = 37, 80, 2, 1, 60
    nb = 9
    K = nb * rpb
    lda, ldb = M + 4, Nn + 4
    sa = _store(rng, nb * T, M, lda)
    sb = _store(rng, nb * T, Nn, ldb)
    A = _mapped_rows(sa, rpb, T * lda, lda, t_mul, t_add, t_limit, K, M)
    Bm = _mapped_rows(sb, rpb, T * ldb, ldb, t_mul, t_add, t_limit, K, Nn)
    ad, bd = torch.from_numpy(sa).to(cuda_dev), torch.from_numpy(sb).to(cuda_dev)
    Mr = nb * rpb
    A2 = _mapped_rows(sa, rpb, T * lda, lda, t_mul, t_add, t_limit, Mr, 64)
    sb2 = _store(rng, Nn, 64, 64)
    bd2 = torch.from_numpy(sb2).to(cuda_dev)

    def probs():
        C = torch.zeros(M, Nn, device=cuda_dev)
        C2 = torch.zeros(Mr, Nn, device=cuda_dev)
        return [ops.gemm_problem(
            ops.operand(ad, 1, ops.rowmap(lda, T * lda, rpb, t_mul, t_add, t_limit)),
            ops.operand(bd, 1, ops.rowmap(ldb, T * ldb, rpb, t_mul, t_add, t_limit)),
            C, ops.rowmap(Nn), M, Nn, K),
            ops.gemm_problem(
            ops.operand(ad, 0, ops.rowmap(lda, T * lda, rpb, t_mul, t_add, t_limit)),
            ops.operand(bd2, 0, ops.rowmap(64)), C2, ops.rowmap(Nn), Mr, Nn, 64)], [C, C2]
    # one launch per layout pair (the fast kernel takes one pair per launch)
    p, o = probs()
    monkeypatch.setenv('ASR_GEMM_F32FAST', '1')
    ops.run_gemm(p[:1], cuda_dev)
    ops.run_gemm(p[1:], cuda_dev)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(o[0].cpu().numpy(), A.T @ Bm)
    np.testing.assert_array_equal(o[1].cpu().numpy(), A2 @ sb2.astype(np.float64).T)


@pytest.mark.parametrize('ci,co,F,sign', [(64, 64, 20, 1), (64, 128, 12, -1), (16, 32, 9, 1)])
def test_f32_fast_kernel_taps_match_generic(ci, co, F, sign, cuda_dev, monkeypatch):
    """3x3 convolutions as tap-addressed products in fp32 mode (forward /
    input-gradient geometry: taps on A's k; weight gradient: taps on B's
    columns in K mode): gemm_f32_fast bitwise equal to gemm_kernel<false>
    (small integers: both exact)."""
    ops = _ops()
    ops.set_compute_dtype('fp32')
    rng = np.random.RandomState(ci + co + F)
    B, T = 3, 11
    P = B * (T + 2) * (F + 2)
    x = torch.from_numpy(rng.randint(-3, 4, (P, ci)).astype(np.float32)).to(cuda_dev)
    w = torch.from_numpy(rng.randint(-3, 4, (co, 9 * ci)).astype(np.float32)).to(cuda_dev)
    dz = torch.from_numpy(rng.randint(-3, 4, (P, co)).astype(np.float32)).to(cuda_dev)

    def fwd():
        out = torch.zeros(P, co, device=cuda_dev)
        return [ops.gemm_problem(ops._tap_operand(x, 0, ci, ci, F + 2, sign),
                                 ops.operand(w, 0, ops.rowmap(9 * ci)), out, ops.rowmap(co),
                                 P, co, 9 * ci)], [out]

    def wgrad():
        packed = torch.zeros(co, 9 * ci, device=cuda_dev)
        return [ops.gemm_problem(ops.operand(dz, 1, ops.rowmap(co)),
                                 ops._tap_operand(x, 1, ci, ci, F + 2, 1), packed,
                                 ops.rowmap(9 * ci), co, 9 * ci, P)], [packed]
    for fn in (fwd, wgrad):
        a = _f32_run(ops, cuda_dev, fn, '1', monkeypatch)[0]
        b = _f32_run(ops, cuda_dev, fn, '0', monkeypatch)[0]
        assert np.abs(b).max() > 0
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('precision,M,N', [('bf16', 700, 10001), ('bf16', 300, 200),
                                           ('fp32', 700, 10001), ('fp32', 50, 1000),
                                           ('fp32', 4000, 60)])
def test_gemm_row_lse_partials(precision, M, N, cuda_dev):
    """asr_gemm_lse_ws: the epilogue's per-row (max, sum exp) over every
    64-column slab of the written C (with the bias) -- the 8-wave / 128 x 128
    bf16 kernels and the f32 fast kernel's three tile shapes: each pair equals
    the slab's max and sum of exp(C - max) computed from the returned C, and
    their fold equals logsumexp of the row (1e-6)."""
    ops = _ops()
    ops.set_compute_dtype(precision)
    try:
        rng = np.random.RandomState(M + N)
        K = 256
        x = torch.from_numpy(rng.randn(M, K).astype(np.float32)).to(cuda_dev)
        w = torch.from_numpy((rng.randn(N, K) * 0.2).astype(np.float32)).to(cuda_dev)
        b = torch.from_numpy(rng.randn(N).astype(np.float32)).to(cuda_dev)
        nq = (N + 63) // 64
        lse = torch.full((nq, M, 2), float('nan'), device=cuda_dev)
        y, _, _, _ = ops._linear_forward(x, w, b, None, lse=lse)
        torch.cuda.synchronize()
        c = y.double().cpu().numpy()
        part = lse.double().cpu().numpy()
        pad = np.full((M, nq * 64), -np.inf)
        pad[:, :N] = c
        slabs = pad.reshape(M, nq, 64)
        mx = slabs.max(axis=2).T
        np.testing.assert_allclose(part[:, :, 0], mx, rtol=1e-6, atol=1e-6)
        sm = np.exp(slabs - mx.T[:, :, None]).sum(axis=2).T
        np.testing.assert_allclose(part[:, :, 1], sm, rtol=2e-6)
        m = part[:, :, 0].max(axis=0)
        tot = (part[:, :, 1] * np.exp(part[:, :, 0] - m)).sum(axis=0)
        ref = np.log(np.exp(c - c.max(axis=1, keepdims=True)).sum(axis=1)) + c.max(axis=1)
        np.testing.assert_allclose(m + np.log(tot), ref, rtol=1e-6)
    finally:
        ops.set_compute_dtype('fp32')


def test_f32_fast_kernel_batch_permutation_matches_generic(cuda_dev, monkeypatch):
    """gemm_f32_fast with the encoder's batch permutation in the row map (the
    first BLSTM layer of a length-sorted batch): an R-mode operand (rows
    permuted once per slot) and a K-mode operand (the permuted utterance
    re-read at every utterance crossing, frame stride 2 / offset 1 / limit),
    bitwise equal to gemm_kernel<false> on small integers."""
    ops = _ops()
    ops.set_compute_dtype('fp32')
    rng = np.random.RandomState(5)
    nb, T, rpb, D, Nn = 7, 90, 45, 132, 200
    perm = torch.from_numpy(rng.permutation(nb).astype(np.int32)).to(cuda_dev)
    x = torch.from_numpy(rng.randint(-3, 4, (nb * T, D)).astype(np.float32)).to(cuda_dev)
    w = torch.from_numpy(rng.randint(-3, 4, (Nn, D)).astype(np.float32)).to(cuda_dev)
    g = torch.from_numpy(rng.randint(-3, 4, (nb * rpb, Nn)).astype(np.float32)).to(cuda_dev)
    M = nb * rpb

    def fwd():
        c = torch.zeros(M, Nn, device=cuda_dev)
        return [ops.gemm_problem(ops.operand(x, 0, ops.rowmap(D, T * D, rpb, 2, 1, T, perm=perm)),
                                 ops.operand(w, 0, ops.rowmap(D)), c, ops.rowmap(Nn), M, Nn, D)], [c]

    def wgrad():
        c = torch.zeros(Nn, D, device=cuda_dev)
        return [ops.gemm_problem(ops.operand(g, 1, ops.rowmap(Nn)),
                                 ops.operand(x, 1, ops.rowmap(D, T * D, rpb, 2, 1, T, perm=perm)),
                                 c, ops.rowmap(D), Nn, D, M)], [c]
    for fn in (fwd, wgrad):
        a = _f32_run(ops, cuda_dev, fn, '1', monkeypatch)[0]
        b = _f32_run(ops, cuda_dev, fn, '0', monkeypatch)[0]
        assert np.abs(b).max() > 0
        np.testing.assert_array_equal(a, b)
