"""Forward / input-gradient GEMM kernel (sae_gemm_nt) with its fused FF-block epilogues, and the
FF block built on it (ff.py:8-34: Dense -> nn.gelu (tanh) -> Dense).

References: float64 products of the same bf16 inputs; GELU / GELU' from torch's fp32
``gelu(approximate="tanh")`` (= Flax ``nn.gelu`` default).  Outputs are bf16, so the bar is bf16
rounding (2e-2 of the largest magnitude, the north_star bf16 tolerance); the pre-activation h and
the weight casts are compared bit for bit where the math is exact."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N)
    (25216, 384, 1536),   # DeiT-S FF Dense_0 forward / Dense_1 input gradient
    (25216, 1536, 384),   # DeiT-S FF Dense_1 forward / Dense_0 input gradient
    (25216, 384, 1152),   # DeiT-S QKV projection
    (197, 768, 1000),     # ragged tokens, head-like N (not a tile multiple)
    (1000, 64, 40),       # one K stage, N below one tile
    (130, 128, 136),
    (4000, 192, 256),     # odd stage count (the epilogue reuses the last stage's LDS buffer)
]


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _inputs(dev, M, K, N, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    bt = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    return a, bt, bias


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_nt_plain(dev, M, K, N, bias):
    import sae_vision_amd.ops as ops
    a, bt, b = _inputs(dev, M, K, N, M + K + N)
    c = ops.gemm_nt(a, bt, b if bias else None)
    ref = a.double() @ bt.double().t()
    if bias:
        ref = ref + b.double()
    assert c.shape == (M, N) and c.dtype == torch.bfloat16
    assert _rel(c, ref) <= 1e-2


# (6000, 768, 3072): the ViT-B FF shape on the 256-token tile (>= 512 tiles), ragged last tile
@pytest.mark.parametrize("M,K,N", [(25216, 384, 1536), (197, 768, 1000), (130, 128, 136), (6000, 768, 3072)])
def test_gemm_nt_gelu(dev, M, K, N):
    import sae_vision_amd.ops as ops
    a, bt, b = _inputs(dev, M, K, N, 11)
    y, h = ops.gemm_nt(a, bt, b, ops.EPI_GELU)
    ref_h = a.double() @ bt.double().t() + b.double()
    assert _rel(h, ref_h) <= 1e-2
    # gelu applied to the kernel's own bf16 pre-activation: only the final rounding differs
    ref_y = F.gelu(h.float(), approximate="tanh")
    assert _rel(y, ref_y) <= 1e-2
    assert float((y.float() - ref_y).abs().max()) <= 2 ** -7 * float(ref_y.abs().max())


# (6000, 768, 3072): the ViT-B FF shape on the 256-token tile (>= 512 tiles), ragged last tile
@pytest.mark.parametrize("M,K,N", [(25216, 384, 1536), (197, 768, 1000), (130, 128, 136), (6000, 768, 3072)])
def test_gemm_nt_dgelu(dev, M, K, N):
    import sae_vision_amd.ops as ops
    a, bt, _ = _inputs(dev, M, K, N, 12)
    g = torch.Generator(device=dev).manual_seed(13)
    h = (torch.randn(M, N, device=dev, generator=g) * 2).to(torch.bfloat16)
    dh = ops.gemm_nt(a, bt, None, ops.EPI_DGELU, aux=h)
    da = (a.double() @ bt.double().t()).to(torch.bfloat16).float()
    hf = h.float().requires_grad_(True)
    F.gelu(hf, approximate="tanh").backward(da)
    assert _rel(dh, hf.grad) <= 1e-2


def test_gemm_nt_strided_out(dev):
    """Row-strided a (a column slice of a wider buffer) and c written into a wider buffer."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(5)
    M, K, N = 777, 128, 64
    aw = torch.randn(M, K + 64, device=dev, generator=g).to(torch.bfloat16)
    a = aw[:, 64:]
    bt = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    cw = torch.zeros(M, N + 16, device=dev, dtype=torch.bfloat16)
    ops.gemm_nt(a, bt, out=cw[:, :N])
    assert _rel(cw[:, :N], a.double() @ bt.double().t()) <= 1e-2
    assert float(cw[:, N:].abs().max()) == 0.0


def test_gemm_nt_rejects(dev):
    import sae_vision_amd.ops as ops
    from sae_vision_amd._lib import SaeError
    a = torch.zeros(64, 100, device=dev, dtype=torch.bfloat16)     # K not a multiple of 8
    bt = torch.zeros(64, 100, device=dev, dtype=torch.bfloat16)
    with pytest.raises(SaeError):
        ops.gemm_nt(a, bt)
    a = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    bt = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    with pytest.raises((SaeError, ValueError)):                     # DGELU without aux
        ops.gemm_nt(a, bt, None, ops.EPI_DGELU)
    with pytest.raises(ValueError):                                 # out of the wrong dtype
        ops.gemm_nt(a, bt, out=torch.empty(64, 64, device=dev))


def test_gemm_nt_strided_out_gelu(dev):
    """A caller-provided out with a row stride larger than N, GELU epilogue: c and the
    pre-activation c2 (allocated with out's row stride) both hold the right values."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(4)
    M, N, K = 200, 96, 128
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    big = torch.full((M, 160), 7.0, device=dev, dtype=torch.bfloat16)
    out = big[:, 16:16 + N]
    c, h = ops.gemm_nt(a, bt, None, ops.EPI_GELU, out=out)
    ref = (a.float() @ bt.float().t()).to(torch.bfloat16)
    assert c.data_ptr() == out.data_ptr() and h.stride(0) == out.stride(0)
    assert float((h.float() - ref.float()).abs().max()) <= 2e-2 * float(ref.float().abs().max())
    gl = torch.nn.functional.gelu(h.float(), approximate="tanh")
    assert float((c.float() - gl).abs().max()) <= 2e-2 * float(gl.abs().max())
    assert torch.all(big[:, :16] == 7.0) and torch.all(big[:, 16 + N:] == 7.0)


def test_weight_cast_exact(dev):
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(9)
    for K, N in ((384, 1536), (1536, 384), (100, 72), (3, 5)):
        w = torch.randn(K, N, device=dev, generator=g)
        w16, wt16 = ops.weight_cast(w)
        assert torch.equal(w16, w.to(torch.bfloat16))
        assert torch.equal(wt16, w.t().contiguous().to(torch.bfloat16))


@pytest.mark.parametrize("M,C", [(2 * 197, 384), (3 * 577, 768)])
def test_ff_block_fwd_bwd(dev, M, C):
    """ops.ff_block against the unfused bf16 path (library GEMMs + torch GELU) and an fp32 one."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(M)
    x = torch.randn(M, C, device=dev, generator=g)
    w0 = torch.randn(C, 4 * C, device=dev, generator=g) / C ** 0.5
    b0 = torch.randn(4 * C, device=dev, generator=g) * 0.1
    w1 = torch.randn(4 * C, C, device=dev, generator=g) / (4 * C) ** 0.5
    b1 = torch.randn(C, device=dev, generator=g) * 0.1
    dy = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)

    leaves = [t.clone().requires_grad_(True) for t in (x, w0, b0, w1, b1)]
    y = ops.ff_block(leaves[0].to(torch.bfloat16), *leaves[1:])
    y.backward(dy)

    ref = [t.clone().double().requires_grad_(True) for t in (x, w0, b0, w1, b1)]
    xb = ref[0].to(torch.bfloat16).double()
    hr = (xb @ ref[1].to(torch.bfloat16).double() + ref[2])
    yr = F.gelu(hr, approximate="tanh") @ ref[3].to(torch.bfloat16).double() + ref[4]
    yr.backward(dy.double())
    assert _rel(y, yr) <= 2e-2
    for got, want, name in zip(leaves, ref, ("x", "w0", "b0", "w1", "b1")):
        assert _rel(got.grad, want.grad) <= 2e-2, name


def test_ff_block_deterministic(dev):
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(1)
    M, C = 4 * 197, 384
    x = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    w0 = torch.randn(C, 4 * C, device=dev, generator=g) / C ** 0.5
    w1 = torch.randn(4 * C, C, device=dev, generator=g) / (4 * C) ** 0.5
    b0, b1 = torch.zeros(4 * C, device=dev), torch.zeros(C, device=dev)
    dy = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        ps = [t.clone().requires_grad_(True) for t in (w0, b0, w1, b1)]
        xx = x.clone().requires_grad_(True)
        y = ops.ff_block(xx, *ps)
        y.backward(dy)
        outs.append([y.detach(), xx.grad] + [p.grad for p in ps])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_cast_weights_multi_exact(dev):
    """sae_weight_cast_multi: column-stacked groups (queries / keys / values kernels into one
    [C, 3HD] projection) in one launch, bit-equal to torch's casts; cache lookups and clearing."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(21)
    C, H, D = 384, 6, 64
    wq, wk, wv = (torch.randn(C, H, D, device=dev, generator=g) for _ in range(3))
    wo = torch.randn(H, D, C, device=dev, generator=g)
    ws = [[w.reshape(C, H * D) for w in (wq, wk, wv)], [wo.reshape(H * D, C)]]
    ws += [[torch.randn(96, 40, device=dev, generator=g)] for _ in range(60)]   # > one launch of items
    ws += [[torch.randn(30, 37, device=dev, generator=g)], [torch.randn(130, 68, device=dev, generator=g)]]
    # (30 x 37: the element-wise 32 x 32 path; 130 x 68: 64 x 64 vector tiles with ragged edges)
    ops.cast_weights(ws)
    try:
        w16, wt16 = ops._cast_lookup(ws[0])
        ref = torch.stack((wq, wk, wv), dim=1).reshape(C, 3 * H * D)
        assert torch.equal(w16, ref.to(torch.bfloat16))
        assert torch.equal(wt16, ref.t().contiguous().to(torch.bfloat16))
        for grp in ws[1:]:
            a, b = ops._cast_lookup(grp)
            assert torch.equal(a, grp[0].to(torch.bfloat16)) and torch.equal(b, grp[0].t().to(torch.bfloat16))
        wq.add_(1.0)                                   # in-place update: the entry is stale
        assert ops._cast_lookup(ws[0]) is None
    finally:
        ops.clear_weight_cache()
    assert ops._cast_lookup(ws[1]) is None


@pytest.mark.parametrize("K", [64, 192, 320])
def test_gemm_nt_odd_stages_repeatable(dev, K):
    """Odd stage counts: the last stage is computed from LDS buffer 0, which the epilogue then
    reuses as scratch -- every rerun must give the same bits (a missing barrier shows up as
    run-to-run differences) and match the reference."""
    import sae_vision_amd.ops as ops
    a, bt, b = _inputs(dev, 25216, K, 1536, K)
    ref = a.double() @ bt.double().t() + b.double()
    first = ops.gemm_nt(a, bt, b)
    assert _rel(first, ref) <= 1e-2
    for _ in range(20):
        assert torch.equal(ops.gemm_nt(a, bt, b), first)


# gemm8.h (the persistent 256-row kernel sae_gemm_nt routes the 384-feature outputs and the wide
# K = 768 forwards to): one tile per workgroup (25216 x 384: 198 tiles), several per workgroup
# (70000 x 384: 548 tiles; 18464 x 2304: 1,152 tiles), ragged last row block (5000, 70000, 18464)
G8_SHAPES = [(25216, 384, 384), (25216, 1152, 384), (25216, 1536, 384), (5000, 384, 384), (70000, 384, 384),
             (18464, 768, 2304),
             # gemm8x (ping-pong wave groups, 256 x 256 tiles): the ViT-B 768-feature outputs
             (18464, 3072, 768), (18464, 768, 768), (5000, 2304, 768)]


@pytest.mark.parametrize("M,K,N", G8_SHAPES)
def test_gemm8_plain_repeatable(dev, M, K, N):
    """gemm8 / gemm8x: against the float64 product (bias in the first K-tile's MFMA C operand) and bit-equal
    over reruns (a stage read before its LDS-DMA landed shows up as run-to-run differences)."""
    import sae_vision_amd.ops as ops
    a, bt, b = _inputs(dev, M, K, N, 3 * M + K)
    ref = a.double() @ bt.double().t() + b.double()
    first = ops.gemm_nt(a, bt, b)
    assert _rel(first, ref) <= 1e-2
    for _ in range(5):
        assert torch.equal(ops.gemm_nt(a, bt, b), first)
    assert _rel(ops.gemm_nt(a, bt), a.double() @ bt.double().t()) <= 1e-2   # no bias


@pytest.mark.parametrize("M,K,N", [(18464, 768, 3072), (3000, 768, 1152)])
def test_gemm8_gelu(dev, M, K, N):
    import sae_vision_amd.ops as ops
    a, bt, b = _inputs(dev, M, K, N, 17)
    y, h = ops.gemm_nt(a, bt, b, ops.EPI_GELU)
    assert _rel(h, a.double() @ bt.double().t() + b.double()) <= 1e-2
    ref_y = F.gelu(h.float(), approximate="tanh")
    assert float((y.float() - ref_y).abs().max()) <= 2 ** -7 * float(ref_y.abs().max())


def test_gemm8_strided(dev):
    """gemm8 with a row-strided a and c written into a wider buffer (columns outside untouched)."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(6)
    M, K, N = 9000, 384, 384
    aw = torch.randn(M, K + 64, device=dev, generator=g).to(torch.bfloat16)
    a = aw[:, 64:]
    bt = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    cw = torch.full((M, N + 64), 3.0, device=dev, dtype=torch.bfloat16)
    ops.gemm_nt(a, bt, out=cw[:, 32:32 + N])
    assert _rel(cw[:, 32:32 + N], a.double() @ bt.double().t()) <= 1e-2
    assert torch.all(cw[:, :32] == 3.0) and torch.all(cw[:, 32 + N:] == 3.0)


# Round 5 routing (capi.hip g8x_route / g8_route, sae_gemm_nt_route): K not a multiple of 64 on the
# 128-row kernel's K-tail instances (CaiT-XXS/XS 288, CvT 368, TNT inner 24 / 40, their FF widths,
# the classifier head's K = 1000 input gradient), and the ViT-L / CvT-W24 1024 / 4096 widths on
# gemm8x.  Each case asserts which kernel the C ABI picked, so the test exercises that kernel.
ROUTE_SHAPES = [  # (M, K, N, epilogue, expected route)
    (6304, 288, 864, 0, 2), (6304, 864, 288, 0, 2), (6304, 288, 1152, 1, 2), (6304, 288, 1152, 2, 2),
    (5000, 368, 1104, 0, 2), (5000, 1472, 368, 0, 1), (3136, 40, 120, 0, 2), (3136, 24, 96, 1, 2),
    (3136, 96, 24, 0, 2), (128, 1000, 384, 0, 2), (197, 40, 40, 2, 2),
    (18464, 1024, 1024, 0, 4), (18464, 4096, 1024, 0, 4), (9000, 1024, 4096, 1, 4), (9000, 1024, 3072, 0, 3),
    (6304, 192, 576, 0, 1), (25216, 576, 576, 0, 3),
]


@pytest.mark.parametrize("M,K,N,epi,route", ROUTE_SHAPES)
def test_gemm_nt_generalised_routes(dev, M, K, N, epi, route):
    import sae_vision_amd.ops as ops
    from sae_vision_amd import _lib as L
    assert L.load().sae_gemm_nt_route(M, N, K, epi) == route
    a, bt, b = _inputs(dev, M, K, N, 7 * M + K + N)
    if epi == ops.EPI_GELU:
        y, h = ops.gemm_nt(a, bt, b, ops.EPI_GELU)
        assert _rel(h, a.double() @ bt.double().t() + b.double()) <= 1e-2
        ref_y = F.gelu(h.float(), approximate="tanh")
        assert float((y.float() - ref_y).abs().max()) <= 2 ** -7 * float(ref_y.abs().max())
    elif epi == ops.EPI_DGELU:
        g = torch.Generator(device=dev).manual_seed(5)
        h = (torch.randn(M, N, device=dev, generator=g) * 2).to(torch.bfloat16)
        dh = ops.gemm_nt(a, bt, None, ops.EPI_DGELU, aux=h)
        da = (a.double() @ bt.double().t()).to(torch.bfloat16).float()
        hf = h.float().requires_grad_(True)
        F.gelu(hf, approximate="tanh").backward(da)
        assert _rel(dh, hf.grad) <= 1e-2
    else:
        c = ops.gemm_nt(a, bt, b)
        assert _rel(c, a.double() @ bt.double().t() + b.double()) <= 1e-2
        assert torch.equal(ops.gemm_nt(a, bt, b), c)


def test_gemm_nt_ktail_rowstride(dev):
    """K-tail kernel reading a row-strided a whose row continues past K (the columns past K of the
    last stage must read as zero, not as the neighbouring data)."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(9)
    M, K, N = 3000, 40, 64
    aw = (torch.randn(M, K + 88, device=dev, generator=g) * 100).to(torch.bfloat16)
    a = aw[:, :K]
    bt = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    c = ops.gemm_nt(a, bt)
    assert _rel(c, a.double() @ bt.double().t()) <= 1e-2


@pytest.mark.parametrize("M,K,N", [(25216, 384, 1536), (197, 768, 1000), (6000, 768, 3072), (300, 368, 1472)])
def test_gemm_nt_gelu_grad_pair(dev, M, K, N):
    """The FF block's epilogue pair: EPI_GELU_GRAD returns gelu(h) bit-equal to EPI_GELU's and
    g = bf16(gelu'(h)) of the same bf16 pre-activation; EPI_MUL_AUX multiplies bf16(acc) by g."""
    import sae_vision_amd.ops as ops
    from sae_vision_amd import _lib as L
    lib = L.load()
    assert lib.sae_gemm_nt_route(M, N, K, ops.EPI_GELU_GRAD) == lib.sae_gemm_nt_route(M, N, K, ops.EPI_GELU)
    # the multiply epilogue may take gemm8 where GELU' does not (K > 384): any kernel, never NONE
    assert lib.sae_gemm_nt_route(M, N, K, ops.EPI_MUL_AUX) != 0
    a, bt, b = _inputs(dev, M, K, N, 21)
    y, g = ops.gemm_nt(a, bt, b, ops.EPI_GELU_GRAD)
    y_ref, h = ops.gemm_nt(a, bt, b, ops.EPI_GELU)
    assert torch.equal(y, y_ref)
    hf = h.float().requires_grad_(True)
    F.gelu(hf, approximate="tanh").sum().backward()
    gref = hf.grad
    assert float((g.float() - gref).abs().max()) <= 2 ** -8 * float(gref.abs().max()) + 1e-6
    # the input-gradient side: dY [M, N'] x W [N', N] -> dA [M, N] times g
    a2, bt2, _ = _inputs(dev, M, N, N, 22)
    dh = ops.gemm_nt(a2, bt2, None, ops.EPI_MUL_AUX, aux=g)
    da = (a2.double() @ bt2.double().t()).to(torch.bfloat16).float()
    assert _rel(dh, da * g.float()) <= 1e-2
    # and against the GELU' epilogue from h: the one extra bf16 rounding of gelu'
    dh_ref = ops.gemm_nt(a2, bt2, None, ops.EPI_DGELU, aux=h)
    assert _rel(dh, dh_ref.float()) <= 2e-2
