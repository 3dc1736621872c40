"""GPU: the MFMA GEMM engine (csrc/ops/mlp.hip) against fp32 PyTorch references.

Exact-integer operands (bf16-representable, fp32 sums exact) catch any fragment / layout / C-map
error bit-for-bit; random operands check the fused epilogue within bf16 tolerance."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from gsc_amd.ops.mlp import gemm  # noqa: E402


def _ints(*shape, lo=-3, hi=4, g=None):
    return torch.randint(lo, hi, shape, generator=g).float()


def _ref(a, b, layout):
    if layout == "nt":
        return a.float() @ b.float().t()
    if layout == "tn":
        return a.float().t() @ b.float()
    return a.float() @ b.float()


def _shapes(layout, M, N, K):
    if layout == "nt":
        return (M, K), (N, K)
    if layout == "tn":
        return (K, M), (K, N)
    return (M, K), (K, N)


@pytest.mark.parametrize("layout", ["nt", "tn", "nn"])
@pytest.mark.parametrize("tile", [0, 1, 2])
@pytest.mark.parametrize("MNK", [(256, 128, 64), (100, 70, 50), (33, 300, 130)])
def test_gemm_exact_integers(layout, tile, MNK):
    g = torch.Generator().manual_seed(hash((layout, tile, MNK)) % 1000)
    M, N, K = MNK
    sa, sb = _shapes(layout, M, N, K)
    a, b = _ints(*sa, g=g), _ints(*sb, g=g)
    # asymmetric operands (row/column swaps cannot cancel)
    a[0, :] += 1
    out = torch.full((M, N), float("nan"), device="cuda")
    gemm(a.cuda().bfloat16(), b.cuda().bfloat16(), layout, out32=out, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), _ref(a, b, layout))


@pytest.mark.parametrize("layout", ["nt", "tn", "nn"])
def test_gemm_strided_unaligned_fp32(layout):
    """Row views at odd column offsets (element-wise staging path) and fp32 operands."""
    g = torch.Generator().manual_seed(5)
    M, N, K = 96, 80, 72
    sa, sb = _shapes(layout, M, N, K)
    A = _ints(sa[0], sa[1] + 11, g=g)
    B = _ints(sb[0], sb[1] + 7, g=g)
    a, b = A[:, 3:3 + sa[1]], B[:, 5:5 + sb[1]]
    out = torch.zeros(M, N + 3, device="cuda")
    gemm(A.cuda().bfloat16()[:, 3:3 + sa[1]], B.cuda()[:, 5:5 + sb[1]], layout, out32=out[:, 1:1 + N])
    torch.cuda.synchronize()
    assert torch.equal(out[:, 1:1 + N].cpu(), _ref(a, b, layout))


def test_gemm_splitk_and_aug():
    """Weight-gradient shape: K = batch, split-K slabs, ones + topology one-hot virtual columns."""
    g = torch.Generator().manual_seed(7)
    K, M, N, T = 4000, 64, 22, 3
    a, b = _ints(K, M, g=g), _ints(K, N, g=g)
    topo = torch.randint(0, T, (K,), generator=g, dtype=torch.int32)
    out = torch.zeros(M, N + 1 + T, device="cuda")
    slabs = torch.empty(16 * M * (N + 1 + T), device="cuda")
    gemm(a.cuda().bfloat16(), b.cuda().bfloat16(), "tn", out32=out, splits=16, slabs=slabs, aug_t=T,
         aug_topo=topo.cuda())
    torch.cuda.synchronize()
    baug = torch.cat([b, torch.ones(K, 1), torch.nn.functional.one_hot(topo.long(), T).float()], 1)
    assert torch.equal(out.cpu(), a.t() @ baug)


def test_gemm_epilogue():
    torch.manual_seed(0)
    M, N, K, T = 300, 96, 40, 2
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.2
    bias = torch.randn(N, device="cuda")
    rowtab = torch.randn(T, N, device="cuda")
    topo = torch.randint(0, T, (M,), device="cuda", dtype=torch.int32)
    prev = torch.randn(M, N, device="cuda")
    gate = torch.randn(M, N, device="cuda").bfloat16()
    colmask = (torch.rand(T, N, device="cuda") > 0.3).float()
    out32 = prev.clone()
    out16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gemm(x.bfloat16(), w.bfloat16(), "nt", out32=out32, out16=out16, alpha=0.5, bias=bias, rowtab=rowtab,
         topo=topo, colmask=colmask, gate=gate, relu=True, clamp=(-1.0, 0.75), accumulate=True)
    ref = 0.5 * (x.bfloat16().float() @ w.bfloat16().float().t()) + bias + rowtab[topo.long()] + prev
    ref = ref * (gate.float() > 0)
    ref = ref.clamp_min(0) * colmask[topo.long()]
    ref = ref.clamp(-1.0, 0.75)
    torch.cuda.synchronize()
    assert torch.allclose(out32, ref, atol=1e-4, rtol=1e-4)
    assert torch.allclose(out16.float(), ref, atol=1e-2, rtol=1e-2)


def test_gemm_large_random_vs_fp32():
    """The learner's largest product ([25600, 256] x [256, 1728]) within bf16 tolerance of fp32."""
    torch.manual_seed(1)
    M, N, K = 25600, 1728, 256
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / 16
    out = torch.empty(M, N, device="cuda")
    gemm(x.bfloat16(), w.bfloat16(), "nt", out32=out)
    ref = x @ w.t()
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item()
    assert err < 0.05 * ref.abs().max().item(), err


@pytest.mark.parametrize("layout", ["nt", "tn"])
def test_gemm_row_indexed_operand(layout):
    """Row-indexed operands (replay-ring rows read in place): exactly the GEMM of the gathered rows --
    nt with A rows indexed (the critic's action projection, split-K) and tn with B rows indexed (its
    weight gradient, K = batch)."""
    g = torch.Generator().manual_seed(7)
    cap, A, B, c1 = 300, 1000, 130, 64
    ring = _ints(cap, 1008, g=g).cuda().bfloat16()        # rows padded to 8 columns
    rows = torch.randint(0, cap, (B,), generator=g).int().cuda()
    gathered = ring[rows.long()][:, :A].contiguous()
    slabs = torch.empty(1 << 22, device="cuda")
    if layout == "nt":
        w = _ints(c1, A, g=g).cuda().bfloat16()
        want = torch.empty(B, c1, device="cuda")
        got = torch.empty(B, c1, device="cuda")
        gemm(gathered, w, "nt", out32=want, splits=4, slabs=slabs)
        gemm(ring[:, :A], w, "nt", out32=got, splits=4, slabs=slabs, a_rows=rows)
        assert torch.equal(got, want)
        torch.testing.assert_close(got, gathered.float() @ w.float().t())
    else:
        dh = _ints(B, c1, g=g).cuda().bfloat16()
        want = torch.empty(c1, A, device="cuda")
        got = torch.empty(c1, A, device="cuda")
        gemm(dh, gathered, "tn", out32=want)
        gemm(dh, ring[:, :A], "tn", out32=got, b_rows=rows)
        assert torch.equal(got, want)
        torch.testing.assert_close(got, dh.float().t() @ gathered.float())
