"""bf16 MFMA GEMM vs a plain torch fp32 reference of the same op.
Tolerance: inputs are bf16 (exact in fp32), accumulation fp32 -> the only
differences are fp32 summation order (rtol 1e-5 scale) and the bf16 rounding
of bf16 outputs (rel 2^-8)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    import dexterous_rl_manipulation_amd  # noqa: F401
    from dexterous_rl_manipulation_amd import _native
    return _native


def gemm(N, A, Bt, *, bias=None, bias_stride=1, act=0, gate=None, out_f32=True, out_rm=False, out_fm=False,
         splits=1):
    M, K = A.shape
    Nn = Bt.shape[0]
    dev = A.device
    Cf = torch.zeros(M, Nn, dtype=torch.float32, device=dev) if out_f32 else None
    Crm = torch.zeros(M, Nn, dtype=torch.bfloat16, device=dev) if out_rm else None
    Cfm = torch.zeros(Nn, M, dtype=torch.bfloat16, device=dev) if out_fm else None
    partial = torch.empty(splits + 16, M, Nn, dtype=torch.float32, device=dev) if splits > 1 else None
    p = N.ptr
    N.call("dxrl_gemm_bf16", dev.index, p(A), A.stride(0), p(Bt), Bt.stride(0), M, Nn, K, p(bias), bias_stride, act,
           p(gate), 0 if gate is None else gate.stride(0), p(Cf), Nn, p(Crm), Nn, p(Cfm), M, None, 0, splits, p(partial),
           N.stream_of(dev))
    torch.cuda.synchronize()
    return Cf, Crm, Cfm


@pytest.mark.parametrize("M,Nn,K", [(128, 128, 32), (300, 256, 64), (4096, 256, 256), (77, 32, 288), (1000, 288, 96)])
def test_gemm_plain(N, M, Nn, K):
    g = torch.Generator(device="cuda").manual_seed(M + Nn + K)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    Bt = torch.randn(Nn, K, device="cuda", generator=g).to(torch.bfloat16)
    Cf, _, _ = gemm(N, A, Bt)
    ref = A.float() @ Bt.float().T
    torch.testing.assert_close(Cf, ref, rtol=1e-5, atol=1e-4 * K ** 0.5)


def test_gemm_asymmetric_identity(N):
    """A = I with an asymmetric B catches a row/col swap in the C write."""
    M = K = 64
    A = torch.eye(M, K, device="cuda").to(torch.bfloat16)
    Bt = (torch.arange(96 * K, device="cuda").reshape(96, K) % 251).float().to(torch.bfloat16)
    Cf, _, _ = gemm(N, A, Bt)
    torch.testing.assert_close(Cf, Bt.float().T[:M], rtol=0, atol=0)


def test_gemm_epilogue_bias_tanh_gate_layouts(N):
    M, Nn, K = 333, 256, 64
    g = torch.Generator(device="cuda").manual_seed(3)
    A = (0.3 * torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
    W = (0.3 * torch.randn(Nn, K + 8, device="cuda", generator=g)).to(torch.bfloat16)  # ld = K + 8
    bias_mat = torch.randn(Nn, 3, device="cuda", generator=g)  # strided bias column
    gate = torch.tanh(torch.randn(M, Nn, device="cuda", generator=g)).to(torch.bfloat16)
    Cf, Crm, Cfm = gemm(N, A, W[:, :K], bias=bias_mat[:, 1], bias_stride=3, act=1, gate=gate, out_rm=True,
                        out_fm=True)
    ref = torch.tanh(A.float() @ W[:, :K].float().T + bias_mat[:, 1]) * (1 - gate.float() ** 2)
    torch.testing.assert_close(Cf, ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(Crm.float(), ref, rtol=2 ** -7, atol=1e-6)
    torch.testing.assert_close(Cfm.float().T, Crm.float(), rtol=0, atol=0)


def test_gemm_split_k_weight_gradient_shape(N):
    """dW[o][i] = sum_m dY[m][o] X[m][i] with both operands feature-major
    (K = samples), split-K partial slabs reduced in fixed order."""
    Ms, O, I = 40000, 256, 288
    g = torch.Generator(device="cuda").manual_seed(9)
    dYfm = (0.1 * torch.randn(O, Ms, device="cuda", generator=g)).to(torch.bfloat16)
    Xfm = torch.randn(I, Ms, device="cuda", generator=g).to(torch.bfloat16)
    Cf, _, _ = gemm(N, dYfm, Xfm, splits=13)
    ref = dYfm.float() @ Xfm.float().T
    torch.testing.assert_close(Cf, ref, rtol=1e-4, atol=2e-3)
    Cf2, _, _ = gemm(N, dYfm, Xfm, splits=13)
    assert torch.equal(Cf, Cf2)  # deterministic


def wgrad(N, Y, O, X, I, splits=1):
    M = Y.shape[0]
    dev = Y.device
    out = torch.full((O, I), float("nan"), dtype=torch.float32, device=dev)
    partial = torch.empty(max(splits, 1) + 16, O, I, dtype=torch.float32, device=dev)
    p = N.ptr
    N.call("dxrl_wgrad_bf16", dev.index, p(Y), Y.stride(0), O, p(X), X.stride(0), I, M, splits, p(partial), p(out),
           N.stream_of(dev))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("M,O,ldy,I,ldx,splits", [(64, 128, 128, 128, 128, 1), (1000, 256, 256, 288, 288, 1),
                                                  (4096, 32, 32, 288, 288, 7), (3232, 256, 256, 64, 64, 5),
                                                  (50016, 256, 256, 288, 288, 33), (1000, 200, 256, 264, 288, 4),
                                                  (819200, 256, 256, 256, 288, 256), (5000, 256, 256, 288, 288, 4),
                                                  (96, 256, 256, 256, 256, 7), (24736, 256, 256, 256, 256, 24)])
def test_wgrad_transposed_lds_reads(N, M, O, ldy, I, ldx, splits):
    """out[o][i] = sum_m Y[m][o] X[m][i] from row-major operands (ds_read_b64_tr_b16 path)."""
    g = torch.Generator(device="cuda").manual_seed(M + O + I)
    Y = (0.1 * torch.randn(M, ldy, device="cuda", generator=g)).to(torch.bfloat16)
    X = torch.randn(M, ldx, device="cuda", generator=g).to(torch.bfloat16)
    out = wgrad(N, Y, O, X, I, splits)
    ref = Y[:, :O].float().T @ X[:, :I].float()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3 * (M / 1000) ** 0.5)


@pytest.mark.parametrize("M,O,I,splits", [(700, 256, 288, 3), (4160, 136, 200, 5)])
def test_wgrad_full_output_exact_integer(N, M, O, I, splits):
    """The whole-output kernel (k_wgrad_full: O > 128) on exact small integers, ragged M chunks."""
    Y = (torch.arange(M * O, device="cuda").reshape(M, O) % 7 - 3).to(torch.bfloat16)
    X = (torch.arange(M * I, device="cuda").reshape(M, I) % 5 - 2).float().mul(torch.arange(I, device="cuda") % 3 + 1)
    X = X.to(torch.bfloat16)
    out = wgrad(N, Y, O, X, I, splits)
    assert torch.equal(out, Y.float().T @ X.float())


def test_wgrad_exact_integer_asymmetric(N):
    """Exact small integers: any transpose / k-order slip shows as a hard mismatch."""
    M, O, I = 128, 32, 64
    Y = (torch.arange(M * O, device="cuda").reshape(M, O) % 7 - 3).to(torch.bfloat16)
    X = (torch.arange(M * I, device="cuda").reshape(M, I) % 5 - 2).float().mul(torch.arange(I, device="cuda") % 3 + 1)
    X = X.to(torch.bfloat16)
    out = wgrad(N, Y, O, X, I)
    ref = Y.float().T @ X.float()
    assert torch.equal(out, ref)
