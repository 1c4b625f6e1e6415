"""Parity of the analytic exact-GP backward (gpk_exact_mll_grad_f32, through the C ABI
and through autograd) against the fp64 oracle gradients (oracle.exact_mll_grads:
torch fp64 autograd of the GPyTorch restatement, pinned by finite differences in
tests/test_oracle.py).

Tolerance: the gradient contains K_hat^{-1}, which an fp32 Cholesky (GPyTorch's own
fp32 path included) only delivers to ~cond(K_hat) * 2^-24; the bound below is
norm-wise relative 1e-4 per gradient block (the north_star bound; measured 1e-7..4e-6), and the fp32 torch-autograd path of the
same model (what GPyTorch computes) is reported beside it as the accuracy the
reference itself achieves. The MLL forward stays at the north_star's 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

LN2 = float(np.log(2.0))
NOISE0 = LN2 + 1e-4
TOL = 1e-4


def _rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _fp32_torch_grads(X, y, ls, s2, c, noise, gout):
    """The reference's own arithmetic: fp32 torch autograd (GPyTorch-like), CPU."""
    Xt = X.clone().requires_grad_(True)
    yt = y.clone().requires_grad_(True)
    lst = torch.tensor(np.atleast_1d(ls), dtype=torch.float32, requires_grad=True)
    s2t = torch.tensor(s2, dtype=torch.float32, requires_grad=True)
    ct = torch.tensor(c, dtype=torch.float32, requires_grad=True)
    nzt = torch.tensor(noise, dtype=torch.float32, requires_grad=True)
    N = X.shape[1]
    xs = Xt / lst
    d = ((xs.unsqueeze(-2) - xs.unsqueeze(-3)) ** 2).sum(-1)
    K = s2t * torch.exp(-0.5 * d) + nzt * torch.eye(N)
    L = torch.linalg.cholesky(K)
    z = torch.linalg.solve_triangular(L, (yt - ct).unsqueeze(-1), upper=False).squeeze(-1)
    mll = -0.5 * ((z * z).sum(-1) + 2 * torch.log(torch.diagonal(L, dim1=-2, dim2=-1)).sum(-1)
                  + N * np.log(2 * np.pi)) / N
    gs = torch.autograd.grad((gout * mll).sum(), [Xt, yt, lst, s2t, ct, nzt])
    return dict(zip(["X", "y", "lengthscale", "outputscale", "mean_constant", "noise"],
                    [g.detach().numpy() for g in gs]))


@pytest.mark.parametrize("B,N,D,ard", [(3, 16, 4, False), (2, 37, 5, True), (4, 64, 8, False),
                                       (2, 96, 32, False), (2, 256, 32, False), (2, 250, 7, True),
                                       (2, 80, 48, True), (2, 256, 64, False)])
def test_exact_grad_abi_vs_oracle(cuda_device, B, N, D, ard):
    from fine_grained_gaussian_process_forcasting_amd import ops
    g = torch.Generator().manual_seed(B * 100 + N)
    X = torch.randn(B, N, D, generator=g) / np.sqrt(D)
    y = torch.randn(B, N, generator=g)
    ls = np.linspace(0.6, 1.4, D) if ard else LN2
    s2, c, noise = 1.3, 0.2, NOISE0
    gout = torch.rand(B, generator=g) + 0.5
    dev = cuda_device
    hyper = ops.pack_exact_hyper(s2, noise, c, torch.tensor(np.atleast_1d(ls), dtype=torch.float32), dev)
    fw = ops.exact_mll(X.to(dev), y.to(dev), None, None, None, None, hyper=hyper, want_L=True, want_z=True)
    assert (fw.info.cpu() == 0).all()
    gr = ops.exact_mll_grad(X.to(dev), fw.L, fw.z, hyper, gout.to(dev))
    torch.cuda.synchronize()
    ref = O.exact_mll_grads(X.double().numpy(), y.double().numpy(), ls, s2, c, noise,
                            gout=gout.double().numpy())
    dh = gr.dhyp.sum(0).cpu().double().numpy()
    got = {"X": gr.dX.cpu().numpy(), "y": gr.dy.cpu().numpy(), "outputscale": dh[0], "noise": dh[1],
           "mean_constant": dh[2], "lengthscale": dh[3:] if ard else dh[3]}
    f32 = _fp32_torch_grads(X, y, ls, s2, c, noise, gout)
    for k in got:
        e = _rel(got[k], ref[k])
        e32 = _rel(f32[k], ref[k])
        print(f"N={N} D={D} {k:14s} hip {e:.2e}   torch-fp32 {e32:.2e}")
        assert e <= TOL, (k, e, e32)


def test_exact_grad_autograd_path(cuda_device):
    """ExactGPModel-style objective through ops_autograd: every parameter's .grad
    comes from the HIP adjoint and matches the oracle."""
    from fine_grained_gaussian_process_forcasting_amd import ops_autograd
    B, N, D = 3, 48, 6
    g = torch.Generator().manual_seed(5)
    X = torch.randn(B, N, D, generator=g) / np.sqrt(D)
    y = torch.randn(B, N, generator=g)
    dev = cuda_device
    Xd = X.to(dev).requires_grad_(True)
    yd = y.to(dev).requires_grad_(True)
    p = {k: torch.tensor(v, device=dev, requires_grad=True)
         for k, v in dict(ls=[0.9], s2=1.1, c=0.05, nz=0.3).items()}
    mll = ops_autograd.exact_log_prob(Xd, yd, p["ls"], p["s2"], p["c"], p["nz"])
    (-mll.mean()).backward()
    ref = O.exact_mll_grads(X.double().numpy(), y.double().numpy(), 0.9, 1.1, 0.05, 0.3,
                            gout=-np.ones(B) / B)
    assert _rel(Xd.grad.cpu(), ref["X"]) <= TOL
    assert _rel(yd.grad.cpu(), ref["y"]) <= TOL
    assert _rel(p["ls"].grad.cpu(), ref["lengthscale"]) <= TOL
    assert _rel(p["s2"].grad.cpu(), ref["outputscale"]) <= TOL
    assert _rel(p["c"].grad.cpu(), ref["mean_constant"]) <= TOL
    assert _rel(p["nz"].grad.cpu(), ref["noise"]) <= TOL


def test_exact_grad_native_kernel_loaded(cuda_device):
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    assert lib.gpk_exact_grad_workspace_bytes(2, 256) == 2 * 36224 * 4
    assert lib.gpk_exact_grad_workspace_bytes(1, 801) == 0
    # a NULL workspace is refused before anything is launched; a real one runs
    import torch
    from fine_grained_gaussian_process_forcasting_amd import ops
    X = torch.randn(2, 40, 3, device=cuda_device) / 2
    y = torch.randn(2, 40, device=cuda_device)
    h = ops.pack_exact_hyper(0.8, 0.5, 0.0, 0.9, cuda_device)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    dh = torch.empty(2, 4, device=cuda_device)
    go = torch.ones(2, device=cuda_device)
    rc = lib.gpk_exact_mll_grad_f32(X.data_ptr(), f.L.data_ptr(), f.z.data_ptr(), h.data_ptr(), 1, 2, 40, 3,
                                    go.data_ptr(), None, None, None, dh.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == -10
    ws = torch.empty(lib.gpk_exact_grad_workspace_bytes(2, 40) // 4, device=cuda_device)
    rc = lib.gpk_exact_mll_grad_f32(X.data_ptr(), f.L.data_ptr(), f.z.data_ptr(), h.data_ptr(), 1, 2, 40, 3,
                                    go.data_ptr(), ws.data_ptr(), None, None, dh.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(dh).all()


def test_exact_grad_full_bench_batch(cuda_device):
    """The backward at the bench / BASELINE configs[3] batch (B=512, N=256, D=32: the
    launch the bench times), checked per window on a sample of 8 windows spread over the
    batch: dX, dy and the per-window hyper-parameter rows vs the fp64 oracle (1e-4)."""
    from fine_grained_gaussian_process_forcasting_amd import ops
    B, N, D = 512, 256, 32
    g = torch.Generator().manual_seed(512)
    X = torch.randn(B, N, D, generator=g) / np.sqrt(D)
    y = torch.randn(B, N, generator=g)
    s2, c, noise = LN2, 0.0, NOISE0
    gout = torch.rand(B, generator=g) + 0.5
    dev = cuda_device
    hyper = ops.pack_exact_hyper(s2, noise, c, LN2, dev)
    fw = ops.exact_mll(X.to(dev), y.to(dev), None, None, None, None, hyper=hyper, want_L=True, want_z=True)
    assert (fw.info.cpu() == 0).all()
    gr = ops.exact_mll_grad(X.to(dev), fw.L, fw.z, hyper, gout.to(dev))
    torch.cuda.synchronize()
    dX, dy, dh = gr.dX.cpu().numpy(), gr.dy.cpu().numpy(), gr.dhyp.cpu().double().numpy()
    for w in np.linspace(0, B - 1, 8).astype(int):
        ref = O.exact_mll_grads(X[w:w + 1].double().numpy(), y[w:w + 1].double().numpy(), LN2, s2, c, noise,
                                gout=gout[w:w + 1].double().numpy())
        got = {"X": dX[w:w + 1], "y": dy[w:w + 1], "outputscale": dh[w, 0], "noise": dh[w, 1],
               "mean_constant": dh[w, 2], "lengthscale": dh[w, 3]}
        for k in got:
            e = _rel(got[k], ref[k])
            assert e <= TOL, (w, k, e)


@pytest.mark.parametrize("N,noise", [(128, 1e-2), (128, 1e-3), (256, 1e-3)])
def test_exact_grad_ill_conditioned_vs_fp32_reference(cuda_device, N, noise):
    """Small noise (cond(K_hat) ~ 1e3..1e4 at N=128, more at the headline's N=256): the HIP
    backward's error vs the fp64 oracle must stay within 1e-4 or within 3x of what the
    reference's own fp32 arithmetic (torch fp32 autograd through cholesky) achieves on the
    same windows. alpha (hence dy and the mean-constant gradient) comes from V^T z with V
    the split-f16 explicit L^-1, so N=256 pins its error growth at the bench shape."""
    from fine_grained_gaussian_process_forcasting_amd import ops
    B, D = 2, 8
    g = torch.Generator().manual_seed(77)
    X = torch.randn(B, N, D, generator=g) / np.sqrt(D)
    y = torch.randn(B, N, generator=g)
    s2, c = 1.0, 0.1
    gout = torch.rand(B, generator=g) + 0.5
    dev = cuda_device
    hyper = ops.pack_exact_hyper(s2, noise, c, LN2, dev)
    fw = ops.exact_mll(X.to(dev), y.to(dev), None, None, None, None, hyper=hyper, want_L=True, want_z=True)
    assert (fw.info.cpu() == 0).all()
    gr = ops.exact_mll_grad(X.to(dev), fw.L, fw.z, hyper, gout.to(dev))
    torch.cuda.synchronize()
    ref = O.exact_mll_grads(X.double().numpy(), y.double().numpy(), LN2, s2, c, noise,
                            gout=gout.double().numpy())
    dh = gr.dhyp.sum(0).cpu().double().numpy()
    got = {"X": gr.dX.cpu().numpy(), "y": gr.dy.cpu().numpy(), "outputscale": dh[0], "noise": dh[1],
           "mean_constant": dh[2], "lengthscale": dh[3]}
    f32 = _fp32_torch_grads(X, y, LN2, s2, c, noise, gout)
    for k in got:
        e = _rel(got[k], ref[k])
        e32 = _rel(f32[k], ref[k])
        print(f"noise={noise} {k:14s} hip {e:.2e}   torch-fp32 {e32:.2e}")
        assert e <= max(TOL, 3 * e32), (k, e, e32)
