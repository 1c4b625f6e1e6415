"""HIP-graph capture of a training step through the GP path (graphs.GraphedStep).

The graphed step must reproduce the eager step (same seeds, same batches, same Adam
arithmetic with capturable=True) and report the same numerical warnings per replay as
the eager call. Reference loop: train.py:152-167; GP branch denoise_model_2.py:42-59,
ELBO forecast_denoising.py:86-89.
"""
import math
import warnings

import pytest
import torch
import torch.nn as nn

from fine_grained_gaussian_process_forcasting_amd import NumericalWarning, settings
from fine_grained_gaussian_process_forcasting_amd.denoising_model.denoise_model_2 import denoise_model_2
from fine_grained_gaussian_process_forcasting_amd.denoising_model.DeepGP import DeepGPp
from fine_grained_gaussian_process_forcasting_amd.graphs import GraphedStep
from fine_grained_gaussian_process_forcasting_amd.mlls import DeepApproximateMLL, VariationalELBO

pytestmark = pytest.mark.gpu


class _Backbone(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.e = nn.Linear(d, d)
        self.d = nn.Linear(d, d)

    def forward(self, enc, dec):
        return torch.tanh(self.e(enc)), torch.tanh(self.d(dec))


class _Model(nn.Module):
    def __init__(self, d, nin=4, seed=7):
        super().__init__()
        torch.manual_seed(seed)
        self.emb_e = nn.Linear(nin, d)
        self.emb_d = nn.Linear(nin, d)
        self.de = denoise_model_2(_Backbone(d), "stand-in", True, d, None, seed)
        self.proj = nn.Linear(d, 1)
        self.d = d

    def forward(self, enc, dec, y):
        out, dist = self.de(self.emb_e(enc), self.emb_d(dec))
        mll = DeepApproximateMLL(VariationalELBO(self.de.deep_gp.likelihood, self.de.deep_gp, self.d))
        return nn.MSELoss()(y, self.proj(out)) - 0.005 * mll(dist, y.permute(2, 0, 1)).mean()


def _batches(n, b, ne, nd, nin, dev, seed=11):
    g = torch.Generator().manual_seed(seed)
    return [tuple(t.to(dev) for t in (torch.randn(b, ne, nin, generator=g), torch.randn(b, nd, nin, generator=g),
                                      torch.randn(b, nd, 1, generator=g))) for _ in range(n)]


def test_graphed_train_step_matches_eager(cuda_device):
    dev = cuda_device
    d, b, ne, nd = 32, 8, 48, 24
    batches = _batches(6, b, ne, nd, 4, dev)
    with settings.num_likelihood_samples(1):
        ma = _Model(d).to(dev)
        mb = _Model(d).to(dev)
        with torch.no_grad():
            ma(*batches[0])          # q(u) initialises lazily on the first call (its own randn)
        mb.load_state_dict(ma.state_dict())
        # SGD: parameter updates proportional to the gradients (Adam's sign-like first
        # steps would amplify float-level gradient differences of near-zero entries)
        oa = torch.optim.SGD(ma.parameters(), lr=1e-2)
        ob = torch.optim.SGD(mb.parameters(), lr=1e-2)

        def eager(batch):
            oa.zero_grad(set_to_none=True)
            loss = ma(*batch)
            loss.backward()
            oa.step()
            return float(loss.detach())

        for _ in range(3):                       # GraphedStep's warm-up steps
            eager(batches[0])
        def fb(e, dd, y):              # (aux, loss) like Forecast_denoising's tuple return
            loss = mb(e, dd, y)
            return 2.0 * loss.detach(), loss

        step = GraphedStep(fb, ob, batches[0], warmup=3, loss_index=1)
        for k in range(1, 6):
            la = eager(batches[k])
            aux, lossb = step(*batches[k])
            lb = float(lossb.detach())
            assert float(aux) == 2.0 * lb
            assert math.isfinite(lb)
            assert abs(la - lb) <= 1e-5 * max(1.0, abs(la)), (k, la, lb)
        for (na, pa), (nb, pb) in zip(ma.named_parameters(), mb.named_parameters()):
            assert na == nb
            assert torch.allclose(pa, pb, rtol=1e-4, atol=1e-6), na


def test_graphed_step_reports_jitter_warnings_per_replay(cuda_device):
    """Near-duplicate inducing points and no variational jitter: GPyTorch's fp64 K_ZZ
    ladder fires on every call. The captured step records the check and must warn on
    every replay, as the eager step does (lr = 0 keeps the points near-duplicate)."""
    dev = cuda_device
    D, B, N = 8, 4, 32
    g = torch.Generator().manual_seed(5)
    with settings.num_likelihood_samples(1):
        model = DeepGPp(D, 1).to(dev)
        vs = model.hidden_layer.variational_strategy
        vs.jitter_val = 0.0
        with torch.no_grad():
            z0 = torch.randn(1, D, generator=g)
            vs.inducing_points.copy_((z0 + 1e-4 * torch.randn(vs.inducing_points.shape[0], D, generator=g)).to(dev))
        x = torch.randn(B, N, D, generator=g).to(dev)
        y = torch.randn(1, B, N, generator=g).to(dev)
        elbo = DeepApproximateMLL(VariationalELBO(model.likelihood, model, D))
        opt = torch.optim.Adam(model.parameters(), lr=0.0, capturable=True)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", NumericalWarning)
            step = GraphedStep(lambda xx, yy: -elbo(model(xx), yy).mean(), opt, (x, y), warmup=2)
        for _ in range(2):
            with pytest.warns(NumericalWarning, match="added jitter of 1.0e-08"):
                loss = step(x, y)
            assert math.isfinite(float(loss))


class _ExactObjective(nn.Module):
    """-mean exact MLL of a ConstantMean + ScaleKernel(RBF) model (GPModel.py:5-13)."""

    def __init__(self, dev):
        super().__init__()
        self.raw = nn.Parameter(torch.zeros(4, device=dev))    # ls, s2, c, noise (pre-softplus)

    def forward(self, X, y):
        from fine_grained_gaussian_process_forcasting_amd.ops_autograd import exact_log_prob
        sp = torch.nn.functional.softplus(self.raw)
        return -exact_log_prob(X, y, sp[0:1], sp[1], self.raw[2], sp[3] + 1e-4).mean()


def _exact_batch(dev, B=4, N=32, D=4, seed=3):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(B, N, D, generator=g) / 2).to(dev), torch.randn(B, N, generator=g).to(dev)


@pytest.mark.parametrize("check_every", [1, 2])
def test_graphed_step_rolls_back_a_failing_replay(cuda_device, check_every):
    """Eager psd_safe_cholesky raises in the forward with the parameters intact. A replay
    has already stepped the optimizer when its verdict is read: GraphedStep must restore
    the parameters and Adam state of the failing check block before raising."""
    from fine_grained_gaussian_process_forcasting_amd import NanError, NotPSDError
    dev = cuda_device
    model = _ExactObjective(dev)
    X, y = _exact_batch(dev)
    opt = torch.optim.Adam(model.parameters(), lr=torch.tensor(1e-2, device=dev), capturable=True)
    step = GraphedStep(model, opt, (X, y), warmup=1, check_every=check_every)
    for _ in range(check_every):
        step(X, y)                                  # a good block: parameters move
    before = model.raw.detach().clone()
    state_before = {k: v.detach().clone() for k, v in opt.state[model.raw].items()}
    Xbad = X.clone()
    Xbad[1, 3, 0] = float("nan")
    with pytest.raises((NanError, NotPSDError)):
        step(Xbad, y)                               # replay 1 of the block fails ...
        if check_every == 2:
            step(X, y)                              # ... and is caught at the block's check
    torch.testing.assert_close(model.raw.detach(), before, rtol=0, atol=0)
    for k, v in opt.state[model.raw].items():
        torch.testing.assert_close(v.detach(), state_before[k], rtol=0, atol=0)
    for _ in range(check_every):
        loss = step(X, y)                           # training continues from the restored state
    assert math.isfinite(float(loss))
    assert not torch.equal(model.raw.detach(), before)


def test_graphed_step_learning_rate_rules(cuda_device):
    """A float lr is fixed inside the graph: changing it after capture must raise; a
    device-tensor lr updated in place is honoured (the NoamOpt schedule, train.py:147)."""
    dev = cuda_device
    X, y = _exact_batch(dev)
    model = _ExactObjective(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)
    step = GraphedStep(model, opt, (X, y), warmup=1)
    step(X, y)
    opt.param_groups[0]["lr"] = 2e-3
    with pytest.raises(ValueError, match="float lr"):
        step(X, y)

    model = _ExactObjective(dev)
    lr = torch.tensor(0.0, device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=lr, capturable=True)
    step = GraphedStep(model, opt, (X, y), warmup=1)
    before = model.raw.detach().clone()
    step(X, y)
    torch.testing.assert_close(model.raw.detach(), before, rtol=0, atol=0)   # lr 0: no move
    lr.fill_(1e-2)
    step(X, y)
    assert (model.raw.detach() - before).abs().max() > 1e-4                  # the new lr is used

