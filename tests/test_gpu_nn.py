"""NN challenger HIP kernels vs PyTorch / scikit-learn oracles (run with -m gpu)."""
import time

import numpy as np
import pytest
import torch

from cobalt_smart_lender_ai_amd.nn import mlp
from cobalt_smart_lender_ai_amd.nn.smote import SMOTE, kneighbors

pytestmark = pytest.mark.gpu


def _toy(n, F=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.random((n, F)).astype(np.float32)
    y = ((X[:, 0] + 0.5 * X[:, 1] + rng.normal(0, 0.15, n)) > 0.9).astype(np.float32)
    return X, y


def test_forward_kernel_matches_torch():
    X, _ = _toy(5003)
    p = mlp.init_params(20, seed=3)
    ref = torch.sigmoid(mlp.forward_torch(torch.as_tensor(p, dtype=torch.float64), torch.as_tensor(X, dtype=torch.float64), 20))
    out = torch.empty(len(X), dtype=torch.float32, device="cuda")
    mlp.mlp_forward_gpu(torch.as_tensor(X, device="cuda"), torch.as_tensor(p, device="cuda"), out)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("kernel", ["mfma", "fma"])
@pytest.mark.parametrize("F", [1, 7, 20, 32])
def test_forward_kernels_all_widths_strided_biased(kernel, F):
    """Both forward kernels vs an fp64 PyTorch reference: non-zero biases, odd widths (layer-1 K
    padding in the MFMA kernel), a row stride wider than F, N not a multiple of the 32-row tile."""
    rng = np.random.default_rng(F)
    n = 70_001
    Xw = rng.normal(0, 1, (n, F + 3)).astype(np.float32)
    p = mlp.init_params(F, seed=F)
    for name, (o, shape) in mlp.layout(F).items():
        if name.startswith("b"):
            p[o:o + int(np.prod(shape))] = rng.normal(0, 0.3, int(np.prod(shape)))
    zref = mlp.forward_torch(torch.as_tensor(p, dtype=torch.float64), torch.as_tensor(Xw[:, :F], dtype=torch.float64), F)
    Xd = torch.as_tensor(Xw, device="cuda")[:, :F]
    assert Xd.stride(0) == F + 3
    prob = torch.full((n,), -1.0, device="cuda")
    z = torch.full((n,), -1.0, device="cuda")
    mlp.mlp_forward_gpu(Xd, torch.as_tensor(p, device="cuda"), prob, z, kernel=kernel)
    zr = zref.numpy()
    np.testing.assert_allclose(z.cpu().numpy(), zr, rtol=1e-5, atol=2e-5 * max(1.0, float(np.abs(zr).max())))
    np.testing.assert_allclose(prob.cpu().numpy(), torch.sigmoid(zref).numpy(), rtol=0, atol=1e-5)


def test_forward_mfma_equals_fma_kernel_at_scale():
    X, _ = _toy(1_000_003, seed=5)
    p = torch.as_tensor(mlp.init_params(20, seed=9), device="cuda")
    Xd = torch.as_tensor(X, device="cuda")
    a = torch.empty(len(X), device="cuda")
    b = torch.empty(len(X), device="cuda")
    mlp.mlp_forward_gpu(Xd, p, a, kernel="mfma")
    mlp.mlp_forward_gpu(Xd, p, b, kernel="fma")
    assert float((a - b).abs().max()) < 2e-6


@pytest.mark.parametrize("kernel", ["mfma", "fma"])
def test_train_epoch_kernel_matches_torch_oracle(kernel):
    X, y = _toy(203)
    cfg = mlp.MLPConfig(epochs=1, shuffle=False)
    rate, dsteps = cfg.decay(len(X))
    p = torch.as_tensor(mlp.init_params(20, 7))
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    step, _ = mlp.train_epoch_torch(torch.as_tensor(X), torch.as_tensor(y), torch.arange(len(X)), p, m, v, 0, cfg,
                                    rate, dsteps)
    models, _ = mlp.fit_many(X, y, cfg=cfg, seeds=(7,), device="cuda", kernel=kernel)
    np.testing.assert_allclose(models[0].params, p.numpy(), rtol=0, atol=2e-6)


@pytest.mark.parametrize("F,batch", [(1, 32), (7, 17), (20, 32), (31, 5)])
def test_train_mfma_widths_batches_vs_torch(F, batch):
    """MFMA trainer vs the PyTorch oracle of the same algorithm: odd widths (K padding, the bias
    column at F), partial and small batches, shuffled order, 3 models in one launch, moments too."""
    rng = np.random.default_rng(F)
    n = 301
    X = rng.random((n, F)).astype(np.float32)
    y = ((X[:, 0] + 0.3 * rng.normal(size=n)) > 0.5).astype(np.float32)
    cfg = mlp.MLPConfig(epochs=1, batch_size=batch)
    rate, dsteps = cfg.decay(n)
    seeds = (3, 4, 5)
    G, P = len(seeds), mlp.num_params(F)
    p0 = np.stack([mlp.init_params(F, s) for s in seeds])
    for g in range(G):  # non-zero biases and moments
        for name, (o, shape) in mlp.layout(F).items():
            if name.startswith("b"):
                p0[g, o:o + int(np.prod(shape))] = rng.normal(0, 0.1, int(np.prod(shape)))
    m0 = rng.normal(0, 1e-3, (G, P)).astype(np.float32)
    v0 = rng.uniform(0, 1e-5, (G, P)).astype(np.float32)
    perms = np.stack([rng.permutation(n) for _ in seeds]).astype(np.int32)
    lib = mlp._native.lib()
    hp = mlp._Hyper(cfg.initial_lr, rate, dsteps, 1, cfg.weight_decay, cfg.beta1, cfg.beta2, cfg.eps, cfg.lambda_l2, batch)
    dev = "cuda"
    pd_, md, vd = (torch.as_tensor(a, device=dev).contiguous() for a in (p0, m0, v0))
    steps = torch.full((G,), 11, dtype=torch.int64, device=dev)
    loss = torch.zeros(G, device=dev)
    Xd, yd, permd = (torch.as_tensor(a, device=dev) for a in (X, y, perms))
    rc = lib.cobalt_mlp_train_epoch_mfma(Xd.data_ptr(), F, yd.data_ptr(), n, F, permd.data_ptr(), pd_.data_ptr(),
                                         md.data_ptr(), vd.data_ptr(), steps.data_ptr(), mlp.ctypes.byref(hp), G,
                                         loss.data_ptr(), None, mlp._native.stream_handle())
    assert rc == 0
    for g in range(G):
        p, m, v = (torch.as_tensor(a[g].copy()) for a in (p0, m0, v0))
        st, ls = mlp.train_epoch_torch(torch.as_tensor(X), torch.as_tensor(y), torch.as_tensor(perms[g], dtype=torch.int64),
                                       p, m, v, 11, cfg, rate, dsteps)
        assert int(steps[g]) == st
        np.testing.assert_allclose(pd_[g].cpu().numpy(), p.numpy(), rtol=0, atol=3e-6)
        np.testing.assert_allclose(md[g].cpu().numpy(), m.numpy(), rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(float(loss[g]), ls, rtol=1e-5)


def test_many_models_in_one_launch_equal_single_runs():
    X, y = _toy(2000)
    cfg = mlp.MLPConfig(epochs=2)
    many, _ = mlp.fit_many(X, y, cfg=cfg, seeds=(0, 1, 2), device="cuda")
    for s, mm in zip((0, 1, 2), many):
        one, _ = mlp.fit_many(X, y, cfg=cfg, seeds=(s,), device="cuda")
        np.testing.assert_array_equal(one[0].params, mm.params)


@pytest.mark.parametrize("kernel", ["mfma", "fma"])
def test_full_size_epoch_speed_and_quality(kernel):
    X, y = _toy(78034, seed=1)
    Xv, yv = _toy(19509, seed=2)
    cfg = mlp.MLPConfig(epochs=3)
    t = time.perf_counter()
    models, hist = mlp.fit_many(X, y, Xv, yv, cfg, seeds=(0,), device="cuda", kernel=kernel)
    dt = (time.perf_counter() - t) / 3
    print(f"[nn] {kernel}: {dt * 1e3:.1f} ms/epoch for 2439 steps of batch 32 ({78034 / dt / 1e6:.2f} M rows/s)")
    assert hist[0]["val_AUC"][-1] > 0.9
    assert dt < 2.0  # the reference's Keras CPU run: 2-4 s per epoch


def test_knn_matches_sklearn():
    from sklearn.neighbors import NearestNeighbors

    rng = np.random.default_rng(4)
    R = rng.normal(size=(3001, 20)).astype(np.float32)
    idx, dist = kneighbors(R, R, 6, device="cuda")
    ref_d, ref_i = NearestNeighbors(n_neighbors=6).fit(R.astype(np.float64)).kneighbors(R.astype(np.float64))
    assert (idx == ref_i).mean() > 0.999
    np.testing.assert_allclose(dist, ref_d, rtol=1e-3, atol=2e-3)
    assert np.all(idx[:, 0] == np.arange(len(R)))


def test_smote_gpu_equals_cpu():
    rng = np.random.default_rng(6)
    X = rng.normal(size=(3000, 20))
    y = (rng.random(3000) < 0.13).astype(np.int64)
    Xg, yg = SMOTE(random_state=123, device="cuda").fit_resample(X, y)
    Xc, yc = SMOTE(random_state=123, device="cpu").fit_resample(X, y)
    np.testing.assert_array_equal(yg, yc)
    np.testing.assert_allclose(Xg, Xc, rtol=0, atol=1e-12)
