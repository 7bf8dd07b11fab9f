"""NN challenger: Dense 128-32-16-1 (ReLU, sigmoid) with L2, AdamW + staircase ExponentialDecay, BCE.

Reference: notebooks/04_model_training.ipynb cell 39 ``build_and_train_nn`` and cell 40 call
(SURVEY.md §2.2 N10, §3.6). Defaults reproduce that call: lambda_l2=1e-3, lr 1e-3 -> 1e-6 over 50
staircase decays of ``int(len(X_train)/32)`` steps, 50 epochs, batch 32, Keras AdamW defaults
(weight_decay 0.004, beta 0.9/0.999, eps 1e-7), Glorot-uniform kernels / zero biases,
EarlyStopping(monitor="val_precision", mode="max", patience=5, restore_best_weights=True).

Execution: on the GPU every epoch is ONE launch of a fused trainer that keeps weights, AdamW
moments and activations on one CU for all steps (``csrc/mlp.hip``). The default is the fp32-MFMA
trainer (``k_mlp_train_mfma``, F <= 31: 4 waves per model, W1/W2 in registers as the MFMA operands
they are, 9.4 us per batch-32 step); ``kernel="fma"`` selects the 1024-thread scalar-FMA trainer
(29.6 us per step). ``fit_many`` trains several models (seeds / learning rates) in the same launch,
one per CU. Bulk inference runs on fp32 MFMA as well (``k_mlp_forward_mfma``). On CPU the same
algorithm runs in plain PyTorch (:func:`train_epoch_torch`), which is also the numerics oracle of
the kernel. History keys follow Keras 3 naming (``loss``, ``val_loss``, ``val_accuracy``,
``val_Precision``, ``val_Recall``, ``val_AUC``): the reference's monitor ``"val_precision"`` is not
among them, so -- exactly as in the notebook run (warning at ``04:3996``) -- early stopping never
triggers with the default config.
"""
from __future__ import annotations

import ctypes
import json
import logging
import math
from dataclasses import asdict, dataclass, field
from pathlib import Path

import numpy as np
import torch

from .. import _native

log = logging.getLogger(__name__)

H1, H2, H3 = 128, 32, 16
MAX_F = 32
MAX_F_MFMA = 31  # the MFMA trainer folds b1 into W1 through a constant-1 input column


def num_params(F: int) -> int:
    return F * H1 + H1 + H1 * H2 + H2 + H2 * H3 + H3 + H3 + 1


def layout(F: int) -> dict[str, tuple[int, tuple[int, ...]]]:
    """name -> (offset, shape) in the flat parameter vector (kernel layout ``[in][out]``)."""
    out, off = {}, 0
    for name, shape in (("W1", (F, H1)), ("b1", (H1,)), ("W2", (H1, H2)), ("b2", (H2,)), ("W3", (H2, H3)),
                        ("b3", (H3,)), ("W4", (H3,)), ("b4", (1,))):
        out[name] = (off, shape)
        off += int(np.prod(shape))
    return out


def l2_mask(F: int) -> np.ndarray:
    """Elements carrying the kernel regulariser (W1, W2, W3 -- not the output layer or biases)."""
    m = np.zeros(num_params(F), dtype=bool)
    lay = layout(F)
    for k in ("W1", "W2", "W3"):
        o, s = lay[k]
        m[o:o + int(np.prod(s))] = True
    return m


@dataclass
class MLPConfig:
    lambda_l2: float = 1e-3
    initial_lr: float = 1e-3
    final_lr: float = 1e-6
    epochs: int = 50
    batch_size: int = 32
    patience: int = 5
    weight_decay: float = 0.004
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-7
    staircase: bool = True
    monitor: str = "val_precision"
    mode: str = "max"
    restore_best_weights: bool = True
    seed: int = 0
    shuffle: bool = True

    def decay(self, n_train: int) -> tuple[float, int]:
        steps = max(1, int(n_train / self.batch_size))
        return (self.final_lr / self.initial_lr) ** (1 / 50), steps


class _Hyper(ctypes.Structure):
    _fields_ = [("lr0", ctypes.c_float), ("decay_rate", ctypes.c_float), ("decay_steps", ctypes.c_int32),
                ("staircase", ctypes.c_int32), ("weight_decay", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("l2", ctypes.c_float), ("batch", ctypes.c_int32),
                ("pad", ctypes.c_int32 * 2)]


assert ctypes.sizeof(_Hyper) == 48

_native.register("cobalt_mlp_num_params", ctypes.c_int, [ctypes.c_int])
_native.register("cobalt_mlp_train_epoch", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p])
_native.register("cobalt_mlp_train_epoch_mfma", ctypes.c_int,
                 [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p])
for _fwd in ("cobalt_mlp_forward", "cobalt_mlp_forward_mfma"):
    _native.register(_fwd, ctypes.c_int,
                     [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p, ctypes.c_void_p])


def init_params(F: int, seed: int = 0) -> np.ndarray:
    """Glorot-uniform kernels, zero biases (Keras Dense defaults), fp32 flat vector."""
    rng = np.random.default_rng(seed)
    p = np.zeros(num_params(F), dtype=np.float32)
    for name, (o, shape) in layout(F).items():
        if name.startswith("W"):
            fan_in, fan_out = (shape[0], shape[1]) if len(shape) == 2 else (shape[0], 1)
            lim = math.sqrt(6.0 / (fan_in + fan_out))
            p[o:o + int(np.prod(shape))] = rng.uniform(-lim, lim, int(np.prod(shape))).astype(np.float32)
    return p


def _unpack(p: torch.Tensor, F: int) -> dict[str, torch.Tensor]:
    return {k: p[o:o + int(np.prod(s))].view(*s) for k, (o, s) in layout(F).items()}


def forward_torch(p: torch.Tensor, X: torch.Tensor, F: int) -> torch.Tensor:
    """Logits [N] (plain PyTorch; any device/dtype)."""
    w = _unpack(p, F)
    h1 = torch.relu(X @ w["W1"] + w["b1"])
    h2 = torch.relu(h1 @ w["W2"] + w["b2"])
    h3 = torch.relu(h2 @ w["W3"] + w["b3"])
    return h3 @ w["W4"] + w["b4"]


def train_epoch_torch(X: torch.Tensor, y: torch.Tensor, perm: torch.Tensor, p: torch.Tensor, m: torch.Tensor,
                      v: torch.Tensor, step: int, cfg: MLPConfig, decay_rate: float, decay_steps: int) -> tuple[int, float]:
    """One epoch of the kernel's algorithm in PyTorch (in-place on p/m/v). Returns (step, mean batch loss sum)."""
    F = X.shape[1]
    reg = torch.as_tensor(l2_mask(F), device=p.device)
    B = cfg.batch_size
    loss_sum = 0.0
    for b0 in range(0, X.shape[0], B):
        idx = perm[b0:b0 + B]
        xb, yb = X[idx], y[idx]
        pp = p.detach().clone().requires_grad_(True)
        z = forward_torch(pp, xb, F)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(z, yb)
        g, = torch.autograd.grad(loss, pp)
        loss_sum += float(loss.detach())
        with torch.no_grad():
            e = math.floor(step / decay_steps) if cfg.staircase else step / decay_steps
            lr = cfg.initial_lr * decay_rate ** e
            t = step + 1
            lr_t = lr * math.sqrt(1 - cfg.beta2 ** t) / (1 - cfg.beta1 ** t)
            g = torch.where(reg, g + 2 * cfg.lambda_l2 * p, g)
            p -= lr * cfg.weight_decay * p
            m += (g - m) * (1 - cfg.beta1)
            v += (g * g - v) * (1 - cfg.beta2)
            p -= lr_t * m / (torch.sqrt(v) + cfg.eps)
        step += 1
    return step, loss_sum


# ------------------------------------------------------------------------------------- model
@dataclass
class MLPModel:
    params: np.ndarray          # flat fp32
    n_features: int
    feature_names: list[str] | None = None
    config: dict = field(default_factory=dict)

    def predict_proba(self, X, device=None) -> np.ndarray:
        Xt = torch.as_tensor(np.asarray(X, dtype=np.float32) if not isinstance(X, torch.Tensor) else X)
        dev = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        if dev.type == "cuda":
            Xd = Xt.to(dev, torch.float32).contiguous()
            pd_ = torch.as_tensor(self.params, device=dev)
            out = torch.empty(Xd.shape[0], dtype=torch.float32, device=dev)
            mlp_forward_gpu(Xd, pd_, out)
            return out.cpu().numpy()
        z = forward_torch(torch.as_tensor(self.params), Xt.float(), self.n_features)
        return torch.sigmoid(z).numpy()

    def predict(self, X, device=None) -> np.ndarray:
        return (self.predict_proba(X, device) > 0.5).astype(np.int64)

    def save(self, path) -> None:
        from safetensors.numpy import save_file

        path = Path(path)
        meta = {"n_features": str(self.n_features), "feature_names": json.dumps(self.feature_names),
                "config": json.dumps(self.config), "architecture": "dense-128-32-16-1-relu-sigmoid"}
        save_file({"params": np.ascontiguousarray(self.params)}, str(path), metadata=meta)

    @classmethod
    def load(cls, path) -> "MLPModel":
        from safetensors import safe_open

        with safe_open(str(path), framework="numpy") as f:
            meta = f.metadata()
            p = f.get_tensor("params")
        return cls(p, int(meta["n_features"]), json.loads(meta["feature_names"]), json.loads(meta["config"]))


def mlp_forward_gpu(X: torch.Tensor, params: torch.Tensor, out_prob: torch.Tensor,
                    out_logit: torch.Tensor | None = None, kernel: str = "mfma") -> None:
    """Sigmoid probabilities (and optionally logits) of fp32 rows ``X`` [N, F] (row stride free, unit
    column stride). ``kernel="mfma"`` (default): every layer on fp32 MFMA with activations in
    registers; ``"fma"``: the LDS-tiled scalar-FMA forward shared with the training kernel."""
    if kernel not in ("mfma", "fma"):
        raise ValueError(f"kernel must be 'mfma' or 'fma', got {kernel!r}")
    N, F = X.shape
    if X.dtype != torch.float32 or X.stride(1) != 1 or params.dtype != torch.float32 or not params.is_contiguous():
        raise ValueError("mlp_forward_gpu needs fp32 X with unit column stride and contiguous fp32 params")
    if params.numel() != num_params(F) or out_prob.numel() < N or (out_logit is not None and out_logit.numel() < N):
        raise ValueError("mlp_forward_gpu: params / output sizes do not match X")
    lib = _native.lib()
    name = "cobalt_mlp_forward_mfma" if kernel == "mfma" else "cobalt_mlp_forward"
    rc = getattr(lib, name)(X.data_ptr(), X.stride(0), N, F, params.data_ptr(), out_prob.data_ptr(),
                            out_logit.data_ptr() if out_logit is not None else None, _native.stream_handle())
    _native.check(rc, name)


# ----------------------------------------------------------------------------------- training
def _val_metrics(y: np.ndarray, p: np.ndarray) -> dict[str, float]:
    from ..metrics.auc import roc_auc

    pred = p > 0.5
    yb = y > 0.5
    tp = float(np.sum(pred & yb))
    fp = float(np.sum(pred & ~yb))
    fn = float(np.sum(~pred & yb))
    eps = 1e-7
    q = np.clip(p.astype(np.float64), eps, 1 - eps)
    return {"val_loss": float(-np.mean(yb * np.log(q) + (~yb) * np.log(1 - q))),
            "val_accuracy": float(np.mean(pred == yb)),
            "val_Precision": tp / (tp + fp) if tp + fp > 0 else 0.0,
            "val_Recall": tp / (tp + fn) if tp + fn > 0 else 0.0,
            "val_AUC": float(roc_auc(y, p)) if 0 < yb.sum() < len(yb) else float("nan")}


def fit_many(X_train, y_train, X_val=None, y_val=None, cfg: MLPConfig | None = None, seeds=(0,),
             device=None, feature_names=None, kernel: str | None = None) -> tuple[list[MLPModel], list[dict]]:
    """Train ``len(seeds)`` independent models (same data, different init/shuffle seeds).

    On the GPU all models train in the same launch (one workgroup each). ``kernel``: ``"mfma"``
    (default for F <= 31: 4 waves per model, every contraction on fp32 MFMA) or ``"fma"`` (1024
    threads per model, scalar FMA through LDS)."""
    cfg = cfg or MLPConfig()
    X = np.ascontiguousarray(np.asarray(X_train, dtype=np.float32))
    y = np.asarray(y_train, dtype=np.float32).reshape(-1)
    N, F = X.shape
    if F > MAX_F:
        raise ValueError(f"at most {MAX_F} input features")
    kernel = kernel or ("mfma" if F <= MAX_F_MFMA else "fma")
    if kernel not in ("mfma", "fma") or (kernel == "mfma" and F > MAX_F_MFMA):
        raise ValueError(f"kernel must be 'fma' or 'mfma' (F <= {MAX_F_MFMA}), got {kernel!r} at F={F}")
    G = len(seeds)
    dev = torch.device(device) if device is not None else (
        torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    rate, dsteps = cfg.decay(N)
    P = num_params(F)
    p0 = np.stack([init_params(F, s) for s in seeds])
    hist = [{"loss": []} for _ in range(G)]
    best = [None] * G
    best_val = [-math.inf if cfg.mode == "max" else math.inf] * G
    wait = [0] * G
    stopped = [False] * G
    rngs = [np.random.RandomState(s) for s in seeds]
    nb = -(-N // cfg.batch_size)
    Xv = None if X_val is None else np.ascontiguousarray(np.asarray(X_val, dtype=np.float32))
    yv = None if y_val is None else np.asarray(y_val, dtype=np.float32).reshape(-1)

    if dev.type == "cuda":
        lib = _native.lib()
        Xd, yd = torch.as_tensor(X, device=dev), torch.as_tensor(y, device=dev)
        pd_ = torch.as_tensor(p0, device=dev).contiguous()
        md = torch.zeros_like(pd_)
        vd = torch.zeros_like(pd_)
        steps = torch.zeros(G, dtype=torch.int64, device=dev)
        loss = torch.zeros(G, dtype=torch.float32, device=dev)
        hp = _Hyper(cfg.initial_lr, rate, dsteps, int(cfg.staircase), cfg.weight_decay, cfg.beta1, cfg.beta2,
                    cfg.eps, cfg.lambda_l2, cfg.batch_size)
        Xvd = torch.as_tensor(Xv, device=dev) if Xv is not None else None
    else:
        Xd, yd = torch.as_tensor(X), torch.as_tensor(y)
        pt = [torch.as_tensor(p0[g].copy()) for g in range(G)]
        mt = [torch.zeros(P) for _ in range(G)]
        vt = [torch.zeros(P) for _ in range(G)]
        st = [0] * G

    for ep in range(cfg.epochs):
        if all(stopped):
            break
        perms = np.stack([r.permutation(N) if cfg.shuffle else np.arange(N) for r in rngs]).astype(np.int32)
        if dev.type == "cuda":
            permd = torch.as_tensor(perms, device=dev)
            if kernel == "mfma":
                rc = lib.cobalt_mlp_train_epoch_mfma(Xd.data_ptr(), F, yd.data_ptr(), N, F, permd.data_ptr(),
                                                     pd_.data_ptr(), md.data_ptr(), vd.data_ptr(), steps.data_ptr(),
                                                     ctypes.byref(hp), G, loss.data_ptr(), None,
                                                     _native.stream_handle())
            else:
                rc = lib.cobalt_mlp_train_epoch(Xd.data_ptr(), F, yd.data_ptr(), N, F, permd.data_ptr(),
                                                pd_.data_ptr(), md.data_ptr(), vd.data_ptr(), steps.data_ptr(),
                                                ctypes.byref(hp), G, loss.data_ptr(), None, _native.stream_handle())
            _native.check(rc, f"mlp train epoch ({kernel})")
            losses = (loss / nb).cpu().numpy()
            cur = pd_.cpu().numpy()
        else:
            losses = []
            for g in range(G):
                st[g], ls = train_epoch_torch(Xd, yd, torch.as_tensor(perms[g], dtype=torch.int64), pt[g], mt[g],
                                              vt[g], st[g], cfg, rate, dsteps)
                losses.append(ls / nb)
            cur = np.stack([t.numpy() for t in pt])
        for g in range(G):
            if stopped[g]:
                continue
            h = hist[g]
            h["loss"].append(float(losses[g]))
            if Xv is not None:
                if dev.type == "cuda":
                    out = torch.empty(Xv.shape[0], dtype=torch.float32, device=dev)
                    mlp_forward_gpu(Xvd, pd_[g], out)
                    pv = out.cpu().numpy()
                else:
                    pv = torch.sigmoid(forward_torch(torch.as_tensor(cur[g]), torch.as_tensor(Xv), F)).numpy()
                for k, val in _val_metrics(yv, pv).items():
                    h.setdefault(k, []).append(val)
            if cfg.monitor in h:
                val = h[cfg.monitor][-1]
                better = val > best_val[g] if cfg.mode == "max" else val < best_val[g]
                if better:
                    best_val[g], best[g], wait[g] = val, cur[g].copy(), 0
                else:
                    wait[g] += 1
                    if wait[g] >= cfg.patience:
                        stopped[g] = True
                        h["stopped_epoch"] = ep
            elif ep == 0 and g == 0:
                log.warning("Early stopping conditioned on metric `%s` which is not available. Available metrics "
                            "are: %s", cfg.monitor, ",".join(h))
        log.info("epoch %d/%d loss %s", ep + 1, cfg.epochs, np.round(losses, 4).tolist())
    models = []
    for g in range(G):
        params = best[g] if (cfg.restore_best_weights and best[g] is not None) else cur[g]
        models.append(MLPModel(np.asarray(params, dtype=np.float32).copy(), F,
                               list(feature_names) if feature_names is not None else None, asdict(cfg)))
    return models, hist


def build_and_train_nn(X_train, y_train, X_val, y_val, input_dim=None, lambda_l2=0.001, initial_lr=0.001,
                       final_lr=1e-6, epochs=50, batch_size=32, patience=5, seed: int = 0, device=None,
                       feature_names=None) -> tuple[MLPModel, dict]:
    """The notebook's function signature (cell 39); returns (model, history)."""
    cfg = MLPConfig(lambda_l2=lambda_l2, initial_lr=initial_lr, final_lr=final_lr, epochs=epochs,
                    batch_size=batch_size, patience=patience, seed=seed)
    if input_dim is not None and input_dim != np.asarray(X_train).shape[1]:
        raise ValueError("input_dim must equal the number of columns")
    models, hists = fit_many(X_train, y_train, X_val, y_val, cfg, seeds=(seed,), device=device,
                             feature_names=feature_names)
    return models[0], hists[0]
