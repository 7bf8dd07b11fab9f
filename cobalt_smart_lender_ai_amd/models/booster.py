"""Tree-ensemble model in the XGBoost 3.0 layout, with checkpoint I/O and inference entry points.

The reference's model artifact is a joblib pickle of ``xgboost.sklearn.XGBClassifier`` whose
``_Booster.handle`` is a UBJSON document (src/model_train_test/
model_tree_train_test.py:215-219; src/api/cobalt_fast_api.py:45). :class:`Booster` holds the same
per-tree arrays (``left_children``, ``right_children``, ``parents``, ``split_indices``,
``split_conditions``, ``default_left``, ``base_weights``, ``loss_changes``, ``sum_hessian``) and
reads/writes that document, so artifacts move both ways between this framework and XGBoost.

Inference (`predict`, `shap_values`) dispatches on device: CUDA tensors / ``device="cuda"`` run the
gfx950 kernels in ``ops/predict_ops.py``; ``device="cpu"`` runs the NumPy reference implementation
(`predict_margin_host`, `treeshap_host`), which is also the oracle of the GPU tests.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Iterable, Sequence

import numpy as np

from ..dataio import safe_pickle, ubjson

ROOT_PARENT = 2147483647


def _fmt_float(x: float) -> str:
    """XGBoost writes float parameters with up to 9 significant digits ('0.0500000007')."""
    if x == int(x) and abs(x) < 1e15:
        return str(int(x))
    return f"{np.float32(x):.9g}"


@dataclass
class Tree:
    left_children: np.ndarray      # int32 [n]; -1 for leaves
    right_children: np.ndarray     # int32 [n]
    parents: np.ndarray            # int32 [n]; root = 2147483647
    split_indices: np.ndarray      # int32 [n]
    split_conditions: np.ndarray   # float32 [n]; leaf value for leaves
    default_left: np.ndarray       # uint8 [n]
    base_weights: np.ndarray       # float32 [n]
    loss_changes: np.ndarray       # float32 [n]
    sum_hessian: np.ndarray        # float32 [n]

    @property
    def num_nodes(self) -> int:
        return int(self.left_children.shape[0])

    @property
    def is_leaf(self) -> np.ndarray:
        return self.left_children == -1

    def depth(self) -> int:
        d = np.zeros(self.num_nodes, dtype=np.int32)
        for i in range(1, self.num_nodes):
            d[i] = d[self.parents[i]] + 1
        return int(d.max()) if self.num_nodes else 0

    def to_doc(self, tree_id: int, num_feature: int) -> dict[str, Any]:
        n = self.num_nodes
        return {
            "base_weights": self.base_weights.astype(np.float32),
            "categories": np.zeros(0, dtype=np.int32),
            "categories_nodes": np.zeros(0, dtype=np.int32),
            "categories_segments": np.zeros(0, dtype=np.int64),
            "categories_sizes": np.zeros(0, dtype=np.int64),
            "default_left": self.default_left.astype(np.uint8),
            "id": int(tree_id),
            "left_children": self.left_children.astype(np.int32),
            "loss_changes": self.loss_changes.astype(np.float32),
            "parents": self.parents.astype(np.int32),
            "right_children": self.right_children.astype(np.int32),
            "split_conditions": self.split_conditions.astype(np.float32),
            "split_indices": self.split_indices.astype(np.int32),
            "split_type": np.zeros(n, dtype=np.uint8),
            "sum_hessian": self.sum_hessian.astype(np.float32),
            "tree_param": {"num_deleted": "0", "num_feature": str(num_feature), "num_nodes": str(n),
                           "size_leaf_vector": "1"},
        }

    @classmethod
    def from_doc(cls, d: dict[str, Any]) -> "Tree":
        def arr(k, dt):
            v = d[k]
            return np.asarray(v, dtype=dt).copy()

        if np.asarray(d.get("split_type", [])).any():
            raise NotImplementedError("categorical splits are not used by the credit-risk models")
        return cls(
            left_children=arr("left_children", np.int32),
            right_children=arr("right_children", np.int32),
            parents=arr("parents", np.int32),
            split_indices=arr("split_indices", np.int32),
            split_conditions=arr("split_conditions", np.float32),
            default_left=arr("default_left", np.uint8),
            base_weights=arr("base_weights", np.float32),
            loss_changes=arr("loss_changes", np.float32),
            sum_hessian=arr("sum_hessian", np.float32),
        )


def _logit(p: float) -> float:
    p = min(max(p, 1e-16), 1 - 1e-16)
    return math.log(p / (1 - p))


@dataclass
class Booster:
    """An additive ensemble of regression trees for ``binary:logistic`` (XGBoost ``gbtree``)."""

    trees: list[Tree]
    feature_names: list[str] | None = None
    feature_types: list[str] | None = None
    base_score: float = 0.5
    num_feature: int = 0
    objective: str = "binary:logistic"
    train_params: dict[str, Any] = field(default_factory=dict)
    attributes: dict[str, str] = field(default_factory=dict)
    # the "Config" section of a loaded model, re-emitted verbatim while the forest is unchanged
    source_config: dict[str, Any] | None = field(default=None, repr=False, compare=False)

    # --------------------------------------------------------------------------------- basics
    @property
    def base_margin(self) -> float:
        """Margin-space intercept: logit(base_score) for binary:logistic, as float32."""
        if self.objective == "binary:logistic":
            return float(np.float32(_logit(float(self.base_score))))
        return float(np.float32(self.base_score))

    @property
    def num_trees(self) -> int:
        return len(self.trees)

    def slice(self, n_trees: int) -> "Booster":
        return Booster(self.trees[:n_trees], self.feature_names, self.feature_types, self.base_score,
                       self.num_feature, self.objective, dict(self.train_params), dict(self.attributes))

    def max_depth(self) -> int:
        return max((t.depth() for t in self.trees), default=0)

    # ------------------------------------------------------------------------- importance
    def get_score(self, importance_type: str = "weight") -> dict[str, float]:
        """Per-feature importance with XGBoost's ``Booster.get_score`` semantics.

        Used by ``/feature_importance_bulk`` (reference: src/api/cobalt_fast_api.py:128-143).
        """
        F = self.num_feature
        weight = np.zeros(F, dtype=np.float64)
        gain = np.zeros(F, dtype=np.float64)
        cover = np.zeros(F, dtype=np.float64)
        for t in self.trees:
            m = ~t.is_leaf
            f = t.split_indices[m]
            np.add.at(weight, f, 1.0)
            np.add.at(gain, f, t.loss_changes[m].astype(np.float64))
            np.add.at(cover, f, t.sum_hessian[m].astype(np.float64))
        names = self.feature_names or [f"f{i}" for i in range(F)]
        out: dict[str, float] = {}
        for i in range(F):
            if weight[i] == 0:
                continue
            if importance_type == "weight":
                v = weight[i]
            elif importance_type == "gain":
                v = gain[i] / weight[i]
            elif importance_type == "total_gain":
                v = gain[i]
            elif importance_type == "cover":
                v = cover[i] / weight[i]
            elif importance_type == "total_cover":
                v = cover[i]
            else:
                raise ValueError(f"unknown importance_type {importance_type!r}")
            out[names[i]] = float(v)
        return out

    def feature_importances(self, importance_type: str = "gain") -> np.ndarray:
        """sklearn ``feature_importances_``: normalised per-feature score (0 for unused features)."""
        sc = self.get_score(importance_type)
        names = self.feature_names or [f"f{i}" for i in range(self.num_feature)]
        v = np.array([sc.get(n, 0.0) for n in names], dtype=np.float32)
        s = v.sum()
        return v / s if s > 0 else v

    # ------------------------------------------------------------------------- inference
    def predict_margin(self, X, device: str | None = None, n_trees: int | None = None):
        """Raw margins (base margin + sum of leaf values). ``X``: [N, F] float array/tensor."""
        from ..ops import predict_ops

        return predict_ops.predict_margin(self, X, device=device, n_trees=n_trees)

    def predict_proba(self, X, device: str | None = None):
        from ..ops import predict_ops

        return predict_ops.predict_proba(self, X, device=device)

    def shap_values(self, X, device: str | None = None):
        """Path-dependent TreeSHAP values [N, F] (+ expected value via :meth:`expected_value`)."""
        from ..ops import predict_ops

        return predict_ops.shap_values(self, X, device=device)

    def expected_value(self) -> float:
        """TreeExplainer ``expected_value``: base margin + cover-weighted mean leaf value per tree."""
        tot = 0.0
        for t in self.trees:
            leaf = t.is_leaf
            cov = t.sum_hessian.astype(np.float64)
            tot += float(np.sum(cov[leaf] * t.split_conditions[leaf].astype(np.float64)) / cov[0])
        return self.base_margin + tot

    # ------------------------------------------------------------------- XGBoost document
    def _config_doc(self) -> dict[str, Any]:
        p = {"eta": 0.3, "gamma": 0.0, "max_depth": 6, "min_child_weight": 1.0, "reg_lambda": 1.0,
             "reg_alpha": 0.0, "subsample": 1.0, "colsample_bytree": 1.0, "max_bin": 256,
             "scale_pos_weight": 1.0, "seed": 0}
        p.update({k: v for k, v in self.train_params.items() if v is not None})
        f = _fmt_float
        return {
            "learner": {
                "generic_param": {"device": "cpu", "fail_on_invalid_gpu_id": "0", "n_jobs": "0", "nthread": "0",
                                  "random_state": str(int(p["seed"])), "seed": str(int(p["seed"])),
                                  "seed_per_iteration": "0", "validate_parameters": "1"},
                "gradient_booster": {
                    "gbtree_model_param": {"num_parallel_tree": "1", "num_trees": str(self.num_trees)},
                    "gbtree_train_param": {"process_type": "default", "tree_method": "hist",
                                           "updater": "grow_quantile_histmaker",
                                           "updater_seq": "grow_quantile_histmaker"},
                    "name": "gbtree",
                    "specified_updater": False,
                    "tree_train_param": {
                        "alpha": f(p["reg_alpha"]), "cache_opt": "1", "colsample_bylevel": "1",
                        "colsample_bynode": "1", "colsample_bytree": f(p["colsample_bytree"]), "eta": f(p["eta"]),
                        "gamma": f(p["gamma"]), "grow_policy": "depthwise", "interaction_constraints": "",
                        "lambda": f(p["reg_lambda"]), "learning_rate": f(p["eta"]), "max_bin": str(int(p["max_bin"])),
                        "max_cat_threshold": "64", "max_cat_to_onehot": "4", "max_delta_step": "0",
                        "max_depth": str(int(p["max_depth"])), "max_leaves": "0",
                        "min_child_weight": f(p["min_child_weight"]), "min_split_loss": f(p["gamma"]),
                        "monotone_constraints": "()", "refresh_leaf": "1", "reg_alpha": f(p["reg_alpha"]),
                        "reg_lambda": f(p["reg_lambda"]), "sampling_method": "uniform", "sketch_ratio": "2",
                        "sparse_threshold": "0.20000000000000001", "subsample": f(p["subsample"])},
                    "updater": [{"hist_train_param": {"debug_synchronize": "0", "extmem_single_page": "0",
                                                      "max_cached_hist_node": "18446744073709551615"},
                                 "name": "grow_quantile_histmaker"}],
                },
                "learner_model_param": self._lmp(),
                "learner_train_param": {"booster": "gbtree", "disable_default_eval_metric": "0",
                                        "multi_strategy": "one_output_per_tree", "objective": self.objective},
                "metrics": [{"name": "logloss"}],
                "objective": {"name": self.objective,
                              "reg_loss_param": {"scale_pos_weight": f(p["scale_pos_weight"])}},
            },
            "version": [3, 0, 0],
        }

    def _lmp(self) -> dict[str, str]:
        bs = np.format_float_scientific(np.float32(self.base_score), unique=True, exp_digits=1).upper()
        bs = bs.replace("E+", "E")
        if "." in bs:
            mant, ex = bs.split("E")
            mant = mant.rstrip("0").rstrip(".")
            bs = f"{mant}E{ex}"
        return {"base_score": bs, "boost_from_average": "1", "num_class": "0",
                "num_feature": str(self.num_feature), "num_target": "1"}

    def to_doc(self) -> dict[str, Any]:
        spw = self.train_params.get("scale_pos_weight", 1.0)
        model = {
            "learner": {
                "attributes": dict(self.attributes),
                "feature_names": list(self.feature_names or []),
                "feature_types": list(self.feature_types or []),
                "gradient_booster": {
                    "model": {
                        "gbtree_model_param": {"num_parallel_tree": "1", "num_trees": str(self.num_trees)},
                        "iteration_indptr": list(range(self.num_trees + 1)),
                        "tree_info": [0] * self.num_trees,
                        "trees": [t.to_doc(i, self.num_feature) for i, t in enumerate(self.trees)],
                    },
                    "name": "gbtree",
                },
                "learner_model_param": self._lmp(),
                "objective": {"name": self.objective,
                              "reg_loss_param": {"scale_pos_weight": _fmt_float(spw if spw is not None else 1.0)}},
            },
            "version": [3, 0, 0],
        }
        cfg = self.source_config
        if cfg is None or cfg.get("learner", {}).get("gradient_booster", {}).get("gbtree_model_param", {}).get(
                "num_trees") != str(self.num_trees):
            cfg = self._config_doc()
        return {"Config": cfg, "Model": model}

    @classmethod
    def from_doc(cls, doc: dict[str, Any]) -> "Booster":
        model = doc["Model"] if "Model" in doc else doc
        lrn = model["learner"]
        gb = lrn["gradient_booster"]
        if gb.get("name", "gbtree") != "gbtree":
            raise NotImplementedError(f"booster {gb.get('name')!r} not supported")
        trees = [Tree.from_doc(t) for t in gb["model"]["trees"]]
        lmp = lrn["learner_model_param"]
        obj = lrn.get("objective", {}).get("name", "binary:logistic")
        params: dict[str, Any] = {}
        cfg = doc.get("Config", {}).get("learner", {})
        ttp = cfg.get("gradient_booster", {}).get("tree_train_param", {})
        for src, dst, typ in (("eta", "eta", float), ("gamma", "gamma", float), ("max_depth", "max_depth", int),
                              ("min_child_weight", "min_child_weight", float), ("lambda", "reg_lambda", float),
                              ("alpha", "reg_alpha", float), ("subsample", "subsample", float),
                              ("colsample_bytree", "colsample_bytree", float), ("max_bin", "max_bin", int)):
            if src in ttp:
                params[dst] = typ(float(ttp[src]))
        spw = lrn.get("objective", {}).get("reg_loss_param", {}).get("scale_pos_weight")
        if spw is not None:
            params["scale_pos_weight"] = float(spw)
        seed = cfg.get("generic_param", {}).get("seed")
        if seed is not None:
            params["seed"] = int(seed)
        return cls(trees=trees,
                   feature_names=list(lrn.get("feature_names") or []) or None,
                   feature_types=list(lrn.get("feature_types") or []) or None,
                   base_score=float(np.float32(lmp.get("base_score", "0.5"))),
                   num_feature=int(lmp.get("num_feature", "0")),
                   objective=obj, train_params=params,
                   attributes=dict(lrn.get("attributes") or {}),
                   source_config=doc.get("Config"))

    # --------------------------------------------------------------------------- file I/O
    def save_raw(self, fmt: str = "ubj") -> bytes:
        if fmt == "ubj":
            return ubjson.dumps(self.to_doc())
        if fmt == "json":
            return json.dumps(_jsonable(self.to_doc())).encode()
        raise ValueError(fmt)

    @classmethod
    def load_raw(cls, raw: bytes) -> "Booster":
        raw = bytes(raw)
        if raw[:1] == b"{" and raw[1:2] in (b'"', b" ", b"\n"):
            return cls.from_doc(json.loads(raw.decode()))
        return cls.from_doc(ubjson.loads(raw))

    def save_model(self, path: str | Path) -> None:
        path = Path(path)
        fmt = "json" if path.suffix == ".json" else "ubj"
        path.write_bytes(self.save_raw(fmt))

    @classmethod
    def load_model(cls, path: str | Path) -> "Booster":
        p = Path(path)
        data = p.read_bytes()
        if p.suffix in (".pkl", ".pickle", ".joblib") or data[:1] == b"\x80":
            return load_pickle_bytes(data)[1]
        return cls.load_raw(data)


def _jsonable(v: Any) -> Any:
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


# ---------------------------------------------------------------------------- pickle checkpoint

def sklearn_state(params: dict[str, Any], n_classes: int = 2) -> dict[str, Any]:
    """The XGBClassifier ``__dict__`` in the reference checkpoint's key order."""
    keys = ["n_estimators", "objective", "max_depth", "max_leaves", "max_bin", "grow_policy", "learning_rate",
            "verbosity", "booster", "tree_method", "gamma", "min_child_weight", "max_delta_step", "subsample",
            "sampling_method", "colsample_bytree", "colsample_bylevel", "colsample_bynode", "reg_alpha",
            "reg_lambda", "scale_pos_weight", "base_score", "missing", "num_parallel_tree", "random_state",
            "n_jobs", "monotone_constraints", "interaction_constraints", "importance_type", "device",
            "validate_parameters", "enable_categorical", "feature_types", "feature_weights", "max_cat_to_onehot",
            "max_cat_threshold", "multi_strategy", "eval_metric", "early_stopping_rounds", "callbacks", "kwargs"]
    st: dict[str, Any] = {k: None for k in keys}
    st["objective"] = "binary:logistic"
    st["missing"] = float("nan")
    st["enable_categorical"] = False
    st["kwargs"] = {}
    for k, v in params.items():
        if k in st:
            st[k] = v
    if st.get("scale_pos_weight") is not None:
        st["scale_pos_weight"] = np.float64(st["scale_pos_weight"])
    st["n_classes_"] = n_classes
    return st


def dump_pickle_bytes(booster: Booster, sk_params: dict[str, Any]) -> bytes:
    return safe_pickle.encode_xgb_classifier(sklearn_state(sk_params), booster.save_raw("ubj"))


def load_pickle_bytes(data: bytes) -> tuple[dict[str, Any], Booster]:
    """Load an ``XGBClassifier`` pickle statically (nothing in the file is executed)."""
    st, raw = safe_pickle.read_xgb_classifier_pickle(data)
    return st, Booster.load_raw(raw)


# ------------------------------------------------------------------------ host reference paths

def predict_margin_host(b: Booster, X: np.ndarray, n_trees: int | None = None) -> np.ndarray:
    """NumPy reference traversal: ``x < cond`` goes left, NaN takes ``default_left``; fp32 sums in
    tree order starting from the base margin (XGBoost CPU predictor semantics)."""
    X = np.asarray(X, dtype=np.float32)
    N = X.shape[0]
    out = np.full(N, np.float32(b.base_margin), dtype=np.float32)
    rows = np.arange(N)
    for t in b.trees[: (n_trees if n_trees is not None else b.num_trees)]:
        nid = np.zeros(N, dtype=np.int32)
        while True:
            lc = t.left_children[nid]
            active = lc != -1
            if not active.any():
                break
            f = t.split_indices[nid]
            v = X[rows, np.where(active, f, 0)]
            c = t.split_conditions[nid]
            go_left = np.where(np.isnan(v), t.default_left[nid] == 1, v < c)
            nxt = np.where(go_left, lc, t.right_children[nid])
            nid = np.where(active, nxt, nid)
        out = (out + t.split_conditions[nid]).astype(np.float32)
    return out


def sigmoid32(m: np.ndarray) -> np.ndarray:
    m = np.asarray(m, dtype=np.float32)
    return (np.float32(1.0) / (np.float32(1.0) + np.exp(-m))).astype(np.float32)


def treeshap_host(b: Booster, X: np.ndarray) -> np.ndarray:
    """Exact path-dependent TreeSHAP (Lundberg et al., Algorithm 2) in NumPy; oracle for the GPU kernel.

    Reproduces ``shap.TreeExplainer(model).shap_values(X)`` for XGBoost models (node covers =
    ``sum_hessian``), as called by the reference at src/api/cobalt_fast_api.py:46,100.
    """
    X = np.asarray(X, dtype=np.float32)
    N, F = X.shape
    phi = np.zeros((N, F), dtype=np.float64)
    for t in b.trees:
        cov = t.sum_hessian.astype(np.float64)
        val = t.split_conditions.astype(np.float64)
        for r in range(N):
            _treeshap_row(t, cov, val, X[r], phi[r])
    return phi


def _treeshap_row(t: Tree, cov, val, x, phi) -> None:
    # path entries: feature index, zero fraction, one fraction, pweight
    def extend(m, pz, po, pi):
        feats, zs, os_, ws = m
        l = len(feats)
        feats = feats + [pi]
        zs = zs + [pz]
        os_ = os_ + [po]
        ws = ws + [1.0 if l == 0 else 0.0]
        for i in range(l - 1, -1, -1):
            ws[i + 1] += po * ws[i] * (i + 1) / (l + 1)
            ws[i] = pz * ws[i] * (l - i) / (l + 1)
        return feats, zs, os_, ws

    def unwind(m, i):
        feats, zs, os_, ws = m
        l = len(feats) - 1
        n = ws[l]
        ws = list(ws)
        if os_[i] != 0:
            for j in range(l - 1, -1, -1):
                tmp = ws[j]
                ws[j] = n * (l + 1) / ((j + 1) * os_[i])
                n = tmp - ws[j] * zs[i] * (l - j) / (l + 1)
        else:
            for j in range(l - 1, -1, -1):
                ws[j] = (ws[j] * (l + 1)) / (zs[i] * (l - j))
        feats = feats[:i] + feats[i + 1:]
        zs = zs[:i] + zs[i + 1:]
        os_ = os_[:i] + os_[i + 1:]
        ws = ws[:l]
        return feats, zs, os_, ws

    def unwound_sum(m, i):
        feats, zs, os_, ws = m
        l = len(feats) - 1
        total = 0.0
        if os_[i] != 0:
            n = ws[l]
            for j in range(l - 1, -1, -1):
                tmp = n / ((j + 1) * os_[i])
                total += tmp
                n = ws[j] - tmp * zs[i] * (l - j)
            return total * (l + 1)
        for j in range(l - 1, -1, -1):
            total += ws[j] / (zs[i] * (l - j))
        return total * (l + 1)

    def recurse(j, m, pz, po, pi):
        m = extend(m, pz, po, pi)
        if t.left_children[j] == -1:
            feats, zs, os_, ws = m
            for i in range(1, len(feats)):
                w = unwound_sum(m, i)
                phi[feats[i]] += w * (os_[i] - zs[i]) * val[j]
            return
        f = int(t.split_indices[j])
        v = x[f]
        left, right = int(t.left_children[j]), int(t.right_children[j])
        if np.isnan(v):
            hot = left if t.default_left[j] else right
        else:
            hot = left if v < t.split_conditions[j] else right
        cold = right if hot == left else left
        iz, io = 1.0, 1.0
        feats = m[0]
        k = next((q for q in range(1, len(feats)) if feats[q] == f), None)
        if k is not None:
            iz, io = m[1][k], m[2][k]
            m = unwind(m, k)
        recurse(hot, m, iz * cov[hot] / cov[j], io, f)
        recurse(cold, m, iz * cov[cold] / cov[j], 0.0, f)

    recurse(0, ([], [], [], []), 1.0, 1.0, -1)


def iter_leaf_paths(t: Tree) -> Iterable[tuple[int, list[tuple[int, int, bool]]]]:
    """Yield (leaf node, [(node, feature, went_left)]) for every root->leaf path."""
    stack = [(0, [])]
    while stack:
        j, path = stack.pop()
        if t.left_children[j] == -1:
            yield j, path
            continue
        f = int(t.split_indices[j])
        stack.append((int(t.right_children[j]), path + [(j, f, False)]))
        stack.append((int(t.left_children[j]), path + [(j, f, True)]))


def trees_from_heap_nodes(nodes: np.ndarray, max_depth: int, native: bool | None = None) -> list[Tree]:
    """Convert heap-ordered node records (NODE_DTYPE, [T, 2^(D+1)-1]) of the trainer into XGBoost
    trees, numbering nodes in XGBoost's depthwise creation order (children allocated in pairs).

    ``native`` (default: whenever the native library is loadable): the one-pass C++ conversion
    (``csrc/treeconv.cpp``, ~0.1 ms for 300 trees); False: the NumPy form below (its oracle)."""
    if native is not False and nodes.ndim == 2 and nodes.shape[0] > 0:
        out = _trees_from_heap_nodes_native(nodes, required=native is True)
        if out is not None:
            return out
    # Heap indices of one level are contiguous and children are allocated in parent order, so the
    # depthwise creation order is simply ascending heap index over the live nodes.
    # Everything is computed for all trees at once and split per tree at the end.
    if nodes.ndim != 2 or nodes.shape[0] == 0:
        return []
    T, M = nodes.shape
    status = nodes["status"]
    live = (status == 2) | (status == 3)
    new_id = (np.cumsum(live, axis=1) - 1).astype(np.int32)       # per-tree position of each live node
    counts = live.sum(1)
    split_full = status == 2
    kid = np.minimum(2 * np.arange(M) + 1, M - 2)
    lc_full = np.where(split_full, new_id[:, kid], -1).astype(np.int32)
    rc_full = np.where(split_full, new_id[:, kid + 1], -1).astype(np.int32)
    par_full = np.full((T, M), ROOT_PARENT, np.int32)
    parent_heap = (np.arange(M) - 1) // 2
    has_par = np.arange(M) > 0
    par_full[:, has_par] = new_id[:, parent_heap[has_par]]
    # the live records gathered as 64-byte rows of an int32 view (a boolean mask on the structured
    # array copied field by field: ~4 ms for 300 trees)
    words = np.ascontiguousarray(nodes).reshape(-1).view(np.int32).reshape(-1, NODE_DTYPE.itemsize // 4)
    r = words[np.flatnonzero(live.reshape(-1))].view(NODE_DTYPE).reshape(-1)
    split = r["status"] == 2
    lc, rc, par = lc_full[live], rc_full[live], par_full[live]
    si = np.where(split, r["feat"], 0).astype(np.int32)
    sc = np.where(split, r["split_cond"], r["leaf_value"]).astype(np.float32)
    dl = np.where(split, r["default_left"], 0).astype(np.uint8)
    lo = np.where(split, r["loss_chg"], 0).astype(np.float32)
    bw = r["base_weight"].astype(np.float32)
    sh = r["sum_hess"].astype(np.float32)
    # per-tree views by offsets (np.split's per-piece swapaxes cost ~9 ms for 300 x 9 arrays)
    ends = np.cumsum(counts).tolist()
    begins = [0] + ends[:-1]
    cols = (lc, rc, par, si, sc, dl, bw, lo, sh)
    return [Tree(*(a[b0:b1] for a in cols)) for b0, b1 in zip(begins, ends)]


def _trees_from_heap_nodes_native(nodes: np.ndarray, required: bool = False) -> list[Tree] | None:
    try:
        from .. import _native

        lib = _native.lib()
    except Exception:  # noqa: BLE001 -- no native library (source-only CPU install): NumPy path
        if required:
            raise
        return None
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    T, M = nodes.shape
    cap = T * M
    counts = np.empty(T, np.int32)
    cols = [np.empty(cap, dt) for dt in (np.int32, np.int32, np.int32, np.int32, np.float32, np.uint8,
                                         np.float32, np.float32, np.float32)]
    lc, rc, par, si, sc, dl, bw, lo, sh = cols
    n = lib.cobalt_heap_to_trees(nodes.ctypes.data, T, M, counts.ctypes.data,
                                 *(a.ctypes.data for a in cols))
    if n < 0:
        raise RuntimeError("cobalt_heap_to_trees: bad arguments")
    ends = np.cumsum(counts).tolist()
    begins = [0] + ends[:-1]
    # Tree fields in their declared order: left, right, parents, split_indices, split_conditions,
    # default_left, base_weights, loss_changes, sum_hessian
    order = (lc, rc, par, si, sc, dl, bw, lo, sh)
    spans = list(zip(begins, ends))
    per_col = [[a[b0:b1] for b0, b1 in spans] for a in order]
    return [Tree(*parts) for parts in zip(*per_col)]


NODE_DTYPE = np.dtype([
    ("G", "<i8"), ("H", "<i8"), ("start", "<i4"), ("count", "<i4"), ("status", "<i4"), ("build", "<i4"),
    ("feat", "<i4"), ("bin", "<i4"), ("default_left", "<i4"), ("split_cond", "<f4"), ("loss_chg", "<f4"),
    ("leaf_value", "<f4"), ("sum_hess", "<f4"), ("base_weight", "<f4"),
])
assert NODE_DTYPE.itemsize == 64


def concat_feature_names(names: Sequence[str] | None, F: int) -> list[str]:
    return list(names) if names is not None else [f"f{i}" for i in range(F)]
