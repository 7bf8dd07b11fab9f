"""FastAPI scoring service with the reference's REST contract (src/api/cobalt_fast_api.py).

Routes (identical paths, request schemas, response keys and error codes):

* ``POST /predict``                 -- one borrower (20 fields, two of them via the aliases
  ``"application_type_Joint App"`` / ``"hardship_status_No Hardship"``) ->
  ``{prob_default, shap_values[20], base_value, features[20], input_row}``; micro-batched onto the
  GPU engine (hipGraph replay of predictor + TreeSHAP).
* ``POST /predict_bulk_csv``        -- multipart field ``file`` with a CSV of the 20 columns ->
  ``{"predictions": [row + prob_default]}`` with NaN/inf rendered ``"null"``; errors -> 500
  ``"Bulk prediction failed: ..."``.
* ``POST /feature_importance_bulk`` -- ``{"data": [...]}`` -> top-10 average-gain features; empty
  -> 400 ``"No data provided."``.
* ``GET /health``                   -- additive: model / device / batcher statistics.
* ``GET /metrics``                  -- additive: Prometheus exposition (request counts and latency
  histograms per route, micro-batch sizes, model info), one registry per app.

With ``COBALT_SCORER_SOCKET`` set the app holds no GPU state: it parses and validates HTTP on the CPU
and forwards rows to the one scorer process (serve/scorer.py) that owns the device, so several
uvicorn workers share one engine and one micro-batcher instead of time-slicing the GPU.

Model loading mirrors the reference lifespan (load at startup, fail fast with ``RuntimeError``) but
reads the checkpoint with the static, non-executing pickle decoder and takes the path from
``COBALT_MODEL_PATH`` (or S3 via ``COBALT_SOURCE=s3`` when boto3 is available).
"""
from __future__ import annotations

import asyncio
import io
import os
import time
import re
from contextlib import asynccontextmanager
from pathlib import Path
from typing import Dict, List

import numpy as np
import pandas as pd
from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, Response
from pydantic import BaseModel, ConfigDict, Field

from ..config import ServeConfig, from_env
from ..models.booster import Booster, load_pickle_bytes
from .batcher import MicroBatcher
from .engine import ScoringEngine


class SingleInput(BaseModel):
    # Aliases are required for the two fields with spaces: the reference's pydantic-v1
    # ``allow_population_by_field_name`` is ignored under pydantic v2, so the
    # underscore spellings are rejected with 422 there too.
    model_config = ConfigDict(populate_by_name=False)

    loan_amnt: float
    term: float
    installment: float
    fico_range_low: float
    last_fico_range_high: float
    open_il_12m: float
    open_il_24m: float
    max_bal_bc: float
    num_rev_accts: float
    pub_rec_bankruptcies: float
    emp_length_num: float
    earliest_cr_line_days: float
    grade_E: int
    home_ownership_MORTGAGE: int
    verification_status_Verified: int
    application_type_Joint_App: int = Field(alias="application_type_Joint App")
    hardship_status_BROKEN: int
    hardship_status_COMPLETE: int
    hardship_status_COMPLETED: int
    hardship_status_No_Hardship: int = Field(alias="hardship_status_No Hardship")


class BulkInput(BaseModel):
    data: List[Dict]


def parse_multipart(body: bytes, content_type: str) -> dict[str, tuple[str | None, bytes]]:
    """Minimal RFC 7578 multipart/form-data parser -> {field name: (filename, payload)}."""
    m = re.search(r'boundary="?([^";]+)"?', content_type or "")
    if not m:
        raise ValueError("multipart request without boundary")
    boundary = b"--" + m.group(1).encode("latin-1")
    out: dict[str, tuple[str | None, bytes]] = {}
    for part in body.split(boundary)[1:]:
        if part.startswith(b"--"):
            break
        part = part[2:] if part.startswith(b"\r\n") else part
        head, sep, payload = part.partition(b"\r\n\r\n")
        if not sep:
            continue
        if payload.endswith(b"\r\n"):
            payload = payload[:-2]
        headers = head.decode("latin-1")
        nm = re.search(r'name="([^"]*)"', headers)
        fn = re.search(r'filename="([^"]*)"', headers)
        if nm:
            out[nm.group(1)] = (fn.group(1) if fn else None, payload)
    return out


def load_model(cfg: ServeConfig) -> Booster:
    if cfg.source == "s3":
        from ..dataio.artifacts import S3Store

        data = S3Store(cfg.s3_bucket).get_bytes(cfg.s3_model_key)
    else:
        p = Path(cfg.model_path)
        if not p.exists():
            raise FileNotFoundError(p)
        data = p.read_bytes()
    if data[:1] == b"\x80":
        return load_pickle_bytes(data)[1]
    return Booster.load_raw(data)


class _Metrics:
    """Prometheus instruments of one app (own registry, so several apps can live in one process)."""

    def __init__(self):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

        self.registry = CollectorRegistry()
        buckets = (1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1.0, 2.5)
        self.requests = Counter("cobalt_requests_total", "HTTP requests", ["route", "status"], registry=self.registry)
        self.latency = Histogram("cobalt_request_seconds", "HTTP request latency", ["route"], buckets=buckets,
                                 registry=self.registry)
        self.batch_rows = Histogram("cobalt_microbatch_rows", "rows per micro-batch of /predict",
                                    buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512), registry=self.registry)
        self.rows = Counter("cobalt_scored_rows_total", "rows scored", ["route"], registry=self.registry)
        self.model = Gauge("cobalt_model_info", "loaded model", ["trees", "features", "device"], registry=self.registry)


# Uploads at least this large are parsed by the GPU CSV reader when the engine runs on a GPU (smaller
# ones parse faster in pandas than a device round trip). Module-level so tests can move it.
GPU_CSV_MIN_BYTES = 1 << 20


def _bulk_inputs(data: bytes, feats: list, state: dict):
    """(frame, device matrix or None) of an uploaded bulk CSV. On a GPU engine a large upload is parsed
    on the device (prep/csv_gpu.py) and scored from HBM without a host copy of the features; the
    response frame is the device frame's pandas export (typed like pd.read_csv). Anything the device
    path cannot take (layout, wrong columns, non-numeric features) goes through pandas, so errors read
    exactly like the reference's (/root/reference/src/api/cobalt_fast_api.py predict_bulk_csv)."""
    eng = state.get("engine")
    dev = getattr(eng, "device", None)
    if dev is not None and dev.type == "cuda" and "remote" not in state and len(data) >= GPU_CSV_MIN_BYTES:
        try:
            import torch

            from ..prep.device_frame import DeviceFrame

            with torch.cuda.device(dev):
                # pandas' default float conversion: the echoed inputs equal pd.read_csv's bit for bit
                fr = DeviceFrame.read_csv(data, dev, engine="gpu", float_precision="high")
                if fr.columns == list(feats):
                    return fr.to_pandas(), fr.matrix(list(feats))
        except Exception:  # noqa: BLE001 -- the pandas path below reports it
            pass
    return pd.read_csv(io.BytesIO(data)), None


def _score_device(booster: Booster, Xd, lock=None) -> np.ndarray:
    """Probabilities of a device-parsed bulk upload. Serialised with the scoring engine (its lock): the
    MicroBatcher thread replays the engine's hipGraphs on the engine stream, and a bulk request must
    neither capture a graph (global capture mode forbids other threads' stream syncs and allocator
    calls meanwhile) nor run concurrently with another bulk capture. Per-request buffers are never
    captured (``capture=False``): a one-off matrix gains nothing from a graph."""
    import contextlib

    import torch

    from .batch_score import score_device_matrix

    with (lock if lock is not None else contextlib.nullcontext()), torch.cuda.device(Xd.device):
        return score_device_matrix(booster, Xd, capture=False).cpu().numpy()


def create_app(cfg: ServeConfig | None = None, booster: Booster | None = None) -> FastAPI:
    cfg = cfg or from_env(ServeConfig)
    state: dict = {}
    metrics = _Metrics()

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        try:
            bst = booster if booster is not None else load_model(cfg)
            state.update(booster=bst, expected_value=float(bst.expected_value()),
                         features=list(bst.feature_names or [f"f{i}" for i in range(bst.num_feature)]))
            if cfg.scorer_socket:
                from .scorer import RemoteScorer

                remote = RemoteScorer(cfg.scorer_socket, bst.num_feature)
                await remote.start()
                state.update(engine=None, batcher=remote, remote=remote)
                where = f"scorer {cfg.scorer_socket}"
            else:
                engine = ScoringEngine(bst, device=cfg.device, use_graphs=cfg.use_graphs)
                batcher = MicroBatcher(engine, max_batch=cfg.max_batch, max_wait_ms=cfg.max_wait_ms)
                await batcher.start()
                batcher.on_batch = lambda n: metrics.batch_rows.observe(n)
                state.update(engine=engine, batcher=batcher)
                where = str(engine.device)
            metrics.model.labels(str(bst.num_trees), str(bst.num_feature), where).set(1)
            print(f"[INFO] Model and SHAP engine ready on {where} ({bst.num_trees} trees).")
        except Exception as e:  # noqa: BLE001
            print(f"[ERROR] Model load failed: {e}")
            raise RuntimeError("Failed to load model.") from e
        yield
        await state["batcher"].stop()

    app = FastAPI(title="Cobalt XGBoost Inference API", lifespan=lifespan)
    app.state.cobalt = state
    app.state.metrics = metrics

    @app.middleware("http")
    async def observe(request: Request, call_next):
        route = request.url.path
        t0 = time.perf_counter()
        status = 500
        try:
            response = await call_next(request)
            status = response.status_code
            return response
        finally:
            if route != "/metrics":
                metrics.latency.labels(route).observe(time.perf_counter() - t0)
                metrics.requests.labels(route, str(status)).inc()

    @app.post("/predict")
    async def predict_single(input_data: SingleInput):
        row = input_data.model_dump(by_alias=True)
        feats = state["features"]
        x = np.array([float(row[f]) for f in feats], dtype=np.float32)
        prob, phi = await state["batcher"].submit(x)
        metrics.rows.labels("/predict").inc()
        # a pre-built JSONResponse skips FastAPI's generic jsonable_encoder walk (same JSON body)
        return JSONResponse({
            "prob_default": float(prob),
            "shap_values": phi.tolist(),
            "base_value": state["expected_value"],
            "features": feats,
            "input_row": {f: float(row[f]) for f in feats},
        })

    @app.post("/predict_bulk_csv")
    async def predict_bulk_csv(request: Request):
        try:
            ctype = request.headers.get("content-type", "")
            parts = parse_multipart(await request.body(), ctype)
            if "file" not in parts:
                raise ValueError("multipart field 'file' is required")
            feats = state["features"]
            loop = asyncio.get_running_loop()
            df, Xd = await loop.run_in_executor(None, _bulk_inputs, parts["file"][1], feats, state)
            if list(df.columns) != feats:
                raise ValueError(f"feature_names mismatch: expected {feats}, got {list(df.columns)}")
            # scored on a worker thread: the reference runs this blocking call on the event loop
            # (SURVEY App. B.8), which stalls every concurrent /predict request behind a bulk file
            if Xd is not None:
                df["prob_default"] = await loop.run_in_executor(None, _score_device, state["booster"], Xd,
                                                                getattr(state.get("engine"), "_lock", None))
            elif "remote" in state:
                X = df.to_numpy(dtype=np.float32, na_value=np.nan)
                df["prob_default"] = (await state["remote"].score_many(X, False))[0]
            else:
                X = df.to_numpy(dtype=np.float32, na_value=np.nan)
                df["prob_default"] = await loop.run_in_executor(None, state["engine"].predict_proba, X)
            metrics.rows.labels("/predict_bulk_csv").inc(len(df))
            df_clean = df.replace([np.inf, -np.inf], np.nan).astype(object).where(
                df.replace([np.inf, -np.inf], np.nan).notna(), "null")
            return {"predictions": df_clean.to_dict(orient="records")}
        except Exception as e:  # noqa: BLE001
            print(f"[ERROR] Bulk prediction failed: {e}")
            raise HTTPException(status_code=500, detail=f"Bulk prediction failed: {e}")

    @app.post("/feature_importance_bulk")
    def feature_importance_bulk(data: BulkInput):
        if not data.data:
            raise HTTPException(status_code=400, detail="No data provided.")
        try:
            imp = state["booster"].get_score(importance_type="gain")
            top = sorted(imp.items(), key=lambda kv: kv[1], reverse=True)[:10]
            return {"top_features": [{"feature": k, "importance": v} for k, v in top]}
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=500, detail=f"Feature importance computation failed: {e}")

    @app.get("/metrics")
    def prometheus_metrics():
        from prometheus_client import CONTENT_TYPE_LATEST, generate_latest

        return Response(generate_latest(metrics.registry), media_type=CONTENT_TYPE_LATEST)

    @app.get("/health")
    async def health():
        if "remote" in state:
            st = await state["remote"].stats()
            return {"status": "ok", "device": st["device"], "scorer": cfg.scorer_socket,
                    "trees": state["booster"].num_trees, "graphs": None, "batches": st["batches"],
                    "rows": st["rows"], "max_batch_seen": st["max_batch_seen"]}
        eng = state.get("engine")
        b = state.get("batcher")
        return {
            "status": "ok" if eng is not None else "loading",
            "device": str(eng.device) if eng else None,
            "trees": state["booster"].num_trees if "booster" in state else None,
            "graphs": bool(eng.use_graphs) if eng else None,
            "batches": b.stats.batches if b else 0,
            "rows": b.stats.rows if b else 0,
            "max_batch_seen": b.stats.max_batch_seen if b else 0,
        }

    return app
