"""Scoring API entry point -- same module path and routes as the reference service
(reference: src/api/cobalt_fast_api.py). Run with ``uvicorn cobalt_fast_api:app --port 8000`` from
this directory, or ``python cobalt_fast_api.py``.

The app is built by :func:`cobalt_smart_lender_ai_amd.serve.app.create_app`; the model comes from
``COBALT_MODEL_PATH`` (default ``models/xgb_model_tree.pkl``) or S3 with ``COBALT_SOURCE=s3``.
"""
import sys
from pathlib import Path

_ROOT = Path(__file__).resolve().parents[2]
if str(_ROOT) not in sys.path:
    sys.path.insert(0, str(_ROOT))

from cobalt_smart_lender_ai_amd.serve.app import BulkInput, SingleInput, create_app  # noqa: E402

app = create_app()

if __name__ == "__main__":
    import uvicorn

    uvicorn.run("cobalt_fast_api:app", host="0.0.0.0", port=8000, reload=False)
