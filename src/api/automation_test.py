"""Automation check (reference: src/api/automation_test.py): write a 10-row label-free sample of the
tree dataset, score it with the deployed model, and print predictions next to the true labels."""
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import pandas as pd  # noqa: E402

from cobalt_smart_lender_ai_amd.config import ServeConfig  # noqa: E402
from cobalt_smart_lender_ai_amd.serve.app import load_model  # noqa: E402
from cobalt_smart_lender_ai_amd.serve.automation import make_sample, score_file  # noqa: E402

original = Path(os.environ.get("AUTOMATION_SOURCE", "../../data/2-intermediate/df_out_dsif3_tree.csv"))
inp = Path("../../data/data-input-automation/test_sample.csv")
out = Path("../../data/3-outputs/latest_output.csv")

if __name__ == "__main__":
    y = make_sample(pd.read_csv(original), inp)
    print(f"Test input saved to: {inp}")
    cfg = ServeConfig(model_path=os.environ.get("MODEL_PATH", "models/xgb_model_tree.pkl"))
    res = score_file(load_model(cfg), inp, out)
    print(pd.DataFrame({"actual": y, "prob_default": res["prob_default"]}))
    print(f"Predictions written to: {out}")
