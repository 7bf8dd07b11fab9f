"""Stage-2 cleaning + feature engineering (reference: src/data_preprocessing/feature_engineering.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from cobalt_smart_lender_ai_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["features"] + sys.argv[1:]))
