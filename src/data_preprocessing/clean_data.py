"""Stage-1 cleaning (reference: src/data_preprocessing/clean_data.py).

Usage:  python clean_data.py        # sample dataset
        python clean_data.py full   # full dataset
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from cobalt_smart_lender_ai_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["clean"] + (["--full"] if len(sys.argv) > 1 and sys.argv[1] == "full" else [])))
